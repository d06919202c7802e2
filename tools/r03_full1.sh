#!/bin/bash
# Full GPU suite on the current build, the C3 stream with inline device builds, and an A/B of the
# previous routing kernels (libddr_mc_prev.so) against the current ones on C5 and C3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_full1
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_objectives.py tests/test_gpu_route.py tests/test_gpu_state.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|error" $OUT/pytest.log | tail -3; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit $rc; }
for b in inline:2 inline:3; do
  bl=${b%%:*}; d=${b#*:}
  DDR_DEBUG_BUILD_TIMING=1 timeout -k 10 400 python3 -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --stream 12 --stream-builder $bl --stream-depth $d > $OUT/c3_$bl$d.json 2> $OUT/c3_$bl$d.err || { tail -5 $OUT/c3_$bl$d.err; exit 1; }
  grep devbuild $OUT/c3_$bl$d.err | tail -2
  python3 -c "import json; d=json.loads(open('$OUT/c3_$bl$d.json').read()); s=d['training_stream']; print('$b fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'wait', round(s['graph_wait_ms_mean'],2)); print([(b['reaches'], b['generations'], b['graph_wait_ms'], b['step_gpu_ms']) for b in s['batches']])"
done
TAG=r03_full1 bash tools/ab_fwd.sh prev: base: prev: base:
WL=c3 TAG=r03_full1 bash tools/ab_fwd.sh prev: base:
