#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_stream4
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_devgraph.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { tail -40 $OUT/pytest.log; exit $rc; }
for b in inline:2 inline:3 device:4; do
  bl=${b%%:*}; d=${b#*:}
  DDR_DEBUG_BUILD_TIMING=1 timeout -k 10 400 python3 -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --stream 12 --stream-builder $bl --stream-depth $d --stream-workers 1 > $OUT/c3_$bl$d.json 2> $OUT/c3_$bl$d.err || { tail -5 $OUT/c3_$bl$d.err; exit 1; }
  grep devbuild $OUT/c3_$bl$d.err | tail -3
  python3 -c "import json; d=json.loads(open('$OUT/c3_$bl$d.json').read()); s=d['training_stream']; print('$b fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'wait', round(s['graph_wait_ms_mean'],2)); print([(b['reaches'], b['generations'], b['graph_wait_ms'], b['step_gpu_ms']) for b in s['batches']])"
done
