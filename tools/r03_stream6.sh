#!/bin/bash
# Device-builder GPU tests, the C3 training stream (pooled device/pinned blocks), then its HIP API trace.
TAG=${1:-r03_stream6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_devgraph.py tests/test_gpu_route.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { tail -40 $OUT/pytest.log; exit $rc; }
DDR_DEBUG_BUILD_TIMING=1 timeout -k 10 400 python3 -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --stream 12 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read()); s=d['training_stream']; print('c3 fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'wait', round(s['graph_wait_ms_mean'],2)); print([(b['reaches'], b['generations'], b['graph_wait_ms'], b['step_gpu_ms']) for b in s['batches']])"
bash tools/r03_stream_trace.sh ${TAG}_trace
