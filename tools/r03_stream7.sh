#!/bin/bash
# Device-builder tests, then the C3 training stream with the benched arithmetic (and its kernel trace).
TAG=${1:-r03_stream7}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_devgraph.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --stream 12 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); s=d['training_stream']; print('c3 fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'gpu', round(s['step_gpu_ms_mean'],2), 'between', round(s['between_steps_ms'],2), 'ratio', round(s['stream_over_gpu_step'],3)); print([(b['reaches'], b['generations'], b['step_gpu_ms']) for b in s['batches']])"
exit 0
