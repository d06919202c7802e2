#!/bin/bash
# Round-3 re-entry baseline on the current build: full -m gpu suite, C3 fixed + training stream
# (inline device builds), C5 default line. Usage: bash tools/r03_base2.sh [TAG]
TAG=${1:-r03_base2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|^E  " $OUT/pytest.log | cut -c1-300 | tail -8; [ $rc -ne 0 ] && exit $rc
DDR_DEBUG_BUILD_TIMING=1 timeout -k 10 400 python3 -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --stream 12 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read()); s=d['training_stream']; print('c3 fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'wait', round(s['graph_wait_ms_mean'],2)); print([(b['reaches'], b['generations'], b['graph_wait_ms'], b['step_gpu_ms']) for b in s['batches']])"
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
cut -c1-700 $OUT/c5.json
