#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_stream3
mkdir -p $OUT
cd $R
DDR_DEBUG_BUILD_TIMING=1 timeout -k 10 400 python3 -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --stream 12 --stream-workers 1 --stream-depth 4 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
grep devbuild $OUT/c3.err | tail -14
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read()); s=d['training_stream']; print('fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'wait', round(s['graph_wait_ms_mean'],2)); print([(b['reaches'], b['generations'], b['graph_wait_ms'], b['step_gpu_ms']) for b in s['batches']])"
