#!/bin/bash
# The C3 training stream (new adjacency + device graph build per step), with the host-ahead count.
TAG=${1:-r03_stream8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --stream 12 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); s=d['training_stream']; print('c3 fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'gpu', round(s['step_gpu_ms_mean'],2), 'between', round(s['between_steps_ms'],2), 'ratio', round(s['stream_over_gpu_step'],3), s['host_ahead_steps']); print([(b['reaches'], b['generations'], b['step_gpu_ms'], b['host_ahead']) for b in s['batches']])"
exit 0
