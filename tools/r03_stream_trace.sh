#!/bin/bash
# HIP API trace of the C3 training stream: which host calls block between steps.
TAG=${1:-r03_trace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --hip-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --stream 8 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
find $OUT/prof -name "*hip_api_stats.csv" -exec cp {} $OUT/hip_api_stats.csv \;
find $OUT/prof -name "*hip_api_trace.csv" -exec cp {} $OUT/hip_api_trace.csv \;
ls -la $OUT/prof/*/* 2>/dev/null | head
head -30 $OUT/hip_api_stats.csv
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read()); s=d['training_stream']; print('stream', round(s['ms_per_step'],2), 'wait', round(s['graph_wait_ms_mean'],2)); print([(b['reaches'], b['graph_wait_ms'], b['step_gpu_ms']) for b in s['batches']])"
gzip -f $OUT/hip_api_trace.csv
find $OUT/prof -name "*.db" -delete
