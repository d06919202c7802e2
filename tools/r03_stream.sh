#!/bin/bash
# Device graph builder in the C3 training stream: isolated build latency, then the stream with each builder.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_stream
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u tools/probe_build.py > $OUT/probe_build.jsonl 2> $OUT/probe_build.err || { tail -5 $OUT/probe_build.err; exit 1; }
cat $OUT/probe_build.jsonl
for b in device host; do
  timeout -k 10 400 python3 -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --stream 12 --stream-builder $b > $OUT/c3_$b.json 2> $OUT/c3_$b.err || { tail -5 $OUT/c3_$b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c3_$b.json').read()); s=d['training_stream']; print('$b fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'wait', round(s['graph_wait_ms_mean'],2)); print([(b['reaches'], b['generations'], b['graph_wait_ms'], b['step_gpu_ms']) for b in s['batches']])"
done
