#!/bin/bash
# Round-4 evidence, part A (one GPU): the -m gpu suite, smoke(), 2-rank rehearsals of the multi-GPU bench
# on the one GPU (gloo; C3 and C5 sharded by basin, and C5 with its largest basin split over both ranks,
# DDR_SPLIT_BASIN=force), all
# workloads, the C3 training stream, the default bench line (with the CPU baseline) and its rocprofv3
# kernel-trace summary.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_pytest.log 2>&1 \
  || { tail -30 $O/gpu_pytest.log; exit 1; }
tail -1 $O/gpu_pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for w in c3 c5; do
  DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 $R/bench.py --workload $w --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
    --dropin-steps 0 > $O/rehearsal_2rank_$w.json 2> $O/rehearsal_2rank_$w.err || { echo "rehearsal $w failed"; tail -5 $O/rehearsal_2rank_$w.err; exit 1; }
  echo "rehearsal $w: $(cut -c1-200 $O/rehearsal_2rank_$w.json)"
done
DDR_SPLIT_BASIN=force DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 $R/bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  --dropin-steps 0 > $O/rehearsal_split_c5.json 2> $O/rehearsal_split_c5.err || { echo "split rehearsal failed"; tail -5 $O/rehearsal_split_c5.err; exit 1; }
echo "split rehearsal: $(cut -c1-200 $O/rehearsal_split_c5.json)"
for w in c3 c4 c2; do
  timeout -k 10 400 python3 -u $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err \
    || { echo "$w failed"; tail -5 $O/bench_$w.err; exit 1; }
done
timeout -k 10 600 python3 -u $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 --stream 12 \
  > $O/bench_c3_stream.json 2> $O/bench_c3_stream.err || { echo "stream failed"; tail -5 $O/bench_c3_stream.err; exit 1; }
( time timeout -k 10 600 python3 -u $R/bench.py ) > $O/bench_default.json 2> $O/bench_default_time.txt \
  || { echo "default bench failed"; tail -5 $O/bench_default_time.txt; exit 1; }
tail -3 $O/bench_default_time.txt
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  --dropin-steps 0 > $O/rocprof_bench.log 2>&1 || { echo "rocprof failed"; tail -5 $O/rocprof_bench.log; exit 1; }
python3 $R/tools/kstats.py $(find $O/prof -name "*.db") > $O/kernel_stats_c5.txt 2>&1
find $O/prof -name "*_stats.csv" -exec cp {} $O/ \;
find $O/prof -name "*.db" -delete
head -6 $O/kernel_stats_c5.txt | cut -c1-130
for f in $O/bench_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), '%.3g' % d['value'], k)"; done
