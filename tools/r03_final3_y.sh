#!/bin/bash
# Final evidence Y: rocprofv3 kernel-trace summaries of all four workloads, strong scaling by shards alone
# (C3, C5 at N = 1 and 8), the split prediction (C5's basin for a 3-rank group alone; the other ranks of the
# split plan alone) and the 2-rank rehearsals.
TAG=${1:-r03_final3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for w in c5 c3 c4 c2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o run -- python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/rocprof_$w.log 2>&1 || exit 1
  python3 $R/tools/kstats.py $(find $OUT/prof_$w -name "*.db") > $OUT/kernel_stats_$w.txt 2>&1
  head -5 $OUT/kernel_stats_$w.txt | cut -c1-130
  find $OUT/prof_$w -name "*.db" -delete
done
cd $R
for w in c3 c5; do
  bash tools/scale_alone.sh $w "1 8" > $OUT/scale_alone_$w.log 2>&1 || { tail -5 $OUT/scale_alone_$w.log; exit 1; }
  cp gpurun_out/scale_$w/summary.json $OUT/scale_alone_$w.json; tail -2 $OUT/scale_alone_$w.log
done
WORLD_SIZE=8 RANK=0 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_TARGET_BLOCKS=768 timeout -k 10 400 python3 bench.py --steps 2 \
  --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/split_predict_c5_k3.json 2> $OUT/split_predict_c5_k3.err || { tail -5 $OUT/split_predict_c5_k3.err; exit 1; }
for r in 3 4 5 6 7; do
  WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --dropin-steps 0 > $OUT/splitplan_n8_r$r.json 2> $OUT/splitplan_n8_r$r.err || { tail -3 $OUT/splitplan_n8_r$r.err; exit 1; }
done
for w in c3 c5; do
  DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --workload $w --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/rehearsal_$w.json 2> $OUT/rehearsal_$w.err
  rc=$?; echo "rehearsal $w rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/rehearsal_$w.err; exit $rc; }
done
DDR_SPLIT_BASIN=force DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $OUT/rehearsal_split_c5.json 2> $OUT/rehearsal_split_c5.err || { tail -5 $OUT/rehearsal_split_c5.err; exit 1; }
echo "split rehearsal ok"
exit 0
