#!/bin/bash
# Round-6 evidence on one GPU, in two calls (each well under gpurun's 20-minute limit):
#   bash tools/final_r06.sh a TAG   full -m gpu suite, smoke, PMC passes of the four workloads (tools/pmc_all.sh)
#                                   -> locally: bash tools/pmc_all.sh --json TAG/pmc (profiles/counters/*.json)
#   bash tools/final_r06.sh b TAG   the four bench lines (counters from profiles/counters), the default bench line
#                                   (C5 + CPU baselines) and its rocprofv3 kernel-trace summary, the C3 line with the
#                                   reference-faithful caller (--pnet torch --tail torch) and its 8-way shards, the C3
#                                   training stream, 2-rank gloo rehearsals of C3 and C5 on the one GPU
STAGE=$1; TAG=${2:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ "$STAGE" = a ]; then
  timeout -k 10 900 python -u -m pytest $R/tests -v -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; grep -E "passed|failed|FAILED|^E  " $OUT/pytest.log | cut -c1-300 | tail -6
  [ $rc -ne 0 ] && { echo "PYTEST FAILED rc=$rc"; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  bash $R/tools/pmc_all.sh $TAG/pmc || exit $?
  exit 0
fi
if [ "$STAGE" = b ]; then
  bash $R/tools/bench_all.sh $TAG/bench || exit $?
  timeout -k 10 300 python3 -u $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --pnet torch --tail torch \
    > $OUT/bench_c3_torchcaller.json 2> $OUT/bench_c3_torchcaller.err || { tail -5 $OUT/bench_c3_torchcaller.err; exit 1; }
  cut -c1-300 $OUT/bench_c3_torchcaller.json
  ( time timeout -k 10 600 python $R/bench.py ) > $OUT/bench_default.log 2>&1 || { tail -5 $OUT/bench_default.log; exit 1; }
  grep '^{' $OUT/bench_default.log > $OUT/bench_default.json; cut -c1-400 $OUT/bench_default.json
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/rocprof_bench.log 2>&1 ) || exit 1
  python3 $R/tools/kstats.py $(find $OUT/prof -name "*.db") > $OUT/kernel_stats_c5.txt 2>&1
  find $OUT/prof -name "*_stats.csv" -exec cp {} $OUT/ \;
  head -6 $OUT/kernel_stats_c5.txt | cut -c1-130
  find $OUT/prof -name "*.db" -delete
  bash $R/tools/scale_alone.sh c3 "1 8" --pnet torch --tail torch > $OUT/scale_c3_torchcaller.log 2>&1 || { tail -5 $OUT/scale_c3_torchcaller.log; exit 1; }
  cat $OUT/scale_c3_torchcaller.log; cp $R/gpurun_out/scale_c3/summary.json $OUT/scale_c3_torchcaller_summary.json
  bash $R/tools/scale_alone.sh c3 "1 8" > $OUT/scale_c3.log 2>&1 || { tail -5 $OUT/scale_c3.log; exit 1; }
  cat $OUT/scale_c3.log; cp $R/gpurun_out/scale_c3/summary.json $OUT/scale_c3_summary.json
  timeout -k 10 500 python3 -u $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --stream 12 > $OUT/bench_c3_stream.log 2>&1 || { tail -5 $OUT/bench_c3_stream.log; exit 1; }
  grep '^{' $OUT/bench_c3_stream.log > $OUT/bench_c3_stream.json
  for w in c3 c5; do
    DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29611 $R/bench.py --workload $w --gpus 2 --steps 2 --warmup 1 > $OUT/rehearsal_$w.json 2> $OUT/rehearsal_$w.err
    rc=$?; echo "rehearsal $w rc=$rc $(cut -c1-300 $OUT/rehearsal_$w.json)"
    [ $rc -ne 0 ] && { tail -5 $OUT/rehearsal_$w.err; exit $rc; }
  done
  exit 0
fi
echo "usage: final_r06.sh a|b TAG"; exit 2
