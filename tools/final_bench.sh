#!/bin/bash
# Second half of the round-end evidence (after tools/check_round.sh): smoke, every workload, the
# default bench line (with the CPU baseline) and its rocprofv3 kernel-trace summary.
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash $R/tools/bench_all.sh ${TAG}_bench || exit $?
( time timeout -k 10 600 python $R/bench.py ) > $OUT/bench_default.log 2>&1 || { tail -5 $OUT/bench_default.log; exit 1; }
grep '^{' $OUT/bench_default.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/rocprof_bench.log 2>&1 || exit $?
python3 $R/tools/kstats.py $(find $OUT/prof -name "*.db") > $OUT/kernel_stats_c5.txt 2>&1
find $OUT/prof -name "*_stats.csv" -exec cp {} $OUT/ \;
head -8 $OUT/kernel_stats_c5.txt | cut -c1-130
find $OUT/prof -name "*.db" -delete
exit 0
