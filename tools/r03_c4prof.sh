#!/bin/bash
# Kernel-trace summary of C4 (forward + the 365-day geometry pipeline) and C2.
TAG=${1:-r03_c4prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for w in c4 c2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o run -- python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/rocprof_$w.log 2>&1 || exit 1
  python3 $R/tools/kstats.py $(find $OUT/prof_$w -name "*.db") > $OUT/kernel_stats_$w.txt 2>&1
  head -10 $OUT/kernel_stats_$w.txt | cut -c1-130
  find $OUT/prof_$w -name "*.db" -delete
done
# the ranks outside C5's split group at N = 8 (shards of the split plan), each alone
for r in 3 4 5 6 7; do
  WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 timeout -k 10 300 python3 $R/bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --dropin-steps 0 > $OUT/splitplan_n8_r$r.json 2> $OUT/splitplan_n8_r$r.err || { tail -3 $OUT/splitplan_n8_r$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/splitplan_n8_r$r.json').read().strip().splitlines()[-1]); print('rank $r', d['config']['reaches'], round(d['ms_per_step'],2))"
done
# C4 counters with the big forward launch separated from the 365-day accumulation launch
cd $R
HASH=$(python3 -c "import sys; sys.path.insert(0, '$R'); from ddr_amd import _lib; print(_lib.load().ddr_version().decode().split()[-1])")
KEEP_DB=1 bash tools/pmc.sh $TAG/pmc_c4 --workload c4 > $OUT/pmc_c4.log 2>&1 || { tail -20 $OUT/pmc_c4.log; exit 1; }
PMC_JSON_DIR=$OUT python3 tools/pmc_to_json.py $OUT/pmc_c4 c4 $HASH 8760 350000 profiles/r03/pmc_c4 | cut -c1-400
find $OUT -name "*.db" -delete
exit 0
