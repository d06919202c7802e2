#!/bin/bash
# Bench lines of every workload with the counter files of this build in place (roofline.traffic /
# valu_frac filled): C2's counters collected first (per-dispatch selection), then all four workloads and the
# default line.
TAG=${1:-r03_lines}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
HASH=$(python3 -c "import sys; sys.path.insert(0, '$R'); from ddr_amd import _lib; print(_lib.load().ddr_version().decode().split()[-1])")
KEEP_DB=1 bash tools/pmc.sh $TAG/pmc_c2 --workload c2 > $OUT/pmc_c2.log 2>&1 || { tail -20 $OUT/pmc_c2.log; exit 1; }
PMC_JSON_DIR=$OUT python3 tools/pmc_to_json.py $OUT/pmc_c2 c2 $HASH 8760 5000 profiles/r03/pmc_c2 | cut -c1-200
find $OUT -name "*.db" -delete
cp $OUT/c2.json profiles/counters/c2.json
bash tools/bench_all.sh $TAG/bench || exit 1
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2>&1 || { tail -5 $OUT/bench_default.log; exit 1; }
grep '^{' $OUT/bench_default.log | cut -c1-200
exit 0
