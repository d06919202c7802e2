#!/bin/bash
# Default bench line (as the driver runs it) + HBM traffic PMC passes of the routing kernels.
# Usage: bash tools/full_bench.sh TAG
TAG=${1:-full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
( time timeout -k 10 600 python $R/bench.py ) > $OUT/bench_default.log 2>&1 || exit $?
grep '^{' $OUT/bench_default.log | cut -c1-2000
tail -4 $OUT/bench_default.log
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/p3 -o run -- python3 $R/bench.py $ARGS > $OUT/p3.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/p4 -o run -- python3 $R/bench.py $ARGS > $OUT/p4.log 2>&1 || exit $?
python3 $R/tools/pmc_report.py $OUT > $OUT/report.txt 2>&1
cat $OUT/report.txt
find $OUT -name "*.db" -delete
