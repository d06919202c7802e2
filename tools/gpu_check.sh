#!/bin/bash
# GPU-side check: parity tests, then one bench line (no CPU baseline) under a kernel trace.
# Usage: bash tools/gpu_check.sh [tag]
TAG=${1:-check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests -v -m gpu -x --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|PASSED|^E  " $OUT/pytest.log | cut -c1-300 | head -60
[ $rc -ne 0 ] && { echo "PYTEST FAILED rc=$rc"; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?
grep '^{' $OUT/bench.log | cut -c1-600
python3 $R/tools/kstats.py $(find $OUT/prof -name "*.db") > $OUT/kernel_stats.txt 2>&1
head -8 $OUT/kernel_stats.txt
find $OUT/prof -name "*.db" -delete
exit $rc
