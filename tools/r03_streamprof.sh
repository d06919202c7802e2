#!/bin/bash
# Kernel trace of the C3 training stream (which device-build kernels run between training steps) and the
# full-size C2 test with the faithful / fast arithmetic.
TAG=${1:-r03_streamprof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k c2_full --timeout 240 --timeout-method thread > $OUT/c2test.log 2>&1
rc=$?; tail -2 $OUT/c2test.log; [ $rc -ne 0 ] && { grep -E "^E |Error" $OUT/c2test.log | head; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --stream 8 > $OUT/stream.log 2>&1 || exit 1
python3 $R/tools/kstats.py $(find $OUT/prof -name "*.db") > $OUT/kernel_stats_stream.txt 2>&1
head -40 $OUT/kernel_stats_stream.txt | cut -c1-130
find $OUT/prof -name "*.db" -delete
exit 0
