#!/bin/bash
# Storer waves for light forward blocks: GPU suite (incl. the bitwise storer test), then A/B against the
# compute-wave stores of the same build (DDR_NO_STORER=1).
TAG=${1:-r03_storer}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TAG=$TAG/ab WLS="c2 c3s8 light c2" bash tools/ab_env.sh DDR_NO_STORER=0 DDR_NO_STORER=1 || exit 1
exit 0
