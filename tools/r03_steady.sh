#!/bin/bash
# Steady-tick specialisation of the routing kernels: GPU suite (incl. the bitwise steady/general test),
# then A/B against the previous build (libddr_mc_head.so) and the general path of this build (DDR_NO_STEADY=1).
TAG=${1:-r03_steady}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; exit $rc; }
TAG=$TAG/ab WLS="c5 c2 c3s8 light c5s8 c3" bash tools/ab_wl.sh base head || exit 1
TAG=$TAG/ns WLS="c5 c2 c3s8" bash tools/ab_env.sh DDR_NO_STEADY=1 || exit 1
exit 0
