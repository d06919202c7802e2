#!/bin/bash
# Forward imports requested one chunk ahead (KR <= 2): GPU suite, then A/B against the previous build.
TAG=${1:-r03_prefimp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
TAG=$TAG/ab WLS="c3s8 light c5s8 c3 c3s8 light" bash tools/ab_wl.sh base prev || exit 1
exit 0
