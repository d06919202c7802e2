#!/bin/bash
# Backward: v_edge opaque per use (no hoisted 64-bit row offsets spilled to scratch at KR = 4): A/B.
TAG=${1:-r03_opq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=$TAG WLS="c5 c3 light c5" bash tools/ab_wl.sh base opq || exit 1
exit 0
