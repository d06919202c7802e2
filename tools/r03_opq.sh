#!/bin/bash
# Backward: v_edge opaque per use (no hoisted 64-bit row offsets spilled to scratch at KR = 4): A/B.
# Build first: git apply tools/patches_bwd_opaque_edge.diff && bash tools/build_variant.sh opq && git checkout ddr_amd/csrc/route.hip
TAG=${1:-r03_opq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=$TAG WLS="c5 c3 light c5" bash tools/ab_wl.sh base opq || exit 1
exit 0
