#!/bin/bash
# A/B of machine-scheduler strategies for the routing kernels (lib variants built by tools/build_variant.sh)
TAG=${1:-r03_sched}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=$TAG WLS="c5 c2 c3s8" bash tools/ab_wl.sh base ilp postra mc
