#!/bin/bash
# q' gather tile height (steps per workgroup: LDS per workgroup and so workgroups per CU): kernel times.
TAG=${1:-r03_gather}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/exp_kernels.sh $TAG base xcd xcdg4 g4 || exit 1
exit 0
