#!/bin/bash
# Bench run with the per-workgroup launch profile: gpurun_out/$1/{bench.log,blocks.json}
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 300 python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --block-profile $R/gpurun_out/$TAG/blocks.json > $R/gpurun_out/$TAG/bench.log 2>&1
rc=$?
grep -E '^\{|profile' $R/gpurun_out/$TAG/bench.log | cut -c1-900
exit $rc
