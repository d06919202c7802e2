#!/bin/bash
# All four workloads on one GPU (short runs, no CPU baseline), JSON lines -> gpurun_out/TAG/
TAG=${1:-benchall}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for w in c5 c3 c4 c2; do
  timeout -k 10 400 python3 -u $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/$w.json 2> $OUT/$w.err
  rc=$?; echo "$w rc=$rc $(cut -c1-400 $OUT/$w.json)"
  [ $rc -ne 0 ] && { tail -5 $OUT/$w.err; exit $rc; }
done
exit 0
