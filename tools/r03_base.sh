#!/bin/bash
# Round-3 baseline on the current build: C3 fixed + training stream, C5 default (no CPU baseline).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_base
mkdir -p $OUT
timeout -k 10 400 python3 -u $R/bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --stream 10 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
cut -c1-300 $OUT/c3.json
timeout -k 10 400 python3 -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
cut -c1-300 $OUT/c5.json
