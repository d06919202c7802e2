#!/bin/bash
# Per-wave phase profile (DDR_PHASE_PROF=1 variant) of the current build at light load: c3s8 and c5s8r5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_phase2}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
L="DDR_LIB=$R/ddr_amd/lib/libddr_mc_phase.so"
env $L WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 timeout -k 10 300 python3 -u $R/bench.py $B --workload c3 --steps 2 --warmup 1 \
  --block-profile $O/c3s8_blocks.json > $O/c3s8.json 2> $O/c3s8.err || { tail -5 $O/c3s8.err; exit 1; }
env $L WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 timeout -k 10 300 python3 -u $R/bench.py $B --steps 2 --warmup 1 \
  --block-profile $O/c5s8r5_blocks.json > $O/c5s8r5.json 2> $O/c5s8r5.err || { tail -5 $O/c5s8r5.err; exit 1; }
grep -h profile $O/*.err
