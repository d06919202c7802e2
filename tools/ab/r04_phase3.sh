#!/bin/bash
# Per-wave phase profile (DDR_PHASE_PROF=1 variant) of the final round-4 kernels at full load: C5 and C3 on one GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_phase3}
mkdir -p $O
B="--no-cpu-baseline --dropin-steps 0"
L="DDR_LIB=$R/ddr_amd/lib/libddr_mc_phase.so"
env $L timeout -k 10 400 python3 -u $R/bench.py $B --steps 2 --warmup 1 --block-profile $O/c5_blocks.json > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
env $L timeout -k 10 400 python3 -u $R/bench.py $B --workload c3 --steps 2 --warmup 1 --block-profile $O/c3_blocks.json > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
grep -h profile $O/c5.err $O/c3.err
