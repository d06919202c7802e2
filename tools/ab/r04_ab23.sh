#!/bin/bash
# Round 4 A/B 23 (experiment): chain-aware split -- reaches on paths of >= DDR_SPLIT_CHAIN_L reaches split at
# DDR_SPLIT_CHAIN_CAP -- on the C3 8-way shards of ranks 1 and 3, two runs each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab23}
mkdir -p $O
B="--no-cpu-baseline --dropin-steps 0 --workload c3 --steps 3 --warmup 1"
run() { local tag=$1; shift; timeout -k 10 300 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
for i in a b; do
  for r in 1 3; do
    run r${r}_L0_$i WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
    run r${r}_L300_$i DDR_SPLIT_CHAIN_L=300 WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
    run r${r}_L400_$i DDR_SPLIT_CHAIN_L=400 WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
    run r${r}_L300c192_$i DDR_SPLIT_CHAIN_L=300 DDR_SPLIT_CHAIN_CAP=192 WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
  done
done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k, d['config']['blocks_rank0'], d['config']['cut_edges_rank0'])"; done
