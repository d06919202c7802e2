#!/bin/bash
# Round 4 A/B 21: light-load block clamp in the packer (no block above half a workgroup while the capacity
# is there; DDR_PACK_NO_LIGHT_CLAMP=1 = previous) and unweighted packing (DDR_PACK_FAC_POW=0), on the C3
# 8-way shards of rank 3 (five 700-reach blocks before) and rank 1 (all blocks <= 512), two runs each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab21}
mkdir -p $O
B="--no-cpu-baseline --dropin-steps 0 --workload c3 --steps 3 --warmup 1"
run() { local tag=$1; shift; timeout -k 10 300 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
for i in a b; do
  run r3_noclamp_$i DDR_PACK_NO_LIGHT_CLAMP=1 WORLD_SIZE=8 RANK=3 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
  run r3_clamp_$i WORLD_SIZE=8 RANK=3 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
  run r3_pow0_$i DDR_PACK_FAC_POW=0 WORLD_SIZE=8 RANK=3 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
  run r1_clamp_$i WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
  run r1_pow0_$i DDR_PACK_FAC_POW=0 WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B
done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k, d['config']['blocks_rank0'], d['config']['cut_edges_rank0'])"; done
