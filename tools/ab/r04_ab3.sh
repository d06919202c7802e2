#!/bin/bash
# Round 4 A/B 3: the light-load packing quantum as the default (C3 8-way shard, C2, a C5 8-way shard), a
# backward import chunk of 4 ticks (variant library) against 8, and PMC counters of the C3 8-way shard.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab3
mkdir -p $O
export TMPDIR=/tmp
S8="WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1"
B="--no-cpu-baseline --dropin-steps 0"
run() { local tag=$1; shift; timeout -k 10 300 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
CB4="DDR_LIB=$R/ddr_amd/lib/libddr_mc_cb4.so"
run c3s8 $S8 python3 -u $R/bench.py --workload c3 $B --steps 3 --warmup 1
run c3s8_cb4 $S8 $CB4 python3 -u $R/bench.py --workload c3 $B --steps 3 --warmup 1
run c2 python3 -u $R/bench.py --workload c2 $B --steps 3 --warmup 1
run c2_noq DDR_PACK_QUANT=1 python3 -u $R/bench.py --workload c2 $B --steps 3 --warmup 1
run c5s8r5 WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 python3 -u $R/bench.py $B --steps 2 --warmup 1
run c5s8r5_noq WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 DDR_PACK_QUANT=1 python3 -u $R/bench.py $B --steps 2 --warmup 1
run c3_cb4 $CB4 python3 -u $R/bench.py --workload c3 $B --steps 3 --warmup 1
run c5_cb4 $CB4 python3 -u $R/bench.py $B --steps 2 --warmup 1
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
cd /tmp
env $S8 bash $R/tools/pmc.sh r04_ab3/pmc_c3s8 --workload c3 > $O/pmc.log 2>&1; tail -60 $O/pmc.log
