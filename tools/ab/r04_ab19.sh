#!/bin/bash
# Round 4 A/B 19: light-load idle-wave roles on the current build: c3s8 and c5s8r5 with and without the
# storer / import waves (DDR_NO_STORER=1: compute waves store and import), three runs each, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab19}
mkdir -p $O
B="--no-cpu-baseline --dropin-steps 0"
run() { local tag=$1; shift; timeout -k 10 300 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
for i in 1 2 3; do
  run c3s8_on_$i WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
  run c3s8_off_$i DDR_NO_STORER=1 WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
done
run c5s8r5_on WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 python3 -u $R/bench.py $B --steps 2 --warmup 1
run c5s8r5_off DDR_NO_STORER=1 WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 python3 -u $R/bench.py $B --steps 2 --warmup 1
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
