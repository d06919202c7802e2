#!/bin/bash
# Round 4 A/B 27: wave priority = slices the wave still has to run (sp2) against priority = 3 - slice index
# (the default build): C5 (two runs each, interleaved) and C3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab27}
mkdir -p $O
B="--no-cpu-baseline --dropin-steps 0"
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
L2="DDR_LIB=$R/ddr_amd/lib/libddr_mc_sp2.so"
run c5_def_a python3 -u $R/bench.py $B --steps 2 --warmup 1
run c5_sp2_a $L2 python3 -u $R/bench.py $B --steps 2 --warmup 1
run c3_def python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
run c3_sp2 $L2 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
run c5_def_b python3 -u $R/bench.py $B --steps 2 --warmup 1
run c5_sp2_b $L2 python3 -u $R/bench.py $B --steps 2 --warmup 1
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
