#!/bin/bash
# Round 4 A/B 28: light-load issue order (DDR_LIGHT_PRIO: KR = 1 routing waves run their step's physics at
# priority 1, the rest at 0) against the age order alone (lp0): steady / route GPU tests, then c3s8 (two
# runs), c5s8r5 and C2 for each library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab28}
mkdir -p $O
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_steady.py $R/tests/test_gpu_route.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
for v in def lp0; do
  L=""; [ $v != def ] && L="DDR_LIB=$R/ddr_amd/lib/libddr_mc_$v.so"
  run c3s8_${v}_a $L WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
  run c5s8r5_$v $L WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 python3 -u $R/bench.py $B --steps 2 --warmup 1
  run c2_$v $L python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c2
  run c3s8_${v}_b $L WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
