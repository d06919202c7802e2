#!/bin/bash
# Round 4 A/B 15: backward import waves (KR = 1 light blocks: the upper half's idle waves run the cut-out
# imports, requested DDR_BWD_IMP_EARLY ticks before the chunk boundary).  Default build = imp waves, E = 2;
# variants: iw0 (compute-wave imports, as before), ie0 / ie4 / ie6 (lead 0 / 4 / 6 ticks).
# Route / split GPU tests on the default, then c3s8 and c5s8r5 lines for each library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab15}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
for v in def iw0 ie0 ie4 ie6; do
  L=""; [ $v != def ] && L="DDR_LIB=$R/ddr_amd/lib/libddr_mc_$v.so"
  run c3s8_$v $L WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
  run c5s8r5_$v $L WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 python3 -u $R/bench.py $B --steps 2 --warmup 1
done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
