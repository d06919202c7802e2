#!/bin/bash
# Round 4 A/B 26: wave priority by remaining slices (DDR_SLICE_PRIO=1: a wave at slice k of KR runs at priority
# KR - 1 - k, 3 at the top of the tick) against the SIMD arbiter's age order alone (sp0).  Route / steady /
# fullsize GPU tests on the default, then C5 (two runs), C3 and C4 kernel times for each library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab26}
mkdir -p $O
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py $R/tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
for v in def sp0; do
  L=""; [ $v != def ] && L="DDR_LIB=$R/ddr_amd/lib/libddr_mc_$v.so"
  run c5_${v}_a $L python3 -u $R/bench.py $B --steps 2 --warmup 1
  run c3_$v $L python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
  run c4_$v $L python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c4
  run c5_${v}_b $L python3 -u $R/bench.py $B --steps 2 --warmup 1
done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
