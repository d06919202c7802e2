#!/bin/bash
# Round 4 A/B 11: double-buffered x slots for the faithful forward at KR = 4 where the LDS allows
# (DDR_FWD_DBL4=0 = the two-barrier tick): the route / steady / fastmath / fullsize GPU tests, C5 and C3.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab11
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py $R/tests/test_gpu_fastmath.py \
  $R/tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
run c5_dbl4 python3 -u $R/bench.py $B --steps 3 --warmup 1
run c5_nodbl4 DDR_FWD_DBL4=0 python3 -u $R/bench.py $B --steps 3 --warmup 1
run c5_dbl4b python3 -u $R/bench.py $B --steps 3 --warmup 1
run c3 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
