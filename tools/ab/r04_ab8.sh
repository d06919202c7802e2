#!/bin/bash
# Round 4 A/B 8: exhaustive check of the scaling-free IEEE sqrt; the GPU suite on the build with it (forward
# physics, geometry) and with the geometry statistics' valid-slot count (KE) and occupancy-sized persistent
# grid; C4 kernel trace; C5 / C2 / c3s8 lines against the round-3 library; the faithful forward with slice
# pairs in packed halves (DDR_FWD_NP_FAITH=2 variant) at C5 / C3 / C4.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab8
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 120 $R/build/chain_lat 20000 > $O/chain_lat.txt 2>&1 || { echo "chain_lat failed"; exit 1; }
grep -E "faithful|bwd" $O/chain_lat.txt
timeout -k 10 120 $R/build/sqrt_check > $O/sqrt_check.txt 2>&1; rc=$?; cat $O/sqrt_check.txt; [ $rc = 0 ] || exit 1
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
(timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4 -o run -- python3 $R/bench.py $B --steps 3 --warmup 1 --workload c4 \
  > $O/c4.json 2> $O/c4.err) || { echo "c4 failed"; tail -5 $O/c4.err; exit 1; }
python3 $R/tools/kstats.py $(find $O/c4 -name "*.db") --limit 8 > $O/c4_kstats.txt; find $O/c4 -name "*.db" -delete
grep geometry $O/c4_kstats.txt
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
L03="DDR_LIB=$R/ddr_amd/lib/libddr_mc_r03.so"
NP2="DDR_LIB=$R/ddr_amd/lib/libddr_mc_np2.so"
env $NP2 timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py $R/tests/test_gpu_fastmath.py \
  -x -q --timeout 300 --timeout-method thread > $O/pytest_np2.log 2>&1 || { tail -30 $O/pytest_np2.log; exit 1; }
tail -1 $O/pytest_np2.log
run c5 python3 -u $R/bench.py $B --steps 2 --warmup 1
run c5_np2 $NP2 python3 -u $R/bench.py $B --steps 2 --warmup 1
run c3_np2 $NP2 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
run c3 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
run c4_np2 $NP2 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c4
run c5_r03 $L03 python3 -u $R/bench.py $B --steps 2 --warmup 1
run c2 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c2
run c3s8 WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
