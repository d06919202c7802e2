#!/bin/bash
# Light-load diagnosis and first A/B of round 4 (C3 8-way shard = rank 1 of 8 alone; C5 one GPU):
# r03 library baseline, the r03 kernels' per-wave phase profile (DDR_PHASE_PROF=1 variant), a kernel
# trace of the shard's step, the routing GPU tests on the new build, the new build's lines, and the
# drop-in dmc() breakdown at C5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_phase
mkdir -p $O
export TMPDIR=/tmp
S8="WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1"
B="--workload c3 --no-cpu-baseline --dropin-steps 0"
L03="DDR_LIB=$R/ddr_amd/lib/libddr_mc_r03.so"
env $S8 $L03 timeout -k 10 240 python3 -u $R/bench.py $B --steps 3 --warmup 1 > $O/c3s8_r03.json 2> $O/c3s8_r03.err || exit 1
env $S8 DDR_LIB=$R/ddr_amd/lib/libddr_mc_phase.so timeout -k 10 240 python3 -u $R/bench.py $B --steps 2 --warmup 1 \
  --block-profile $O/c3s8_blocks.json > $O/c3s8_phase.json 2> $O/c3s8_phase.err || exit 1
(cd /tmp && env $S8 $L03 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c3s8_trace -o run -- python3 $R/bench.py $B --steps 3 --warmup 1 > $O/c3s8_trace.log 2>&1) || exit 1
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_steady.py $R/tests/test_gpu_route.py -x -q --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
env $S8 timeout -k 10 240 python3 -u $R/bench.py $B --steps 3 --warmup 1 > $O/c3s8_new.json 2> $O/c3s8_new.err || exit 1
env $S8 DDR_PACK_QUANT=256 timeout -k 10 240 python3 -u $R/bench.py $B --steps 3 --warmup 1 > $O/c3s8_new_q256.json 2> $O/c3s8_new_q256.err || exit 1
timeout -k 10 300 python3 -u $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $O/c5_new.json 2> $O/c5_new.err || exit 1
env $L03 timeout -k 10 300 python3 -u $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $O/c5_r03.json 2> $O/c5_r03.err || exit 1
timeout -k 10 400 python3 -u $R/tools/dropin_breakdown.py > $O/dropin.json 2> $O/dropin.err || exit 1
grep -h profile $O/*.err
find $O -name "*.db" -delete
