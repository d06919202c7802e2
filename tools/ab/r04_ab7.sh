#!/bin/bash
# Round 4 A/B 7: DPP lane mapping check; geometry statistics without LDS-crossbar shuffles (wave_rol
# neighbour, ballot counts, DPP fp64 wave sum, readlane order statistics) at C4 + its golden tests;
# per-wave phase profiles of the current routing kernels (DDR_PHASE_PROF=1 variant) at c3s8 and C5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab7
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 60 $R/build/dpp_check > $O/dpp_check.txt 2>&1; rc=$?; cat $O/dpp_check.txt; [ $rc = 0 ] || exit 1
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_objectives.py $R/tests/test_gpu_fullsize.py -x -q --timeout 300 \
  --timeout-method thread -k "geo or stat or long" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
(timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4 -o run -- python3 $R/bench.py $B --steps 3 --warmup 1 --workload c4 \
  > $O/c4.json 2> $O/c4.err) || { echo "c4 failed"; tail -5 $O/c4.err; exit 1; }
python3 $R/tools/kstats.py $(find $O/c4 -name "*.db") --limit 8 > $O/c4_kstats.txt; find $O/c4 -name "*.db" -delete
grep geometry $O/c4_kstats.txt
PH="DDR_LIB=$R/ddr_amd/lib/libddr_mc_phase.so"
env WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 $PH timeout -k 10 300 python3 -u $R/bench.py $B --workload c3 --steps 2 \
  --warmup 1 --block-profile $O/c3s8_blocks.json > $O/c3s8_phase.json 2> $O/c3s8_phase.err || { tail -5 $O/c3s8_phase.err; exit 1; }
grep profile $O/c3s8_phase.err
env $PH timeout -k 10 400 python3 -u $R/bench.py $B --steps 1 --warmup 1 --block-profile $O/c5_blocks.json \
  > $O/c5_phase.json 2> $O/c5_phase.err || { tail -5 $O/c5_phase.err; exit 1; }
grep profile $O/c5_phase.err
