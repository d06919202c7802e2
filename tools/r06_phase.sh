# phase profile (-DDDR_PHASE_PROF=1 build) of the C3 8-way rank-1 shard alone: per-wave phase cycles + block profile
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06_phase; mkdir -p $OUT
WORLD_SIZE=8 RANK=1 DDR_BENCH_ALONE=1 DDR_LIB=$PWD/ddr_amd/lib/libddr_mc_phase.so timeout -k 10 300 python3 bench.py --workload c3 \
  --steps 2 --warmup 1 --no-cpu-baseline --block-profile $OUT/c3s8.json > $OUT/c3s8.log 2>&1 || { tail -5 $OUT/c3s8.log; exit 1; }
grep profile $OUT/c3s8.log
