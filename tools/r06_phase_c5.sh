# phase profile (-DDDR_PHASE_PROF=1 build) of the C5 step (KR = 4): per-wave phase cycles + block profile
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06_phase_c5; mkdir -p $OUT
DDR_LIB=$PWD/ddr_amd/lib/libddr_mc_phase.so timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
  --block-profile $OUT/c5.json > $OUT/c5.log 2>&1 || { tail -5 $OUT/c5.log; exit 1; }
grep profile $OUT/c5.log
