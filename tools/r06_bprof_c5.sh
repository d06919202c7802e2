# per-workgroup launch profile of the C5 step (start / end / tick stamps every 1024 ticks per block)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06_bprof_c5; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 --block-profile $OUT/c5.json > $OUT/c5.log 2>&1 || { tail -5 $OUT/c5.log; exit 1; }
grep -E "profile|^\{" $OUT/c5.log | cut -c1-200
