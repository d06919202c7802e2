# depth-aware basin assignment (distributed.shard_network / split.plan_ranks with steps = T): every shard alone on one GPU
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_shard; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" LOCAL_RANK=0 DDR_BENCH_ALONE=1 timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 $EXTRA \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -3 $O/$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config']['reaches'], {k: round(v['kernel_ms'],2) for k,v in d['kernels'].items()})")"
}
run n2_r0 WORLD_SIZE=2 RANK=0 && run n2_r1 WORLD_SIZE=2 RANK=1 &&
run n4_r2 WORLD_SIZE=4 RANK=2 DDR_BENCH_SPLIT_PLAN=1 && run n4_r3 WORLD_SIZE=4 RANK=3 DDR_BENCH_SPLIT_PLAN=1 &&
for r in 3 4 5 6 7; do run n8_r$r WORLD_SIZE=8 RANK=$r DDR_BENCH_SPLIT_PLAN=1 || exit 1; done &&
bash $R/tools/scale_alone.sh c3 "1 8" > $O/scale_c3.log 2>&1 && cat $O/scale_c3.log && cp $R/gpurun_out/scale_c3/summary.json $O/scale_c3_summary.json
