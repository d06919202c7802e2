# C5 at N = 2 and 4 on one GPU (each shard alone): the current plan (split factor 2: no split below N = 8) against a
# 2-rank split group at N = 4 (factor 1.2: the giant basin packed for 512 workgroups, routed alone = two generations)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_n4; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" LOCAL_RANK=0 DDR_BENCH_ALONE=1 timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -3 $O/$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config']['reaches'], d['config']['blocks_rank0'], {k: round(v['kernel_ms'],2) for k,v in d['kernels'].items()})")"
}
run n2_r0 WORLD_SIZE=2 RANK=0 && run n2_r1 WORLD_SIZE=2 RANK=1 &&
run n4_r0 WORLD_SIZE=4 RANK=0 && run n4_r1 WORLD_SIZE=4 RANK=1 &&
run n4f_group WORLD_SIZE=4 RANK=0 DDR_BENCH_TARGET_BLOCKS=512 &&
run n4f_r2 WORLD_SIZE=4 RANK=2 DDR_BENCH_SPLIT_PLAN=1 DDR_SPLIT_FACTOR=1.2 && run n4f_r3 WORLD_SIZE=4 RANK=3 DDR_BENCH_SPLIT_PLAN=1 DDR_SPLIT_FACTOR=1.2
