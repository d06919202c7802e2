# C5 N = 8 ceiling on this build: (1) the giant basin packed for its 3-rank split group (768 workgroups) routed alone
# on one GPU as three generations; (2) the five non-split ranks' shards of the split plan, each alone
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_split; mkdir -p $O
WORLD_SIZE=8 RANK=0 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_TARGET_BLOCKS=768 timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 \
  --no-cpu-baseline --dropin-steps 0 > $O/split_predict_c5_k3.json 2> $O/split_predict_c5_k3.err || { tail -3 $O/split_predict_c5_k3.err; exit 1; }
echo "giant basin, 768 blocks: $(python3 -c "import json; d=json.loads(open('$O/split_predict_c5_k3.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config']['reaches'], d['config']['blocks_rank0'], d['config']['generations_rank0'], {k: round(v['kernel_ms'],2) for k,v in d['kernels'].items()})")"
EVTAG=r06_split bash $R/tools/ev_shards.sh 2>&1 | grep "^c5"
