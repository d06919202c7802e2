R=$GRAFT_REPO_ROOT
for v in base scap50; do
  lib=$R/ddr_amd/lib/libddr_mc_$v.so; [ $v = base ] && lib=$R/ddr_amd/lib/libddr_mc.so
  for r in 0 1 2 3 4 5 6 7; do
    WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_MC_LIB=$lib timeout -k 10 200 python3 $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $R/gpurun_out/ab_scap/${v}_r$r.json 2>/dev/null || { echo "$v $r failed"; exit 1; }
    echo "$v r$r $(python3 -c "import json; d=json.loads(open('$R/gpurun_out/ab_scap/${v}_r$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), {k: round(v['kernel_ms'],2) for k,v in d['kernels'].items()}, d['config']['blocks_rank0'], d['config']['cut_edges_rank0'])")"
  done
done
