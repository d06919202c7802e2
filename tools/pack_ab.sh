# C5 step time under packer settings (env knobs of graph.cpp): "FAC_POW,QUANT" pairs as arguments
mkdir -p gpurun_out/pk
for cfg in "$@"; do
  fp=${cfg%,*}; q=${cfg#*,}
  DDR_PACK_FAC_POW=$fp DDR_PACK_QUANT=$q timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 > gpurun_out/pk/f${fp}_q$q.log 2>&1 || exit 1
  echo "pow $fp quant $q" $(grep '^{' gpurun_out/pk/f${fp}_q$q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v['kernel_ms'],2) for k, v in d['kernels'].items()}, d['config']['blocks_rank0'])")
done
