mkdir -p gpurun_out/pk
for fp in 1.0 1.5 2.0 0.5; do
  DDR_PACK_FAC_POW=$fp timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 > gpurun_out/pk/f$fp.log 2>&1 || exit 1
  echo "pow $fp" $(grep '^{' gpurun_out/pk/f$fp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v['kernel_ms'],2) for k, v in d['kernels'].items()}, d['config']['blocks_rank0'])")
done
