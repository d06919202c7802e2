# packer: exponent of the chain-pacing weight ((T + L) / T)^p (DDR_PACK_FAC_POW; the build's 1) at C5
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_facpow; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 $EXTRA \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -3 $O/$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config'].get('blocks_rank0'), {k: round(v['kernel_ms'],2) for k,v in d['kernels'].items()})")"
}
for p in ${PS:-1 1.5 2 3 1 2}; do run c5_p$p DDR_PACK_FAC_POW=$p || exit 1; done
