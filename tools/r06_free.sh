# packer: free pieces (single-piece basins) filling any height class (DDR_PACK_FREE=1, the build's default) against
# the height-class packing of every piece (DDR_PACK_FREE=0); bench lines' own HIP-event kernel times
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_free; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 $EXTRA \
    > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -3 $O/$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config'].get('blocks_rank0'), {k: round(v['kernel_ms'],2) for k,v in d['kernels'].items()})")"
}
for fr in 0 1 0 1; do
  run c5_f$fr DDR_PACK_FREE=$fr || exit 1
done
for fr in 0 1; do
  EXTRA="--workload c4" run c4_f$fr DDR_PACK_FREE=$fr || exit 1
  EXTRA="--workload c3" run c3_f$fr DDR_PACK_FREE=$fr || exit 1
  EXTRA="--workload c3" run c3s8_f$fr DDR_PACK_FREE=$fr WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 || exit 1
  EXTRA="--reaches 100000 --basins 400" run light_f$fr DDR_PACK_FREE=$fr || exit 1
done
