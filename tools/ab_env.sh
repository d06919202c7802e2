#!/bin/bash
# A/B of packer environment knobs: WLS="c3 c3s8" bash tools/ab_env.sh "DDR_PACK_FAC_POW=1" "DDR_PACK_FAC_POW=0.5" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abe}
mkdir -p $OUT
for size in ${WLS:-c3}; do
  for e in "$@"; do
    envs="$e"; fl=""
    case $size in
      light) fl="--reaches 100000 --basins 400";;
      c5) fl="";;
      c3s8) fl="--workload c3"; envs="$envs WORLD_SIZE=8 RANK=1 DDR_BENCH_ALONE=1";;
      c5s8) fl=""; envs="$envs WORLD_SIZE=8 RANK=0 DDR_BENCH_ALONE=1";;
      *) fl="--workload $size";;
    esac
    tag=$(echo "$e" | tr '= ' '__')
    env $envs timeout -k 10 300 python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 $fl > $OUT/${tag}_$size.log 2>&1 || { echo "$e $size failed"; tail -3 $OUT/${tag}_$size.log; exit 1; }
    echo "$e $size" $(grep '^{' $OUT/${tag}_$size.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v['kernel_ms'],2) for k, v in d['kernels'].items()}, d['config']['blocks_rank0'], d['config']['cut_edges_rank0'])")
  done
done
