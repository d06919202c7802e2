#!/bin/bash
# A/B of one library under environment settings: ENVS="A=0|A=1" WLS="c5" bash tools/ab_env.sh   (TAG: output dir)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abe}
mkdir -p $OUT
IFS='|' read -ra SETS <<< "${ENVS:-X=0}"
for size in ${WLS:-c5}; do
  for rep in $(seq 1 ${REPS:-1}); do
    for e in "${SETS[@]}"; do
      case $size in
        light) fl="--reaches 100000 --basins 400";;
        c5) fl="";;
        c3s8) fl="--workload c3"; e="$e WORLD_SIZE=8 RANK=1 DDR_BENCH_ALONE=1";;
        *) fl="--workload $size";;
      esac
      tag=$(echo "$e" | tr ' =' '__')
      env $e timeout -k 10 300 python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 $fl > $OUT/${tag}_$size.log 2>&1 || { echo "$e $size failed"; tail -3 $OUT/${tag}_$size.log; exit 1; }
      echo "$e $size" $(grep '^{' $OUT/${tag}_$size.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v['kernel_ms'],2) for k, v in d['kernels'].items()})")
    done
  done
done
