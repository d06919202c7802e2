#!/bin/bash
# A/B of library variants over workloads: WLS="light c5 c3 c2" bash tools/ab_wl.sh base variant ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abw}
mkdir -p $OUT
for size in ${WLS:-light c5}; do
  for v in "$@"; do
    lib=$R/ddr_amd/lib/libddr_mc_$v.so; [ "$v" = base ] && lib=$R/ddr_amd/lib/libddr_mc.so
    envs=""
    case $size in
      light) fl="--reaches 100000 --basins 400";;
      c5) fl="";;
      c3s8) fl="--workload c3 $C3FL"; envs="WORLD_SIZE=8 RANK=1 DDR_BENCH_ALONE=1";;  # one 8-way C3 shard alone
      c5s8) fl=""; envs="WORLD_SIZE=8 RANK=0 DDR_BENCH_ALONE=1";;               # the giant-basin C5 shard
      c3) fl="--workload c3 $C3FL";;
      *) fl="--workload $size";;
    esac
    env $envs DDR_MC_LIB=$lib timeout -k 10 300 python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps ${DROPIN:-0} $fl > $OUT/${v}_$size.log 2>&1 || { echo "$v $size failed"; tail -3 $OUT/${v}_$size.log; exit 1; }
    echo "$v $size" $(grep '^{' $OUT/${v}_$size.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v['kernel_ms'],2) for k, v in d['kernels'].items()}, d.get('dropin_dmc', {}).get('route_timestep_ms'))")
  done
done
