#!/bin/bash
# A/B of library variants on C5 (short runs): VARIANT:FLAGS pairs, e.g. base: fnp2:--fast-math
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ab}
mkdir -p $OUT
for spec in "$@"; do
  v=${spec%%:*}; fl=${spec#*:}
  lib=$R/ddr_amd/lib/libddr_mc_$v.so; [ "$v" = base ] && lib=$R/ddr_amd/lib/libddr_mc.so
  DDR_MC_LIB=$lib timeout -k 10 200 python $R/bench.py --workload ${WL:-c5} --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 $fl > $OUT/$v$fl.log 2>&1 || { echo "$spec failed"; tail -3 $OUT/$v$fl.log; exit 1; }
  echo "$spec" $(grep '^{' $OUT/$v$fl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v['kernel_ms'],2) for k, v in d['kernels'].items()})")
done
