#!/bin/bash
# Kernel-time A/B of library variants under rocprofv3 (one short bench per variant).
# Usage: bash tools/exp_kernels.sh TAG v1 v2 ...   ("base" = ddr_amd/lib/libddr_mc.so)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then unset DDR_LIB; else export DDR_LIB=$R/ddr_amd/lib/libddr_mc_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$v.log 2>&1 || exit $?
  echo "== $v $(grep '^{' $OUT/$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],1))')"
  python3 $R/tools/kstats.py $(find $OUT/$v -name "*.db") | sed -n 3,7p | cut -c1-110
  find $OUT/$v -name "*.db" -delete
done
