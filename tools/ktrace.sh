#!/bin/bash
# Kernel-trace a short bench run per library: gpurun_out/TAG/<lib>_<wl>/ (rocpd db) + <lib>_<wl>.txt (tools/kstats.py).
# Usage: LIBS="cur r05" WLS="c5 c3s8" TAG=kt bash tools/ktrace.sh   (lib "cur" = ddr_amd/lib/libddr_mc.so,
# any other name X = ddr_amd/lib/libddr_mc_X.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-kt}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for wl in ${WLS:-c5}; do
  case $wl in
    c5) fl="";;
    light) fl="--reaches 100000 --basins 400";;
    c3s8) fl="--workload c3";;
    *) fl="--workload $wl";;
  esac
  for lib in ${LIBS:-cur}; do
    if [ "$lib" = cur ]; then L=$R/ddr_amd/lib/libddr_mc.so; else L=$R/ddr_amd/lib/libddr_mc_$lib.so; fi
    if [ "$wl" = c3s8 ]; then export WORLD_SIZE=8 RANK=1 DDR_BENCH_ALONE=1; else unset WORLD_SIZE RANK DDR_BENCH_ALONE; fi
    DDR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${lib}_$wl -o run -- \
      python3 $R/bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --dropin-steps 0 $fl $EXTRA \
      > $OUT/${lib}_$wl.log 2>&1 || { echo "$lib $wl failed"; tail -5 $OUT/${lib}_$wl.log; exit 1; }
    db=$(find $OUT/${lib}_$wl -name "*.db" | head -1)
    python3 $R/tools/kstats.py $db --limit 12 > $OUT/${lib}_$wl.txt
    [ "${KEEP_DB:-0}" = 1 ] || find $OUT/${lib}_$wl -name "*.db" -delete
    echo "== $lib $wl: $(grep '^{' $OUT/${lib}_$wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), 'ms/step')")"
    head -8 $OUT/${lib}_$wl.txt | cut -c1-120
  done
done
