#!/bin/bash
# cost of the exact adjoint on this build (C5, c3s8 rank 1 alone), default vs --exact-adjoint
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06_exact; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for wl in c5 c3s8; do
  case $wl in c5) fl="";; c3s8) fl="--workload c3";; esac
  for mode in default exact; do
    ex=""; [ $mode = exact ] && ex="--exact-adjoint"
    if [ $wl = c3s8 ]; then export WORLD_SIZE=8 RANK=1 DDR_BENCH_ALONE=1; else unset WORLD_SIZE RANK DDR_BENCH_ALONE; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${mode}_$wl -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 $fl $ex > $OUT/${mode}_$wl.log 2>&1 \
      || { echo "$mode $wl failed"; tail -5 $OUT/${mode}_$wl.log; exit 1; }
    db=$(find $OUT/${mode}_$wl -name "*.db" | head -1)
    python3 $R/tools/kstats.py $db --limit 6 > $OUT/${mode}_$wl.txt
    find $OUT/${mode}_$wl -name "*.db" -delete
    echo "== $mode $wl: $(grep '^{' $OUT/${mode}_$wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), 'ms/step')")"
    head -5 $OUT/${mode}_$wl.txt | cut -c1-120
  done
done
