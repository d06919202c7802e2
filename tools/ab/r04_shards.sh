#!/bin/bash
# Every 8-way shard routed alone on one GPU with the full bench step: C3 (basin-sharded) and C5 under the
# split plan (ranks of the split group cannot run alone and are skipped).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_shards}
mkdir -p $O
B="--no-cpu-baseline --dropin-steps 0"
for r in 0 1 2 3 4 5 6 7; do
  WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 timeout -k 10 300 python3 $R/bench.py --workload c3 --steps 3 --warmup 1 $B \
    > $O/c3_r$r.json 2> $O/c3_r$r.err || { echo "c3 rank $r failed"; tail -3 $O/c3_r$r.err; exit 1; }
done
for r in 0 1 2 3 4 5 6 7; do
  WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 timeout -k 10 300 python3 $R/bench.py --steps 2 --warmup 1 $B \
    > $O/c5_r$r.json 2> $O/c5_r$r.err
  rc=$?
  if [ $rc != 0 ]; then grep -q "split-group rank" $O/c5_r$r.err && { echo "c5 rank $r: split group, skipped"; rm -f $O/c5_r$r.json; continue; }
    echo "c5 rank $r failed rc=$rc"; tail -3 $O/c5_r$r.err; exit 1; fi
done
for f in $O/c3_r*.json $O/c5_r*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f .json)', d['config']['reaches'], round(d['ms_per_step'],2), k)"; done | tee $O/summary.txt
