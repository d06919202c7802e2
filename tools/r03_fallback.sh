#!/bin/bash
# Rehearsal of the split-basin fallback: rank 1 fails its hand-shake, rank 0's hand-shake times out on the
# device, both fall back to whole-basin sharding and the bench completes (forced 2-rank split, one GPU).
TAG=${1:-r03_fallback}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
DDR_SPLIT_FAIL_RANK=1 DDR_SPLIT_BASIN=force DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $OUT/fallback_c5.json 2> $OUT/fallback_c5.err
rc=$?; echo "rc=$rc"; grep -E "hand-shake|falling back|RiverGraph" $OUT/fallback_c5.err | cut -c1-300
python3 -c "import json; d=json.loads(open('$OUT/fallback_c5.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['split_basin'], d['config']['reaches'], d['config']['reaches_per_rank'])"
exit $rc
