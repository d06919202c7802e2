#!/bin/bash
# The split bench's hand-shake (720-step forward + backward) in the forced 2-rank rehearsal, then the
# fallback rehearsal (rank 1 fails its hand-shake on purpose).
TAG=${1:-r03_handshake}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
DDR_SPLIT_BASIN=force DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $OUT/split_c5.json 2> $OUT/split_c5.err || { tail -5 $OUT/split_c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/split_c5.json').read().strip().splitlines()[-1]); print('split', round(d['ms_per_step'],1), d['config']['split_basin'])"
grep -E "hand-shake|falling" $OUT/split_c5.err | head -3
bash tools/r03_fallback.sh $TAG/fallback || exit 1
exit 0
