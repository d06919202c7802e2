#!/bin/bash
# Round-3 evidence, part B: PMC counters of C5, C3 and C4 (-> profiles/counters via tools/pmc_to_json.py,
# run afterwards in the build container), strong-scaling prediction (every rank's shard alone) for C3 and C5
# at N = 1 and 8, and 2-rank gloo rehearsals of the multi-GPU bench on the one GPU.
TAG=${1:-r03_final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for w in c5 c3 c4; do
  bash tools/pmc.sh $TAG/pmc_$w --workload $w > $OUT/pmc_$w.log 2>&1 || { tail -20 $OUT/pmc_$w.log; exit 1; }
  echo "pmc $w done"
done
for w in c3 c5; do
  bash tools/scale_alone.sh $w "1 8" > $OUT/scale_alone_$w.log 2>&1 || { tail -5 $OUT/scale_alone_$w.log; exit 1; }
  cp gpurun_out/scale_$w/summary.json $OUT/scale_alone_$w.json; tail -2 $OUT/scale_alone_$w.log
done
# split-basin prediction: C5's largest basin packed for a 3-GPU split group (768 workgroups) routed alone on
# this one GPU, i.e. as three generations one after another; a split rank runs one of them concurrently
WORLD_SIZE=8 RANK=0 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_TARGET_BLOCKS=768 timeout -k 10 400 python3 bench.py --steps 2 \
  --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/split_predict_c5_k3.json 2> $OUT/split_predict_c5_k3.err || { tail -5 $OUT/split_predict_c5_k3.err; exit 1; }
cut -c1-300 $OUT/split_predict_c5_k3.json
for w in c3 c5; do
  DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --workload $w --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/rehearsal_$w.json 2> $OUT/rehearsal_$w.err
  rc=$?; echo "rehearsal $w rc=$rc $(cut -c1-200 $OUT/rehearsal_$w.json)"
  [ $rc -ne 0 ] && { tail -5 $OUT/rehearsal_$w.err; exit $rc; }
done
exit 0
