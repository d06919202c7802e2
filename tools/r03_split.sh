#!/bin/bash
# Split basin on one GPU: the two-process bitwise test, a forced 2-rank rehearsal of the C5 bench with the
# largest basin split (both ranks on device 0, gloo), then the whole -m gpu suite.
TAG=${1:-r03_split}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread > $OUT/split_test.log 2>&1
rc=$?; tail -3 $OUT/split_test.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error|error" $OUT/split_test.log | head -40; exit $rc; }
DDR_SPLIT_BASIN=force DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $OUT/rehearsal_split_c5.json 2> $OUT/rehearsal_split_c5.err
rc=$?; echo "rehearsal rc=$rc $(cut -c1-700 $OUT/rehearsal_split_c5.json)"; grep -E "split|hand-shake" $OUT/rehearsal_split_c5.err | head
[ $rc -ne 0 ] && { tail -20 $OUT/rehearsal_split_c5.err; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -30; exit $rc; }
exit 0
