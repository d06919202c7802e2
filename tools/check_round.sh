#!/bin/bash
# GPU-side round check: full -m gpu suite, PMC counters of a workload -> profiles/counters JSON,
# and a 2-rank rehearsal of the multi-GPU bench on the one GPU (gloo, both ranks on device 0).
# Usage: bash tools/check_round.sh TAG [workload]
TAG=${1:-check}; WL=${2:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests -v -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|^E  " $OUT/pytest.log | cut -c1-300 | tail -8
[ $rc -ne 0 ] && { echo "PYTEST FAILED rc=$rc"; exit $rc; }
bash $R/tools/pmc.sh $TAG/pmc --workload $WL > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
HASH=$(python3 -c "import sys; sys.path.insert(0, '$R'); from ddr_amd import _lib; print(_lib.load().ddr_version().decode().split()[-1])")
python3 $R/tools/pmc_to_json.py $OUT/pmc $WL $HASH $(python3 -c "print({'c5':'8760 800000','c3':'2136 896201','c4':'8760 350000','c2':'8760 5000'}['$WL'])") profiles/r02/pmc_$WL
cp $OUT/pmc/report.txt $R/gpurun_out/$TAG/pmc_report.txt
for w in c3 c5; do
  DDR_BENCH_SAME_DEVICE=1 DDR_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 $R/bench.py --workload $w --gpus 2 --steps 2 --warmup 1 > $OUT/rehearsal_$w.json 2> $OUT/rehearsal_$w.err
  rc=$?; echo "rehearsal $w rc=$rc $(cut -c1-300 $OUT/rehearsal_$w.json)"
  [ $rc -ne 0 ] && { tail -5 $OUT/rehearsal_$w.err; exit $rc; }
done
exit 0
