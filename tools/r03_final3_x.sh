#!/bin/bash
# Final evidence X: -m gpu suite + smoke, PMC counters of all four workloads keyed to this build's kernel
# hash (per-dispatch selection, written into profiles/counters on the box so the bench lines carry them),
# every workload's bench line, the C3 training stream and the default line with its CPU baseline.
TAG=${1:-r03_final3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 240 --timeout-method thread > $OUT/gpu_pytest.log 2>&1
rc=$?; tail -1 $OUT/gpu_pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/gpu_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
HASH=$(python3 -c "import sys; sys.path.insert(0, '$R'); from ddr_amd import _lib; print(_lib.load().ddr_version().decode().split()[-1])")
for w in c5 c3 c4 c2; do
  case $w in c5) A="8760 800000";; c3) A="2136 896201";; c4) A="8760 350000";; c2) A="8760 5000";; esac
  KEEP_DB=1 bash tools/pmc.sh $TAG/pmc_$w --workload $w > $OUT/pmc_$w.log 2>&1 || { tail -20 $OUT/pmc_$w.log; exit 1; }
  PMC_JSON_DIR=$OUT python3 tools/pmc_to_json.py $OUT/pmc_$w $w $HASH $A profiles/r03/pmc_$w > /dev/null || exit 1
  find $OUT/pmc_$w -name "*.db" -delete
  cp $OUT/$w.json profiles/counters/$w.json
  echo "pmc $w done"
done
bash tools/bench_all.sh $TAG/bench || exit 1
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --stream 12 > $OUT/bench_c3_stream.json 2> $OUT/bench_c3_stream.err || { tail -5 $OUT/bench_c3_stream.err; exit 1; }
( time timeout -k 10 600 python bench.py ) > $OUT/bench_default.log 2>&1 || { tail -5 $OUT/bench_default.log; exit 1; }
grep '^{' $OUT/bench_default.log | cut -c1-200
exit 0
