# round 6 re-entry: GPU suite on HEAD, C5 / c3s8 kernel traces, C3 fused vs torch-caller lines, C3 8-way shards alone
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06_base; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
LIBS="cur" WLS="c5 c3s8" TAG=r06_base bash tools/ktrace.sh || exit 1
for c in fused torch; do
  timeout -k 10 300 python3 -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --pnet $c --tail $c > $OUT/c3_$c.json 2> $OUT/c3_$c.err || { tail -5 $OUT/c3_$c.err; exit 1; }
  cut -c1-300 $OUT/c3_$c.json
done
bash tools/scale_alone.sh c3 "1 8" > $OUT/scale_c3.log 2>&1 || { tail -5 $OUT/scale_c3.log; exit 1; }
cat $OUT/scale_c3.log; cp gpurun_out/scale_c3/summary.json $OUT/scale_c3_summary.json
