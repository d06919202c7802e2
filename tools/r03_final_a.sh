#!/bin/bash
# Round-3 evidence, part A: full -m gpu suite + smoke, every workload's bench line, the C3 training stream,
# the default bench line (with the CPU baseline) and rocprofv3 kernel-trace summaries of C5 and C3.
TAG=${1:-r03_final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 240 --timeout-method thread > $OUT/gpu_pytest.log 2>&1
rc=$?; tail -1 $OUT/gpu_pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/gpu_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/bench_all.sh $TAG/bench || exit 1
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --stream 12 > $OUT/bench_c3_stream.json 2> $OUT/bench_c3_stream.err || { tail -5 $OUT/bench_c3_stream.err; exit 1; }
( time timeout -k 10 600 python bench.py ) > $OUT/bench_default.log 2>&1 || { tail -5 $OUT/bench_default.log; exit 1; }
grep '^{' $OUT/bench_default.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
for w in c5 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o run -- python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/rocprof_$w.log 2>&1 || exit 1
  python3 $R/tools/kstats.py $(find $OUT/prof_$w -name "*.db") > $OUT/kernel_stats_$w.txt 2>&1
  find $OUT/prof_$w -name "*_stats.csv" -exec cp {} $OUT/ \; 2>/dev/null
  head -4 $OUT/kernel_stats_$w.txt | cut -c1-130
  find $OUT/prof_$w -name "*.db" -delete
done
exit 0
