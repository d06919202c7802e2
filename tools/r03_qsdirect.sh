#!/bin/bash
# Direct q' read in the forward (no gather pass) vs the gather: GPU suite, A/B over workloads, the C3 training
# stream with the inline device builder vs host builder threads, and a kernel trace of C5 with the direct read.
TAG=${1:-r03_qsd}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; exit $rc; }
TAG=$TAG/ab WLS="c5 c2 light c5s8" bash tools/ab_env.sh DDR_QS_DIRECT=1 DDR_QS_DIRECT=0 || exit 1
# upper bound of what the forward's x_save / runoff stores cost (variant without them; timing only)
TAG=$TAG/nost WLS="c2 c3s8 light c5" bash tools/ab_wl.sh base nost || exit 1
for b in inline host; do
  timeout -k 10 400 python3 -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --stream 12 --stream-builder $b > $OUT/c3_$b.json 2> $OUT/c3_$b.err || { tail -5 $OUT/c3_$b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c3_$b.json').read()); s=d['training_stream']; print('$b c3 fixed', round(d['ms_per_step'],2), 'stream', round(s['ms_per_step'],2), 'wait', round(s['graph_wait_ms_mean'],2)); print([(b['reaches'], b['generations'], b['graph_wait_ms'], b['step_gpu_ms']) for b in s['batches']])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/bench_prof.log 2>&1 || exit 1
python3 $R/tools/kstats.py $(find $OUT/prof -name "*.db") > $OUT/kernel_stats_c5.txt 2>&1
head -8 $OUT/kernel_stats_c5.txt | cut -c1-140
find $OUT/prof -name "*.db" -delete
# dynamic instruction mix at light load (C2) and full load (C5)
cd $R
BENCH_ARGS="--workload c2" bash tools/pmc_valu.sh $TAG/mix_c2 > /dev/null 2>&1; head -40 $OUT/mix_c2/report.txt
bash tools/pmc_valu.sh $TAG/mix_c5 > /dev/null 2>&1; head -40 $OUT/mix_c5/report.txt
exit 0
