R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${EVTAG:-r05_ev2}; mkdir -p $O
for r in 3 4 5 6 7; do
  WORLD_SIZE=8 RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=${SPLIT_PLAN:-1} timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $O/c5s8_r$r.json 2> $O/c5s8_r$r.err || { echo "c5 rank $r failed"; tail -3 $O/c5s8_r$r.err; exit 1; }
  echo "c5 r$r $(python3 -c "import json; d=json.loads(open('$O/c5s8_r$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config']['reaches'], {k: round(v['kernel_ms'],2) for k,v in d['kernels'].items()})")"
done
cd /tmp && export TMPDIR=/tmp
WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $O/c3s8_prof.log 2>&1 || exit 1
python3 $R/tools/kstats.py --per-step 5 $(find $O/prof -name "*.db") > $O/kernel_stats_c3s8.txt 2>&1; head -20 $O/kernel_stats_c3s8.txt | cut -c1-140
find $O/prof -name "*.db" -delete
