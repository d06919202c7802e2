#!/bin/bash
# GPU iteration: parity tests, profiled bench, then optional variant benches.
# Usage: bash tools/exp_run.sh TAG [variant ...]   (variants: ddr_amd/lib/libddr_mc_<v>.so)
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $OUT/pytest.log | head -20; exit $rc; }
bash $R/tools/exp_profile.sh $TAG || exit $?
for v in "$@"; do
  DDR_LIB=$R/ddr_amd/lib/libddr_mc_$v.so timeout -k 10 300 python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b_$v.log 2>&1 || exit $?
  echo "$v" $(grep '^{' $OUT/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v['kernel_ms'],1) for k, v in d['kernels'].items()})")
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/rocprof_bench.log 2>&1 || exit $?
python3 $R/tools/kstats.py $(find $OUT/prof -name "*.db") > $OUT/kernel_stats.txt 2>&1
head -9 $OUT/kernel_stats.txt | cut -c1-130
find $OUT/prof -name "*.db" -delete
