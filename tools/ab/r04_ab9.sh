#!/bin/bash
# Round 4 A/B 9: the GPU suite on the current build (backward compute loop as pre / adjoint / post per
# slice, geometry statistics with the split-run sort for 6-of-8 slots), C4 kernel trace, and the
# C5 / C3 / C2 / c3s8 / c5s8r5 lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab9
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
(timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4 -o run -- python3 $R/bench.py $B --steps 3 --warmup 1 --workload c4 \
  > $O/c4.json 2> $O/c4.err) || { echo "c4 failed"; tail -5 $O/c4.err; exit 1; }
python3 $R/tools/kstats.py $(find $O/c4 -name "*.db") --limit 8 > $O/c4_kstats.txt; find $O/c4 -name "*.db" -delete
grep geometry $O/c4_kstats.txt
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
run c5 python3 -u $R/bench.py $B --steps 2 --warmup 1
run c3 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
run c2 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c2
run c3s8 WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1 python3 -u $R/bench.py $B --steps 3 --warmup 1 --workload c3
run c5s8r5 WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1 python3 -u $R/bench.py $B --steps 2 --warmup 1
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
