#!/bin/bash
# Round 4 A/B 17: the hourly q' gather with its grid dealt by XCD (DDR_GATHER_XCD=1: XCD x takes step tiles
# x, x + 8, ..., the blocks of a tile back to back) against the two-dimensional grid (=0).  Route GPU
# tests on the new build, then kernel traces of C5, C4 and c5s8r5 with each setting.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab17}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
tr() { local tag=$1; shift; (timeout -k 10 400 env "$@" rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python3 $R/bench.py $B --steps 2 --warmup 1 $EXTRA \
  > $O/$tag.json 2> $O/$tag.err) || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 $R/tools/kstats.py $(find $O/$tag -name "*.db") --limit 12 > $O/${tag}_kstats.txt; find $O/$tag -name "*.db" -delete
  echo "$tag $(grep gather_qprime_kernel $O/${tag}_kstats.txt | head -1 | cut -c1-60) $(grep gather_qprime_kernel $O/${tag}_kstats.txt | head -1 | awk '{print $(NF-3)}')"; }
EXTRA="" tr c5_x1 DDR_GATHER_XCD=1
EXTRA="" tr c5_x0 DDR_GATHER_XCD=0
EXTRA="--workload c4" tr c4_x1 DDR_GATHER_XCD=1
EXTRA="--workload c4" tr c4_x0 DDR_GATHER_XCD=0
EXTRA="" tr c5s8r5_x1 DDR_GATHER_XCD=1 WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1
EXTRA="" tr c5s8r5_x0 DDR_GATHER_XCD=0 WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
