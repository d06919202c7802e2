#!/bin/bash
# Round 4 A/B 18: the persistent software-pipelined hourly q' gather for heavy blocks (DDR_GATHER_PIPE=1,
# work items of 16 four-step tiles dealt round robin) against the two-dimensional grid (=0).  Route GPU
# tests on the new build, then kernel traces of C5, C4 with each setting.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab18}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py $R/tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
tr() { local tag=$1; shift; (timeout -k 10 400 env "$@" rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python3 $R/bench.py $B --steps 2 --warmup 1 $EXTRA \
  > $O/$tag.json 2> $O/$tag.err) || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 $R/tools/kstats.py $(find $O/$tag -name "*.db") --limit 12 > $O/${tag}_kstats.txt; find $O/$tag -name "*.db" -delete
  echo "$tag $(grep gather_qprime $O/${tag}_kstats.txt | head -1 | cut -c1-60) $(grep gather_qprime $O/${tag}_kstats.txt | head -1 | awk '{print $(NF-3)}')"; }
EXTRA="" tr c5_p1 DDR_GATHER_PIPE=1
EXTRA="" tr c5_p0 DDR_GATHER_PIPE=0
EXTRA="--workload c4" tr c4_p1 DDR_GATHER_PIPE=1
EXTRA="--workload c4" tr c4_p0 DDR_GATHER_PIPE=0
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
