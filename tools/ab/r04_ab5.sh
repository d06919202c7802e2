#!/bin/bash
# Round 4 A/B 5: the step-major row layout of an hourly q' store (DDR_QS_HOURLY_ROWS=1: the gather becomes a
# row permutation written in whole rows; the routing kernels read a position's step t from row t) against
# the tick-major layout, at C5 (one GPU and an 8-way shard) and C4; the geometry statistics kernel rewrite
# (one v_med3 per compare-exchange, no scratch, persistent XCD-dealt workgroups) at C4.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab5
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py $R/tests/test_gpu_state.py \
  $R/tests/test_gpu_objectives.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
DDR_QS_HOURLY_ROWS=1 timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py \
  $R/tests/test_gpu_state.py $R/tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > $O/pytest_rows.log 2>&1 \
  || { tail -30 $O/pytest_rows.log; exit 1; }
tail -1 $O/pytest_rows.log
cd /tmp
trace() {  # tag env... --steps ... (bench args from --steps on)
  local tag=$1; shift
  local e=(); while [ "$1" != "--steps" ]; do e+=("$1"); shift; done
  timeout -k 10 400 env "${e[@]}" rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python3 $R/bench.py $B "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 $R/tools/kstats.py $(find $O/$tag -name "*.db") --limit 10 > $O/${tag}_kstats.txt
  find $O/$tag -name "*.db" -delete
  sed -n 3,6p $O/${tag}_kstats.txt
}
trace c5_rows DDR_QS_HOURLY_ROWS=1 --steps 2 --warmup 1
trace c4 DDR_QS_HOURLY_ROWS=0 --steps 3 --warmup 1 --workload c4
trace c4_rows DDR_QS_HOURLY_ROWS=1 --steps 3 --warmup 1 --workload c4
S8="WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1"
trace c5s8r5 $S8 DDR_QS_HOURLY_ROWS=0 --steps 2 --warmup 1
trace c5s8r5_rows $S8 DDR_QS_HOURLY_ROWS=1 --steps 2 --warmup 1
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
