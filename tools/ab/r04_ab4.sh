#!/bin/bash
# Round 4 A/B 4: the GPU suite on the new build (DPP lane exchanges in the geometry statistics' sort, the
# light-load packing quantum as default, device-build cleanup), the output-tiled q' gather
# (DDR_GATHER_OUT=1) against the step-tiled one: its parity tests and C5 kernel traces; C4 kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab4
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
DDR_GATHER_OUT=1 timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py \
  $R/tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread > $O/pytest_out.log 2>&1 \
  || { tail -30 $O/pytest_out.log; exit 1; }
tail -2 $O/pytest_out.log
cd /tmp
trace() {  # tag, env..., -- bench args
  local tag=$1; shift
  local e=(); while [ "$1" != "--steps" ]; do e+=("$1"); shift; done
  timeout -k 10 400 env "${e[@]}" rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python3 $R/bench.py $B "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 $R/tools/kstats.py $(find $O/$tag -name "*.db") --limit 12 > $O/${tag}_kstats.txt
  find $O/$tag -name "*.db" -delete
  head -8 $O/${tag}_kstats.txt
}
trace c5 DDR_GATHER_OUT=0 --steps 2 --warmup 1
trace c5_out DDR_GATHER_OUT=1 --steps 2 --warmup 1
trace c4 DDR_GATHER_OUT=0 --steps 3 --warmup 1 --workload c4
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
