#!/bin/bash
# Round 4 A/B 6: the q' gather with light-load tiles (32 steps x 256/512-thread workgroups for blocks of
# <= 512 reaches, 16 steps for <= 1024; DDR_GATHER_SEL=0 is the previous 8-step, 1024-thread tile) at a
# C5 8-way shard, C2 and the C3 8-way shard; its parity tests; the dependent-chain latency of one
# reach-step (tools/chain_lat.hip, built in-tree: build/chain_lat).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab6
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 120 $R/build/chain_lat 20000 > $O/chain_lat.txt 2>&1 || { echo "chain_lat failed"; cat $O/chain_lat.txt; exit 1; }
cat $O/chain_lat.txt
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_route.py $R/tests/test_gpu_steady.py $R/tests/test_gpu_state.py \
  $R/tests/test_gpu_split.py $R/tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
trace() {  # tag env... --steps ... (bench args from --steps on)
  local tag=$1; shift
  local e=(); while [ "$1" != "--steps" ]; do e+=("$1"); shift; done
  timeout -k 10 400 env "${e[@]}" rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python3 $R/bench.py $B "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 $R/tools/kstats.py $(find $O/$tag -name "*.db") --limit 10 > $O/${tag}_kstats.txt
  find $O/$tag -name "*.db" -delete
  grep gather $O/${tag}_kstats.txt
}
S8="WORLD_SIZE=8 RANK=5 LOCAL_RANK=0 DDR_BENCH_ALONE=1 DDR_BENCH_SPLIT_PLAN=1"
trace c5s8r5_g0 $S8 DDR_GATHER_SEL=0 --steps 2 --warmup 1
trace c5s8r5 $S8 DDR_GATHER_SEL=1 --steps 2 --warmup 1
trace c2_g0 DDR_GATHER_SEL=0 --steps 3 --warmup 1 --workload c2
trace c2 DDR_GATHER_SEL=1 --steps 3 --warmup 1 --workload c2
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k)"; done
