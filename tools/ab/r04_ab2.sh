#!/bin/bash
# Round 4 A/B 2: the full GPU suite on the new build, then the lines that matter (C3 8-way shard, C3, C5
# with the drop-in line, C4, C2), the light-load packing quantum as an arm, and a kernel trace of the
# C3 shard step (non-routing kernels).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
S8="WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1"
B="--no-cpu-baseline --dropin-steps 0"
run() { local tag=$1; shift; timeout -k 10 300 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
run c3s8 $S8 python3 -u $R/bench.py --workload c3 $B --steps 3 --warmup 1
run c3s8_q256 $S8 DDR_PACK_QUANT=256 python3 -u $R/bench.py --workload c3 $B --steps 3 --warmup 1
run c3 python3 -u $R/bench.py --workload c3 $B --steps 3 --warmup 1
run c3_q256 DDR_PACK_QUANT=256 python3 -u $R/bench.py --workload c3 $B --steps 3 --warmup 1
run c5 python3 -u $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
run c5_q256 DDR_PACK_QUANT=256 python3 -u $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0
run c4 python3 -u $R/bench.py --workload c4 $B --steps 2 --warmup 1
run c2 python3 -u $R/bench.py --workload c2 $B --steps 3 --warmup 1
(cd /tmp && env $S8 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c3s8_trace -o run -- python3 $R/bench.py \
  --workload c3 $B --steps 3 --warmup 1 > $O/c3s8_trace.log 2>&1) || exit 1
python3 $R/tools/kstats.py $(find $O/c3s8_trace -name "*.db") --limit 60 > $O/c3s8_kstats.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4_trace -o run -- python3 $R/bench.py \
  --workload c4 $B --steps 1 --warmup 1 > $O/c4_trace.log 2>&1) || exit 1
python3 $R/tools/kstats.py $(find $O/c4_trace -name "*.db") --limit 20 > $O/c4_kstats.txt
find $O -name "*.db" -delete
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k={a:round(b['kernel_ms'],2) for a,b in d['kernels'].items()}
print('$(basename $f)', round(d['ms_per_step'],2), k, (d.get('dropin_dmc') or {}).get('ms_per_step'))"; done
