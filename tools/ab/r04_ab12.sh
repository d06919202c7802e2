#!/bin/bash
# Round 4 A/B 12 (13: + wave-aggregated atomics): the device builder's level walks with the basin's values in LDS (k_sub_ht_lds, k_split_lds:
# child table and split table rows requested a level ahead; DDR_DEVBUILD_LEVEL_LDS=0 = the global walks):
# the device-build GPU tests (schedule bit-identical to the host builder), the C3 training stream, and a
# kernel trace of the stream's builds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab12}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_devgraph.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local tag=$1; shift; timeout -k 10 500 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }; }
run stream_lds python3 -u $R/bench.py $B --workload c3 --steps 1 --warmup 1 --stream 12
#run stream_glob DDR_DEVBUILD_LEVEL_LDS=0 python3 -u $R/bench.py $B --workload c3 --steps 1 --warmup 1 --stream 12
for f in $O/stream_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); t=d['training_stream']
print('$(basename $f)', round(t['ms_per_step'],2), 'gpu', round(t['step_gpu_ms_mean'],2), 'between', round(t['between_steps_ms'],2), 'ratio', round(t['stream_over_gpu_step'],3))"; done
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/tr -o run -- python3 $R/bench.py $B --workload c3 --steps 1 --warmup 1 \
  --stream 6 > $O/trace.json 2> $O/trace.err || { echo "trace failed"; tail -5 $O/trace.err; exit 1; }
python3 $R/tools/kstats.py $(find $O/tr -name "*.db") --limit 40 > $O/stream_kstats.txt; find $O/tr -name "*.db" -delete
grep -E "k_sub_ht|k_split|k_child|k_inv|k_split_tab|sort|Scan|k_emit|k_piece" $O/stream_kstats.txt | head -20
