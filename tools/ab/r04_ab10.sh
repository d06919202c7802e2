#!/bin/bash
# Round 4 A/B 10: the q' gather's step tile for heavy blocks (DDR_GATHER_HEAVY_G = 2 / 4 / default 8, and 16
# where blocks hold <= 2048 reaches) at C5 and C4, kernel traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_ab10
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
cd /tmp
trace() {  # tag env... --steps ... (bench args from --steps on)
  local tag=$1; shift
  local e=(); while [ "$1" != "--steps" ]; do e+=("$1"); shift; done
  timeout -k 10 400 env "${e[@]}" rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python3 $R/bench.py $B "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 $R/tools/kstats.py $(find $O/$tag -name "*.db") --limit 10 > $O/${tag}_kstats.txt
  find $O/$tag -name "*.db" -delete
  echo "$tag: $(grep gather_qprime $O/${tag}_kstats.txt | head -2)"
}
trace c5_g8 DDR_GATHER_HEAVY_G=0 --steps 2 --warmup 1
trace c5_g4 DDR_GATHER_HEAVY_G=4 --steps 2 --warmup 1
trace c5_g2 DDR_GATHER_HEAVY_G=2 --steps 2 --warmup 1
trace c4_g8 DDR_GATHER_HEAVY_G=0 --steps 2 --warmup 1 --workload c4
trace c4_g4 DDR_GATHER_HEAVY_G=4 --steps 2 --warmup 1 --workload c4
trace c4_g16 DDR_GATHER_HEAVY_G=16 --steps 2 --warmup 1 --workload c4
