#!/bin/bash
# Round 4 A/B 16: kernel trace of the c3s8 shard step (C3 8-way shard, rank 1 alone) and of C3 on one GPU
# on the current build: the non-routing kernels' share of the step (parameter network, objective, Adam).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab16}
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --dropin-steps 0"
cd /tmp
S8="WORLD_SIZE=8 RANK=1 LOCAL_RANK=0 DDR_BENCH_ALONE=1"
(env $S8 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c3s8 -o run -- python3 $R/bench.py $B --steps 4 --warmup 1 --workload c3 \
  > $O/c3s8.json 2> $O/c3s8.err) || { echo "c3s8 failed"; tail -5 $O/c3s8.err; exit 1; }
python3 $R/tools/kstats.py $(find $O/c3s8 -name "*.db") --limit 60 > $O/c3s8_kstats.txt; find $O/c3s8 -name "*.db" -delete
(timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c3 -o run -- python3 $R/bench.py $B --steps 3 --warmup 1 --workload c3 \
  > $O/c3.json 2> $O/c3.err) || { echo "c3 failed"; tail -5 $O/c3.err; exit 1; }
python3 $R/tools/kstats.py $(find $O/c3 -name "*.db") --limit 60 > $O/c3_kstats.txt; find $O/c3 -name "*.db" -delete
head -30 $O/c3s8_kstats.txt
