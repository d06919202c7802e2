#!/bin/bash
# PMC passes over a short bench run (one counter group per pass; no tracing domains mixed in).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
ARGS="--steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/p1 -o run -- python3 $R/bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS -d $OUT/p2 -o run -- python3 $R/bench.py $ARGS > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $OUT/p3 -o run -- python3 $R/bench.py $ARGS > $OUT/p3.log 2>&1
echo PMC_DONE
