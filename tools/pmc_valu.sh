#!/bin/bash
# Dynamic instruction mix of the routing kernels (one counter group per pass).
# Usage: bash tools/pmc_valu.sh TAG [variant]   (variant: ddr_amd/lib/libddr_mc_<v>.so)
TAG=${1:-mix}; V=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
[ -n "$V" ] && export DDR_LIB=$R/ddr_amd/lib/libddr_mc_$V.so
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --dropin-steps 0 ${BENCH_ARGS:-}"
run() {
  local n=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d $OUT/$n -o run -- python3 $R/bench.py $ARGS > $OUT/$n.log 2>&1
  local rc=$?; echo "pass $n rc=$rc"; return $rc
}
run p1 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU &&
run p2 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU &&
run p3 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM
rc=$?
python3 $R/tools/pmc_report.py $OUT > $OUT/report.txt 2>&1
head -60 $OUT/report.txt
find $OUT -name "*.db" -delete
exit $rc
