#!/bin/bash
# PMC passes over a short bench run, one counter group per pass (no tracing domains mixed in).
# Usage: bash tools/pmc.sh TAG [bench args...]   -> gpurun_out/TAG/{p1..p5}, report.txt
TAG=${1:-pmc}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --dropin-steps 0 $*"
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d $OUT/$n -o run -- python3 $R/bench.py $ARGS > $OUT/$n.log 2>&1
  local rc=$?; echo "pass $n rc=$rc"; return $rc
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU &&
run p2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM &&
run p3 FETCH_SIZE &&
run p4 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum &&
run p5 GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum &&
{ run p6 TCC_ATOMIC_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum || echo "p6 (atomics) failed: optional"; }
rc=$?
python3 $R/tools/pmc_report.py $OUT > $OUT/report.txt 2>&1
cat $OUT/report.txt
[ "${KEEP_DB:-0}" = 1 ] || find $OUT -name "*.db" -delete
exit $rc
