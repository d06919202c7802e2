#!/bin/bash
# Round-4 evidence, PMC part: tools/pmc.sh passes (one counter group per pass) for the given workloads,
# turned into counter files keyed to the loaded library's build (tools/pmc_to_json.py, written under
# gpurun_out/TAG/counters/ -> profiles/counters/), plus the readable reports.
# Usage: bash tools/ab/r04_final_pmc.sh TAG c5 [c3 c4 c2]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O/counters
export TMPDIR=/tmp
HASH=$(python3 -c "import sys; sys.path.insert(0, '$R'); from ddr_amd import _lib; print(_lib.load().ddr_version().decode().split()[-1])")
echo "kernel build $HASH"
for WL in "$@"; do
  KEEP_DB=1 bash $R/tools/pmc.sh $TAG/pmc_$WL --workload $WL > $O/pmc_$WL.log 2>&1 || { echo "pmc $WL failed"; tail -20 $O/pmc_$WL.log; exit 1; }
  ARGS=$(python3 -c "print({'c5':'8760 800000','c3':'2136 896201','c4':'8760 350000','c2':'8760 5000'}['$WL'])")
  PMC_JSON_DIR=$O/counters python3 $R/tools/pmc_to_json.py $O/pmc_$WL $WL $HASH $ARGS profiles/r04/pmc_$WL > $O/pmc_to_json_$WL.log 2>&1 \
    || { echo "pmc_to_json $WL failed"; tail -5 $O/pmc_to_json_$WL.log; exit 1; }
  cp $O/pmc_$WL/report.txt $O/pmc_${WL}_report.txt
  find $O/pmc_$WL -name "*.db" -delete
  echo "$WL done: $(head -c 300 $O/pmc_to_json_$WL.log)"
done
