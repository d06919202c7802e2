#!/bin/bash
# PMC passes (tools/pmc.sh) for every bench workload on the current build: gpurun_out/TAG/<wl>/{p1..p6, report.txt}.
# Then, locally: bash tools/pmc_all.sh --json TAG   -> profiles/counters/<wl>.json (tools/pmc_to_json.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
if [ "$1" = "--json" ]; then
  TAG=$2
  HASH=$(python3 -c "import sys; sys.path.insert(0, '$R'); from ddr_amd import _lib; print(_lib.load().ddr_version().decode().split()[-1])")
  for wl in ${WLS:-c5 c3 c4 c2}; do
    python3 $R/tools/pmc_to_json.py $R/gpurun_out/$TAG/$wl $wl $HASH \
      $(python3 -c "print({'c5':'8760 800000','c3':'2136 896201','c4':'8760 350000','c2':'8760 5000'}['$wl'])") profiles/r06/pmc_$wl || exit 1
  done
  exit 0
fi
TAG=${1:-pmcall}
mkdir -p $R/gpurun_out/$TAG
for wl in ${WLS:-c5 c3 c4 c2}; do
  bash $R/tools/pmc.sh $TAG/$wl --workload $wl > $R/gpurun_out/$TAG/$wl.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/$wl.log; exit 1; }
  echo "pmc $wl done"
done
exit 0
