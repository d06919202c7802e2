#!/bin/bash
# Round 4 A/B 22: the packer's light-load rule (blocks <= half a workgroup while the capacity is there; the
# unweighted packing at that capacity before it grows): device-builder and routing GPU tests, then every
# C3 8-way shard alone (tools/ab/r04_shards.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04_ab22}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_devgraph.py $R/tests/test_gpu_route.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash $R/tools/ab/r04_shards.sh ${1:-r04_ab22}/shards
