#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_probe2
mkdir -p $OUT
cd $R
DDR_DEBUG_PART=1 timeout -k 10 300 python3 -u -c "
import sys, time, torch
sys.path.insert(0, '.')
from ddr_amd import synthetic
from ddr_amd.graph import RiverGraph
for k in (0, 2):
    net = synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 100 + k), seed=100 + k, single_inflow=0.25)
    rows, cols = torch.from_numpy(net.rows).cuda(), torch.from_numpy(net.cols).cuda()
    for rep in range(2):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        g = RiverGraph(net.n, rows, cols, steps_hint=2136)
        print('build', k, rep, (time.perf_counter() - t0) * 1e3, file=sys.stderr, flush=True)
" > $OUT/dpart.log 2>&1 || { tail -5 $OUT/dpart.log; exit 1; }
grep -v "^\[part\]   slots\|amdgpu.ids" $OUT/dpart.log | tail -60
TAG=r03_probe2 bash tools/ab_fwd.sh base: fnp2: base:--math=faithful 2>&1 | tail -5
