"""Predicted strong scaling: route every rank's shard of the global network ALONE on one GPU (the
shards share nothing on the data path, so a rank's time is its shard's time) and report, per N,
max over ranks of the fwd+bwd step time.  Usage: python tools/scale_predict.py [c5|c3] [N ...]"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddr_amd import synthetic  # noqa: E402
from ddr_amd.distributed import shard_network  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402
from ddr_amd.ops import RouteConsts, route  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
Ns = [int(a) for a in sys.argv[2:]] or [1, 2, 4, 8]
if wl == "c5":
    net, T = synthetic.forest(synthetic.zipf_sizes(800_000, 3000, 0.35), seed=5, single_inflow=0.35), 8760
else:
    net, T = synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 3), seed=3, single_inflow=0.25), 2136
dev = torch.device("cuda:0")
at = synthetic.reach_attributes(net.n, 11)
u = synthetic.unit_parameters(net.n, 11)
res = {}
for N in Ns:
    per = []
    for r in range(N):
        n_loc, rows, cols, ids = shard_network(net.n, net.rows, net.cols, r, N) if N > 1 else (
            net.n, net.rows, net.cols, np.arange(net.n))
        g = RiverGraph(n_loc, rows, cols, steps_hint=T)
        tt = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a)[ids])).to(dev)  # noqa: E731
        qp = synthetic.lateral_inflow_torch(net.n, T, seed=11, device=dev, ids=ids)
        W = torch.rand((n_loc, T), device=dev)
        un, uq, up = (tt(u[k]).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial"))

        def step():
            n = un * 0.235 + 0.015
            q = uq * 1.0
            p = torch.exp(up * (np.log(200.0) - np.log(1.0 + 1e-6)) + np.log(1.0 + 1e-6))
            out, _, _, _ = route(g, qp, n, q, p, tt(at.length), tt(np.maximum(at.slope, np.float32(1e-3))), tt(at.x),
                                 consts=RouteConsts(), math=os.environ.get("DDR_MATH", "faithful"))
            out.backward(W)

        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 2 * 1e3
        per.append({"rank": r, "reaches": int(n_loc), "blocks": g.info.n_blocks, "max_depth": g.info.max_depth,
                    "ms": round(ms, 1)})
        print(N, per[-1], flush=True)
        del qp, W, g
        torch.cuda.empty_cache()
    tmax = max(p["ms"] for p in per)
    res[N] = {"ms_max": tmax, "ranks": per}
t1 = res[Ns[0]]["ms_max"] if Ns[0] == 1 else None
for N in Ns:
    if t1:
        res[N]["speedup"] = round(t1 / res[N]["ms_max"], 2)
print(json.dumps({"workload": wl, "T": T, "reaches": net.n, "math": os.environ.get("DDR_MATH", "faithful"),
                  "predicted": res}))
