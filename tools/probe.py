"""Kernel timing probe on the C5 workload: forward / backward under flag variants.

python tools/probe.py [--T 8760] [--variants base,norunoff,coal]   (DDR_LIB selects the library build)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ddr_amd import _lib, ops, synthetic  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402

PROBE = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8760)
    ap.add_argument("--reaches", type=int, default=800_000)
    ap.add_argument("--variants", default="base,norunoff")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    ns = argparse.Namespace(reaches=args.reaches, basins=3000, largest=0.35, single_inflow=0.35, seed=5)
    net, _ = bench.build_rank_network(ns, 0, 1)
    dev = torch.device("cuda", 0)
    g = RiverGraph(net.n, net.rows, net.cols)
    info = g.info
    T = args.T
    at = synthetic.reach_attributes(net.n, 5)
    u = synthetic.unit_parameters(net.n, 5)
    tt = lambda a: torch.from_numpy(np.asarray(a)).to(dev, torch.float32)  # noqa: E731
    R = bench.RANGES
    n = tt(u["n"]) * (R["n"][1] - R["n"][0]) + R["n"][0]
    q = tt(u["q_spatial"]) * (R["q_spatial"][1] - R["q_spatial"][0]) + R["q_spatial"][0]
    p = tt(u["p_spatial"]) * 20 + 1
    length, slope, xs = tt(at.length), tt(np.maximum(at.slope, np.float32(1e-3))), tt(at.x)
    qprime = synthetic.lateral_inflow_torch(net.n, T, seed=5, device=dev)
    W = torch.rand((net.n, T), device=dev)
    consts = ops.RouteConsts().as_list()
    gid = ops.register_graph(g)
    out = {"lib": os.environ.get("DDR_LIB", "default"), "blocks": info.n_blocks, "kr": info.reaches_per_thread,
           "n_cut": info.n_cut}

    def timed(fn):
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return min(ts), r

    for v in args.variants.split(","):
        fl = _lib.DDR_FWD_SAVE_X | {"base": 0, "norunoff": _lib.DDR_FWD_NO_RUNOFF}[v]
        tf, res = timed(lambda: ops.mc_route(qprime, n, q, p, length, slope, xs, None, None, None, None, None, None,
                                             gid, consts, fl))
        x_save, bnd = res[4], res[5]
        bfl = 0
        tb, _ = timed(lambda: ops.mc_route_backward(W, qprime, n, q, p, length, slope, xs, None, x_save, bnd, None,
                                                    None, gid, consts, bfl))
        out[v] = {"fwd_ms": round(tf, 2), "bwd_ms": round(tb, 2)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
