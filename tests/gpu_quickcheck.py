"""Quick end-to-end check of the HIP routing path against the oracle (run on a GPU box).

python tests/gpu_quickcheck.py
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from ddr_amd import synthetic  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402
from ddr_amd.ops import RouteConsts, route  # noqa: E402
from oracle import mc_oracle as O  # noqa: E402

RANGES = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}


def case(net, T, seed, dtype, **gkw):
    attrs = synthetic.reach_attributes(net.n, seed)
    qp = synthetic.lateral_inflow(net.n, T, seed)
    u = synthetic.unit_parameters(net.n, seed)
    nn_ = O.denormalize(u["n"], RANGES["n"])
    qq = O.denormalize(u["q_spatial"], RANGES["q_spatial"])
    pp = O.denormalize(u["p_spatial"], RANGES["p_spatial"], True)
    slope = np.maximum(attrs.slope, np.float32(1e-3))
    W = np.random.default_rng(seed + 4000).uniform(0, 1, (net.n, T)).astype(np.float32)
    g = RiverGraph(net.n, net.rows, net.cols, **gkw)
    dev = torch.device("cuda")
    tt = lambda a: torch.from_numpy(np.asarray(a)).to(dev, dtype)  # noqa: E731
    n_t, q_t, p_t = (tt(v).requires_grad_(True) for v in (nn_, qq, pp))
    t0 = time.time()
    runoff, q_last, tw, ss = route(g, tt(qp), n_t, q_t, p_t, tt(attrs.length), tt(slope), tt(attrs.x),
                                   consts=RouteConsts())
    (runoff * tt(W)).sum().backward()
    torch.cuda.synchronize()
    el = time.time() - t0
    net_o = O.Network.from_coo(net.n, net.rows, net.cols)
    r = O.Reaches(nn_, qq, pp, attrs.length, slope, attrs.x)
    odt = np.float64 if dtype == torch.float64 else np.float32
    ref = O.route(net_o, r, qp, O.Bounds(), dtype=odt)
    bw = O.route_backward(net_o, r, qp, ref["x"], W, O.Bounds())
    out = runoff.detach().cpu().numpy()
    rel = np.max(np.abs(out - ref["runoff"]) / np.maximum(np.abs(ref["runoff"]), 1e-30))
    res = {"graph": repr(g), "dtype": str(dtype), "runoff_maxrel": float(rel), "sec": el,
           "q_last_maxrel": float(np.max(np.abs(q_last.detach().cpu().numpy() - ref["q_last"]) / np.abs(ref["q_last"])))}
    for name, t, o in (("n", n_t, bw["n"]), ("q", q_t, bw["q_spatial"]), ("p", p_t, bw["p_spatial"])):
        gg = t.grad.detach().cpu().numpy().astype(np.float64)
        res[f"grad_{name}_normrel"] = float(np.linalg.norm(gg - o) / np.linalg.norm(o))
    return res


def main():
    torch.manual_seed(0)
    nets = [("chain5", synthetic.SyntheticNetwork(5, np.arange(1, 5, dtype=np.int32), np.arange(0, 4, dtype=np.int32),
                                                  np.array([5])), 20),
            ("tree300", synthetic.random_binary_tree(300, seed=3), 40),
            ("c1", synthetic.random_binary_tree(2000, seed=0), 720),
            ("forest", synthetic.forest(synthetic.loguniform_sizes(40, 20, 3000, 1), seed=1), 200)]
    for name, net, T in nets:
        for dtype in (torch.float64, torch.float32):
            for kw in ({}, {"max_block_reaches": 64, "target_blocks": 64}):
                try:
                    res = case(net, T, 7, dtype, **kw)
                    print(name, kw, res, flush=True)
                except Exception as e:  # noqa: BLE001
                    print(name, kw, dtype, "FAILED", repr(e), flush=True)
                    if "co-resident" not in str(e):
                        raise


if __name__ == "__main__":
    main()
