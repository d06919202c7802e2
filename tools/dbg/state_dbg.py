"""Debug: state-gradient kernel vs oracle, per row / reach (fp32 and fp64, with/without flow_scale)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from ddr_amd import synthetic
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import RouteConsts, route
from oracle import mc_oracle as O
from conftest import normrel

dev = torch.device("cuda:0")
net = synthetic.random_binary_tree(300, seed=31); T = 60
at = synthetic.reach_attributes(net.n, 31); rng = np.random.default_rng(31)
u = synthetic.unit_parameters(net.n, 31)
n = O.denormalize(u['n'], [0.015, 0.25]).astype(np.float64); q = O.denormalize(u['q_spatial'], [0, 1]).astype(np.float64)
p = O.denormalize(u['p_spatial'], [1, 200], True).astype(np.float64)
slope = np.maximum(at.slope, 1e-3).astype(np.float64)
qstore = synthetic.lateral_inflow(net.n, T, 32).astype(np.float64); qstore[:2, 5] = 1e-6
fs = rng.uniform(0.5, 1.5, net.n)
W = rng.uniform(0, 1, (net.n, T))
netO = O.Network.from_coo(net.n, net.rows, net.cols); bd = O.Bounds(discharge=1e-4, velocity=0.01, depth=0.01, bottom_width=0.01)
C = RouteConsts(discharge_lb=1e-4)
for dt in (torch.float64, torch.float32):
    for use_fs in (False, True):
        tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)
        qp = tt(qstore).requires_grad_(True)
        g = RiverGraph(net.n, net.rows, net.cols)
        out, _, _, _ = route(g, qp, tt(n), tt(q), tt(p), tt(at.length), tt(slope), tt(at.x),
                             flow_scale=tt(fs) if use_fs else None, consts=C)
        out.backward(tt(W))
        qh = qstore * (fs[None, :] if use_fs else 1.0)
        r = O.Reaches(n, q, p, at.length.astype(np.float64), slope, at.x.astype(np.float64))
        res = O.route(netO, r, qh, bd, dtype=np.float64)
        bw = O.route_backward(netO, r, qh, res['x'], W, bd, want_qprime=True)
        gref = bw['qprime'] * (fs[None, :] if use_fs else 1.0)
        gk = qp.grad.cpu().numpy()
        err = np.abs(gk - gref)
        print(dt, "fs" if use_fs else "nofs", "normrel", normrel(gk, gref), "row0", normrel(gk[0], gref[0]),
              "rows1+", normrel(gk[1:], gref[1:]))
        bad = np.argwhere(err > 1e-6 * np.abs(gref).max())
        print("  bad count", len(bad), bad[:10].tolist())
        if len(bad):
            t, i = bad[0]
            print("  kernel", gk[t, i], "oracle", gref[t, i], "down", netO.down[i] if hasattr(netO, 'down') else None)
