"""Gradient accuracy vs depth: the C5 giant basin (281k reaches, depth 2215) routed alone over a
short horizon; the fp32 kernel's gradients against
  n, q_spatial, p_spatial    the fp64 oracle adjoint on the oracle's own fp32 forward states
  own:*                      the fp64 oracle adjoint on the kernel's fp32 states (its runoff; exact where no step
                             is clamped -- the count is printed)
  f64:*                      the fp64 kernel (fp64 states and adjoint: the fp64 model's gradient)
Usage: DDR_MC_LIB=... python tools/grad_depth.py [T] [cache.npz]"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddr_amd import synthetic  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402
from ddr_amd.ops import RouteConsts, route  # noqa: E402
from ddr_amd.partition import basin_labels, extract_basins  # noqa: E402
from oracle import mc_oracle as O  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 72
cache = Path(sys.argv[2]) if len(sys.argv) > 2 else None
net = synthetic.forest(synthetic.zipf_sizes(800_000, 3000, 0.35), seed=5, single_inflow=0.35)
lab = basin_labels(net.n, net.rows, net.cols)
ids = np.flatnonzero(lab == np.bincount(lab).argmax())
keep = np.zeros(net.n, bool)
keep[ids] = True
ns, rs, cs, sel = extract_basins(net.n, net.rows, net.cols, keep)
at = synthetic.reach_attributes(ns, 9)
u = synthetic.unit_parameters(ns, 9)
r = O.Reaches(O.denormalize(u["n"], [0.015, 0.25]), O.denormalize(u["q_spatial"], [0.0, 1.0]),
              O.denormalize(u["p_spatial"], [1.0, 200.0], True), at.length, np.maximum(at.slope, np.float32(1e-3)), at.x)
qp = synthetic.lateral_inflow(ns, T, 9)
W = np.random.default_rng(9).uniform(0, 1, (ns, T)).astype(np.float32)
dev = torch.device("cuda:0")
tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
n, q, p = (tt(v).requires_grad_(True) for v in (r.n, r.q, r.p))
g = RiverGraph(ns, rs, cs, steps_hint=T)
runoff, _, _, _ = route(g, tt(qp), n, q, p, tt(r.length), tt(r.slope), tt(r.x), consts=RouteConsts())
runoff.backward(tt(W))
torch.cuda.synchronize()
if cache is not None and cache.exists():
    ref = dict(np.load(cache))
else:
    t0 = time.time()
    no = O.Network.from_coo(ns, rs, cs)
    fw = O.route(no, r, qp, O.Bounds(), dtype=np.float32)
    bw = O.route_backward(no, r, qp, fw["x"], W, O.Bounds())
    ref = {"runoff": fw["runoff"], "n": bw["n"], "q_spatial": bw["q_spatial"], "p_spatial": bw["p_spatial"]}
    print(f"oracle {time.time() - t0:.1f}s", flush=True)
    if cache is not None:
        np.savez(cache, **ref)
d = np.abs(runoff.detach().cpu().numpy().astype(np.float64) - ref["runoff"]) / np.abs(ref["runoff"])
out = {"runoff_maxrel": float(d.max())}
for k, t in (("n", n), ("q_spatial", q), ("p_spatial", p)):
    a = t.grad.cpu().numpy().astype(np.float64)
    b = ref[k]
    out[k] = float(np.linalg.norm(a - b) / np.linalg.norm(b))
xk = runoff.detach().cpu().numpy().astype(np.float64).T.copy()  # (T, N) = clamp(x) of the kernel
out["clamped"] = int((xk <= O.Bounds().discharge).sum())
bo = O.route_backward(O.Network.from_coo(ns, rs, cs), r, qp, xk, W, O.Bounds())
for k, t in (("n", n), ("q_spatial", q), ("p_spatial", p)):
    a = t.grad.cpu().numpy().astype(np.float64)
    out["own:" + k] = float(np.linalg.norm(a - bo[k]) / np.linalg.norm(bo[k]))
td = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
n64, q64, p64 = (td(v).requires_grad_(True) for v in (r.n, r.q, r.p))
g64 = RiverGraph(ns, rs, cs, steps_hint=T, max_block_reaches=1024)
ro64, _, _, _ = route(g64, td(qp), n64, q64, p64, td(r.length), td(r.slope), td(r.x), consts=RouteConsts())
ro64.backward(td(W))
for k, t, t64 in (("n", n, n64), ("q_spatial", q, q64), ("p_spatial", p, p64)):
    a = t.grad.cpu().numpy().astype(np.float64)
    b = t64.grad.cpu().numpy()
    out["f64:" + k] = float(np.linalg.norm(a - b) / np.linalg.norm(b))
print({k: (f"{v:.3g}" if isinstance(v, float) else v) for k, v in out.items()}, flush=True)
