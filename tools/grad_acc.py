"""Gradient accuracy of the fp32 adjoint against the fp64 oracle on one case (A/B of library builds).

Usage: python tools/grad_acc.py [path/to/libddr_mc.so]   (other builds may lack newer symbols)
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from ddr_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = Path(sys.argv[1])
    import ctypes

    probe = ctypes.CDLL(sys.argv[1])
    for name in list(_lib._SIGS):
        if not hasattr(probe, name):
            _lib._SIGS.pop(name)
from conftest import normrel, synthetic_case  # noqa: E402
from ddr_amd import synthetic  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402
from ddr_amd.ops import route  # noqa: E402
from oracle import mc_oracle as O  # noqa: E402

dev = torch.device("cuda:0")
for name, net, T in (("hack30k", synthetic.hack_basin(30000, seed=21, single_inflow=0.3), 96),
                     ("tree300", synthetic.random_binary_tree(300, 3), 200)):
    case = synthetic_case(net, T, 21)
    n, q, p, slope = case.physical()
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, torch.float32)  # noqa: E731
    nt, qt, pt = (tt(v).requires_grad_(True) for v in (n, q, p))
    g = RiverGraph(net.n, net.rows, net.cols)
    runoff, _, _, _ = route(g, tt(case.qprime), nt, qt, pt, tt(case.length), tt(slope), tt(case.x))
    runoff.backward(tt(case.W))
    torch.cuda.synchronize()
    r = O.Reaches(n, q, p, case.length, slope, case.x)
    ref64 = O.route(case.network(), r, case.qprime, case.bounds, dtype=np.float64)
    bw = O.route_backward(case.network(), r, case.qprime, ref64["x"], case.W, case.bounds)
    errs = {k: normrel(t.grad.cpu().numpy(), bw[k]) for k, t in (("n", nt), ("q_spatial", qt), ("p_spatial", pt))}
    print(name, g, {k: f"{v:.2e}" for k, v in errs.items()}, flush=True)
