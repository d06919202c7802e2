"""Diagnostic: element-wise gradient error of the fp32 kernel (default and exact adjoint) on the reference's
golden networks, against the fp64 oracle adjoint of the kernel's own fp32 trajectory (bit-identical forward,
exact math) and against the fp64 model gradient.  Prints max-rel over the elements above 1e-3 of the largest."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import PARAMS_DEFAULT, PARAMS_MOCK, golden_case  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402
from ddr_amd.ops import route  # noqa: E402
from oracle import mc_oracle as O  # noqa: E402
from test_gpu_route import consts_of  # noqa: E402


def mx(a, b, frac=1e-3):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    m = np.abs(b) >= frac * np.abs(b).max()
    return float(np.max(np.abs(a[m] - b[m]) / np.abs(b[m])))


dev = torch.device("cuda:0")
for name, params in (("sandbox", PARAMS_MOCK), ("tree300", PARAMS_DEFAULT), ("c1", PARAMS_DEFAULT)):
    case, d = golden_case(name, params)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    rngs = params["parameter_ranges"]
    nn_ = O.denormalize(case.u["n"], rngs["n"])
    qq = O.denormalize(case.u["q_spatial"], rngs["q_spatial"])
    pp = (O.denormalize(case.u["p_spatial"], rngs["p_spatial"], True) if case.u.get("p_spatial") is not None
          else np.full(case.n, params["defaults"]["p_spatial"], np.float32))
    slope = np.maximum(case.slope, np.float32(params["attribute_minimums"]["slope"]))
    r = O.Reaches(nn_, qq, pp.astype(np.float32), case.length, slope, case.x)
    net = case.network()
    fw = O.route(net, r, case.qprime, case.bounds, dtype=np.float32)
    bw = O.route_backward(net, r, case.qprime, fw["x"], case.W, case.bounds)
    r64 = O.Reaches(*(np.asarray(v, np.float64) for v in (nn_, qq, pp, case.length, slope, case.x)))
    fw64 = O.route(net, r64, case.qprime.astype(np.float64), case.bounds, dtype=np.float64)
    bw64 = O.route_backward(net, r64, case.qprime.astype(np.float64), fw64["x"], case.W.astype(np.float64), case.bounds)
    for exact in (False, True):
        n, q, p = (tt(v).requires_grad_(True) for v in (nn_, qq, pp.astype(np.float32)))
        g = RiverGraph(case.n, case.rows, case.cols)
        ro, _, _, _ = route(g, tt(case.qprime), n, q, p, tt(case.length), tt(slope), tt(case.x), consts=consts_of(case),
                            exact_adjoint=exact, math="exact")
        ro.backward(tt(case.W))
        torch.cuda.synchronize()
        fwd_eq = bool(np.array_equal(ro.detach().cpu().numpy(), fw["runoff"]))
        e_same = {k: mx(t.grad.cpu().numpy(), bw[k]) for k, t in (("n", n), ("q_spatial", q), ("p_spatial", p))}
        e_model = {k: mx(t.grad.cpu().numpy(), bw64[k]) for k, t in (("n", n), ("q_spatial", q), ("p_spatial", p))}
        print(f"{name:8s} exact={exact!s:5s} fwd==oracle {fwd_eq}  vs fp64 adjoint of the same trajectory "
              + " ".join(f"{k} {v:.2e}" for k, v in e_same.items()) + "  vs fp64 model "
              + " ".join(f"{k} {v:.2e}" for k, v in e_model.items()), flush=True)
