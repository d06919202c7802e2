"""The approximate-math forwards: route(math="fast") (DDR_FWD_FAST_MATH: the Muskingum coefficients in
hardware-approximate fp32 math, v_rcp / v_log / v_exp / v_rsq) and route(math="faithful")
(DDR_FWD_FAITHFUL_MATH: the reference's operation sequence with IEEE divisions and the pows in fp32
faithful-class arithmetic, like the reference's own Sleef powf).  Neither is bit-identical to the
oracle; both are held to the north star's stated fp32 tolerance (BASELINE.json: max rel err <= 1e-4 vs
the reference fp32) on

* the reference's own golden outputs (tests/golden, made by running the reference),
* the fp32 oracle (same inputs, exact recipe),
* the exact kernel at the full C5 size (800k reaches x 8760 h) and on the C3 daily objective, where
  the oracle cannot run: the exact kernel is itself bit-identical to the oracle
  (test_gpu_fullsize.py), so this pins the fast path to the oracle transitively.

Gradients: the adjoint is the same kernel either way (it recomputes the physics in fast math from the
saved states); only the saved states differ, by the forward's rounding.
"""

import numpy as np
import pytest
import torch

from conftest import PARAMS_DEFAULT, PARAMS_MOCK, golden_case, maxrel, normrel
from ddr_amd import synthetic
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import DailyWindow, GaugeMap, RouteConsts, route
from ddr_amd.routing.utils import denormalize
from oracle import mc_oracle as O
from test_gpu_route import consts_of

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north star: max rel err vs the reference fp32
GOLDEN = [("sandbox", PARAMS_MOCK), ("tree300", PARAMS_DEFAULT), ("c1", PARAMS_DEFAULT)]
MODES = ["fast", "faithful"]


def _run(case, dev, math, gkw=None):
    rng = case.params["parameter_ranges"]
    ls = case.params["log_space_parameters"]
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, torch.float32)  # noqa: E731
    u = {k: (tt(v).requires_grad_(True) if v is not None else None) for k, v in case.u.items()}
    n = denormalize(u["n"], rng["n"], "n" in ls)
    q = denormalize(u["q_spatial"], rng["q_spatial"], "q_spatial" in ls)
    p = (denormalize(u["p_spatial"], rng["p_spatial"], "p_spatial" in ls) if u.get("p_spatial") is not None
         else torch.tensor(float(case.params["defaults"]["p_spatial"]), device=dev))
    slope = torch.clamp(tt(case.slope), min=case.params["attribute_minimums"]["slope"])
    g = RiverGraph(case.n, case.rows, case.cols, **(gkw or {}))
    runoff, q_last, tw, ss = route(g, tt(case.qprime), n, q, p, tt(case.length), slope, tt(case.x),
                                   consts=consts_of(case), math=math)
    runoff.backward(tt(case.W))
    out = {"runoff": runoff.detach().cpu().numpy(), "q_last": q_last.detach().cpu().numpy(),
           "top_width": tw.detach().cpu().numpy(), "side_slope": ss.detach().cpu().numpy(),
           "reaches": O.Reaches(n.detach().cpu().numpy(), q.detach().cpu().numpy(),
                                p.detach().cpu().numpy().astype(np.float32), case.length, slope.detach().cpu().numpy(),
                                case.x)}
    for k, v in u.items():
        if v is not None:
            out[f"grad_{k}"] = v.grad.detach().cpu().numpy()
    return out


@pytest.mark.parametrize("math", MODES)
@pytest.mark.parametrize("name,params", GOLDEN, ids=[g[0] for g in GOLDEN])
@pytest.mark.parametrize("gkw", [None, {"max_block_reaches": 64, "target_blocks": 1 << 20}], ids=["whole", "cut"])
def test_fast_math_matches_reference_golden(cuda, name, params, gkw, math):
    case, d = golden_case(name, params)
    res = _run(case, cuda, math, gkw)
    if "ref_runoff" in d:
        err = maxrel(res["runoff"], d["ref_runoff"])
        print(f"{name} {math}: forward vs reference golden max-rel {err:.2e}")
        assert err <= TOL
    else:
        assert maxrel(res["runoff"][d["sample"]], d["ref_runoff_sample"]) <= TOL
        assert maxrel(res["runoff"][-1], d["ref_outlet"]) <= TOL
    for k in ("q_last", "top_width", "side_slope"):
        assert maxrel(res[k], d[f"ref_{k}"]) <= TOL, k
    for k in ("n", "q_spatial", "p_spatial"):
        if f"ref_grad_{k}" in d:
            assert normrel(res[f"grad_{k}"], d[f"ref_grad_{k}"]) <= 5e-5, k


@pytest.mark.parametrize("math", MODES)
@pytest.mark.parametrize("name,params", GOLDEN, ids=[g[0] for g in GOLDEN])
def test_fast_math_vs_oracle_and_exact_kernel(cuda, name, params, math):
    case, _ = golden_case(name, params)
    fast = _run(case, cuda, math)
    exact = _run(case, cuda, "exact")
    ref = O.route(case.network(), fast["reaches"], case.qprime, case.bounds, dtype=np.float32)
    err = maxrel(fast["runoff"], ref["runoff"])
    print(f"{name}: {math} forward vs fp32 oracle max-rel {err:.2e}")
    assert err <= TOL
    assert maxrel(fast["runoff"], exact["runoff"]) <= TOL
    for k in ("n", "q_spatial", "p_spatial"):
        if f"grad_{k}" in exact:
            assert normrel(fast[f"grad_{k}"], exact[f"grad_{k}"]) <= 5e-5, k


def _chunked_maxrel(a, b, rows=50_000):
    m = 0.0
    for i in range(0, a.shape[0], rows):
        x, y = a[i:i + rows], b[i:i + rows]
        m = max(m, float(((x - y).abs() / y.abs().clamp_min(1e-30)).max()))
    return m


@pytest.mark.parametrize("math", MODES)
def test_fast_math_full_c5_within_tolerance_of_exact(cuda, math):
    """800k reaches x 8760 h: fast vs exact forward (itself bit-identical to the oracle), max-rel over
    all 7e9 values; gradients of a random linear loss norm-rel."""
    net = synthetic.forest(synthetic.zipf_sizes(800_000, 3000, 0.35), seed=5, single_inflow=0.35)
    T = 8760
    at = synthetic.reach_attributes(net.n, 5)
    u = synthetic.unit_parameters(net.n, 5)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    n = tt((u["n"] * np.float32(0.235) + np.float32(0.015)).astype(np.float32))
    q = tt(u["q_spatial"].astype(np.float32))
    lo, hi = np.log(np.float32(1.0 + 1e-6)), np.log(np.float32(200.0))
    p = tt(np.exp(u["p_spatial"] * np.float32(hi - lo) + np.float32(lo)).astype(np.float32))
    length, slope, x = tt(at.length), tt(np.maximum(at.slope, np.float32(1e-3))), tt(at.x)
    qp = synthetic.lateral_inflow_torch(net.n, T, seed=5, device=cuda)
    g = RiverGraph(net.n, net.rows, net.cols)
    gen = torch.Generator(device=cuda).manual_seed(77)
    W = torch.rand((net.n, T), device=cuda, generator=gen)
    outs = {}
    for mode in ("exact", math):
        nt, qt, pt = (v.clone().requires_grad_(True) for v in (n, q, p))
        runoff, _, _, _ = route(g, qp, nt, qt, pt, length, slope, x, consts=RouteConsts(), math=mode)
        runoff.backward(W)
        outs[mode] = (runoff.detach(), nt.grad, qt.grad, pt.grad)
        del runoff
    err = _chunked_maxrel(outs[math][0], outs["exact"][0])
    print(f"C5 full size: {math} vs exact forward max-rel {err:.2e}")
    assert err <= TOL
    for a, b in zip(outs[math][1:], outs["exact"][1:]):
        assert normrel(a.cpu().numpy(), b.cpu().numpy()) <= 5e-5


@pytest.mark.parametrize("math", MODES)
def test_fast_math_c3_daily_objective(cuda, math):
    """The C3 training objective (gauge mode, fused daily pooling) with the fast forward: daily series and
    L1 loss within tolerance of the exact kernel, parameter gradients norm-rel."""
    net = synthetic.forest(synthetic.loguniform_sizes(64, 100, 20000, 3), seed=13, single_inflow=0.25)
    T = 2136
    at = synthetic.reach_attributes(net.n, 13)
    u = synthetic.unit_parameters(net.n, 13)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    n = tt((u["n"] * np.float32(0.235) + np.float32(0.015)).astype(np.float32))
    q = tt(u["q_spatial"].astype(np.float32))
    p = tt((u["p_spatial"] * np.float32(199.0) + np.float32(1.0)).astype(np.float32))
    length, slope, x = tt(at.length), tt(np.maximum(at.slope, np.float32(1e-3))), tt(at.x)
    qp = synthetic.lateral_inflow_torch(net.n, T, seed=13, device=cuda)
    outlets = np.flatnonzero(net.down < 0)
    gz = GaugeMap.build([np.array([o]) for o in outlets], net.n, cuda)
    w = DailyWindow.for_training(T, 3)
    obs = torch.from_numpy(np.random.default_rng(1).lognormal(0, 1, (len(outlets), w.D)).astype(np.float32)).to(cuda)
    g = RiverGraph(net.n, net.rows, net.cols, steps_hint=T)
    res = {}
    for mode in ("exact", math):
        nt, qt, pt = (v.clone().requires_grad_(True) for v in (n, q, p))
        daily, _, _, _ = route(g, qp, nt, qt, pt, length, slope, x, gauges=gz, daily=w, math=mode)
        loss = torch.nn.functional.l1_loss(daily[:, 3:], obs[:, 3:])
        loss.backward()
        res[mode] = (daily.detach().cpu().numpy(), float(loss), nt.grad.cpu().numpy(), qt.grad.cpu().numpy(),
                     pt.grad.cpu().numpy())
    f, e = res[math], res["exact"]
    assert maxrel(f[0], e[0]) <= TOL
    assert abs(f[1] - e[1]) <= TOL * abs(e[1])
    for a, b in zip(f[2:], e[2:]):
        assert normrel(a, b) <= 5e-5
