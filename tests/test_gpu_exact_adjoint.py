"""The exact adjoint of the fp32 trajectory (ops.route ``exact_adjoint=True``, DDR_BWD_EXACT_ADJOINT).

dL/dk of a Muskingum step is a sum of O(Q) terms that cancels to the step's discharge change.  The default
fp32 adjoint takes that change as Q(t-1) - x(t) from the stored fp32 state; the exact adjoint forms the
step's mass imbalances Q(t-1) - qc - sum_j x_j(t) and Q(t-1) - qc - I(t) exactly (physics.h
adjoint_step_fast).  Checked here against the fp64 oracle adjoint (mc_oracle.route_backward, the hand VJP
of routing/mmc.py:487-559 and utils.py:188-242) run on the kernel's own fp32 states: the default kernel
forward is bit-identical to the oracle's fp32 forward, which the tests assert first, so the oracle's saved
states are the kernel's.

Bars: 1e-5 norm-relative (measured 1.8e-7 / 2.4e-7 / 1.6e-7 for n / q / p on the 2215-deep basin; the
default is 1.6e-3 / 4.7e-3 / 2.4e-3 there).  The forward is the same launch either way (bitwise).
"""

import numpy as np
import pytest
import torch

from conftest import deep_case, normrel
from ddr_amd import synthetic
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import RouteConsts, route
from oracle import mc_oracle as O

pytestmark = pytest.mark.gpu

RANGES = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}
BAR = 1e-5
MAXREL_BAR = 1e-4


def _reaches(u, attrs):
    return O.Reaches(O.denormalize(u["n"], RANGES["n"]), O.denormalize(u["q_spatial"], RANGES["q_spatial"]),
                     O.denormalize(u["p_spatial"], RANGES["p_spatial"], True), attrs.length,
                     np.maximum(attrs.slope, np.float32(1e-3)), attrs.x)


def _kernel(dev, n_reach, rows, cols, r, qp, W, exact, q0=None, gkw=None):
    """fp32 kernel forward + backward; returns runoff and the gradients of sum(W * runoff)."""
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    n, q, p = (tt(v).requires_grad_(True) for v in (r.n, r.q, r.p))
    qpt = tt(qp).requires_grad_(True)
    q0t = tt(q0).requires_grad_(True) if q0 is not None else None
    g = RiverGraph(n_reach, rows, cols, steps_hint=qp.shape[0], **(gkw or {}))
    runoff, _, _, _ = route(g, qpt, n, q, p, tt(r.length), tt(r.slope), tt(r.x), q0=q0t, consts=RouteConsts(),
                            exact_adjoint=exact)
    runoff.backward(tt(W))
    torch.cuda.synchronize()
    out = {"runoff": runoff.detach().cpu().numpy(), "qprime": qpt.grad.cpu().numpy(),
           **{k: t.grad.cpu().numpy().astype(np.float64) for k, t in (("n", n), ("q_spatial", q), ("p_spatial", p))}}
    if q0t is not None:
        out["q0"] = q0t.grad.cpu().numpy()
    return out


def _check(res, bw, keys, bar):
    errs = {k: normrel(res[k], bw[k]) for k in keys}
    for k, e in errs.items():
        assert e <= bar, (k, errs)
    # element-wise: north_star's max-rel bar (1e-4 for an fp32 result) over the elements above 1e-3 of the
    # gradient's largest magnitude (smaller ones carry the fp32 cancellation of their own sums)
    mx = {k: maxrel_above(res[k], bw[k], 1e-3) for k in keys}
    print("normrel", errs, "maxrel", mx)
    for k, e in mx.items():
        assert e <= MAXREL_BAR, (k, mx)
    return errs


def maxrel_above(a, b, frac):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    m = np.abs(b) >= frac * np.abs(b).max()
    return float(np.max(np.abs(a[m] - b[m]) / np.abs(b[m]))) if m.any() else 0.0


def test_exact_adjoint_on_the_deep_basin(cuda):
    """C5's 281k-reach, 2215-deep basin over 24 h (the chain where the default fp32 adjoint is ~1e-3 off)."""
    c = deep_case(24)
    r = _reaches(c.u, c.attrs)
    net = O.Network.from_coo(c.n, c.rows, c.cols)
    fw = O.route(net, r, c.qprime, O.Bounds(), dtype=np.float32)
    bw = O.route_backward(net, r, c.qprime, fw["x"], c.W, O.Bounds())
    base = _kernel(cuda, c.n, c.rows, c.cols, r, c.qprime, c.W, exact=False)
    ex = _kernel(cuda, c.n, c.rows, c.cols, r, c.qprime, c.W, exact=True)
    np.testing.assert_array_equal(base["runoff"], fw["runoff"])   # the oracle's states are the kernel's
    np.testing.assert_array_equal(ex["runoff"], base["runoff"])   # the forward is unchanged
    errs = _check(ex, bw, ("n", "q_spatial", "p_spatial"), BAR)
    base_errs = {k: normrel(base[k], bw[k]) for k in errs}
    print("exact", errs, "default", base_errs)
    assert all(errs[k] < base_errs[k] / 100 for k in errs), (errs, base_errs)


# max_block_reaches 1024 / 2048 / 4096: one, two and four reaches per thread (kr_of_load), each its own kernel
@pytest.mark.parametrize("blk", [1024, 2048, 4096], ids=["kr1", "kr2", "kr4"])
@pytest.mark.parametrize("mode", ["hot", "carry"])
def test_exact_adjoint_state_gradients(cuda, blk, mode):
    """A 529-deep Hack basin over 48 h with dL/dq' (and dL/dQ0 of a carried state): the state-gradient
    kernels (GS) with the exact adjoint, against the fp64 oracle adjoint on the same fp32 states."""
    net = synthetic.hack_basin(30000, seed=21, single_inflow=0.3)
    T = 48
    at = synthetic.reach_attributes(net.n, 21)
    r = _reaches(synthetic.unit_parameters(net.n, 21), at)
    qp = synthetic.lateral_inflow(net.n, T, 21)
    W = np.random.default_rng(21).uniform(0, 1, (net.n, T)).astype(np.float32)
    q0 = np.random.default_rng(22).uniform(0.5, 5.0, net.n).astype(np.float32) if mode == "carry" else None
    netO = O.Network.from_coo(net.n, net.rows, net.cols)
    fw = O.route(netO, r, qp, O.Bounds(), q0=q0, dtype=np.float32)
    bw = O.route_backward(netO, r, qp, fw["x"], W, O.Bounds(), want_qprime=True, carry=q0 is not None)
    ex = _kernel(cuda, net.n, net.rows, net.cols, r, qp, W, exact=True, q0=q0, gkw={"max_block_reaches": blk})
    np.testing.assert_array_equal(ex["runoff"], fw["runoff"])
    keys = ("n", "q_spatial", "p_spatial", "qprime") + (("q0",) if q0 is not None else ())
    _check(ex, bw, keys, BAR)
    if blk == 1024:
        # partition invariance: many small workgroups with cut edges give the same bits
        cut = _kernel(cuda, net.n, net.rows, net.cols, r, qp, W, exact=True, q0=q0,
                      gkw={"max_block_reaches": 64, "target_blocks": 1 << 20})
        for k in keys:
            np.testing.assert_array_equal(cut[k], ex[k], err_msg=k)


def test_exact_adjoint_gauge_daily_store(cuda):
    """Gauge mode over a daily q' store with flow_scale and a missing divide (the C3 training layout: the qc
    re-read goes through the store's row layout), against the fp64 oracle adjoint on the oracle's fp32
    states (the kernel's, bit for bit: exact forward math)."""
    from ddr_amd.ops import GaugeMap

    net = synthetic.hack_basin(30000, seed=23, single_inflow=0.3)
    T, hours = 72, 24
    at = synthetic.reach_attributes(net.n, 23)
    r = _reaches(synthetic.unit_parameters(net.n, 23), at)
    rng = np.random.default_rng(23)
    qstore = synthetic.lateral_inflow(net.n, T // hours, 24)
    fs = rng.uniform(0.5, 1.5, net.n).astype(np.float32)
    valid = np.ones(net.n, np.uint8)
    valid[7] = 0
    outflow = [np.array([net.n - 1]), np.array([100, 200, 300]), np.array([5000])]
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    n, q, p = (tt(v).requires_grad_(True) for v in (r.n, r.q, r.p))
    qp = tt(qstore).requires_grad_(True)
    g = RiverGraph(net.n, net.rows, net.cols, steps_hint=T)
    gz = GaugeMap.build(outflow, net.n, cuda)
    runoff, _, _, _ = route(g, qp, n, q, p, tt(r.length), tt(r.slope), tt(r.x), flow_scale=tt(fs), gauges=gz,
                            consts=RouteConsts(), steps=T, qprime_hours=hours, qprime_valid=torch.from_numpy(valid),
                            exact_adjoint=True)
    W = rng.uniform(0, 1, tuple(runoff.shape)).astype(np.float32)
    runoff.backward(tt(W))
    # the oracle on the hourly, scaled, filled series the kernel routes (fp32, as the kernel's gather forms it)
    qh = np.repeat(qstore, hours, axis=0)[:T].copy()
    qh[:, valid == 0] = np.float32(0.001)
    qh = (qh * fs[None, :]).astype(np.float32)
    netO = O.Network.from_coo(net.n, net.rows, net.cols)
    fw = O.route(netO, r, qh, O.Bounds(), dtype=np.float32, outflow_idx=outflow)
    bw = O.route_backward(netO, r, qh, fw["x"], W, O.Bounds(), outflow_idx=outflow, want_qprime=True)
    gh = bw["qprime"] * fs[None, :].astype(np.float64)
    gh[:, valid == 0] = 0.0
    gstore = np.zeros(qstore.shape)
    for t in range(T):
        gstore[t // hours] += gh[t]
    res = {"n": n.grad, "q_spatial": q.grad, "p_spatial": p.grad}
    for k, v in res.items():
        assert normrel(v.cpu().numpy(), bw[k]) <= BAR, k
    assert normrel(qp.grad.cpu().numpy(), gstore) <= BAR
