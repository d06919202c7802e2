"""Which fp32 rounding carries the deep-chain gradient error?  CPU only.

The fp32 kernel's gradients on C5's 281k-reach, 2215-deep basin are ~1e-3 norm-relative from the fp64 adjoint
(the reference's own fp32 autograd: 2.6e-3 .. 7.9e-3).  This re-runs the oracle's fp64 adjoint (mc_oracle.
route_backward) on the same fp32 forward states with fp32 rounding injected at ONE place at a time:

  coef32   the recomputed celerity and Muskingum coefficients c1..c4 rounded to fp32 (cel32: the celerity
           only; c1_32: c1 only; c234_32: c2, c3, c4 only) (the kernel's recompute
           is fp32; its hardware rcp / log / exp add ~1e-6 relative on top -- coefhw emulates that as a
           relative perturbation of 1e-6 on c)
  gb32     the transposed solve's per-hop product c1_down gb_down rounded to fp32 (the kernel publishes
           A = fp32(c1 gb64) into LDS; the solve itself accumulates in fp64)
  vjp32    the step's VJP terms (dL/dQ through the coefficients and the parameter terms) rounded to fp32
  lam32    the adjoint state lambda (dL/dQ carried across time) rounded to fp32 each step
  acc32    the parameter gradients accumulated over time in fp32
  all32    all of the above at once

Usage: python tools/grad_terms.py [T=24] [--small]   (prints norm-relative errors vs the fp64 adjoint)
"""
from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddr_amd import synthetic  # noqa: E402
from ddr_amd.partition import basin_labels, extract_basins  # noqa: E402
from oracle import mc_oracle as O  # noqa: E402

F32 = np.float32


def r32(a, on):
    return a.astype(F32).astype(np.float64) if on else a


def adjoint(net, r, qprime, xs, grad_runoff, bd, knobs, dt=3600.0, rng=None):
    """mc_oracle.route_backward (all-output mode, hot start) with fp32 rounding injected per `knobs`."""
    f = np.float64
    r = r.astype(f)
    xs = np.asarray(xs, f)
    qprime = np.asarray(qprime, f)
    T, N = xs.shape
    qlb = bd.discharge
    g_all = np.asarray(grad_runoff, f).T
    Qall = np.maximum(xs, qlb)
    lam = np.zeros(N)
    gn = np.zeros(N)
    gq = np.zeros(N)
    gp = np.zeros(N)
    p_full = np.broadcast_to(r.p, (N,)).astype(f)
    has_down = net.down >= 0
    for t in range(T - 1, 0, -1):
        lam = r32(lam + g_all[t], "lam32" in knobs)
        gx = lam * (xs[t] >= qlb)
        Qp = Qall[t - 1]
        c, _, _ = O.trapezoid_celerity(Qp, r.n, r.q, p_full, r.slope, bd, f)
        if "coefhw" in knobs:
            c = c * (1.0 + 1e-6 * rng.standard_normal(N))
        c = r32(c, "coef32" in knobs or "cel32" in knobs)
        c1, c2, c3, c4 = O.muskingum_coefficients(r.length, c, r.x, dt, f)
        c1 = r32(c1, "coef32" in knobs or "c1_32" in knobs)
        c2, c3, c4 = (r32(v, "coef32" in knobs or "c234_32" in knobs) for v in (c2, c3, c4))
        if "coefhw" in knobs:
            c1, c2, c3, c4 = (v * (1.0 + 1e-6 * rng.standard_normal(N)) for v in (c1, c2, c3, c4))
        # transposed solve (I - C1 N)^T gb = gx, downstream first; the hop product optionally rounded
        gb = gx.copy()
        for nodes in net._down_levels[1:]:
            d = net.down[nodes]
            gb[nodes] = gb[nodes] + r32(c1[d] * gb[d], "gb32" in knobs)
        Sx = net.spmv(xs[t])
        I = net.spmv(Qp)
        qc = np.maximum(qprime[t - 1], qlb)
        gc1, gc2, gc3, gc4 = gb * Sx, gb * I, gb * Qp, gb * qc
        X = r.x
        two_k = 2.0 * (r.length / c)
        den = two_k * (1.0 - X) + dt
        if "xstored" in knobs:       # the r04 kernel's form: Q_{t-1} - x~ taken as Q_{t-1} - (stored fp32 x_t)
            g_twok = gb * (X * (I - Sx) + (1.0 - X) * (Qp - xs[t])) / den
        elif "dform" in knobs:       # x~ = c . (Sx, I, Qp, qc) folded in exactly: coefficients times imbalances
            Sx32, I32 = r32(Sx, "sum32" in knobs), r32(I, "sum32" in knobs)
            D1, D2 = Qp - qc - Sx32, Qp - qc - I32
            g_twok = gb * (D1 * (X + (1.0 - X) * c1) + D2 * ((1.0 - X) * c2 - X)) / den
        else:
            g_twok = (gc1 * (-X - c1 * (1.0 - X)) + gc2 * (X - c2 * (1.0 - X))
                      + gc3 * (1.0 - X) * (1.0 - c3) - gc4 * c4 * (1.0 - X)) / den
        g_c = -2.0 * g_twok * (r.length / c) / c
        gQc, gn_t, gq_t, gp_t = (r32(v, "vjp32" in knobs) for v in O._celerity_vjp(Qp, r.n, r.q, p_full, r.slope, bd, g_c))
        acc = "acc32" in knobs
        gn, gq, gp = r32(gn + gn_t, acc), r32(gq + gq_t, acc), r32(gp + gp_t, acc)
        up_push = np.zeros(N)
        dn = net.down[has_down]
        up_push[has_down] = r32(gb[dn] * c2[dn], "vjp32" in knobs)
        lam = up_push + r32(gb * c3, "vjp32" in knobs) + gQc
    return dict(n=gn, q_spatial=gq, p_spatial=gp)


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 24
    small = "--small" in sys.argv
    t0 = time.time()
    if small:
        net = synthetic.hack_basin(30000, seed=21, single_inflow=0.3)
        ns, rs, cs = net.n, net.rows, net.cols
    else:
        net = synthetic.forest(synthetic.zipf_sizes(800_000, 3000, 0.35), seed=5, single_inflow=0.35)
        lab = basin_labels(net.n, net.rows, net.cols)
        keep = lab == np.bincount(lab).argmax()
        ns, rs, cs, _ = extract_basins(net.n, net.rows, net.cols, keep)
    at = synthetic.reach_attributes(ns, 9)
    u = synthetic.unit_parameters(ns, 9)
    r = O.Reaches(O.denormalize(u["n"], [0.015, 0.25]), O.denormalize(u["q_spatial"], [0.0, 1.0]),
                  O.denormalize(u["p_spatial"], [1.0, 200.0], True), at.length,
                  np.maximum(at.slope, np.float32(1e-3)), at.x)
    qp = synthetic.lateral_inflow(ns, T, 9)
    W = np.random.default_rng(9).uniform(0, 1, (ns, T)).astype(np.float32)
    no = O.Network.from_coo(ns, rs, cs)
    fw = O.route(no, r, qp, O.Bounds(), dtype=np.float32)
    print(f"basin {ns} reaches, depth {int(no.dist.max()) + 1 if hasattr(no, 'dist') else '?'}, T {T}; "
          f"setup + fp32 forward {time.time() - t0:.0f}s", flush=True)
    ref = adjoint(no, r, qp, fw["x"], W, O.Bounds(), set())
    if "--states" in sys.argv:       # the fp64 adjoint on the fp64 forward's states vs on the fp32 forward's
        fw64 = O.route(no, r, qp, O.Bounds(), dtype=np.float64)
        g = adjoint(no, r, qp, fw64["x"], W, O.Bounds(), set())
        print("fp64 states", {k: f"{np.linalg.norm(g[k] - ref[k]) / np.linalg.norm(ref[k]):.2e}" for k in ref}, flush=True)
        g = adjoint(no, r, qp, fw64["x"], W, O.Bounds(), {"xstored"})
        print("fp64 states, xstored", {k: f"{np.linalg.norm(g[k] - ref[k]) / np.linalg.norm(ref[k]):.2e}" for k in ref}, flush=True)
    rng = np.random.default_rng(0)
    sets = [["coef32"], ["cel32"], ["c1_32"], ["c234_32"], ["coefhw"], ["gb32"], ["vjp32"], ["lam32"], ["acc32"],
            ["coef32", "gb32", "vjp32", "lam32", "acc32"]]
    if "--knobs" in sys.argv:
        sets = [k.split("+") for k in sys.argv[sys.argv.index("--knobs") + 1].split(",")]
    for knobs in sets:
        t1 = time.time()
        g = adjoint(no, r, qp, fw["x"], W, O.Bounds(), set(knobs), rng=rng)
        errs = {k: float(np.linalg.norm(g[k] - ref[k]) / np.linalg.norm(ref[k])) for k in ref}
        print("+".join(knobs), {k: f"{v:.2e}" for k, v in errs.items()}, f"({time.time() - t1:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
