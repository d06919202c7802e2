"""Parity at BASELINE.json's full sizes (C2: 5k reaches x 8760 h; C3: 256 gauged subnetworks, 896k
reaches x 2136 h; C5: 800k reaches x 8760 h; a 1.0M-reach C5-shaped forest that needs two
generations of workgroups).

The oracle cannot route 800k reaches over a water year in seconds, so the full-size checks use the
properties the domain offers:

* **Basin independence + oracle on samples.** Outlet basins do not interact, so a basin's discharge and
  its reaches' parameter gradients inside the full C5 forest must equal the oracle routing that basin
  alone.  The samples include a basin the partitioner split across several workgroups (cut edges,
  cross-block hand-off over all 8760 steps) and small single-block basins.
* **Partition invariance at full size.** The same multi-block basin routed alone (a different
  workgroup split) gives bitwise the same discharge and gradients as inside the 800k forest.
* **C2 end to end.** The whole 5k-reach Hack-law basin over 8760 h against the oracle (fp32 recipe,
  bitwise expected), which also pins the hot start and the clamp path over a full seasonal cycle.

Tolerances as in test_gpu_route.py: fp32 kernel vs fp32 oracle max-rel <= 1e-6 (observed 0);
gradients vs the fp64 oracle adjoint norm-rel <= 5e-5 (the fp32 adjoint's own rounding).
"""

import numpy as np
import pytest
import torch

from conftest import maxrel, normrel
from ddr_amd import synthetic
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import GaugeMap, RouteConsts, route
from ddr_amd.partition import basin_labels, extract_basins
from oracle import mc_oracle as O

pytestmark = pytest.mark.gpu

RANGES = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}
T_FULL = 8760
T_C3 = 2136  # rho = 90 days: (90 - 1) * 24 hourly steps (dataclasses.py:115-137, example_config rho 90)


def _physical(u):
    """denormalize (utils.py:166-185) in fp32 on the host; the kernel is fed exactly these values."""
    n = (u["n"] * np.float32(RANGES["n"][1] - RANGES["n"][0]) + np.float32(RANGES["n"][0])).astype(np.float32)
    q = (u["q_spatial"] * np.float32(1.0) + np.float32(0.0)).astype(np.float32)
    lo, hi = np.log(np.float32(1.0 + 1e-6)), np.log(np.float32(200.0))
    p = np.exp(u["p_spatial"] * np.float32(hi - lo) + np.float32(lo)).astype(np.float32)
    return n, q, p


class FullForest:
    """One synthetic network resident on the device, routed fwd+bwd once; per-reach inputs kept on host."""

    def __init__(self, net, seed, dev, T=T_FULL, **gkw):
        self.net, self.T, self.dev = net, T, dev
        at = synthetic.reach_attributes(net.n, seed)
        u = synthetic.unit_parameters(net.n, seed)
        self.n, self.q, self.p = _physical(u)
        self.length, self.slope, self.x = at.length, np.maximum(at.slope, np.float32(1e-3)), at.x
        self.qprime = synthetic.lateral_inflow_torch(net.n, T, seed=seed, device=dev)
        gen = torch.Generator(device=dev).manual_seed(seed + 4000)
        self.W = torch.rand((net.n, T), device=dev, dtype=torch.float32, generator=gen)
        self.graph = RiverGraph(net.n, net.rows, net.cols, **gkw)
        self.run(self.graph, np.arange(net.n))

    def run(self, graph, ids):
        tt = lambda a: torch.from_numpy(np.ascontiguousarray(a[ids])).to(self.dev)  # noqa: E731
        n, q, p = (tt(a).requires_grad_(True) for a in (self.n, self.q, self.p))
        full = len(ids) == self.net.n
        qp = self.qprime if full else self.qprime[:, torch.from_numpy(ids).to(self.dev)].contiguous()
        W = self.W if full else self.W[torch.from_numpy(ids).to(self.dev)].contiguous()
        runoff, _, _, _ = route(graph, qp, n, q, p, tt(self.length), tt(self.slope), tt(self.x),
                                consts=RouteConsts())
        runoff.backward(W)
        torch.cuda.synchronize()
        out = {"runoff": runoff.detach(), "gn": n.grad, "gq": q.grad, "gp": p.grad}
        if full:
            self.out = out
        return out

    def basin(self, ids):
        """Subnetwork (topologically ordered COO) of the reaches `ids` (sorted, whole basins)."""
        keep = np.zeros(self.net.n, bool)
        keep[ids] = True
        ns, rs, cs, sel = extract_basins(self.net.n, self.net.rows, self.net.cols, keep)
        assert np.array_equal(sel, ids)
        return ns, rs, cs

    def oracle(self, ids, grads=True):
        ns, rs, cs = self.basin(ids)
        net = O.Network.from_coo(ns, rs, cs)
        r = O.Reaches(self.n[ids], self.q[ids], self.p[ids], self.length[ids], self.slope[ids], self.x[ids])
        qp = self.qprime[:, torch.from_numpy(ids).to(self.dev)].cpu().numpy()
        ref = O.route(net, r, qp, O.Bounds(), dtype=np.float32)
        if grads:
            W = self.W[torch.from_numpy(ids).to(self.dev)].cpu().numpy()
            ref["grads"] = O.route_backward(net, r, qp, ref["x"], W, O.Bounds())
        return ref


@pytest.fixture(scope="module")
def c5(cuda):
    net = synthetic.forest(synthetic.zipf_sizes(800_000, 3000, 0.35), seed=5, single_inflow=0.35)
    ff = FullForest(net, 5, cuda)
    yield ff
    del ff.qprime, ff.W, ff.out
    torch.cuda.empty_cache()


def _basins_by_blocks(ff):
    s = ff.graph.structure()
    lab = basin_labels(ff.net.n, ff.net.rows, ff.net.cols)
    order = np.argsort(lab, kind="stable")
    starts = np.r_[0, np.flatnonzero(np.diff(lab[order])) + 1]
    members = np.split(order, starts[1:])
    nblk = np.array([len(np.unique(s["block"][m])) for m in members])
    return members, nblk


def test_c5_multiblock_basin_matches_oracle_and_is_partition_invariant(c5):
    members, nblk = _basins_by_blocks(c5)
    assert c5.graph.info.n_cut > 0
    multi = [i for i in range(len(members)) if nblk[i] >= 2]
    assert multi, "no basin of the C5 forest spans several workgroups"
    b = min(multi, key=lambda i: len(members[i]))  # the smallest split basin keeps the oracle fast
    ids = np.sort(members[b])
    ref = c5.oracle(ids, grads=False)
    got = c5.out["runoff"][torch.from_numpy(ids).to(c5.dev)].cpu().numpy()
    assert maxrel(got, ref["runoff"]) <= 1e-6
    # the same basin alone: a different partition, bitwise-identical discharge and gradients
    ns, rs, cs = c5.basin(ids)
    alone = c5.run(RiverGraph(ns, rs, cs), ids)
    np.testing.assert_array_equal(alone["runoff"].cpu().numpy(), got)
    sel = torch.from_numpy(ids).to(c5.dev)
    for k in ("gn", "gq", "gp"):
        np.testing.assert_array_equal(alone[k].cpu().numpy(), c5.out[k][sel].cpu().numpy())


def test_c5_small_basins_match_oracle_with_gradients(c5):
    members, nblk = _basins_by_blocks(c5)
    sizes = np.array([len(m) for m in members])
    rng = np.random.default_rng(0)
    cand = np.flatnonzero((sizes >= 20) & (sizes <= 400))
    pick = rng.choice(cand, size=min(4, len(cand)), replace=False)
    ids = np.sort(np.concatenate([members[i] for i in pick]))
    ref = c5.oracle(ids)
    sel = torch.from_numpy(ids).to(c5.dev)
    assert maxrel(c5.out["runoff"][sel].cpu().numpy(), ref["runoff"]) <= 1e-6
    for k, rk in (("gn", "n"), ("gq", "q_spatial"), ("gp", "p_spatial")):
        assert normrel(c5.out[k][sel].cpu().numpy(), ref["grads"][rk]) <= 5e-5, k


def test_c5_giant_basin_oracle_and_partition_invariance(c5):
    """The 281k-reach basin (0.35 N, depth 2215): the longest chain of inter-workgroup hand-offs.
    (1) Routed alone over the first 72 hours, its discharge matches the oracle.  (2) Over the full
    8760 h, routed alone under two other partitions (the basin's own default packing, and 1024-reach
    workgroups), discharge and gradients are bitwise those of the basin inside the 800k forest.
    Gradient accuracy along this chain is pinned against the reference by test_deep_basin_gradients."""
    members, nblk = _basins_by_blocks(c5)
    b = int(np.argmax([len(m) for m in members]))
    ids = np.sort(members[b])
    assert len(ids) > 250_000 and nblk[b] >= 50
    ns, rs, cs = c5.basin(ids)
    sel = torch.from_numpy(ids).to(c5.dev)
    Ts = 72
    short = FullForest.__new__(FullForest)
    short.net, short.T, short.dev = c5.net, Ts, c5.dev
    short.n, short.q, short.p, short.length, short.slope, short.x = c5.n, c5.q, c5.p, c5.length, c5.slope, c5.x
    short.qprime = c5.qprime[:Ts].contiguous()
    short.W = c5.W[:, :Ts].contiguous()
    got = short.run(RiverGraph(ns, rs, cs, steps_hint=Ts), ids)
    ref = short.oracle(ids, grads=False)
    assert maxrel(got["runoff"].cpu().numpy(), ref["runoff"]) <= 1e-6
    del short, got
    full = c5.out["runoff"][sel].cpu().numpy()
    for gkw in ({}, {"max_block_reaches": 1024}):
        g = RiverGraph(ns, rs, cs, **gkw)
        assert g.info.n_cut > 0
        alone = c5.run(g, ids)
        np.testing.assert_array_equal(alone["runoff"].cpu().numpy(), full)
        for k in ("gn", "gq", "gp"):
            np.testing.assert_array_equal(alone[k].cpu().numpy(), c5.out[k][sel].cpu().numpy())
        del alone, g
        torch.cuda.empty_cache()


@pytest.mark.parametrize("t0", [2000, 5000, 8700])
def test_c5_giant_basin_windows_across_the_water_year(c5, t0):
    """The 281k-reach, 2215-deep basin pinned against the oracle across the whole year, not only its first
    hours: the kernel's own state at hour t0 of the full 8760-h run (runoff[:, t0] = Q(t0)) is carried into
    a 36-h window (the reference's carry_state, mmc.py:330-333; scripts/router.py:160-166) and routed
    (1) by the kernel from that state, which must reproduce the full run's hours t0 .. t0 + 35 bit for bit;
    (2) by the fp32 oracle from the same state (max-rel <= 1e-6, bitwise expected); and (3) the window's
    parameter gradients: the fp64 kernel equals the fp64 oracle adjoint (norm-rel <= 1e-10, the algorithm
    is exact), and the fp32 kernel is within the fp32 rounding that accumulates along this chain in any
    fp32 adjoint (the reference's own fp32 gradients on this basin are 2.6e-3 / 7.9e-3 / 4.3e-3 from the
    fp64 adjoint, tests/golden/deep.npz; bar 5e-3 / 1e-2 / 5e-3)."""
    L = 36
    members, _ = _basins_by_blocks(c5)
    ids = np.sort(members[int(np.argmax([len(m) for m in members]))])
    assert len(ids) > 250_000
    ns, rs, cs = c5.basin(ids)
    sel = torch.from_numpy(ids).to(c5.dev)
    full = c5.out["runoff"][sel]
    q0 = full[:, t0].contiguous()
    qp = c5.qprime[t0:t0 + L][:, sel].contiguous()
    gen = torch.Generator(device=c5.dev).manual_seed(t0)
    W = torch.rand((len(ids), L), device=c5.dev, dtype=torch.float32, generator=gen)
    at = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a[ids])).to(c5.dev, dt)  # noqa: E731
    res = {}
    for dt, gkw in ((torch.float32, {}), (torch.float64, {"max_block_reaches": 1024})):
        g = RiverGraph(ns, rs, cs, steps_hint=L, **gkw)
        n, q, p = (at(a, dt).requires_grad_(True) for a in (c5.n, c5.q, c5.p))
        runoff, _, _, _ = route(g, qp.to(dt), n, q, p, at(c5.length, dt), at(c5.slope, dt), at(c5.x, dt),
                                q0=q0.to(dt), consts=RouteConsts())
        runoff.backward(W.to(dt))
        torch.cuda.synchronize()
        res[dt] = {"runoff": runoff.detach().cpu().numpy(),
                   **{k: v.grad.cpu().numpy().astype(np.float64) for k, v in (("n", n), ("q_spatial", q), ("p_spatial", p))}}
        del g, runoff, n, q, p
    got = res[torch.float32]["runoff"]
    np.testing.assert_array_equal(got, full[:, t0:t0 + L].cpu().numpy())  # the full run, continued bit for bit
    net = O.Network.from_coo(ns, rs, cs)
    r = O.Reaches(c5.n[ids], c5.q[ids], c5.p[ids], c5.length[ids], c5.slope[ids], c5.x[ids])
    qn, q0n, Wn = qp.cpu().numpy(), q0.cpu().numpy(), W.cpu().numpy()
    ref = O.route(net, r, qn, O.Bounds(), q0=q0n, dtype=np.float32)
    assert maxrel(got, ref["runoff"]) <= 1e-6
    r64 = O.route(net, r, qn, O.Bounds(), q0=q0n, dtype=np.float64)
    assert maxrel(res[torch.float64]["runoff"], r64["runoff"]) <= 1e-12
    gref = O.route_backward(net, r, qn, r64["x"], Wn, O.Bounds(), carry=True)
    for k, bar in (("n", 5e-3), ("q_spatial", 1e-2), ("p_spatial", 5e-3)):
        assert normrel(res[torch.float64][k], gref[k]) <= 1e-10, k
        assert normrel(res[torch.float32][k], gref[k]) <= bar, k
    torch.cuda.empty_cache()


def test_deep_basin_gradients_vs_reference(cuda):
    """Gradients along a 2215-hop chain (tests/golden/deep.npz: the reference itself on C5's 281k-reach
    basin over 24 h).  fp32 rounding accumulates along the chain in ANY fp32 adjoint: the reference's
    own gradients are 2.6e-3 / 7.9e-3 / 4.3e-3 (norm-rel, n / q / p) from the fp64 adjoint here.  The
    bar: the fp32 kernel is at least as close to the fp64 oracle as the reference, its discharge is
    within the north star's 1e-4 of the reference, and the fp64 kernel agrees with the fp64 oracle to
    1e-10 (the algorithm is exact)."""
    from conftest import deep_case, load_golden

    d = load_golden("deep")
    c = deep_case(int(d["T"]))
    rngs = RANGES
    net = O.Network.from_coo(c.n, c.rows, c.cols)
    tt = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(cuda, dt)  # noqa: E731
    res = {}
    for dt in (torch.float32, torch.float64):
        u = {k: tt(c.u[k], dt).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial")}
        n = u["n"] * (rngs["n"][1] - rngs["n"][0]) + rngs["n"][0]
        q = u["q_spatial"] * (rngs["q_spatial"][1] - rngs["q_spatial"][0]) + rngs["q_spatial"][0]
        lo, hi = np.log(rngs["p_spatial"][0] + 1e-6), np.log(rngs["p_spatial"][1])
        p = torch.exp(u["p_spatial"] * (hi - lo) + lo)
        slope = torch.clamp(tt(c.attrs.slope, dt), min=1e-3)
        # fp64 statics and slots take twice the LDS: smaller workgroups
        g = RiverGraph(c.n, c.rows, c.cols, steps_hint=int(d["T"]),
                       max_block_reaches=1024 if dt == torch.float64 else 0)
        runoff, _, _, _ = route(g, tt(c.qprime, dt), n, q, p, tt(c.attrs.length, dt), slope, tt(c.attrs.x, dt),
                                consts=RouteConsts())
        runoff.backward(tt(c.W, dt))
        torch.cuda.synchronize()
        res[dt] = {"outlet": runoff[c.n - 1].detach().cpu().numpy(),
                   **{k: v.grad.cpu().numpy().astype(np.float64) for k, v in u.items()},
                   "reaches": O.Reaches(n.detach().cpu().numpy(), q.detach().cpu().numpy(), p.detach().cpu().numpy(),
                                        c.attrs.length.astype(np.float64 if dt == torch.float64 else np.float32),
                                        slope.cpu().numpy(), c.attrs.x.astype(np.float64 if dt == torch.float64 else np.float32))}
    assert maxrel(res[torch.float32]["outlet"], d["ref_outlet"]) <= 1e-4
    r64 = res[torch.float64]["reaches"]
    qp64 = c.qprime.astype(np.float64)
    f64 = O.route(net, r64, qp64, O.Bounds(), dtype=np.float64)
    bw = O.route_backward(net, r64, qp64, f64["x"], c.W.astype(np.float64), O.Bounds())
    u64 = {k: c.u[k].astype(np.float64) for k in c.u}
    g64 = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], u64["n"], u64["q_spatial"],
                                  u64["p_spatial"], rngs)
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(res[torch.float64][k], g64[k]) <= 1e-10, k
        ref_err = normrel(d[f"ref_grad_{k}"], g64[k])
        ours = normrel(res[torch.float32][k], g64[k])
        assert ours <= ref_err, (k, ours, ref_err)
        assert normrel(res[torch.float32][k], d[f"ref_grad_{k}"]) <= 2.5 * ref_err, k


def test_c5_outputs_finite_and_bounded(c5):
    r = c5.out["runoff"]
    assert r.shape == (800_000, T_FULL)
    assert bool(torch.isfinite(r).all()) and float(r.min()) >= np.float32(1e-4)
    for k in ("gn", "gq", "gp"):
        assert bool(torch.isfinite(c5.out[k]).all()), k


def test_c2_full_water_year_matches_oracle(cuda):
    net = synthetic.hack_basin(5000, seed=2)
    ff = FullForest(net, 2, cuda)
    ref = ff.oracle(np.arange(net.n), grads=False)
    assert maxrel(ff.out["runoff"].cpu().numpy(), ref["runoff"]) <= 1e-6
    # the benched arithmetic (faithful: IEEE divisions, fp32 pow within 1 ulp) and the fast one, over the
    # whole water year against the same fp32 oracle (correctly rounded pow): north star 1e-4 max-rel
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    for math, tol in (("faithful", 1e-5), ("fast", 1e-4)):
        with torch.no_grad():
            runoff, _, _, _ = route(ff.graph, ff.qprime, tt(ff.n), tt(ff.q), tt(ff.p), tt(ff.length), tt(ff.slope),
                                    tt(ff.x), consts=RouteConsts(), save=False, math=math)
        err = maxrel(runoff.cpu().numpy(), ref["runoff"])
        assert err <= tol, (math, err)


# ---- C3: the training batch of 256 gauged subnetworks ------------------------------------------


@pytest.fixture(scope="module")
def c3(cuda):
    net = synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 3), seed=3, single_inflow=0.25)
    ff = FullForest(net, 3, cuda, T=T_C3, steps_hint=T_C3)
    yield ff
    del ff.qprime, ff.W, ff.out
    torch.cuda.empty_cache()


def test_c3_batch_on_one_gpu_split_basin_matches_oracle(c3):
    """Round 1 could not build C3 (305 co-resident workgroups needed); it now packs into one resident
    generation.  The 20k-reach basin is split across workgroups; it matches the oracle with gradients
    and is bitwise partition invariant (routed alone, it gets a different split)."""
    info = c3.graph.info
    assert info.n == 896_201 and info.n_cut > 0
    assert info.generations == 1 and info.n_blocks <= 256
    members, nblk = _basins_by_blocks(c3)
    sizes = np.array([len(m) for m in members])
    b = int(np.argmax(sizes))
    assert sizes[b] >= 19_000 and nblk[b] >= 2
    ids = np.sort(members[b])
    ref = c3.oracle(ids)
    sel = torch.from_numpy(ids).to(c3.dev)
    got = c3.out["runoff"][sel].cpu().numpy()
    assert maxrel(got, ref["runoff"]) <= 1e-6
    for k, rk in (("gn", "n"), ("gq", "q_spatial"), ("gp", "p_spatial")):
        assert normrel(c3.out[k][sel].cpu().numpy(), ref["grads"][rk]) <= 5e-5, k
    ns, rs, cs = c3.basin(ids)
    alone = c3.run(RiverGraph(ns, rs, cs, steps_hint=T_C3), ids)
    np.testing.assert_array_equal(alone["runoff"].cpu().numpy(), got)
    for k in ("gn", "gq", "gp"):
        np.testing.assert_array_equal(alone[k].cpu().numpy(), c3.out[k][sel].cpu().numpy())


def test_c3_gauge_mode_is_the_outlet_rows(c3):
    """Gauge mode (one gauge per subnetwork outlet, mmc.py:344-363, 405-411) returns exactly the outlet
    rows of the full output, and its adjoint equals the full adjoint with dL/drunoff on those rows."""
    down = c3.net.down
    outlets = np.flatnonzero(down < 0)
    assert len(outlets) == 256
    gz = GaugeMap.build([np.array([o]) for o in outlets], c3.net.n, c3.dev)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(c3.dev)  # noqa: E731
    sel = torch.from_numpy(outlets).to(c3.dev)
    Wg = c3.W[sel].contiguous()
    outs = {}
    for mode in ("gauge", "masked"):
        n, q, p = (tt(a).requires_grad_(True) for a in (c3.n, c3.q, c3.p))
        runoff, _, _, _ = route(c3.graph, c3.qprime, n, q, p, tt(c3.length), tt(c3.slope), tt(c3.x),
                                gauges=gz if mode == "gauge" else None)
        if mode == "gauge":
            runoff.backward(Wg)
            outs[mode] = (runoff.detach()[:, :], n.grad, q.grad, p.grad)
        else:
            Wm = torch.zeros_like(c3.W)
            Wm[sel] = Wg
            runoff.backward(Wm)
            outs[mode] = (runoff.detach()[sel], n.grad, q.grad, p.grad)
            del Wm
        torch.cuda.synchronize()
    for a, b in zip(outs["gauge"], outs["masked"]):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())


# ---- beyond one resident generation -----------------------------------------------------------


def test_1m_forest_two_generations(cuda):
    """1.0M reaches (C5-shaped) exceed 256 workgroups of <= 4096 reaches: the schedule packs into two
    generations of ticket-ordered workgroups and still matches the oracle on sampled basins."""
    net = synthetic.forest(synthetic.zipf_sizes(1_000_000, 3750, 0.35), seed=6, single_inflow=0.35)
    ff = FullForest(net, 6, cuda, T=2190)
    assert ff.graph.info.generations >= 2 and ff.graph.info.n_blocks > 256
    members, nblk = _basins_by_blocks(ff)
    sizes = np.array([len(m) for m in members])
    rng = np.random.default_rng(1)
    cand = np.flatnonzero((sizes >= 20) & (sizes <= 400))
    pick = rng.choice(cand, size=4, replace=False)
    ids = np.sort(np.concatenate([members[i] for i in pick]))
    ref = ff.oracle(ids)
    sel = torch.from_numpy(ids).to(cuda)
    assert maxrel(ff.out["runoff"][sel].cpu().numpy(), ref["runoff"]) <= 1e-6
    for k, rk in (("gn", "n"), ("gq", "q_spatial"), ("gp", "p_spatial")):
        assert normrel(ff.out[k][sel].cpu().numpy(), ref["grads"][rk]) <= 5e-5, k
    multi = [i for i in range(len(members)) if nblk[i] >= 2]
    b = min(multi, key=lambda i: len(members[i]))
    ids = np.sort(members[b])
    ref = ff.oracle(ids, grads=False)
    assert maxrel(ff.out["runoff"][torch.from_numpy(ids).to(cuda)].cpu().numpy(), ref["runoff"]) <= 1e-6
    r = ff.out["runoff"]
    assert bool(torch.isfinite(r).all()) and float(r.min()) >= np.float32(1e-4)
    for k in ("gn", "gq", "gp"):
        assert bool(torch.isfinite(ff.out[k]).all()), k
    del ff.qprime, ff.W, ff.out
    torch.cuda.empty_cache()


# ---- C4: MERIT-shaped 350k reaches, water-year forward + 365-day geometry statistics --------------


def test_c4_full_size_sampled_basins(cuda):
    """BASELINE config 4 at full size: the 350k-reach MERIT-shaped forest (x = 0.3) routed forward over
    8760 h (exact mode) and its 365-day geometry statistics in the fused pipeline.  Basins are
    independent in both, so sampled basins (small ones and a basin split across workgroups) are checked
    against the oracle routing / accumulating that basin alone."""
    from ddr_amd.geometry.statistics import geometry_statistics_from_inflow

    net = synthetic.forest(synthetic.zipf_sizes(350_000, 1000, 0.35), seed=4, single_inflow=0.15)
    T = T_FULL
    at = synthetic.reach_attributes(net.n, 4, x_const=0.3)
    u = synthetic.unit_parameters(net.n, 4)
    n, q, p = _physical(u)
    slope = np.maximum(at.slope, np.float32(1e-3))
    qp = synthetic.lateral_inflow_torch(net.n, T, seed=4, device=cuda)
    g = RiverGraph(net.n, net.rows, net.cols)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    with torch.no_grad():
        runoff, _, _, _ = route(g, qp, tt(n), tt(q), tt(p), tt(at.length), tt(slope), tt(at.x),
                                consts=RouteConsts(), math="exact")
        q_daily = qp[::24][:365].contiguous()
        stats = geometry_statistics_from_inflow(g, q_daily, tt(n), tt(p), tt(q), tt(slope))
    torch.cuda.synchronize()
    assert runoff.shape == (net.n, T) and bool(torch.isfinite(runoff).all())
    ff = FullForest.__new__(FullForest)
    ff.net, ff.T, ff.dev, ff.graph = net, T, cuda, g
    members, nblk = _basins_by_blocks(ff)
    sizes = np.array([len(m) for m in members])
    rng = np.random.default_rng(3)
    cand = np.flatnonzero((sizes >= 20) & (sizes <= 300))
    pick = list(rng.choice(cand, size=3, replace=False))
    multi = [i for i in range(len(members)) if nblk[i] >= 2]
    assert multi
    pick.append(min(multi, key=lambda i: len(members[i])))
    for b in pick:
        ids = np.sort(members[b])
        keep = np.zeros(net.n, bool)
        keep[ids] = True
        ns, rs, cs, _ = extract_basins(net.n, net.rows, net.cols, keep)
        onet = O.Network.from_coo(ns, rs, cs)
        r = O.Reaches(n[ids], q[ids], p[ids], at.length[ids], slope[ids], at.x[ids])
        sel = torch.from_numpy(ids).to(cuda)
        qb = qp[:, sel].cpu().numpy()
        ref = O.route(onet, r, qb, O.Bounds(), dtype=np.float32)
        assert maxrel(runoff[sel].cpu().numpy(), ref["runoff"]) <= 1e-6, b
        acc = O.accumulate_daily(onet, q_daily[:, sel].cpu().numpy())
        orc = O.geometry_statistics(n[ids], p[ids], q[ids], slope[ids], acc)
        for k, v in stats.items():
            # means: the kernel sums the 365 days in fp64, the reference (numpy nanmean on fp32,
            # statistics.py:20-83) pairwise in fp32 -- a few ulp apart at 365 terms; min/max/median exact
            tol = 5e-6 if k.endswith("_mean") else 0.0
            assert maxrel(v[ids], orc[k]) <= tol, (b, k)
    del runoff, qp
    torch.cuda.empty_cache()


def test_c3_as_benched_daily_store_and_objective(cuda):
    """The C3 configuration exactly as bench.py runs it (scripts/train.py:54-104): the 896k-reach batch of
    256 gauged subnetworks over T = 2136 h from a DAILY q' store (89 rows, q'[t // 24], the reader's
    repeat(24), readers.py:513-519) with missing divides filled with 0.001 (readers.py:523-530), one
    gauge per subnetwork outlet, the fused daily objective (trim [13 : -11 + tau], area pooling) and the
    L1 loss over all gauges, backward into n / q / p.

    * exact mode: the daily series of the split 20k-reach basin and of sampled small basins equal the
      oracle's objective on the same hourly inputs; their parameter gradients equal the fp64 oracle
      adjoint seeded by the objective's gradient (norm-rel 5e-5);
    * faithful mode (what the bench times) against exact over the WHOLE batch: daily series within
      1e-5 max-rel, gradients within the north star's 1e-4 (norm-rel)."""
    from ddr_amd.ops import DailyWindow

    net = synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 3), seed=3, single_inflow=0.25)
    T, H = T_C3, 24
    rows = -(-T // H)
    at = synthetic.reach_attributes(net.n, 11)
    u = synthetic.unit_parameters(net.n, 11)
    n, q, p = _physical(u)
    slope = np.maximum(at.slope, np.float32(1e-3))
    qd = synthetic.lateral_inflow_torch(net.n, rows, seed=11, device=cuda)
    valid = np.random.default_rng(12).random(net.n) > 0.02
    outlets = np.flatnonzero(net.down < 0)
    G = len(outlets)
    gz = GaugeMap.build([np.array([o]) for o in outlets], net.n, cuda)
    w = DailyWindow.for_training(T, 3)
    wd = 3
    obs = np.random.default_rng(100).lognormal(np.log(5.0), 1.0, (G, w.D)).astype(np.float32)
    g = RiverGraph(net.n, net.rows, net.cols, steps_hint=T)
    assert g.info.generations == 1
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    res = {}
    for mode in ("exact", "faithful"):
        nt, qt, pt = (tt(a).requires_grad_(True) for a in (n, q, p))
        daily, _, _, _ = route(g, qd, nt, qt, pt, tt(at.length), tt(slope), tt(at.x), gauges=gz, daily=w, steps=T,
                               qprime_hours=H, qprime_valid=tt(valid), consts=RouteConsts(), math=mode)
        loss = torch.nn.functional.l1_loss(daily[:, wd:], tt(obs)[:, wd:], reduction="sum") / (G * (w.D - wd))
        loss.backward()
        torch.cuda.synchronize()
        res[mode] = (daily.detach().cpu().numpy(), nt.grad.cpu().numpy(), qt.grad.cpu().numpy(), pt.grad.cpu().numpy())
    ex, fa = res["exact"], res["faithful"]
    assert maxrel(fa[0], ex[0]) <= 1e-5
    for a, b in zip(fa[1:], ex[1:]):
        assert normrel(a, b) <= 1e-4
    # exact mode vs the oracle on sampled basins (the split 20k basin and four small ones)
    ff = FullForest.__new__(FullForest)
    ff.net, ff.graph = net, g
    members, nblk = _basins_by_blocks(ff)
    sizes = np.array([len(m) for m in members])
    big = int(np.argmax(sizes))
    assert sizes[big] >= 19_000 and nblk[big] >= 2
    cand = np.flatnonzero((sizes >= 50) & (sizes <= 600))
    pick = [big] + list(np.random.default_rng(2).choice(cand, size=4, replace=False))
    ids = np.sort(np.concatenate([members[b] for b in pick]))
    keep = np.zeros(net.n, bool)
    keep[ids] = True
    ns, rs, cs, _ = extract_basins(net.n, net.rows, net.cols, keep)
    onet = O.Network.from_coo(ns, rs, cs)
    r = O.Reaches(n[ids], q[ids], p[ids], at.length[ids], slope[ids], at.x[ids])
    qh = np.repeat(qd[:, torch.from_numpy(ids).to(cuda)].cpu().numpy(), H, axis=0)[:T]
    qh[:, ~valid[ids]] = np.float32(0.001)
    loc_out = np.flatnonzero(net.down[ids] < 0)  # the sampled gauges, in global gauge order
    gsel = np.searchsorted(outlets, ids[loc_out])
    ref = O.route(onet, r, qh, O.Bounds(), dtype=np.float32, outflow_idx=[np.array([o]) for o in loc_out])
    _, daily_o, gh = O.daily_l1_objective(ref["runoff"], obs[gsel], 3, wd)
    assert maxrel(ex[0][gsel], daily_o) <= 1e-6
    # the global loss's gradient on these gauges: the subset objective's, rescaled from its own mean
    Wg = np.zeros((ns, T))
    Wg[loc_out] = gh * (len(gsel) / G)
    ref64 = O.route(onet, r, qh, O.Bounds(), dtype=np.float64)
    bw = O.route_backward(onet, r, qh, ref64["x"], Wg, O.Bounds())
    for a, k in zip(ex[1:], ("n", "q_spatial", "p_spatial")):
        assert normrel(a[ids], bw[k]) <= 5e-5, k
    del qd
    torch.cuda.empty_cache()
