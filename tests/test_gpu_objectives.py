"""SURVEY §8(f) rows on the HIP path: the fused gauge-mode training objective (f1), the daily q' feed
(f2) and the per-day geometry statistics with the C4 pipeline (f4).

Checkers: the reference's own outputs (tests/golden/daily.npz, geostats.npz, made by running the
reference's io/functions.py, scripts/train.py objective and geometry/statistics.py), the oracle, and
for the daily feed the hourly-expanded input (the reader's repeat(24)), bitwise.
"""

import ctypes as C

import numpy as np
import pytest
import torch

from conftest import load_golden, maxrel, normrel, synthetic_case
from ddr_amd import _lib, synthetic
from ddr_amd.geometry.statistics import compute_geometry_statistics, geometry_statistics_from_inflow
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import DailyWindow, GaugeMap, RouteConsts, route
from oracle import mc_oracle as O

pytestmark = pytest.mark.gpu


def _tt(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


# ---- (f2) daily q' -------------------------------------------------------------------------------


def test_daily_qprime_equals_hourly_repeat(cuda):
    """q'[t / 24] in-kernel == the reader's np.repeat(daily, 24)[:T] (readers.py:513-519), bitwise,
    forward and adjoint; a missing-divide mask == 0.001 columns (readers.py:523-530)."""
    net = synthetic.forest(synthetic.zipf_sizes(3000, 12, 0.4), seed=31, single_inflow=0.3)
    T = 24 * 9 - 24  # (rho - 1) * 24 hourly steps from rho = 9 daily rows
    case = synthetic_case(net, T, 31)
    n, q, p, slope = case.physical()
    daily = synthetic.lateral_inflow(net.n, 9, 32)  # (9, N) daily store
    valid = np.random.default_rng(3).random(net.n) > 0.1
    hourly = np.repeat(daily, 24, axis=0)[:T].copy()
    hourly_filled = hourly.copy()
    hourly_filled[:, ~valid] = np.float32(0.001)
    g = RiverGraph(net.n, net.rows, net.cols, max_block_reaches=512, target_blocks=1 << 20)
    outs = []
    for qp, hours, mask in ((hourly_filled, 1, None), (daily, 24, valid)):
        nt, qt, pt = (_tt(v, cuda).requires_grad_(True) for v in (n, q, p))
        runoff, _, _, _ = route(g, _tt(qp, cuda), nt, qt, pt, _tt(case.length, cuda), _tt(slope, cuda),
                                _tt(case.x, cuda), steps=T, qprime_hours=hours,
                                qprime_valid=None if mask is None else _tt(mask, cuda))
        runoff.backward(_tt(case.W, cuda))
        outs.append([runoff.detach().cpu().numpy(), nt.grad.cpu().numpy(), qt.grad.cpu().numpy(),
                     pt.grad.cpu().numpy()])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


# ---- (f1) fused gauge-mode objective ------------------------------------------------------------


def test_daily_seed_matches_reference_autograd(cuda):
    """The pooling adjoint kernel reproduces torch autograd of the reference objective (daily.npz)."""
    d = load_golden("daily")
    G, T = d["runoff"].shape
    w = DailyWindow.for_training(T, int(d["tau"]))
    assert (w.t0, w.L, w.D) == (13, T - 21, 88)
    # dloss/ddaily of the reference objective (mean absolute error over kept gauges, days >= warmup)
    daily = O.area_downsample(d["runoff"][:, 13:T - 8], w.D)
    keep = ~np.isnan(d["obs"]).any(axis=1)
    diff = daily[keep][:, 3:].astype(np.float64) - d["obs"][keep][:, 3:]
    gd = np.zeros((G, w.D), np.float32)
    gd[np.flatnonzero(keep)[:, None], np.arange(3, w.D)[None, :]] = (np.sign(diff) / diff.size).astype(np.float32)
    gh = torch.empty((G, T), device=cuda)
    _lib.check(_lib.load().ddr_gauge_daily_seed_f32(G, T, w.t0, w.L, w.D, _tt(gd, cuda).data_ptr(), gh.data_ptr(),
                                                    _lib.stream_ptr(cuda)))
    assert maxrel(gh.cpu().numpy(), d["ref_grad"], floor=1e-12) <= 1e-6


def test_fused_daily_objective_matches_unfused_and_oracle(cuda):
    """route(..., gauges, daily=window) == gauge-mode (G, T) output pooled by F.interpolate(area) (the
    reference downsample), values and parameter gradients of the L1 training loss; and equals the
    oracle's objective gradient pushed through its adjoint."""
    net = synthetic.forest(synthetic.loguniform_sizes(12, 50, 800, 5), seed=5, single_inflow=0.25)
    T = 24 * 13
    case = synthetic_case(net, T, 5)
    n, q, p, slope = case.physical()
    down = net.down
    outlets = np.flatnonzero(down < 0)
    outflow = [np.array([o]) for o in outlets]
    outflow[1] = np.array([outlets[1], outlets[2]])  # a two-reach gauge
    gz = GaugeMap.build(outflow, net.n, cuda)
    w = DailyWindow.for_training(T, 3)
    rng = np.random.default_rng(9)
    obs = rng.lognormal(np.log(5.0), 1.0, (len(outflow), w.D)).astype(np.float32)
    obs[4, 2] = np.nan
    keep = torch.from_numpy(~np.isnan(obs).any(axis=1)).to(cuda)
    g = RiverGraph(net.n, net.rows, net.cols, max_block_reaches=256, target_blocks=1 << 20)
    res = {}
    for mode in ("fused", "unfused"):
        nt, qt, pt = (_tt(v, cuda).requires_grad_(True) for v in (n, q, p))
        args = (g, _tt(case.qprime, cuda), nt, qt, pt, _tt(case.length, cuda), _tt(slope, cuda), _tt(case.x, cuda))
        if mode == "fused":
            daily, _, _, _ = route(*args, gauges=gz, daily=w)
        else:
            hourly, _, _, _ = route(*args, gauges=gz)
            daily = torch.nn.functional.interpolate(hourly[:, w.t0:w.t0 + w.L].unsqueeze(1), size=(w.D,),
                                                    mode="area").squeeze(1)
        loss = torch.nn.functional.l1_loss(daily[keep].transpose(0, 1)[3:], _tt(obs, cuda)[keep].transpose(0, 1)[3:])
        loss.backward()
        res[mode] = (daily.detach().cpu().numpy(), float(loss), nt.grad.cpu().numpy(), qt.grad.cpu().numpy(),
                     pt.grad.cpu().numpy())
    f, u = res["fused"], res["unfused"]
    assert maxrel(f[0], u[0]) <= 1e-6
    assert abs(f[1] - u[1]) <= 1e-6 * abs(u[1])
    for a, b in zip(f[2:], u[2:]):
        assert normrel(a, b) <= 1e-5
    # oracle: forward, gauge reduce, objective, adjoint seeded by the objective's hourly gradient
    r = O.Reaches(n, q, p, case.length, slope, case.x)
    ref = O.route(case.network(), r, case.qprime, O.Bounds(), dtype=np.float32, outflow_idx=outflow)
    loss_o, daily_o, gh = O.daily_l1_objective(ref["runoff"], obs, 3, 3)
    assert maxrel(f[0], daily_o) <= 1e-6
    assert abs(f[1] - loss_o) <= 1e-5 * abs(loss_o)
    ref64 = O.route(case.network(), r, case.qprime, O.Bounds(), dtype=np.float64)
    Wg = np.zeros((net.n, T))
    for gi, idx in enumerate(outflow):
        for j in idx:
            Wg[j] += gh[gi]
    bw = O.route_backward(case.network(), r, case.qprime, ref64["x"], Wg, O.Bounds())
    for a, k in zip(f[2:], ("n", "q_spatial", "p_spatial")):
        assert normrel(a, bw[k]) <= 5e-5, k


# ---- (f4) geometry statistics and the C4 pipeline ------------------------------------------------


def test_geometry_statistics_match_reference_golden(cuda):
    d = load_golden("geostats")
    for D in (31, 30):
        for tag, mins in (("default", {"depth": 0.01, "bottom_width": 0.01}), ("mock", {"depth": 0.01, "bottom_width": 0.1})):
            got = compute_geometry_statistics(torch.from_numpy(d["n"]), torch.from_numpy(d["p"]), torch.from_numpy(d["q"]),
                                              torch.from_numpy(d["slope"]), d[f"d{D}_q"], mins)
            orc = O.geometry_statistics(d["n"], d["p"], d["q"], d["slope"], d[f"d{D}_q"],
                                        O.Bounds(bottom_width=mins["bottom_width"]))
            for k, v in got.items():
                ref = d[f"d{D}_{tag}_{k}"]
                assert np.array_equal(np.isnan(v), np.isnan(ref)), k
                ok = ~np.isnan(ref)
                assert maxrel(v[ok], ref[ok]) <= 2e-6, (D, tag, k)  # vs the reference (Sleef powf)
                # vs the oracle (same correctly rounded pow): min / max / median exact; mean within
                # the fp32 rounding of numpy's pairwise sum vs the kernel's fp64 sum
                tol = 1e-6 if k.endswith("_mean") else 0.0
                assert maxrel(v[ok], orc[k][ok]) <= tol, (D, tag, k)


def test_c4_pipeline_matches_oracle(cuda):
    """Daily accumulation of a whole MERIT-shaped forest in one launch (every step a hot start) +
    geometry statistics, against the oracle's day-by-day compute_hotstart_discharge + statistics."""
    net = synthetic.forest(synthetic.zipf_sizes(6000, 20, 0.35), seed=44, single_inflow=0.15)
    D = 45
    at = synthetic.reach_attributes(net.n, 44, x_const=0.3)
    u = synthetic.unit_parameters(net.n, 44)
    n = (u["n"] * np.float32(0.235) + np.float32(0.015)).astype(np.float32)
    q = u["q_spatial"].astype(np.float32)
    lo, hi = np.log(np.float32(1.0 + 1e-6)), np.log(np.float32(200.0))
    p = np.exp(u["p_spatial"] * np.float32(hi - lo) + np.float32(lo)).astype(np.float32)
    slope = np.maximum(at.slope, np.float32(1e-3))
    hourly = synthetic.lateral_inflow(net.n, D * 24, 44)
    q_daily = hourly[::24].copy()  # q'[d * 24] (geometry_predictor.py:206)
    g = RiverGraph(net.n, net.rows, net.cols, max_block_reaches=400, target_blocks=1 << 20)
    got = geometry_statistics_from_inflow(g, _tt(q_daily, cuda), n, p, q, slope)
    acc = O.accumulate_daily(O.Network.from_coo(net.n, net.rows, net.cols), q_daily)
    orc = O.geometry_statistics(n, p, q, slope, acc)
    for k, v in got.items():
        tol = 1e-6 if k.endswith("_mean") else 0.0
        assert maxrel(v, orc[k]) <= tol, k


@pytest.mark.parametrize("D", [513, 1100])
def test_geometry_statistics_long_window(cuda, D):
    """Windows beyond 512 days (multi-year predictor runs; the reference has no cap,
    statistics.py:20-83) take the workgroup-per-reach LDS sort: equal to the oracle, NaN days skipped."""
    rng = np.random.default_rng(D)
    N = 300
    n = rng.uniform(0.015, 0.25, N).astype(np.float32)
    p = rng.uniform(1.0, 200.0, N).astype(np.float32)
    q = rng.uniform(0.0, 1.0, N).astype(np.float32)
    slope = rng.uniform(1e-3, 0.05, N).astype(np.float32)
    qd = rng.lognormal(0.0, 2.0, (D, N)).astype(np.float32)
    qd[rng.random((D, N)) < 0.01] = np.nan
    qd[:, 7] = np.nan  # a reach without a valid day
    got = compute_geometry_statistics(torch.from_numpy(n), torch.from_numpy(p), torch.from_numpy(q),
                                      torch.from_numpy(slope), qd)
    orc = O.geometry_statistics(n, p, q, slope, qd)
    for k, v in got.items():
        assert np.array_equal(np.isnan(v), np.isnan(orc[k])), k
        ok = ~np.isnan(orc[k])
        # means: the kernel sums in fp64, numpy's nanmean pairwise in fp32 -- a few ulp apart over
        # hundreds of days (as test_c4_full_size_sampled_basins); min / max / median exact
        tol = 5e-6 if k.endswith("_mean") else 0.0
        assert maxrel(v[ok], orc[k][ok]) <= tol, (D, k)


def _uniform_params(n_reaches):
    """tests/geometry/test_geometry_stats.py:9-16: uniform parameters for a small network."""
    return {"n": torch.full((n_reaches,), 0.035), "p_spatial": torch.full((n_reaches,), 21.0),
            "q_spatial": torch.full((n_reaches,), 0.5), "slope": torch.full((n_reaches,), 0.001)}


GEO_VARS = ("depth", "top_width", "bottom_width", "side_slope", "hydraulic_radius", "discharge")


def test_geometry_statistics_properties(cuda):
    """The reference's property tests of compute_geometry_statistics (tests/geometry/test_geometry_stats.py:19-58):
    min <= median, mean <= max; a constant discharge gives equal statistics; a reach with higher discharge every
    day is deeper and wider; a custom depth lower bound is respected."""
    q = np.random.default_rng(42).uniform(1.0, 500.0, (30, 10)).astype(np.float32)
    r = compute_geometry_statistics(**_uniform_params(10), daily_accumulated_discharge=q)
    for v in GEO_VARS:
        assert (r[f"{v}_min"] <= r[f"{v}_median"] + 1e-6).all() and (r[f"{v}_median"] <= r[f"{v}_max"] + 1e-6).all()
        assert (r[f"{v}_min"] <= r[f"{v}_mean"] + 1e-6).all() and (r[f"{v}_mean"] <= r[f"{v}_max"] + 1e-6).all()
    r = compute_geometry_statistics(**_uniform_params(5), daily_accumulated_discharge=np.full((10, 5), 25.0, np.float32))
    for v in GEO_VARS:
        for s in ("max", "median", "mean"):
            np.testing.assert_allclose(r[f"{v}_min"], r[f"{v}_{s}"], rtol=1e-5)
    q = np.array([[1.0, 100.0], [2.0, 200.0], [3.0, 300.0]], np.float32)
    r = compute_geometry_statistics(**_uniform_params(2), daily_accumulated_discharge=q)
    assert r["depth_mean"][1] > r["depth_mean"][0] and r["top_width_mean"][1] > r["top_width_mean"][0]
    r = compute_geometry_statistics(**_uniform_params(3), daily_accumulated_discharge=np.full((2, 3), 1e-8, np.float32),
                                    attribute_minimums={"depth": 0.5, "bottom_width": 0.01})
    assert (r["depth_min"] >= 0.5).all()
