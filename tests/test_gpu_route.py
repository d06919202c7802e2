"""GPU parity of the fused HIP routing path (``ddrx::mc_route`` -> libddr_mc.so) against the oracle
and the reference's golden vectors.

Tolerances (BASELINE.json north star):
  * fp32 kernel vs reference fp32 (golden): discharge max-rel <= 1e-4; gradients norm-rel <= 5e-5
    (the reference's own fp32 autograd noise).
  * fp32 kernel vs fp32 oracle (same recipe, correctly rounded pow): max-rel <= 1e-6 (observed 0).
  * fp64 kernel vs fp64 oracle: max-rel <= 1e-6 required, asserted at 1e-12; gradients 1e-10.
Size-independent properties at larger sizes: partition invariance and basin independence (bitwise),
determinism, finite differences.
"""

import numpy as np
import pytest
import torch

from conftest import PARAMS_DEFAULT, PARAMS_MOCK, golden_case, maxrel, normrel, synthetic_case
from ddr_amd import synthetic
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import GaugeMap, RouteConsts, route
from ddr_amd.routing.utils import denormalize
from oracle import mc_oracle as O

pytestmark = pytest.mark.gpu


def consts_of(case):
    m = case.params["attribute_minimums"]
    return RouteConsts(discharge_lb=m["discharge"], velocity_lb=m["velocity"], depth_lb=m["depth"],
                       bottom_width_lb=m["bottom_width"])


def run_hip(case, dev, dtype=torch.float32, gkw=None, gauges=None, q0=None, qprime=None, W=None, grads=True,
            graph=None, math="exact"):
    """Reference recipe on the device: denormalize in torch, fused route, backward(W)."""
    rng = case.params["parameter_ranges"]
    ls = case.params["log_space_parameters"]
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype)  # noqa: E731
    u = {k: (tt(v).requires_grad_(grads) if v is not None else None) for k, v in case.u.items()}
    n = denormalize(u["n"], rng["n"], "n" in ls)
    q = denormalize(u["q_spatial"], rng["q_spatial"], "q_spatial" in ls)
    p = (denormalize(u["p_spatial"], rng["p_spatial"], "p_spatial" in ls) if u.get("p_spatial") is not None
         else torch.tensor(float(case.params["defaults"]["p_spatial"]), device=dev, dtype=dtype))
    slope = torch.clamp(tt(case.slope), min=case.params["attribute_minimums"]["slope"])
    g = graph if graph is not None else RiverGraph(case.n, case.rows, case.cols, **(gkw or {}))
    qp = tt(case.qprime if qprime is None else qprime)
    runoff, q_last, tw, ss = route(g, qp, n, q, p, tt(case.length), slope, tt(case.x), gauges=gauges,
                                   q0=None if q0 is None else tt(q0), consts=consts_of(case), math=math)
    out = {"runoff": runoff.detach().cpu().numpy(), "q_last": q_last.detach().cpu().numpy(),
           "top_width": tw.detach().cpu().numpy(), "side_slope": ss.detach().cpu().numpy(), "graph": g}
    # the exact physical inputs the kernel saw (torch's device expf in the log-space denormalize may
    # differ from NumPy's by an ulp): oracle comparisons use these
    npd = np.float64 if dtype == torch.float64 else np.float32
    out["reaches"] = O.Reaches(n.detach().cpu().numpy(), q.detach().cpu().numpy(),
                               p.detach().cpu().numpy().astype(npd), case.length.astype(npd),
                               slope.detach().cpu().numpy(), case.x.astype(npd))
    if grads:
        runoff.backward(tt(case.W if W is None else W))
        for k, v in u.items():
            if v is not None:
                out[f"grad_{k}"] = v.grad.detach().cpu().numpy()
    torch.cuda.synchronize()
    return out


GOLDEN = [("sandbox", PARAMS_MOCK), ("tree300", PARAMS_DEFAULT), ("c1", PARAMS_DEFAULT)]
PARTITIONS = [None, {"max_block_reaches": 64, "target_blocks": 1 << 20}]


@pytest.mark.parametrize("name,params", GOLDEN, ids=[g[0] for g in GOLDEN])
@pytest.mark.parametrize("gkw", PARTITIONS, ids=["whole", "cut"])
def test_fp32_matches_reference_golden(cuda, name, params, gkw):
    case, d = golden_case(name, params)
    res = run_hip(case, cuda, gkw=gkw)
    if "ref_runoff" in d:
        assert maxrel(res["runoff"], d["ref_runoff"]) <= 1e-4
    else:
        assert maxrel(res["runoff"][d["sample"]], d["ref_runoff_sample"]) <= 1e-4
        assert maxrel(res["runoff"][-1], d["ref_outlet"]) <= 1e-4
    assert maxrel(res["q_last"], d["ref_q_last"]) <= 1e-4
    assert maxrel(res["top_width"], d["ref_top_width"]) <= 1e-4
    assert maxrel(res["side_slope"], d["ref_side_slope"]) <= 1e-4
    for k in ("n", "q_spatial", "p_spatial"):
        if f"ref_grad_{k}" in d:
            assert normrel(res[f"grad_{k}"], d[f"ref_grad_{k}"]) <= 5e-5, k


@pytest.mark.parametrize("name,params", GOLDEN, ids=[g[0] for g in GOLDEN])
def test_fp32_matches_oracle_recipe(cuda, name, params):
    case, _ = golden_case(name, params)
    res = run_hip(case, cuda, grads=False)
    ref = O.route(case.network(), res["reaches"], case.qprime, case.bounds, dtype=np.float32)
    assert maxrel(res["runoff"], ref["runoff"]) <= 1e-6
    assert maxrel(res["q_last"], ref["q_last"]) <= 1e-6


@pytest.mark.parametrize("name,params", GOLDEN[:2], ids=[g[0] for g in GOLDEN[:2]])
@pytest.mark.parametrize("gkw", PARTITIONS, ids=["whole", "cut"])
def test_fp64_matches_fp64_oracle(cuda, name, params, gkw):
    case, _ = golden_case(name, params)
    res = run_hip(case, cuda, dtype=torch.float64, gkw=gkw)
    net, r, bd = case.network(), res["reaches"], case.bounds
    ref = O.route(net, r, case.qprime, bd, dtype=np.float64)
    assert maxrel(res["runoff"], ref["runoff"]) <= 1e-12
    bw = O.route_backward(net, r, case.qprime, ref["x"], case.W, bd)
    u64 = {k: (None if v is None else v.astype(np.float64)) for k, v in case.u.items()}
    g = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], u64["n"], u64["q_spatial"],
                                u64.get("p_spatial"), case.params["parameter_ranges"])
    for k, v in g.items():
        assert normrel(res[f"grad_{k}"], v) <= 1e-10, k
        # north_star's element-wise bar against an fp64 oracle (max rel <= 1e-6), on every gradient element
        # (the floor only keeps exact zeros out of the division)
        assert maxrel(res[f"grad_{k}"], v, floor=1e-30 * float(np.abs(v).max())) <= 1e-6, k


def test_gauge_mode_and_carry_state(cuda):
    case, d = golden_case("gauge", PARAMS_DEFAULT)
    offs = d["outflow_offsets"]
    outflow = [d["outflow_flat"][offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    gz = GaugeMap.build(outflow, case.n, cuda)
    res = run_hip(case, cuda, gauges=gz)
    assert res["runoff"].shape == d["ref_runoff"].shape == (len(outflow), 30)
    assert maxrel(res["runoff"], d["ref_runoff"]) <= 1e-4
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(res[f"grad_{k}"], d[f"ref_grad_{k}"]) <= 5e-5, k
    res2 = run_hip(case, cuda, gauges=gz, q0=d["ref_q_last"], qprime=d["qprime2"], W=d["W2"])
    assert maxrel(res2["runoff"], d["ref2_runoff"]) <= 1e-4
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(res2[f"grad_{k}"], d[f"ref2_grad_{k}"]) <= 5e-5, k


def test_partition_invariance_and_determinism(cuda):
    """Outputs are bitwise identical for any workgroup partition (exchange is exact) and run."""
    net = synthetic.forest(synthetic.zipf_sizes(30000, 60, 0.4), seed=11, single_inflow=0.35)
    case = synthetic_case(net, 200, 11)
    base = run_hip(case, cuda)
    again = run_hip(case, cuda)
    for k in ("runoff", "grad_n", "grad_q_spatial", "grad_p_spatial"):
        np.testing.assert_array_equal(base[k], again[k])
    # cap 64: ~470 blocks, more than the 256 CUs hold at once (ticket-ordered, not co-resident);
    # max_resident 8: the packer's multi-generation mode
    for gkw in ({"max_block_reaches": 160, "target_blocks": 1 << 20}, {"max_block_reaches": 500, "target_blocks": 1 << 20},
                {"max_block_reaches": 64, "target_blocks": 1 << 20},
                {"max_block_reaches": 500, "target_blocks": 1 << 20, "max_resident": 8}):
        alt = run_hip(case, cuda, gkw=gkw)
        assert alt["graph"].info.n_cut > 0
        np.testing.assert_array_equal(alt["runoff"], base["runoff"])
        for k in ("grad_n", "grad_q_spatial", "grad_p_spatial"):
            np.testing.assert_array_equal(alt[k], base[k])


def test_faithful_partition_invariance_with_full_workgroups(cuda):
    """The faithful forward (the drop-in default) is bitwise partition-invariant too, including blocks of
    more than 2048 reaches (KR = 4, whose x slots are double-buffered when the LDS allows) against one
    reach per thread (KR = 1, storer waves) and two (KR = 2)."""
    net = synthetic.forest(synthetic.zipf_sizes(30000, 60, 0.4), seed=12, single_inflow=0.35)
    case = synthetic_case(net, 120, 12)
    big = run_hip(case, cuda, gkw={"target_blocks": 8}, math="faithful")
    assert big["graph"].info.reaches_per_thread == 4 and big["graph"].info.n_cut > 0
    for gkw in ({"max_block_reaches": 500, "target_blocks": 1 << 20}, {"max_block_reaches": 1500, "target_blocks": 1 << 20}):
        alt = run_hip(case, cuda, gkw=gkw, math="faithful")
        assert alt["graph"].info.reaches_per_thread in (1, 2)
        np.testing.assert_array_equal(alt["runoff"], big["runoff"])
        np.testing.assert_array_equal(alt["q_last"], big["q_last"])
        for k in ("grad_n", "grad_q_spatial", "grad_p_spatial"):
            np.testing.assert_array_equal(alt[k], big[k])


def test_basin_independence(cuda):
    """Routing a subset of basins alone equals routing them inside the full forest (bitwise)."""
    from ddr_amd.partition import basin_labels, extract_basins

    net = synthetic.forest(synthetic.zipf_sizes(20000, 40, 0.4), seed=12)
    case = synthetic_case(net, 120, 12)
    full = run_hip(case, cuda, grads=False)
    lab = basin_labels(net.n, net.rows, net.cols)
    keep = np.isin(lab, np.unique(lab)[::3])
    ns, rs, cs, ids = extract_basins(net.n, net.rows, net.cols, keep)
    sub = synthetic.SyntheticNetwork(ns, rs, cs, np.array([ns]))
    sc = synthetic_case(sub, 120, 12)
    sc.length, sc.slope, sc.x = case.length[ids], case.slope[ids], case.x[ids]
    sc.qprime = case.qprime[:, ids]
    sc.u = {k: v[ids] for k, v in case.u.items()}
    part = run_hip(sc, cuda, grads=False)
    np.testing.assert_array_equal(part["runoff"], full["runoff"][ids])


def test_finite_difference_gradient_fp64(cuda):
    net = synthetic.random_binary_tree(40, 9)
    case = synthetic_case(net, 30, 9)
    res = run_hip(case, cuda, dtype=torch.float64)
    rng = np.random.default_rng(0)
    for k in ("n", "q_spatial", "p_spatial"):
        idx = rng.integers(0, net.n, 3)
        for i in idx:
            h = 1e-6
            vals = []
            for s in (+1, -1):
                c2 = synthetic_case(net, 30, 9)
                c2.u = {kk: vv.astype(np.float64).copy() for kk, vv in case.u.items()}
                c2.u[k][i] += s * h
                r = run_hip(c2, cuda, dtype=torch.float64, grads=False)
                vals.append(float(np.sum(r["runoff"] * case.W.astype(np.float64))))
            fd = (vals[0] - vals[1]) / (2 * h)
            assert abs(fd - res[f"grad_{k}"][i]) <= 1e-5 * max(1.0, abs(fd)), (k, i, fd, res[f"grad_{k}"][i])


def test_edge_cases(cuda):
    dev = cuda
    # single reach, T = 1 (hot start only), isolated reaches, a 4-inflow confluence
    for n, rows, cols, T in ((1, [], [], 1), (1, [], [], 5), (6, [], [], 7), (6, [5, 5, 5, 5, 5], [0, 1, 2, 3, 4], 9)):
        net = synthetic.SyntheticNetwork(n, np.array(rows, np.int32), np.array(cols, np.int32), np.array([n]))
        case = synthetic_case(net, T, 3)
        res = run_hip(case, dev, dtype=torch.float64, grads=T > 1)
        ref = O.route(case.network(), res["reaches"], case.qprime, case.bounds, dtype=np.float64)
        assert maxrel(res["runoff"], ref["runoff"]) <= 1e-12
        res32 = run_hip(case, dev, grads=False)
        ref32 = O.route(case.network(), res32["reaches"], case.qprime, case.bounds, dtype=np.float32)
        assert maxrel(res32["runoff"], ref32["runoff"]) <= 1e-6


def test_flow_scale_and_scalar_p(cuda):
    net = synthetic.random_binary_tree(200, 4)
    case = synthetic_case(net, 50, 4, learn_p=False)
    fs = np.random.default_rng(1).uniform(0.3, 1.0, net.n).astype(np.float32)
    n, q, p, slope = case.physical()
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda, torch.float32)  # noqa: E731
    g = RiverGraph(net.n, net.rows, net.cols)
    runoff, _, _, _ = route(g, tt(case.qprime), tt(n), tt(q), torch.tensor(21.0, device=cuda), tt(case.length),
                            tt(slope), tt(case.x), flow_scale=tt(fs), consts=consts_of(case))
    ref = O.route(case.network(), O.Reaches(n, q, np.float32(21.0), case.length, slope, case.x),
                  (case.qprime * fs[None, :]).astype(np.float32), case.bounds)
    assert maxrel(runoff.cpu().numpy(), ref["runoff"]) <= 1e-6


def test_carry_state_below_lower_bound(cuda):
    """Carried Q0 below q_lb enters the first step unclamped; out[:, 0] is clamped (mmc.py:385)."""
    net = synthetic.random_binary_tree(50, 8)
    case = synthetic_case(net, 12, 8)
    q0 = np.full(net.n, 1e-6, np.float32)
    res = run_hip(case, cuda, q0=q0, grads=False)
    ref = O.route(case.network(), res["reaches"], case.qprime, case.bounds, q0=q0, dtype=np.float32)
    assert maxrel(res["runoff"], ref["runoff"]) <= 1e-6
    assert np.all(res["runoff"][:, 0] == np.float32(1e-4))


def test_more_blocks_than_cus_match_oracle(cuda):
    """A schedule of ~470 workgroups (1024 threads each, one per CU) on 256 CUs: later workgroups
    start only when earlier ones finish; ticket ordering keeps it deadlock-free and exact."""
    net = synthetic.hack_basin(30000, seed=21, single_inflow=0.3)
    case = synthetic_case(net, 96, 21)
    res = run_hip(case, cuda, gkw={"max_block_reaches": 64, "target_blocks": 1 << 20})
    assert res["graph"].info.n_blocks > 256
    ref = O.route(case.network(), res["reaches"], case.qprime, case.bounds, dtype=np.float32)
    assert maxrel(res["runoff"], ref["runoff"]) <= 1e-6
    ref64 = O.route(case.network(), res["reaches"], case.qprime, case.bounds, dtype=np.float64)
    bw = O.route_backward(case.network(), res["reaches"], case.qprime, ref64["x"], case.W, case.bounds)
    g = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], case.u["n"], case.u["q_spatial"],
                                case.u["p_spatial"], case.params["parameter_ranges"])
    # a 529-deep Hack basin: fp32 gradients drift further from the fp64 oracle than on the shallow
    # golden trees -- each parameter gradient sums ~T mixed-sign per-step terms in fp32 (as the
    # reference's fp32 autograd accumulates them) and the adjoint recompute uses hardware rcp/log/exp
    # (physics.h adjoint_step_fast); measured 5.5e-5 / 1.3e-4 / 5.4e-5 for n / q / p.  The fp64
    # kernel on the same schedule agrees with the fp64 oracle to 1e-10 (the algorithm is exact).
    for k, v in g.items():
        assert normrel(res[f"grad_{k}"], v) <= 2e-4, k
    res64 = run_hip(case, cuda, dtype=torch.float64, gkw={"max_block_reaches": 64, "target_blocks": 1 << 20})
    u64 = {k: v.astype(np.float64) for k, v in case.u.items()}
    ref64b = O.route(case.network(), res64["reaches"], case.qprime, case.bounds, dtype=np.float64)
    assert maxrel(res64["runoff"], ref64b["runoff"]) <= 1e-12
    bw64 = O.route_backward(case.network(), res64["reaches"], case.qprime, ref64b["x"], case.W, case.bounds)
    g64 = O.param_grads_from_unit(bw64["n"], bw64["q_spatial"], bw64["p_spatial"], u64["n"], u64["q_spatial"],
                                  u64["p_spatial"], case.params["parameter_ranges"])
    for k, v in g64.items():
        assert normrel(res64[f"grad_{k}"], v) <= 1e-10, k
    base = run_hip(case, cuda)
    np.testing.assert_array_equal(base["runoff"], res["runoff"])
    for k in ("grad_n", "grad_q_spatial", "grad_p_spatial"):
        np.testing.assert_array_equal(base[k], res[k])


def test_forced_timeout_raises_on_next_call(cuda):
    """A timed-out inter-workgroup hand-off yields NaN and DDR_ERR_TIMEOUT at the next library call,
    with no DDR_CHECK_STATUS and no host sync in the routing call itself."""
    from ddr_amd import _lib
    from ddr_amd.ops import check_status

    net = synthetic.hack_basin(3000, seed=4)
    case = synthetic_case(net, 40, 4)
    gkw = {"max_block_reaches": 256, "target_blocks": 1 << 20}
    lib = _lib.load()
    check_status()
    _lib.check(lib.ddr_set_debug_flags(_lib.DDR_DEBUG_FORCE_TIMEOUT))
    try:
        bad = run_hip(case, cuda, gkw=gkw, grads=False)
    finally:
        _lib.check(lib.ddr_set_debug_flags(0))
    assert bad["graph"].info.n_cut > 0
    assert np.isnan(bad["runoff"]).any()
    with pytest.raises(_lib.DDRError) as e:
        run_hip(case, cuda, gkw=gkw, grads=False)
    assert e.value.code == _lib.DDR_ERR_TIMEOUT
    # the message names the launch that timed out (its graph handle), not the call that reported it
    assert f"graph {hex(bad['graph'].handle.value)}" in str(e.value), str(e.value)
    assert "forward launch" in str(e.value)
    check_status()  # reported once
    ok = run_hip(case, cuda, gkw=gkw)
    assert np.isfinite(ok["runoff"]).all()
    check_status()


def test_prefetched_batches_match_oracle(cuda):
    """Training-style use: every batch a new adjacency, built on worker threads (GraphPrefetcher) and
    uploaded on the consumer's thread; each routes exactly as the oracle."""
    from ddr_amd.graph import GraphPrefetcher

    cases = [synthetic_case(synthetic.forest(synthetic.loguniform_sizes(6, 50, 800, s), seed=s), 40, s)
             for s in range(3)]
    pf = GraphPrefetcher(((c.n, c.rows, c.cols, c) for c in cases), workers=2, max_block_reaches=128,
                         target_blocks=1 << 20)
    seen = 0
    for g, case in pf:
        assert not g.host_only and g.info.n_cut > 0
        res = run_hip(case, cuda, graph=g)
        ref = O.route(case.network(), res["reaches"], case.qprime, case.bounds, dtype=np.float32)
        assert maxrel(res["runoff"], ref["runoff"]) <= 1e-6
        seen += 1
    assert seen == 3


def test_host_only_graph_is_refused_until_uploaded(cuda):
    from ddr_amd import _lib

    case = synthetic_case(synthetic.random_binary_tree(200, 5), 12, 5)
    g = RiverGraph(case.n, case.rows, case.cols, host_only=True)
    with pytest.raises(_lib.DDRError):
        run_hip(case, cuda, graph=g, grads=False)
    g.upload(cuda)
    res = run_hip(case, cuda, graph=g, grads=False)
    ref = O.route(case.network(), res["reaches"], case.qprime, case.bounds, dtype=np.float32)
    assert maxrel(res["runoff"], ref["runoff"]) <= 1e-6


@pytest.mark.parametrize("which", ["sandbox", "hack5k"])
def test_downstream_accumulation_positive_flow_mass_balance(cuda, which):
    """tests/benchmarks/test_ddr.py:13-91 (the reference's integration checks of DDR routing): after a 50-step
    spin-up the outlet's mean discharge is at least every contributor's, every reach's mean discharge is
    positive, and the outlet's total discharge equals the total lateral inflow within 5 %.  On the RAPID
    Sandbox network of the golden fixture (its 80-hour q' repeated over 2000 h) and on a 5000-reach Hack
    basin (synthetic q', 2000 h)."""
    T = 2000
    if which == "sandbox":
        case, _ = golden_case("sandbox", PARAMS_MOCK)
        case.qprime = np.tile(case.qprime, (T // case.qprime.shape[0] + 1, 1))[:T].copy()
        case.W = np.ones((case.n, T), np.float32)
    else:
        case = synthetic_case(synthetic.hack_basin(5000, seed=8), T, 8)
    res = run_hip(case, cuda, grads=False, math="faithful")
    q = res["runoff"].astype(np.float64)
    down = np.full(case.n, -1)
    down[case.cols] = case.rows
    outlet = int(np.flatnonzero(down < 0)[0])
    assert np.count_nonzero(down < 0) == 1
    spin = 50
    mean = q[:, spin:].mean(axis=1)
    assert np.all(mean > 0)
    for j in np.flatnonzero(down == outlet):
        assert mean[outlet] >= mean[j]
    total_in = float(case.qprime.astype(np.float64).sum())
    total_out = float(q[outlet].sum())
    assert abs(total_out - total_in) / total_in < 0.05, (total_in, total_out)


@pytest.mark.parametrize("name,params", GOLDEN, ids=[g[0] for g in GOLDEN])
def test_fp32_gradients_elementwise_vs_fp64_model(cuda, name, params):
    """north_star's element-wise gradient bar for an fp32 result (max rel <= 1e-4), against the fp64 model (the
    fp64 oracle's forward and adjoint), over the gradient elements above 1e-3 of the largest: the default fp32
    adjoint on the reference's golden networks (measured 5e-6 / 5.2e-5 / 8.8e-5 for Sandbox / tree300 / C1;
    tools/dbg/grad_elementwise.py)."""
    case, _ = golden_case(name, params)
    res = run_hip(case, cuda)
    r32 = res["reaches"]
    r64 = O.Reaches(*(np.asarray(v, np.float64) for v in (r32.n, r32.q, r32.p, r32.length, r32.slope, r32.x)))
    net = case.network()
    fw = O.route(net, r64, case.qprime.astype(np.float64), case.bounds, dtype=np.float64)
    bw = O.route_backward(net, r64, case.qprime.astype(np.float64), fw["x"], case.W.astype(np.float64), case.bounds)
    u64 = {k: (None if v is None else v.astype(np.float64)) for k, v in case.u.items()}
    g = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], u64["n"], u64["q_spatial"],
                                u64.get("p_spatial"), case.params["parameter_ranges"])
    for k, v in g.items():
        a = np.asarray(res[f"grad_{k}"], np.float64)
        m = np.abs(v) >= 1e-3 * np.abs(v).max()
        err = float(np.max(np.abs(a[m] - v[m]) / np.abs(v[m])))
        assert err <= 1e-4, (k, err)
