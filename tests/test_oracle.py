"""The CPU oracle reproduces the reference's own outputs (golden vectors) -- pins the oracle.

Tolerances: the oracle's fp32 path differs from the reference only through PyTorch's 1-ulp Sleef
``powf`` (the oracle's pow is correctly rounded), measured <= 6e-7 max-rel on discharge; the hand
adjoint (fp64) vs the reference's fp32 autograd is ~1e-5 norm-relative (the reference gradient's own
fp32 noise: SURVEY §8(c)).
"""

import numpy as np
import pytest

from conftest import PARAMS_DEFAULT, PARAMS_MOCK, golden_case, load_golden, maxrel, normrel
from oracle import mc_oracle as O

FWD_TOL = 1e-5     # max relative error, discharge
GRAD_TOL = 5e-5    # norm-relative error, parameter gradients


def _grads(case, net, r, res_x, bd, outflow_idx=None, W=None):
    bw = O.route_backward(net, r, case.qprime, res_x, case.W if W is None else W, bd, outflow_idx=outflow_idx)
    return O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], case.u["n"], case.u["q_spatial"],
                                   case.u.get("p_spatial"), case.params["parameter_ranges"])


@pytest.mark.parametrize("name,params", [("sandbox", PARAMS_MOCK), ("tree300", PARAMS_DEFAULT), ("c1", PARAMS_DEFAULT)])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_oracle_matches_reference(name, params, dtype):
    case, d = golden_case(name, params)
    net, r, bd = case.network(), case.reaches(), case.bounds
    res = O.route(net, r, case.qprime, bd, dtype=dtype)
    if "ref_runoff" in d:
        assert maxrel(res["runoff"], d["ref_runoff"]) < FWD_TOL
    else:
        assert maxrel(res["runoff"][d["sample"]], d["ref_runoff_sample"]) < FWD_TOL
        assert maxrel(res["runoff"][-1], d["ref_outlet"]) < FWD_TOL
    assert maxrel(res["q_last"], d["ref_q_last"]) < FWD_TOL
    assert maxrel(res["top_width"], d["ref_top_width"]) < FWD_TOL
    assert maxrel(res["side_slope"], d["ref_side_slope"]) < FWD_TOL
    if name == "c1" and dtype == np.float32:
        return  # one fp64 adjoint check at this size is enough for the CPU suite's time budget
    res64 = res if dtype == np.float64 else O.route(net, r, case.qprime, bd, dtype=np.float64)
    g = _grads(case, net, r, res64["x"], bd)
    for k, v in g.items():
        assert normrel(v, d[f"ref_grad_{k}"]) < GRAD_TOL, k


def test_oracle_gauge_mode_and_carry_state():
    case, d = golden_case("gauge", PARAMS_DEFAULT)
    offs = d["outflow_offsets"]
    outflow = [d["outflow_flat"][offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    net, r, bd = case.network(), case.reaches(), case.bounds
    res = O.route(net, r, case.qprime, bd, outflow_idx=outflow)
    assert res["runoff"].shape == d["ref_runoff"].shape
    assert maxrel(res["runoff"], d["ref_runoff"]) < FWD_TOL
    assert maxrel(res["q_last"], d["ref_q_last"]) < FWD_TOL
    res64 = O.route(net, r, case.qprime, bd, dtype=np.float64, outflow_idx=outflow)
    g = _grads(case, net, r, res64["x"], bd, outflow_idx=outflow)
    for k, v in g.items():
        assert normrel(v, d[f"ref_grad_{k}"]) < GRAD_TOL, k
    # second batch continues from the carried state (mmc.py:330-333)
    res2 = O.route(net, r, d["qprime2"], bd, q0=res["q_last"], outflow_idx=outflow)
    assert maxrel(res2["runoff"], d["ref2_runoff"]) < FWD_TOL
    res2_64 = O.route(net, r, d["qprime2"], bd, q0=res["q_last"], dtype=np.float64, outflow_idx=outflow)
    bw = O.route_backward(net, r, d["qprime2"], res2_64["x"], d["W2"], bd, outflow_idx=outflow)
    g2 = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], case.u["n"], case.u["q_spatial"],
                                 case.u["p_spatial"], case.params["parameter_ranges"])
    for k, v in g2.items():
        assert normrel(v, d[f"ref2_grad_{k}"]) < GRAD_TOL, k


def test_oracle_known_answers():
    """Reference KATs (tests/routing/test_mmc.py:564-602, test_routing_utils.py:18-53)."""
    d = load_golden("kat")
    for name in ("uniform5", "nonuniform4", "single", "clamp3"):
        q = d[f"hot_{name}_q"]
        n = len(q)
        net = O.Network.from_coo(n, np.arange(1, n), np.arange(0, n - 1))
        out = O.hotstart(net, q, O.Bounds(discharge=0.001))
        np.testing.assert_array_equal(out, d[f"hot_{name}_out"])
    np.testing.assert_array_equal(O.hotstart(O.Network.from_coo(5, np.arange(1, 5), np.arange(4)),
                                             np.full(5, 2.0, np.float32), O.Bounds()), [2, 4, 6, 8, 10])
    np.testing.assert_array_equal(O.denormalize(d["den_u"], [0.015, 0.25]), d["den_lin"])
    np.testing.assert_allclose(O.denormalize(d["den_u"], [1.0, 200.0], True), d["den_log"], rtol=2e-7)


def test_coo_to_csr_matches_scipy():
    import scipy.sparse as sp

    rng = np.random.default_rng(0)
    n = 500
    rows = rng.integers(1, n, 3000)
    cols = (rows * rng.uniform(0, 1, 3000)).astype(np.int64)
    vals = rng.uniform(0, 1, 3000).astype(np.float32)
    crow, col, v = O.coo_to_csr(n, rows, cols, vals)
    a = sp.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    np.testing.assert_array_equal(crow, a.indptr)
    np.testing.assert_array_equal(col, a.indices)
    np.testing.assert_allclose(v, a.data, rtol=1e-6)


def test_scipy_recipe_equals_level_sweep():
    from ddr_amd import synthetic

    net = synthetic.forest(synthetic.zipf_sizes(3000, 20, 0.35), seed=2)
    from conftest import synthetic_case

    case = synthetic_case(net, 24, 2)
    a, b = case.network(), case.network()
    b.solver = "scipy"
    r = case.reaches()
    ra, rb = O.route(a, r, case.qprime), O.route(b, r, case.qprime)
    np.testing.assert_array_equal(ra["runoff"], rb["runoff"])


def test_geometry_statistics_oracle_matches_reference_golden():
    """oracle.geometry_statistics restates statistics.py:20-83 (fixture from the reference itself)."""
    d = load_golden("geostats")
    for D in (31, 30):
        for tag, bd in (("default", O.Bounds()), ("mock", O.Bounds(bottom_width=0.1))):
            got = O.geometry_statistics(d["n"], d["p"], d["q"], d["slope"], d[f"d{D}_q"], bd)
            for k, v in got.items():
                ref = d[f"d{D}_{tag}_{k}"]
                assert np.array_equal(np.isnan(v), np.isnan(ref)), k
                ok = ~np.isnan(ref)
                # correctly rounded pow vs the reference's 1-ulp Sleef powf
                assert maxrel(v[ok], ref[ok]) <= 2e-6, (D, tag, k)


def test_daily_objective_oracle_matches_reference_golden():
    """oracle.daily_l1_objective restates train.py:78-97 (downsample + NaN-gauge mask + L1 + warmup)."""
    d = load_golden("daily")
    loss, daily, grad = O.daily_l1_objective(d["runoff"], d["obs"], int(d["tau"]), int(d["warmup"]))
    assert maxrel(daily, d["ref_daily"]) <= 1e-6
    assert abs(loss - float(d["ref_loss"])) <= 1e-6 * abs(float(d["ref_loss"]))
    assert maxrel(grad, d["ref_grad"], floor=1e-12) <= 1e-6


def _state_case():
    from conftest import Case

    d = load_golden("state")
    u = {k: d[f"u_{k}"] for k in ("n", "q_spatial", "p_spatial")}
    case = Case(int(d["n"]), d["rows"], d["cols"], d["length"], d["slope"], d["x"], d["qprime_a"], d["W_a"], u,
                PARAMS_DEFAULT)
    return case, d


def route_timestep_chain(net, r, bd, q0, qclamp, W):
    """The reference's BMI update (mmc.py:487-559) chained K times: loss = sum_k W_k . Q_{k+1}; returns
    (states, dL/dQ0, dL/dq_prime_clamp (K, N), physical parameter gradients summed over the steps)."""
    K = qclamp.shape[0]
    states, xs = [], []
    s = np.asarray(q0, np.float64)
    for k in range(K):
        qp = np.stack([qclamp[k], qclamp[k]]).astype(np.float64)
        res = O.route(net, r, qp, bd, q0=s, dtype=np.float64)
        xs.append(res["x"])
        s = res["q_last"]
        states.append(s)
    g_state = np.zeros(net.n)
    gq = np.zeros((K, net.n))
    gpar = {"n": 0.0, "q_spatial": 0.0, "p_spatial": 0.0}
    for k in range(K - 1, -1, -1):
        G = np.zeros((net.n, 2))
        G[:, 1] = W[k] + g_state
        qp = np.stack([qclamp[k], qclamp[k]]).astype(np.float64)
        bw = O.route_backward(net, r, qp, xs[k], G, bd, want_qprime=True, carry=True)
        g_state = bw["q0"]
        gq[k] = bw["qprime"][0] + bw["qprime"][1]
        for key in gpar:
            gpar[key] = gpar[key] + bw[key]
    return np.stack(states), g_state, gq, gpar


def test_oracle_state_gradients_match_reference():
    """dL/dq' (incl. the hot start's) and dL/dQ0 (carried state, gauge mode with a gauge sum below
    q_lb), and a route_timestep chain, against the reference's autograd (F11)."""
    case, d = _state_case()
    net, r, bd = case.network(), case.reaches(), case.bounds
    # (a) hot-started forward: dL/dstreamflow
    res = O.route(net, r, d["qprime_a"], bd, dtype=np.float64)
    assert maxrel(res["runoff"], d["ref_a_runoff"]) < FWD_TOL
    bw = O.route_backward(net, r, d["qprime_a"], res["x"], d["W_a"], bd, want_qprime=True)
    assert normrel(bw["qprime"], d["ref_a_grad_qprime"]) < GRAD_TOL
    assert maxrel(bw["qprime"][0], d["ref_a_grad_qprime"][0], 1e-3) < 1e-4   # the hot start row
    assert np.all(bw["qprime"][-1] == 0) and np.all(d["ref_a_grad_qprime"][-1] == 0)
    # (b) gauge mode, carried state
    offs = d["outflow_offsets"]
    outflow = [d["outflow_flat"][offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    res = O.route(net, r, d["qprime_b"], bd, q0=d["q0_b"], dtype=np.float64, outflow_idx=outflow)
    assert maxrel(res["runoff"], d["ref_b_runoff"]) < FWD_TOL
    bw = O.route_backward(net, r, d["qprime_b"], res["x"], d["W_b"], bd, outflow_idx=outflow, want_qprime=True,
                          carry=True)
    assert normrel(bw["qprime"], d["ref_b_grad_qprime"]) < GRAD_TOL
    assert normrel(bw["q0"], d["ref_b_grad_q0"]) < GRAD_TOL
    assert d["ref_b_grad_q0"][44] != 0.0  # Q0 below q_lb still feeds step 1 unclamped
    g = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], case.u["n"], case.u["q_spatial"],
                                case.u["p_spatial"], case.params["parameter_ranges"])
    for k, v in g.items():
        assert normrel(v, d[f"ref_b_grad_{k}"]) < GRAD_TOL, k
    # (c) route_timestep chain
    qcl = np.maximum(d["qprime_c"], np.float32(1e-4))
    states, g0, gq, gpar = route_timestep_chain(net, r, bd, d["q0_c"], qcl, d["W_c"])
    assert maxrel(states, d["ref_c_states"]) < FWD_TOL
    assert normrel(g0, d["ref_c_grad_q0"]) < GRAD_TOL
    assert normrel(gq, d["ref_c_grad_qclamp"]) < GRAD_TOL
    g = O.param_grads_from_unit(gpar["n"], gpar["q_spatial"], gpar["p_spatial"], case.u["n"], case.u["q_spatial"],
                                case.u["p_spatial"], case.params["parameter_ranges"])
    for k, v in g.items():
        assert normrel(v, d[f"ref_c_grad_{k}"]) < GRAD_TOL, k


def _chain_case():
    from conftest import Case

    d = load_golden("chain")
    u = {k: d[f"u_{k}"] for k in ("n", "q_spatial", "p_spatial")}
    case = Case(int(d["n"]), d["rows"], d["cols"], d["length"], d["slope"], d["x"], d["qprime_a1"], d["W_a1"], u,
                PARAMS_DEFAULT)
    offs = d["outflow_offsets"]
    outflow = [d["outflow_flat"][offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    return case, d, outflow


def oracle_seeded_grads(case, net, r, bd, qprime, W, outflow, V, T):
    """Forward + adjoint with the loss also on _discharge_t (V[0]), top_width (V[1]) and side_slope (V[2]):
    the geometry's VJP at Q_{T-2} seeds the adjoint's state at T - 2 and adds its own parameter terms."""
    res = O.route(net, r, qprime, bd, dtype=np.float64, outflow_idx=outflow)
    Qp = np.maximum(res["x"][T - 2], bd.discharge)
    gQ, gn2, gq2, gp2 = O.geometry_vjp(Qp, r.n, r.q, r.p, r.slope, bd, V[1], V[2])
    bw = O.route_backward(net, r, qprime, res["x"], W, bd, outflow_idx=outflow, state_seed=np.stack([V[0], gQ]))
    g = O.param_grads_from_unit(bw["n"] + gn2, bw["q_spatial"] + gq2, bw["p_spatial"] + gp2, case.u["n"],
                                case.u["q_spatial"], case.u["p_spatial"], case.params["parameter_ranges"])
    return res, g


def test_oracle_chain_and_geometry_gradients_match_reference():
    """F12: (a) two chained gauge-mode batches, the second carrying the first one's state with its graph --
    dL/dQ0 of batch 2 seeds batch 1's final state; (b, c) a loss also on _discharge_t, top_width and
    side_slope (gauge and all-output mode): the state seeds + the geometry VJP against the reference's
    autograd."""
    case, d, outflow = _chain_case()
    net, r, bd = case.network(), case.reaches(), case.bounds
    T = d["qprime_a1"].shape[0]
    # (a)
    r1 = O.route(net, r, d["qprime_a1"], bd, dtype=np.float64, outflow_idx=outflow)
    r2 = O.route(net, r, d["qprime_a2"], bd, q0=r1["q_last"], dtype=np.float64, outflow_idx=outflow)
    assert maxrel(r1["runoff"], d["ref_a_out1"]) < FWD_TOL
    assert maxrel(r2["runoff"], d["ref_a_out2"]) < FWD_TOL
    b2 = O.route_backward(net, r, d["qprime_a2"], r2["x"], d["W_a2"], bd, outflow_idx=outflow, carry=True)
    b1 = O.route_backward(net, r, d["qprime_a1"], r1["x"], d["W_a1"], bd, outflow_idx=outflow,
                          state_seed=np.stack([b2["q0"], np.zeros(case.n)]))
    assert np.abs(b2["q0"]).max() > 0
    g = O.param_grads_from_unit(b1["n"] + b2["n"], b1["q_spatial"] + b2["q_spatial"], b1["p_spatial"] + b2["p_spatial"],
                                case.u["n"], case.u["q_spatial"], case.u["p_spatial"], case.params["parameter_ranges"])
    for k, v in g.items():
        assert normrel(v, d[f"ref_a_grad_{k}"]) < GRAD_TOL, k
    # (b) gauge mode, (c) all-output mode
    for tag, ofx in (("b", outflow), ("c", None)):
        res, g = oracle_seeded_grads(case, net, r, bd, d[f"qprime_{tag}"], d[f"W_{tag}"], ofx, d[f"V_{tag}"], T)
        assert maxrel(res["runoff"], d[f"ref_{tag}_out"]) < FWD_TOL
        assert maxrel(res["top_width"], d[f"ref_{tag}_top_width"]) < FWD_TOL
        for k, v in g.items():
            assert normrel(v, d[f"ref_{tag}_grad_{k}"]) < GRAD_TOL, (tag, k)
