"""GPU parity of the state-gradient adjoint: dL/dq' (including the hot start's transposed solve,
mmc.py:25-66) and dL/dQ0 of a carried discharge state, which the reference's autograd delivers
because ``route_timestep`` (mmc.py:487-559) is differentiable w.r.t. ``q_prime_clamp`` and
``_discharge_t``.  Against the reference's own gradients (F11, tests/golden/state.npz) and the fp64
oracle (tests/test_oracle.py pins the oracle to F11 at ~1e-7).

Tolerances: fp32 kernel vs reference fp32 autograd, norm-relative 5e-5 (as the parameter gradients,
SURVEY §8(c)); fp64 kernel vs fp64 oracle, norm-relative 1e-10.
"""

import numpy as np
import pytest
import torch

from conftest import PARAMS_DEFAULT, load_golden, maxrel, normrel
from ddr_amd import synthetic
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import GaugeMap, RouteConsts, route
from ddr_amd.routing.utils import denormalize
from oracle import mc_oracle as O
from test_oracle import _state_case, route_timestep_chain

pytestmark = pytest.mark.gpu

PARTITIONS = [None, {"max_block_reaches": 16, "target_blocks": 1 << 20}]
C = RouteConsts(discharge_lb=1e-4, velocity_lb=0.01, depth_lb=0.01, bottom_width_lb=0.01)


def physical(case, dev, dtype):
    rng = case.params["parameter_ranges"]
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype)  # noqa: E731
    u = {k: tt(v).requires_grad_(True) for k, v in case.u.items()}
    n = denormalize(u["n"], rng["n"])
    q = denormalize(u["q_spatial"], rng["q_spatial"])
    p = denormalize(u["p_spatial"], rng["p_spatial"], True)
    slope = torch.clamp(tt(case.slope), min=case.params["attribute_minimums"]["slope"])
    return u, n, q, p, slope, tt


def reaches_of(n, q, p, slope, case, npd):
    return O.Reaches(n.detach().cpu().numpy(), q.detach().cpu().numpy(), p.detach().cpu().numpy(),
                     case.length.astype(npd), slope.detach().cpu().numpy(), case.x.astype(npd))


@pytest.mark.parametrize("gkw", PARTITIONS, ids=["whole", "cut"])
def test_hotstart_qprime_gradient_matches_reference(cuda, gkw):
    case, d = _state_case()
    u, n, q, p, slope, tt = physical(case, cuda, torch.float32)
    qp = tt(d["qprime_a"]).requires_grad_(True)
    g = RiverGraph(case.n, case.rows, case.cols, **(gkw or {}))
    runoff, _, _, _ = route(g, qp, n, q, p, tt(case.length), slope, tt(case.x), consts=C)
    runoff.backward(tt(d["W_a"]))
    assert maxrel(runoff.detach().cpu().numpy(), d["ref_a_runoff"]) <= 1e-4
    gq = qp.grad.cpu().numpy()
    assert normrel(gq, d["ref_a_grad_qprime"]) <= 5e-5
    assert maxrel(gq[0], d["ref_a_grad_qprime"][0], 1e-2) <= 1e-4  # the hot start's transposed solve
    assert np.all(gq[-1] == 0)                                      # q'[T-1] feeds no step
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(u[k].grad.cpu().numpy(), d[f"ref_a_grad_{k}"]) <= 5e-5, k


@pytest.mark.parametrize("gkw", PARTITIONS, ids=["whole", "cut"])
def test_gauge_carry_state_gradients_match_reference(cuda, gkw):
    case, d = _state_case()
    offs = d["outflow_offsets"]
    outflow = [d["outflow_flat"][offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    u, n, q, p, slope, tt = physical(case, cuda, torch.float32)
    qp = tt(d["qprime_b"]).requires_grad_(True)
    q0 = tt(d["q0_b"]).requires_grad_(True)
    g = RiverGraph(case.n, case.rows, case.cols, **(gkw or {}))
    runoff, _, _, _ = route(g, qp, n, q, p, tt(case.length), slope, tt(case.x), q0=q0,
                            gauges=GaugeMap.build(outflow, case.n, cuda), consts=C)
    runoff.backward(tt(d["W_b"]))
    assert maxrel(runoff.detach().cpu().numpy(), d["ref_b_runoff"]) <= 1e-4
    assert normrel(qp.grad.cpu().numpy(), d["ref_b_grad_qprime"]) <= 5e-5
    g0 = q0.grad.cpu().numpy()
    assert normrel(g0, d["ref_b_grad_q0"]) <= 5e-5
    assert maxrel(g0[[20, 44]], d["ref_b_grad_q0"][[20, 44]]) <= 1e-4  # carried Q0 below q_lb
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(u[k].grad.cpu().numpy(), d[f"ref_b_grad_{k}"]) <= 5e-5, k


def test_route_timestep_chain_gradients_match_reference(cuda):
    """The drop-in MuskingumCunge.route_timestep chained three times (the BMI update): gradients reach
    the initial state, every step's lateral inflow and the parameters, as in the reference."""
    from types import SimpleNamespace

    import scipy.sparse as sp

    from ddr_amd.routing.mmc import MuskingumCunge

    case, d = _state_case()
    a = sp.coo_matrix((np.ones(len(case.rows), np.float32), (case.rows, case.cols)), shape=(case.n, case.n)).tocsr()
    adj = torch.sparse_csr_tensor(torch.from_numpy(a.indptr.astype(np.int64)), torch.from_numpy(a.indices.astype(np.int64)),
                                  torch.from_numpy(a.data), size=(case.n, case.n))
    dc = SimpleNamespace(adjacency_matrix=adj, length=torch.from_numpy(case.length), slope=torch.from_numpy(case.slope),
                         x=torch.from_numpy(case.x), top_width=torch.empty(0), side_slope=torch.empty(0),
                         outflow_idx=None, gage_catchment=None, observations=None, flow_scale=None)
    cfg = SimpleNamespace(params=SimpleNamespace(**PARAMS_DEFAULT))
    mc = MuskingumCunge(cfg, device=cuda)
    sp_params = {k: torch.from_numpy(v).to(cuda).requires_grad_(True) for k, v in case.u.items()}
    mc.setup_inputs(dc, torch.from_numpy(d["qprime_c"]).to(cuda), sp_params)
    s0 = torch.from_numpy(d["q0_c"]).to(cuda).requires_grad_(True)
    mc._discharge_t = s0
    mapper, _, _ = mc.create_pattern_mapper()
    qcl = [torch.clamp(torch.from_numpy(d["qprime_c"][k]).to(cuda), min=1e-4).requires_grad_(True) for k in range(3)]
    loss = 0.0
    states = []
    for k in range(3):
        q1 = mc.route_timestep(q_prime_clamp=qcl[k], mapper=mapper)
        mc._discharge_t = q1
        states.append(q1.detach().cpu().numpy())
        loss = loss + (q1 * torch.from_numpy(d["W_c"][k]).to(cuda)).sum()
    loss.backward()
    assert maxrel(np.stack(states), d["ref_c_states"]) <= 1e-4
    assert normrel(s0.grad.cpu().numpy(), d["ref_c_grad_q0"]) <= 5e-5
    assert normrel(np.stack([v.grad.cpu().numpy() for v in qcl]), d["ref_c_grad_qclamp"]) <= 5e-5
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(sp_params[k].grad.cpu().numpy(), d[f"ref_c_grad_{k}"]) <= 5e-5, k


def test_route_timestep_chain_geometry_gradients_match_reference(cuda):
    """F13 (tests/golden/timestep_geo.npz): three chained route_timestep calls whose loss also takes every
    step's reported top_width / side_slope -- the geometry of the carried state the step starts from
    (mmc.py:527-538, 161-162; two carried values below q_lb, which the geometry reads unclamped).  Its gradient
    reaches the carried state, each step's lateral inflow and the parameters as in the reference's autograd."""
    from types import SimpleNamespace

    import scipy.sparse as sp

    from ddr_amd.routing.mmc import MuskingumCunge

    d = load_golden("timestep_geo")
    n = int(d["n"])
    a = sp.coo_matrix((np.ones(len(d["rows"]), np.float32), (d["rows"], d["cols"])), shape=(n, n)).tocsr()
    adj = torch.sparse_csr_tensor(torch.from_numpy(a.indptr.astype(np.int64)), torch.from_numpy(a.indices.astype(np.int64)),
                                  torch.from_numpy(a.data), size=(n, n))
    dc = SimpleNamespace(adjacency_matrix=adj, length=torch.from_numpy(d["length"]), slope=torch.from_numpy(d["slope"]),
                         x=torch.from_numpy(d["x"]), top_width=torch.empty(0), side_slope=torch.empty(0),
                         outflow_idx=None, gage_catchment=None, observations=None, flow_scale=None)
    mc = MuskingumCunge(SimpleNamespace(params=SimpleNamespace(**PARAMS_DEFAULT)), device=cuda)
    sp_params = {k: torch.from_numpy(d[f"u_{k}"]).to(cuda).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial")}
    mc.setup_inputs(dc, torch.from_numpy(d["qprime"]).to(cuda), sp_params)
    s0 = torch.from_numpy(d["q0"]).to(cuda).requires_grad_(True)
    mc._discharge_t = s0
    mapper, _, _ = mc.create_pattern_mapper()
    qcl = [torch.clamp(torch.from_numpy(d["qprime"][k]).to(cuda), min=1e-4).requires_grad_(True) for k in range(3)]
    t = lambda a_: torch.from_numpy(a_).to(cuda)  # noqa: E731
    loss = 0.0
    states, tws, sss = [], [], []
    for k in range(3):
        q1 = mc.route_timestep(q_prime_clamp=qcl[k], mapper=mapper)
        loss = loss + (q1 * t(d["W"][k])).sum() + (mc.top_width * t(d["V"][k, 0])).sum() \
            + (mc.side_slope * t(d["V"][k, 1])).sum()
        states.append(q1.detach().cpu().numpy())
        tws.append(mc.top_width.detach().cpu().numpy())
        sss.append(mc.side_slope.detach().cpu().numpy())
        mc._discharge_t = q1
    loss.backward()
    assert maxrel(np.stack(states), d["ref_states"]) <= 1e-4
    assert maxrel(np.stack(tws), d["ref_top_width"]) <= 1e-4
    assert maxrel(np.stack(sss), d["ref_side_slope"]) <= 1e-4
    assert normrel(s0.grad.cpu().numpy(), d["ref_grad_q0"]) <= 5e-5
    assert normrel(np.stack([v.grad.cpu().numpy() for v in qcl]), d["ref_grad_qclamp"]) <= 5e-5
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(sp_params[k].grad.cpu().numpy(), d[f"ref_grad_{k}"]) <= 5e-5, k


@pytest.mark.parametrize("gkw", PARTITIONS, ids=["whole", "cut"])
@pytest.mark.parametrize("mode", ["hot", "carry", "gauge_carry", "daily"])
def test_fp64_state_gradients_match_fp64_oracle(cuda, gkw, mode):
    """fp64 kernel vs the fp64 oracle, incl. flow_scale and a daily store with a missing divide (its
    0.001 fill has no gradient)."""
    net = synthetic.random_binary_tree(300, seed=31)
    T = 60
    at = synthetic.reach_attributes(net.n, 31)
    rng = np.random.default_rng(31)
    from conftest import Case

    case = Case(net.n, net.rows, net.cols, at.length, at.slope, at.x, None, None,
                synthetic.unit_parameters(net.n, 31), PARAMS_DEFAULT)
    u, n, q, p, slope, tt = physical(case, cuda, torch.float64)
    hours = 24 if mode == "daily" else 1
    rows = -(-T // hours)
    qstore = synthetic.lateral_inflow(net.n, rows, 32).astype(np.float64)
    qstore[:2, 5] = 1e-6  # below the clamp
    fs = rng.uniform(0.5, 1.5, net.n)
    valid = np.ones(net.n, np.uint8)
    if mode == "daily":
        valid[7] = 0
    q0 = rng.uniform(0.5, 5.0, net.n) if "carry" in mode else None
    if q0 is not None:
        q0[11] = 5e-5
    outflow = [np.array([-1]), np.array([3, 40, 41]), np.array([11]), np.array([100, 200])] if mode == "gauge_carry" else None
    gz = GaugeMap.build(outflow, net.n, cuda) if outflow is not None else None
    qp = tt(qstore).requires_grad_(True)
    q0t = tt(q0).requires_grad_(True) if q0 is not None else None
    g = RiverGraph(net.n, net.rows, net.cols, **(gkw or {}))
    runoff, _, _, _ = route(g, qp, n, q, p, tt(at.length), slope, tt(at.x), flow_scale=tt(fs), q0=q0t, gauges=gz,
                            consts=C, steps=T, qprime_hours=hours,
                            qprime_valid=torch.from_numpy(valid) if mode == "daily" else None)
    W = rng.uniform(0, 1, tuple(runoff.shape))
    runoff.backward(tt(W))
    # the oracle on the hourly, scaled, filled series the kernel routes
    qh = np.repeat(qstore, hours, axis=0)[:T]
    qh[:, valid == 0] = float(np.float32(0.001))  # the reader's fill is a float32 0.001 (readers.py:523-530)
    qh = qh * fs[None, :]
    r = reaches_of(n, q, p, slope, case, np.float64)
    netO = O.Network.from_coo(net.n, net.rows, net.cols)
    bd = O.Bounds(discharge=1e-4, velocity=0.01, depth=0.01, bottom_width=0.01)
    res = O.route(netO, r, qh, bd, q0=q0, dtype=np.float64, outflow_idx=outflow)
    assert maxrel(runoff.detach().cpu().numpy(), res["runoff"]) <= 1e-12
    bw = O.route_backward(netO, r, qh, res["x"], W, bd, outflow_idx=outflow, want_qprime=True, carry=q0 is not None)
    gh = bw["qprime"] * fs[None, :]          # d/dq' of q' * flow_scale
    gh[:, valid == 0] = 0.0                  # the fill is a constant
    gstore = np.zeros_like(qstore)
    for t in range(T):
        gstore[t // hours] += gh[t]
    assert normrel(qp.grad.cpu().numpy(), gstore) <= 1e-10
    if q0 is not None:
        assert normrel(q0t.grad.cpu().numpy(), bw["q0"]) <= 1e-10
    gpar = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], case.u["n"].astype(np.float64),
                                   case.u["q_spatial"].astype(np.float64), case.u["p_spatial"].astype(np.float64),
                                   case.params["parameter_ranges"])
    for k, v in gpar.items():
        assert normrel(u[k].grad.cpu().numpy(), v) <= 1e-10, k


def test_state_gradient_off_by_default_and_partition_invariant(cuda):
    """Without a grad on q' / Q0 the adjoint is the parameter-only kernel (same parameter gradients
    bit for bit); the q' gradient is identical across partitions."""
    case, d = _state_case()
    outs = []
    for gkw, want in ((None, False), (None, True), (PARTITIONS[1], True)):
        u, n, q, p, slope, tt = physical(case, cuda, torch.float32)
        qp = tt(d["qprime_a"]).requires_grad_(want)
        g = RiverGraph(case.n, case.rows, case.cols, **(gkw or {}))
        runoff, _, _, _ = route(g, qp, n, q, p, tt(case.length), slope, tt(case.x), consts=C)
        runoff.backward(tt(d["W_a"]))
        outs.append(({k: v.grad.cpu().numpy() for k, v in u.items()}, qp.grad.cpu().numpy() if want else None))
    for k in outs[0][0]:
        assert np.array_equal(outs[0][0][k], outs[1][0][k]), k
        assert np.array_equal(outs[1][0][k], outs[2][0][k]), k
    assert np.array_equal(outs[1][1], outs[2][1])


def _dropin(case, outflow, cuda):
    """A drop-in MuskingumCunge on the case's network (RoutingDataclass stand-in: CSR adjacency)."""
    from types import SimpleNamespace

    import scipy.sparse as sp

    from ddr_amd.routing.mmc import MuskingumCunge

    a = sp.coo_matrix((np.ones(len(case.rows), np.float32), (case.rows, case.cols)), shape=(case.n, case.n)).tocsr()
    adj = torch.sparse_csr_tensor(torch.from_numpy(a.indptr.astype(np.int64)), torch.from_numpy(a.indices.astype(np.int64)),
                                  torch.from_numpy(a.data), size=(case.n, case.n))
    dc = SimpleNamespace(adjacency_matrix=adj, length=torch.from_numpy(case.length), slope=torch.from_numpy(case.slope),
                         x=torch.from_numpy(case.x), top_width=torch.empty(0), side_slope=torch.empty(0),
                         outflow_idx=outflow, gage_catchment=None, observations=None, flow_scale=None)
    cfg = SimpleNamespace(params=SimpleNamespace(**PARAMS_DEFAULT))
    return MuskingumCunge(cfg, device=cuda), dc


def test_chained_gauge_batches_backpropagate_into_the_first_state(cuda):
    """F12 (a): the second gauge-mode batch carries the first one's _discharge_t with its graph
    (mmc.py:330-333, 433-441); one loss over both batches reaches the first batch through its final state
    (the adjoint's q_last seed in gauge mode), as the reference's autograd does."""
    from test_oracle import _chain_case

    case, d, outflow = _chain_case()
    mc, dc = _dropin(case, outflow, cuda)
    sp_params = {k: torch.from_numpy(v).to(cuda).requires_grad_(True) for k, v in case.u.items()}
    mc.setup_inputs(dc, torch.from_numpy(d["qprime_a1"]).to(cuda), sp_params)
    o1 = mc.forward()
    mc.setup_inputs(dc, torch.from_numpy(d["qprime_a2"]).to(cuda), sp_params, carry_state=True)
    o2 = mc.forward()
    ((o1 * torch.from_numpy(d["W_a1"]).to(cuda)).sum() + (o2 * torch.from_numpy(d["W_a2"]).to(cuda)).sum()).backward()
    assert maxrel(o1.detach().cpu().numpy(), d["ref_a_out1"]) <= 1e-4
    assert maxrel(o2.detach().cpu().numpy(), d["ref_a_out2"]) <= 1e-4
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(sp_params[k].grad.cpu().numpy(), d[f"ref_a_grad_{k}"]) <= 5e-5, k


@pytest.mark.parametrize("tag", ["b", "c"], ids=["gauge", "all_output"])
def test_final_state_and_geometry_gradients_match_reference(cuda, tag):
    """F12 (b, c): a loss on the output, on _discharge_t (retained by dmc, torch_mc.py:196-216) and on the
    reported top_width / side_slope (mmc.py:161-162) -- gauge and all-output mode."""
    from test_oracle import _chain_case

    case, d, outflow = _chain_case()
    mc, dc = _dropin(case, outflow if tag == "b" else None, cuda)
    sp_params = {k: torch.from_numpy(v).to(cuda).requires_grad_(True) for k, v in case.u.items()}
    mc.setup_inputs(dc, torch.from_numpy(d[f"qprime_{tag}"]).to(cuda), sp_params)
    out = mc.forward()
    V = torch.from_numpy(d[f"V_{tag}"]).to(cuda)
    loss = ((out * torch.from_numpy(d[f"W_{tag}"]).to(cuda)).sum() + (mc._discharge_t * V[0]).sum()
            + (mc.top_width * V[1]).sum() + (mc.side_slope * V[2]).sum())
    loss.backward()
    assert maxrel(out.detach().cpu().numpy(), d[f"ref_{tag}_out"]) <= 1e-4
    assert maxrel(mc.top_width.detach().cpu().numpy(), d[f"ref_{tag}_top_width"]) <= 1e-4
    for k in ("n", "q_spatial", "p_spatial"):
        assert normrel(sp_params[k].grad.cpu().numpy(), d[f"ref_{tag}_grad_{k}"]) <= 5e-5, (tag, k)


@pytest.mark.parametrize("gkw", PARTITIONS, ids=["whole", "cut"])
@pytest.mark.parametrize("gauge", [False, True], ids=["all_output", "gauge"])
def test_fp64_seeded_adjoint_matches_fp64_oracle(cuda, gkw, gauge):
    """fp64 kernel vs the fp64 oracle with the state seeds (dL/d q_last) and the geometry VJP, plus dL/dq'
    (the state-gradient kernel reads the seeds too)."""
    from test_oracle import _chain_case, oracle_seeded_grads

    case, d, outflow = _chain_case()
    ofx = outflow if gauge else None
    u, n, q, p, slope, tt = physical(case, cuda, torch.float64)
    T = 24
    qp = tt(d["qprime_b"]).requires_grad_(True)
    g = RiverGraph(case.n, case.rows, case.cols, **(gkw or {}))
    gz = GaugeMap.build(ofx, case.n, cuda) if gauge else None
    runoff, q_last, tw, ss = route(g, qp, n, q, p, tt(case.length), slope, tt(case.x), gauges=gz, consts=C)
    rng = np.random.default_rng(5)
    W = rng.uniform(0, 1, tuple(runoff.shape))
    V = rng.uniform(-1, 1, (3, case.n))
    loss = (runoff * tt(W)).sum() + (q_last * tt(V[0])).sum() + (tw * tt(V[1])).sum() + (ss * tt(V[2])).sum()
    loss.backward()
    net, r, bd = case.network(), reaches_of(n, q, p, slope, case, np.float64), case.bounds
    res, gpar = oracle_seeded_grads(case, net, r, bd, d["qprime_b"].astype(np.float64), W, ofx, V, T)
    assert maxrel(runoff.detach().cpu().numpy(), res["runoff"]) <= 1e-12
    for k, v in gpar.items():
        assert normrel(u[k].grad.cpu().numpy(), v) <= 1e-10, k
    assert qp.grad is not None and bool(torch.isfinite(qp.grad).all())


def test_fp64_backward_single_buffer_at_kr2(cuda):
    """fp64 at two reaches per thread: the double-buffered backward slots (96 B per slot) do not fit the LDS
    for blocks above ~1.67K reaches, so the launch takes the single-buffered variant (bwd_xb_of) instead of failing
    with DDR_ERR_CAPACITY; gradients equal the fp64 oracle's."""
    net = synthetic.random_binary_tree(1900, seed=41)
    T = 24
    at = synthetic.reach_attributes(net.n, 41)
    from conftest import Case

    case = Case(net.n, net.rows, net.cols, at.length, at.slope, at.x, None, None,
                synthetic.unit_parameters(net.n, 41), PARAMS_DEFAULT)
    u, n, q, p, slope, tt = physical(case, cuda, torch.float64)
    g = RiverGraph(net.n, net.rows, net.cols, target_blocks=1)  # one 1900-reach block
    assert g.info.reaches_per_thread == 2 and g.info.n_blocks == 1
    qs = synthetic.lateral_inflow(net.n, T, 41).astype(np.float64)
    runoff, _, _, _ = route(g, tt(qs), n, q, p, tt(at.length), slope, tt(at.x), consts=C)
    W = np.random.default_rng(41).uniform(0, 1, tuple(runoff.shape))
    runoff.backward(tt(W))
    r = reaches_of(n, q, p, slope, case, np.float64)
    netO = O.Network.from_coo(net.n, net.rows, net.cols)
    res = O.route(netO, r, qs, case.bounds, dtype=np.float64)
    assert maxrel(runoff.detach().cpu().numpy(), res["runoff"]) <= 1e-12
    bw = O.route_backward(netO, r, qs, res["x"], W, case.bounds)
    gpar = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], case.u["n"].astype(np.float64),
                                   case.u["q_spatial"].astype(np.float64), case.u["p_spatial"].astype(np.float64),
                                   case.params["parameter_ranges"])
    for k, v in gpar.items():
        assert normrel(u[k].grad.cpu().numpy(), v) <= 1e-10, k
