"""World-size-2 (gloo, CPU) test of the multi-rank path: basin sharding + gradient all-reduce.

Each rank routes only its outlet basins (oracle as the per-rank compute -- CPU test), back-propagates
into a shared parameter network, and the all-reduced gradient equals the single-process gradient.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PARAMS_DEFAULT, synthetic_case

T = 16


def _problem():
    from ddr_amd import synthetic

    net = synthetic.forest(synthetic.loguniform_sizes(12, 20, 400, 1), seed=3)
    case = synthetic_case(net, T, 3)
    feats = np.random.default_rng(5).normal(size=(net.n, 4)).astype(np.float32)
    return net, case, feats


def _loss_grad(net_rows, net_cols, n, ids, case, feats, weight):
    """dL/dweight for the reaches `ids` (loss = sum W * runoff, routed by the oracle)."""
    from oracle import mc_oracle as O

    w = torch.tensor(weight, requires_grad=True)
    u = torch.sigmoid(torch.from_numpy(feats[ids]) @ w)  # (n_sub, 3): KAN-like parameter net
    uu = u.detach().numpy().astype(np.float32)
    rngs = PARAMS_DEFAULT["parameter_ranges"]
    nn_ = O.denormalize(uu[:, 0], rngs["n"])
    qq = O.denormalize(uu[:, 1], rngs["q_spatial"])
    pp = O.denormalize(uu[:, 2], rngs["p_spatial"], True)
    slope = np.maximum(case.slope[ids], np.float32(1e-3))
    r = O.Reaches(nn_, qq, pp, case.length[ids], slope, case.x[ids])
    net = O.Network.from_coo(n, net_rows, net_cols)
    qp = case.qprime[:, ids]
    res = O.route(net, r, qp, dtype=np.float64)
    bw = O.route_backward(net, r, qp, res["x"], case.W[ids])
    g = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], uu[:, 0], uu[:, 1], uu[:, 2], rngs)
    gu = torch.from_numpy(np.stack([g["n"], g["q_spatial"], g["p_spatial"]], 1).astype(np.float32))
    u.backward(gu)
    return w.grad.numpy()


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from ddr_amd.distributed import allreduce_gradients, shard_network

    dist.init_process_group("gloo", rank=rank, world_size=world)
    net, case, feats = _problem()
    weight = np.random.default_rng(9).normal(size=(4, 3)).astype(np.float32) * 0.3
    ns, rs, cs, ids = shard_network(net.n, net.rows, net.cols, rank, world)
    p = torch.nn.Parameter(torch.zeros(4, 3))
    p.grad = torch.from_numpy(_loss_grad(rs, cs, ns, ids, case, feats, weight))
    allreduce_gradients([p])
    n_local = torch.tensor([float(ns)])
    dist.all_reduce(n_local)
    out[rank] = (p.grad.numpy().copy(), float(n_local), ids)
    dist.destroy_process_group()


def test_two_rank_basin_sharding_and_grad_allreduce():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = 2
    ctx = mp.get_context("spawn")
    manager = ctx.Manager()
    out = manager.dict()
    procs = [ctx.Process(target=_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    net, case, feats = _problem()
    weight = np.random.default_rng(9).normal(size=(4, 3)).astype(np.float32) * 0.3
    full = _loss_grad(net.rows, net.cols, net.n, np.arange(net.n), case, feats, weight)
    g0, n0, ids0 = out[0]
    g1, n1, ids1 = out[1]
    assert n0 == n1 == net.n  # every reach routed exactly once
    assert len(np.intersect1d(ids0, ids1)) == 0
    np.testing.assert_allclose(g0, g1)
    # fp32 sums over reaches in a different grouping: equal to summation-order rounding
    np.testing.assert_allclose(g0, full, rtol=2e-4, atol=1e-5)


def test_lpt_balance():
    from ddr_amd.partition import lpt_assign, shard_basins

    sizes = np.array([100, 90, 50, 40, 30, 20, 10, 5, 5, 1])
    owner = lpt_assign(sizes, 3)
    loads = np.bincount(owner, weights=sizes, minlength=3)
    assert loads.max() - loads.min() <= sizes.max()
    shards = shard_basins(sizes, 3)
    assert sorted(np.concatenate(shards).tolist()) == list(range(len(sizes)))


@pytest.mark.parametrize("world", [1, 2, 4])
def test_shard_network_covers_every_reach(world):
    from ddr_amd.distributed import shard_network

    net, _, _ = _problem()
    seen = []
    for r in range(world):
        ns, rs, cs, ids = shard_network(net.n, net.rows, net.cols, r, world)
        assert ns == len(ids)
        if len(rs):
            assert np.all(rs > cs)  # still topologically ordered
        seen.append(ids)
    np.testing.assert_array_equal(np.sort(np.concatenate(seen)), np.arange(net.n))


# ---- C3 training objective over ranks: gauges sharded with their basins ---------------------------

T_DAILY = 96  # 4 days: window [13, 88), 3 pooled days


def _objective_grad(rows, cols, n, ids, case, feats, weight, outlets_global, obs, g_global, warmup=1):
    """This rank's share of the global mean daily L1 (train.py:78-97, one gauge per basin outlet) and
    its gradient w.r.t. the parameter-network weight; plus its (G_local, D) daily series."""
    from oracle import mc_oracle as O

    w = torch.tensor(weight, requires_grad=True)
    u = torch.sigmoid(torch.from_numpy(feats[ids]) @ w)
    uu = u.detach().numpy().astype(np.float32)
    rngs = PARAMS_DEFAULT["parameter_ranges"]
    r = O.Reaches(O.denormalize(uu[:, 0], rngs["n"]), O.denormalize(uu[:, 1], rngs["q_spatial"]),
                  O.denormalize(uu[:, 2], rngs["p_spatial"], True), case.length[ids],
                  np.maximum(case.slope[ids], np.float32(1e-3)), case.x[ids])
    net = O.Network.from_coo(n, rows, cols)
    qp = case.qprime[:, ids]
    local_out = np.flatnonzero(np.isin(ids, outlets_global))  # local gauge reaches (ascending)
    gidx = np.searchsorted(outlets_global, ids[local_out])    # their global gauge numbers
    res = O.route(net, r, qp, dtype=np.float64, outflow_idx=[np.array([o]) for o in local_out])
    loss_l, daily, gh = O.daily_l1_objective(res["runoff"], obs[gidx], tau=3, warmup=warmup)
    share = len(local_out) / g_global  # local mean -> this rank's part of the global mean
    Wg = np.zeros((n, T_DAILY))
    Wg[local_out] = gh * share
    res64 = O.route(net, r, qp, dtype=np.float64)
    bw = O.route_backward(net, r, qp, res64["x"], Wg)
    g = O.param_grads_from_unit(bw["n"], bw["q_spatial"], bw["p_spatial"], uu[:, 0], uu[:, 1], uu[:, 2], rngs)
    u.backward(torch.from_numpy(np.stack([g["n"], g["q_spatial"], g["p_spatial"]], 1).astype(np.float32)))
    return w.grad.numpy(), loss_l * share, daily, gidx


def _objective_problem():
    from ddr_amd import synthetic

    net = synthetic.forest(synthetic.loguniform_sizes(10, 20, 300, 4), seed=6)
    case = synthetic_case(net, T_DAILY, 6)
    feats = np.random.default_rng(7).normal(size=(net.n, 4)).astype(np.float32)
    outlets = np.flatnonzero(net.down < 0)
    obs = np.random.default_rng(8).lognormal(0.0, 1.0, (len(outlets), 3)).astype(np.float32)
    weight = np.random.default_rng(10).normal(size=(4, 3)).astype(np.float32) * 0.3
    return net, case, feats, outlets, obs, weight


def _objective_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from ddr_amd.distributed import allreduce_gradients, gather_rows, shard_network

    dist.init_process_group("gloo", rank=rank, world_size=world)
    net, case, feats, outlets, obs, weight = _objective_problem()
    ns, rs, cs, ids = shard_network(net.n, net.rows, net.cols, rank, world)
    grad, loss, daily, gidx = _objective_grad(rs, cs, ns, ids, case, feats, weight, outlets, obs, len(outlets))
    p = torch.nn.Parameter(torch.zeros(4, 3))
    p.grad = torch.from_numpy(grad)
    allreduce_gradients([p])
    lt = torch.tensor([loss], dtype=torch.float64)
    dist.all_reduce(lt)
    full_daily = gather_rows(torch.from_numpy(daily.astype(np.float64)), torch.from_numpy(gidx), len(outlets))
    out[rank] = (p.grad.numpy().copy(), float(lt), full_daily.numpy())
    dist.destroy_process_group()


def _gather_grad_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from ddr_amd.distributed import gather_rows

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows_of = [np.array([4, 0, 2]), np.array([1, 3])]  # global row index of each rank's local rows
    base = torch.arange(15, dtype=torch.float64).reshape(5, 3)
    local = (base[torch.from_numpy(rows_of[rank])] + 1.0).requires_grad_(True)
    full = gather_rows(local, torch.from_numpy(rows_of[rank]), 5)
    W = torch.arange(15, dtype=torch.float64).reshape(5, 3) * 0.5 - 2.0
    (full * W).sum().backward()
    out[rank] = (full.detach().numpy(), local.grad.numpy().copy(), rows_of[rank])
    dist.destroy_process_group()


def test_two_rank_gather_rows_backpropagates():
    """A loss over the gathered rows gives every rank the gradient of its own rows: the same
    gradient a single process gets from ``loss(full).backward()``."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    procs = [ctx.Process(target=_gather_grad_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    W = np.arange(15, dtype=np.float64).reshape(5, 3) * 0.5 - 2.0
    full_ref = np.arange(15, dtype=np.float64).reshape(5, 3) + 1.0
    for r in range(world):
        full, g, rows = out[r]
        np.testing.assert_array_equal(full, full_ref)
        np.testing.assert_array_equal(g, W[rows])  # single-process gradient of these rows


def test_two_rank_c3_objective_allreduce_and_gather():
    """The multi-GPU C3 step at world size 2 (gloo): gauges follow their basins, each rank's L1 is its
    share of the global mean, the all-reduced gradient equals the single-process one and gather_rows
    reassembles the (G, D) daily series in global gauge order on every rank."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    procs = [ctx.Process(target=_objective_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    net, case, feats, outlets, obs, weight = _objective_problem()
    full_grad, full_loss, full_daily, _ = _objective_grad(net.rows, net.cols, net.n, np.arange(net.n), case, feats,
                                                         weight, outlets, obs, len(outlets))
    for r in range(world):
        g, loss, daily = out[r]
        np.testing.assert_allclose(g, full_grad, rtol=2e-4, atol=1e-6)
        assert abs(loss - full_loss) <= 1e-9 * abs(full_loss)
        np.testing.assert_allclose(daily, full_daily, rtol=1e-8)  # SciPy solves of sub- vs whole network


def test_basin_depths_and_depth_aware_shards():
    """partition.basin_depths against a per-reach walk to the outlet; the depth-aware refinement of the LPT
    shards lowers the modelled slowest rank, (T + deepest basin) x reaches, and still covers every basin once."""
    from ddr_amd import synthetic
    from ddr_amd.partition import basin_depths, basin_labels, shard_basins

    net = synthetic.forest(synthetic.zipf_sizes(30000, 120, 0.3), seed=7, single_inflow=0.3)
    lab, dep = basin_depths(net.n, net.rows, net.cols)
    np.testing.assert_array_equal(lab, basin_labels(net.n, net.rows, net.cols))
    down = np.full(net.n, -1)
    down[net.cols] = net.rows
    dist = np.zeros(net.n, dtype=np.int64)
    for i in range(net.n - 1, -1, -1):  # rows > cols: a reach's downstream has the larger index
        dist[i] = 0 if down[i] < 0 else dist[down[i]] + 1
    ref = np.zeros(net.n, dtype=np.int64)
    np.maximum.at(ref, lab, dist + 1)
    np.testing.assert_array_equal(dep, ref[lab])
    outlets, first, inv, sizes = np.unique(lab, return_index=True, return_inverse=True, return_counts=True)
    bd = dep[first]
    T = 720
    for world in (2, 3, 4):
        model = lambda sh: max((T + bd[i].max()) * sizes[i].sum() for i in sh)  # noqa: E731
        plain, deep = shard_basins(sizes, world), shard_basins(sizes, world, bd, T)
        assert model(deep) <= model(plain)
        np.testing.assert_array_equal(np.sort(np.concatenate(deep)), np.arange(len(sizes)))
