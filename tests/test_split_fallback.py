"""World-size-3 (gloo, CPU) test of bench.setup_split's agreement and fallback logic.

C5 at N > 1 routes the largest outlet basin with a group of ranks and checks the cross-rank path with a
hand-shake launch first; if any rank fails (setup or hand-shake), EVERY rank must fall back to
whole-basin sharding, and the ranks outside the group must take part in the same collectives.  The
GPU pieces (graph build, IPC receive memory, the routing launch) are replaced by CPU fakes here; the
plan, the exchange of the group's handles, the hand-shake comparison and the MIN-reduction of the
verdict are bench.py's own code.  The GPU side of the hand-shake is covered by tests/test_gpu_split.py.
"""

import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

WORLD = 3
SIZES = [600, 50, 50, 50, 50]  # largest basin 600 > 2 x the mean share (800 / 3): a 2-rank split group


def _net():
    from ddr_amd import synthetic

    return synthetic.forest(SIZES, seed=11)


def _worker(rank, world, port, mode, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if mode == "fail_handshake":
        os.environ["DDR_SPLIT_FAIL_RANK"] = "1"
    import types

    import torch.distributed as dist

    import bench
    import ddr_amd.ops as ops
    import ddr_amd.split as split_mod

    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = {"exchange": 0, "closed": 0, "graphs": 0}

    class FakeGraph:
        def __init__(self, n, rows, cols, **kw):
            self.n = n
            calls["graphs"] += 1

        def close(self):
            calls["closed"] += 1

    class FakeSplit:
        def __init__(self, g, br, idx, k, T, exchange):
            peers = exchange(("handle", rank))  # the group's IPC handle exchange
            calls["exchange"] += 1
            assert sorted(p[1] for p in peers) == list(range(k))
            if mode == "fail_setup" and rank == 0:
                raise RuntimeError("simulated IPC open failure")
            self.owned_reaches = np.arange(g.n)[idx::k]

        def close(self):
            calls["closed"] += 1

    def fake_route(graph, qp, zn, *a, steps=None, math=None):
        ro = zn[:, None] * qp.t()  # (n_loc, steps), differentiable in zn
        if mode == "mismatch" and rank == 1 and calls["graphs"] == 1:  # (the split graph's trial)
            ro = ro * 1.01
        return ro, None, None, None

    split_mod.SplitBasin = FakeSplit
    split_mod.block_edges = lambda g: (np.ones(4, dtype=np.int64), np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64))
    split_mod.plan_block_ranks = lambda nloc, k, prod, cons: np.arange(len(nloc)) % k
    ops.check_status = lambda *a, **k: None
    bench.RiverGraph = FakeGraph
    bench.route = fake_route
    torch.cuda.get_device_properties = lambda dev: types.SimpleNamespace(multi_processor_count=4)

    net = _net()
    args = types.SimpleNamespace(math=None)
    res = bench.setup_split(args, net, rank, world, dist, torch.device("cpu"), 48)
    # every rank takes part in one more collective: a rank stuck in a mismatched one would hang here
    t = torch.ones(1)
    dist.all_reduce(t)
    out[rank] = (res is not None, args.split_handshake, dict(calls), None if res is None else int(res[2]))
    dist.destroy_process_group()


def _run(mode):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, mode, out)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return [out[r] for r in range(WORLD)]


def test_plan_puts_largest_basin_on_a_two_rank_group():
    from ddr_amd.split import plan_ranks

    net = _net()
    plan = plan_ranks(net.n, net.rows, net.cols, WORLD)
    assert [sp for _, sp in plan] == [([0, 1], 0), ([0, 1], 1), None]
    assert len(plan[0][0]) == len(plan[1][0]) == max(SIZES)


def test_split_handshake_passes_on_every_rank():
    res = _run("pass")
    for r, (used, msg, calls, n_loc) in enumerate(res):
        assert used and msg.startswith("passed"), (r, msg)
        assert calls["closed"] == (1 if r < 2 else 0)  # the whole-basin check graph of the group ranks
    assert res[0][3] == res[1][3] == max(SIZES)
    assert res[2][3] == sum(SIZES) - max(SIZES)


def test_split_handshake_failure_on_one_rank_falls_back_everywhere():
    res = _run("fail_handshake")  # DDR_SPLIT_FAIL_RANK=1: rank 1's hand-shake raises
    for r, (used, msg, calls, _) in enumerate(res):
        assert not used and msg.startswith("failed"), (r, msg)
    # the group ranks release the split graph and its receive memory; rank 0 also its check graph
    assert res[0][2]["closed"] == 3 and res[1][2]["closed"] == 2 and res[2][2]["closed"] == 0


def test_split_setup_failure_falls_back_everywhere():
    res = _run("fail_setup")  # rank 0 cannot open a peer's receive memory
    assert all(not used and msg.startswith("failed") for used, msg, _, _ in res)
    assert res[0][2]["exchange"] == res[1][2]["exchange"] == 1


def test_split_handshake_mismatch_falls_back_everywhere():
    res = _run("mismatch")  # rank 1's split route differs from its whole-basin route
    assert all(not used and msg.startswith("failed") for used, msg, _, _ in res)
