"""Worker of tests/test_gpu_split.py: one rank of a basin split across processes that share cuda:0
(the single-GPU rehearsal of ddr_amd.split; the receive memory is exchanged by IPC handle exactly as
across GPUs).  Usage: python tests/split_worker.py RANK WORLD PORT OUT.npz MATH"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

N, T, SEED = 6000, 160, 21
GRAPH_KW = {"max_block_reaches": 256, "target_blocks": 1 << 20}


def case():
    from ddr_amd import synthetic

    net = synthetic.hack_basin(N, seed=SEED)
    at = synthetic.reach_attributes(net.n, SEED)
    u = synthetic.unit_parameters(net.n, SEED)
    qp = synthetic.lateral_inflow(net.n, T, SEED)
    W = np.random.default_rng(SEED).uniform(0, 1, (net.n, T)).astype(np.float32)
    return net, at, u, qp, W


def route_forward(g, net, at, u, qp, math, dev):
    """Forward only: (runoff, the unit parameters it depends on, last-step Q); backward later."""
    import torch

    from ddr_amd.ops import route

    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, torch.float32)  # noqa: E731
    un = {k: tt(u[k]).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial")}
    n = un["n"] * 0.2 + 0.02
    p = torch.exp(un["p_spatial"] * 5.0)
    runoff, q_last, _, _ = route(g, tt(qp), n, un["q_spatial"], p, tt(at.length), tt(np.maximum(at.slope, 1e-3)),
                                 tt(at.x), math=math)
    return runoff, un, q_last


def route_backward(runoff, un, W, dev):
    import torch

    (runoff * torch.from_numpy(W).to(dev)).sum().backward()
    torch.cuda.synchronize()
    return {"runoff": runoff.detach().cpu().numpy(), **{f"g_{k}": v.grad.cpu().numpy() for k, v in un.items()}}


def route_once(g, net, at, u, qp, W, math, dev):
    runoff, un, _ = route_forward(g, net, at, u, qp, math, dev)
    return route_backward(runoff, un, W, dev)


def second_inputs(qp):
    """A second batch of lateral inflow (the interleaved forward / forward / backward / backward case)."""
    return (qp * np.float32(1.7) + np.float32(0.05)).astype(np.float32)


def main():
    rank, world, port, out, math = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    import ctypes as C

    import torch
    import torch.distributed as dist

    from ddr_amd import _lib
    from ddr_amd.graph import RiverGraph
    from ddr_amd.ops import check_status
    from ddr_amd.split import SplitBasin, block_edges, plan_block_ranks

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    net, at, u, qp, W = case()
    g = RiverGraph(net.n, net.rows, net.cols, **GRAPH_KW)
    nloc, prod, cons = block_edges(g)
    br = plan_block_ranks(nloc, world, prod, cons)

    def exchange(obj):
        res = [None] * world
        dist.all_gather_object(res, obj)
        return res

    sb = SplitBasin(g, br, rank, world, T, exchange)
    res = [route_once(g, net, at, u, qp, W, math, dev) for _ in range(2)]  # two launches: epochs advance
    check_status()
    # forward A, forward B, backward A, backward B: forward B rewrites the shared receive rows before
    # backward A runs (each backward must read its own forward's cross-rank x)
    ra, ua, qa = route_forward(g, net, at, u, qp, math, dev)
    rb, ub, _ = route_forward(g, net, at, u, second_inputs(qp), math, dev)
    res.append(route_backward(ra, ua, W, dev))
    res.append(route_backward(rb, ub, W, dev))
    check_status()
    # outputs of reaches another rank routes are marked, never stale memory
    notown = np.setdiff1d(np.arange(net.n), sb.owned_reaches)
    extra = {"nan_col0": bool(np.isnan(res[2]["runoff"][notown, 0]).all()),
             "nan_qlast": bool(torch.isnan(qa[torch.from_numpy(notown).to(dev)]).all().item()),
             "own_finite": bool(np.isfinite(res[2]["runoff"][sb.owned_reaches]).all())}
    from ddr_amd.ops import GaugeMap, route

    try:  # gauge mode on a split graph is refused
        gz = GaugeMap.build([np.array([net.n - 1])], net.n, dev)
        z = torch.ones(net.n, device=dev)
        route(g, torch.from_numpy(qp).to(dev), z * 0.05, z * 0.5, z * 20, z * 1000, z * 0.01, z * 0.3, gauges=gz,
              math=math)
        extra["gauge_refused"] = False
    except Exception as e:  # noqa: BLE001
        extra["gauge_refused"] = "split basin" in str(e)
    dist.barrier()
    dist.barrier()
    sb.close()
    np.savez(out, owned=sb.owned_reaches, n_x=sb.n_x, kind=sb.kind, fp=np.uint64(g.fingerprint()), **extra,
             **{f"{i}_{k}": v for i, r in enumerate(res) for k, v in r.items()})
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
