"""Headline benchmark: differentiable Muskingum-Cunge routing, forward + backward.

Metric (BASELINE.json): reach-timesteps/s fwd+bwd on a CONUS-shaped network (Hydrofabric-like,
800k reaches, ~3k outlet basins, largest basin 0.35 N, deep Hack's-law main stems) over an 8760-hour
water year (config C5), plus the fraction of HBM peak of the dominant kernel.

One "step" = one full forward (hot start + 8759 routing steps) and one full backward (adjoint w.r.t.
n, q_spatial, p_spatial) over the whole water year, with loss = sum(W * runoff), W ~ U(0, 1).

Multi-GPU (``torchrun --nproc-per-node N bench.py --gpus N``): weak scaling -- the global forest has
N x (C5-shaped forest); outlet basins are LPT-sharded across ranks (no data-path collective; basins
are independent).  Barrier + synchronize bracket the K timed steps; time is the max over ranks.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--reaches 800000] [--T 8760]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from ddr_amd import synthetic  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402
from ddr_amd.ops import RouteConsts, route  # noqa: E402
from ddr_amd.partition import shard_basins  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
FWD_BYTES = 12  # q' read + runoff write + x_save write per reach-step
BWD_BYTES = 12  # grad read + x_save read + q' read per reach-step
RANGES = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_rank_network(args, rank: int, world: int):
    """This rank's basins of a world x C5 forest (Zipf sizes, largest 0.35 of each C5 block)."""
    sizes = np.concatenate([synthetic.zipf_sizes(args.reaches, args.basins, args.largest) for _ in range(world)])
    owner = shard_basins(sizes, world)
    mine = np.sort(owner[rank])
    my_sizes = sizes[mine]
    net = synthetic.forest(my_sizes, seed=args.seed + 7919 * rank, single_inflow=args.single_inflow)
    return net, int(sizes.sum())


def cpu_baseline(args):
    """Time the oracle port of the reference recipe on a bounded sample (1 core)."""
    from oracle import mc_oracle as O

    os.environ.setdefault("OMP_NUM_THREADS", "1")
    sample_n, sample_T = args.cpu_reaches, args.cpu_T
    net = synthetic.forest(synthetic.zipf_sizes(sample_n, max(1, args.basins * sample_n // args.reaches),
                                                args.largest), seed=args.seed, single_inflow=args.single_inflow)
    no = O.Network.from_coo(net.n, net.rows, net.cols)
    no.solver = "scipy"
    at = synthetic.reach_attributes(net.n, args.seed)
    u = synthetic.unit_parameters(net.n, args.seed)
    r = O.Reaches(O.denormalize(u["n"], RANGES["n"]), O.denormalize(u["q_spatial"], RANGES["q_spatial"]),
                  O.denormalize(u["p_spatial"], RANGES["p_spatial"], True), at.length,
                  np.maximum(at.slope, np.float32(1e-3)), at.x)
    qp = synthetic.lateral_inflow(net.n, sample_T, args.seed)
    W = np.random.default_rng(1).uniform(0, 1, (net.n, sample_T)).astype(np.float32)
    t0 = time.perf_counter()
    res = O.route(no, r, qp, O.Bounds(), dtype=np.float32)
    O.route_backward(no, r, qp, res["x"], W, O.Bounds())
    el = time.perf_counter() - t0
    return {"value": net.n * (sample_T - 1) / el, "unit": "reach-timesteps/s", "cores": 1, "kind": "port",
            "sample": f"{net.n} reaches x {sample_T} h C5-shaped sub-forest, fwd (fp32 + SciPy fp64 "
                      f"spsolve_triangular per step) + bwd (hand adjoint + SciPy transposed solve), {el:.1f} s"}


def measured_traffic(kernel: str, args) -> float | None:
    """HBM bytes per launch of `kernel` from the committed PMC measurement (profiles/), if it was taken
    on this workload; None otherwise (rocprofv3 counters cannot be read from inside the run)."""
    f = ROOT / "profiles" / "r01_traffic_c5.json"
    try:
        d = json.loads(f.read_text())
    except (OSError, ValueError):
        return None
    if d.get("config") != {"reaches_per_gpu": args.reaches, "T": args.T} or args.dtype != "f32":
        return None
    k = d["kernels"].get(kernel)
    return None if k is None else float(k["bytes_per_launch"])


def block_profile(path, g, step, lib):
    """One extra step with the per-workgroup profile on: start/end/import-wait per block (µs)."""
    nb = g.info.n_blocks
    bufs = [torch.zeros(16 * nb, dtype=torch.int64, device=g.device) for _ in range(2)]
    for w in (0, 1):
        lib.ddr_set_block_profile(w, ctypes.c_void_p(bufs[w].data_ptr()))
    step(False)
    torch.cuda.synchronize()
    for w in (0, 1):
        lib.ddr_set_block_profile(w, None)
    s = g.structure()
    sizes = np.bincount(s["block"], minlength=nb)
    out = {}
    for w, key in ((0, "forward"), (1, "backward")):
        p = bufs[w].view(nb, 16).cpu().numpy()
        t0 = p[:, 0].min()
        out[key] = {"start_us": ((p[:, 0] - t0) / 100.0).tolist(), "end_us": ((p[:, 1] - t0) / 100.0).tolist(),
                    "wait_us": (p[:, 2] / 100.0).tolist(), "hwid": (p[:, 3] & 0xFFFFFFFF).tolist(),
                    "xcc": (p[:, 3] >> 32).tolist(),
                    "tick1024_us": np.where(p[:, 4:] > 0, (p[:, 4:] - t0) / 100.0, -1).tolist()}
        e = (p[:, 1] - t0) / 100.0
        log(f"[profile] {key}: end min/median/max {e.min():.0f}/{np.median(e):.0f}/{e.max():.0f} us, "
            f"wait max {p[:, 2].max() / 100:.0f} us")
    out["nloc"] = sizes.tolist()
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    Path(path).write_text(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reaches", type=int, default=800_000)
    ap.add_argument("--basins", type=int, default=3000)
    ap.add_argument("--largest", type=float, default=0.35)
    ap.add_argument("--single-inflow", type=float, default=0.35)
    ap.add_argument("--T", type=int, default=8760)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--cpu-reaches", type=int, default=40_000)
    ap.add_argument("--cpu-T", type=int, default=720)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--block-profile", default="", help="write a per-workgroup launch profile (JSON) here")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)

    t_setup = time.perf_counter()
    net, global_n = build_rank_network(args, rank, world)
    g = RiverGraph(net.n, net.rows, net.cols)
    log(f"[rank {rank}] {g} built in {time.perf_counter() - t_setup:.1f}s")
    T = args.T
    dt = torch.float32 if args.dtype == "f32" else torch.float64
    at = synthetic.reach_attributes(net.n, args.seed + rank)
    u = synthetic.unit_parameters(net.n, args.seed + rank)
    tt = lambda a: torch.from_numpy(np.asarray(a)).to(dev, dt)  # noqa: E731
    u_n, u_q, u_p = (tt(u[k]).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial"))
    length, slope, xs = tt(at.length), tt(np.maximum(at.slope, np.float32(1e-3))), tt(at.x)
    qprime = synthetic.lateral_inflow_torch(net.n, T, seed=args.seed + rank, device=dev).to(dt)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    W = torch.rand((net.n, T), device=dev, dtype=dt, generator=gen)  # dL/drunoff of loss = sum(W * runoff)
    consts = RouteConsts()

    def denorm():
        # utils.py:166-185 (torch, autograd reaches the unit-interval parameters)
        n = u_n * (RANGES["n"][1] - RANGES["n"][0]) + RANGES["n"][0]
        q = u_q * (RANGES["q_spatial"][1] - RANGES["q_spatial"][0]) + RANGES["q_spatial"][0]
        lo, hi = math.log(RANGES["p_spatial"][0] + 1e-6), math.log(RANGES["p_spatial"][1])
        p = torch.exp(u_p * (hi - lo) + lo)
        return n, q, p

    ev = {k: [] for k in ("f0", "f1", "b1")}
    kms = {"forward": [], "backward": []}  # main routing kernels, HIP events on the launch stream
    from ddr_amd import _lib

    lib = _lib.load()

    def step(record: bool):
        for t_ in (u_n, u_q, u_p):
            t_.grad = None
        n, q, p = denorm()
        if record:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        runoff, q_last, _, _ = route(g, qprime, n, q, p, length, slope, xs, consts=consts)
        if record:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
        runoff.backward(W)
        if record:
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record()
            ev["f0"].append(e0)
            ev["f1"].append(e1)
            ev["b1"].append(e2)
            for w, key in ((0, "forward"), (1, "backward")):
                ms = ctypes.c_float()
                _lib.check(lib.ddr_kernel_ms(w, ctypes.byref(ms)))
                kms[key].append(ms.value)
        return runoff

    torch.cuda.synchronize()
    log(f"[rank {rank}] inputs resident ({torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB); warmup {args.warmup}")
    for _ in range(args.warmup):
        step(False)
    _lib.check(lib.ddr_set_kernel_timing(1))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(True)
        log(f"[rank {rank}] step {i + 1}/{args.steps}")
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _lib.check(lib.ddr_set_kernel_timing(0))
    if args.block_profile and rank == 0:
        block_profile(args.block_profile, g, step, lib)
    fwd_ms = float(np.mean([a.elapsed_time(b) for a, b in zip(ev["f0"], ev["f1"])]))
    bwd_ms = float(np.mean([a.elapsed_time(b) for a, b in zip(ev["f1"], ev["b1"])]))
    local = torch.tensor([float(net.n)], device=dev, dtype=torch.float64)
    tmax = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(local, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    total_reaches = int(local.item())
    elapsed = float(tmax.item())
    value = total_reaches * (T - 1) * args.steps / elapsed
    if rank == 0:
        reach_steps = net.n * (T - 1)
        kf, kb = float(np.mean(kms["forward"])), float(np.mean(kms["backward"]))
        kern = {"forward": {"op_ms": fwd_ms, "kernel_ms": kf, "GB/s": FWD_BYTES * reach_steps / (kf * 1e-3) / 1e9},
                "backward": {"op_ms": bwd_ms, "kernel_ms": kb, "GB/s": BWD_BYTES * reach_steps / (kb * 1e-3) / 1e9}}
        dom = "backward" if kb >= kf else "forward"
        achieved = kern[dom]["GB/s"]
        cpu = None if args.no_cpu_baseline else cpu_baseline(args)
        out = {
            "metric": "reach-timesteps/sec fwd+bwd (CONUS 800k reaches, 8760 h)",
            "value": value,
            "unit": "reach-timesteps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic",
            "config": {"workload": "C5: Hydrofabric-shaped synthetic forest per GPU, fwd+bwd over a water year",
                       "reaches_per_gpu": args.reaches, "reaches_total": total_reaches, "T": T,
                       "basins_per_gpu": args.basins, "largest_basin_frac": args.largest,
                       "max_depth_rank0": g.info.max_depth, "blocks_rank0": g.info.n_blocks,
                       "cut_edges_rank0": g.info.n_cut, "parallelism": f"basin-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": measured_traffic(f"route_{dom}_kernel", args),
                         "kernel": f"route_{dom}_kernel",
                         "bytes_per_reach_step": FWD_BYTES if dom == "forward" else BWD_BYTES,
                         "note": "VALU-issue bound, not HBM bound: see DESIGN.md section 4"},
            "kernels": kern,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
