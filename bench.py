"""Headline benchmark: differentiable Muskingum-Cunge routing on MI355X (BASELINE.json configs).

Workloads (``--workload``; the default is the headline metric):

* ``c5`` -- BASELINE metric: forward + backward over an 8760-hour water year of a Hydrofabric-shaped
  CONUS network (800k reaches, 3000 outlet basins, Zipf sizes with the largest 0.35 N, Hack's-law main
  stems, 35 % single-inflow reaches), loss = sum(W * runoff).  One step = one full forward (hot start +
  8759 routing steps) and one full adjoint (gradients w.r.t. n, q_spatial, p_spatial).
* ``c3`` -- the training batch: 256 gauged subnetworks (log-uniform 100..20k reaches), rho = 90 days
  (T = 2136 h) from a daily q' store (the reference default), one gauge per subnetwork outlet.  One step = parameter network forward (a KAN
  stand-in: pykan is not installed here) -> denormalize -> fused gauge-mode routing with the daily
  objective (trim [13 : -11 + tau], area pooling) -> L1 loss vs synthetic observations -> backward ->
  RCCL all-reduce of the network's gradients -> clip + Adam step (scripts/train.py:54-104).
* ``c4`` -- MERIT-CONUS-shaped network (350k reaches, ~1k outlets, x = 0.3): water-year forward route
  + per-day accumulation and geometry statistics over the 365 days (geometry_predictor.py:176-212).
* ``c2`` -- one 5k-reach gauged subnetwork, water-year forward route, parameters fixed.

Multi-GPU (``torchrun --nproc-per-node N bench.py --gpus N``): STRONG scaling -- every rank builds the
same global network and routes the outlet basins LPT-assigned to it (no data-path collective: basins
are independent).  RCCL carries the C3 gradient all-reduce and the timing/size
reductions.  Barrier + synchronize bracket the K timed steps; the time is the max over ranks; value =
all ranks' reach-steps / that time.

Usage:  python bench.py [--workload c5] [--gpus N] [--steps K] [--warmup W]
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

from ddr_amd import _lib, synthetic  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402
from ddr_amd.ops import DailyWindow, GaugeMap, RouteConsts, route  # noqa: E402
from ddr_amd.distributed import shard_network  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
RANGES = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}

WORKLOADS = {
    "c5": dict(metric="reach-timesteps/sec fwd+bwd (CONUS 800k reaches, 8760 h)", T=8760, grad=True,
               desc="C5: Hydrofabric-shaped CONUS network, fwd+bwd over a water year"),
    "c3": dict(metric="reach-timesteps/sec fwd+bwd (256 gauged subnetworks, KAN backprop, RCCL grad all-reduce)",
               T=2136, grad=True, desc="C3: training batch of 256 gauged subnetworks (rho 90 d), daily L1 objective"),
    "c4": dict(metric="reach-timesteps/sec fwd (MERIT-CONUS 350k reaches, 8760 h) + 365-day geometry statistics",
               T=8760, grad=False, desc="C4: MERIT-shaped network, water-year forward + geometry statistics"),
    "c2": dict(metric="reach-timesteps/sec fwd (5k-reach gauged subnetwork, 8760 h, parameters fixed)", T=8760,
               grad=False, desc="C2: one Hack-law subnetwork, water-year forward"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def global_network(args):
    """The workload's whole network (deterministic: every rank builds the same one)."""
    w = args.workload
    if w == "c5":
        sizes = synthetic.zipf_sizes(args.reaches, args.basins, args.largest)
        return synthetic.forest(sizes, seed=5, single_inflow=0.35), None
    if w == "c3":
        return synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 3), seed=3, single_inflow=0.25), None
    if w == "c4":
        return synthetic.forest(synthetic.zipf_sizes(350_000, 1000, 0.35), seed=4, single_inflow=0.15), 0.3
    return synthetic.hack_basin(5000, seed=2), None





class _LinearSplitK(torch.autograd.Function):
    """y = x W^T + b whose weight gradient over ~1M rows (a (out x in) result with K = rows) is summed
    from 128 row-chunks by one batched GEMM: hipBLASLt's single GEMM for that shape runs at ~18 TF/s
    (1.0-1.8 ms per layer at C3 size), the batched split 5-12x faster (tools/dbg/mlp_wgrad.py)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gy @ w
        rows, B = x.shape[0], 128
        k = rows // B
        m = B * k
        gw = torch.bmm(gy[:m].view(B, k, -1).transpose(1, 2), x[:m].view(B, k, -1)).sum(0) if k > 0 else 0
        if m < rows:
            gw = gw + gy[m:].t() @ x[m:]
        return gx, gw, gy.sum(0)


class ParamNet(torch.nn.Module):
    """KAN stand-in for C3 (pykan is not installed): attributes -> (n, q_spatial, p_spatial) in [0, 1]
    through sigmoid, the reference nn's output contract (src/ddr/nn/kan.py:11-62); ~35k parameters."""

    def __init__(self, n_attr=10, hidden=128):
        super().__init__()
        g = torch.Generator().manual_seed(0)  # identical replicas on every rank
        self.layers = torch.nn.ModuleList([torch.nn.Linear(n_attr, hidden), torch.nn.Linear(hidden, hidden),
                                           torch.nn.Linear(hidden, hidden), torch.nn.Linear(hidden, 3)])
        with torch.no_grad():
            for m in self.layers:
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) / math.sqrt(m.weight.shape[1]))
                m.bias.zero_()

    def forward(self, x):
        lin = lambda m, v: _LinearSplitK.apply(v, m.weight, m.bias)  # noqa: E731
        for m in self.layers[:-1]:
            x = torch.nn.functional.silu(lin(m, x))
        return torch.sigmoid(lin(self.layers[-1], x))


class FusedNet:
    """C3's parameter network as bench.py uses it: ``--pnet fused`` (default) is ddr_amd.pnet.ParamNet (the same
    architecture and initialisation as ParamNet, forward + backward in two HIP launches, denormalisation fused);
    ``--pnet torch`` is ParamNet + denorm in PyTorch ops.  Both return denormalised (n, q_spatial, p_spatial)."""

    def __init__(self, kind, dev):
        if kind == "fused":
            from ddr_amd.pnet import ParamNet as Fused

            self.net = Fused(10, RANGES).to(dev)
        else:
            self.net = ParamNet().to(dev)
        self.kind = kind

    def parameters(self):
        return self.net.parameters()

    def __call__(self, feats):
        if self.kind == "fused":
            return self.net(feats)
        un = self.net(feats)
        return denorm(un[:, 0].contiguous(), un[:, 1].contiguous(), un[:, 2].contiguous())


class TorchTail:
    """clip_grad_norm_(max_norm=1) + fused Adam in PyTorch ops (the step tail of --tail torch)."""

    def __init__(self, params):
        self.params = list(params)
        self.opt = torch.optim.Adam(self.params, lr=1e-3, fused=True)  # one launch per step, not per tensor

    def zero_grad(self, set_to_none=True):
        self.opt.zero_grad(set_to_none=set_to_none)

    def step(self):
        torch.nn.utils.clip_grad_norm_(self.params, max_norm=1.0, foreach=True)
        self.opt.step()


def make_tail(args, model):
    """(optimizer, loss_fn) of the C3 step: loss_fn(daily, obs, warmup_days, inv_count) is the mean absolute
    error over gauges x days after the warm-up (train.py:91-94); the optimizer clips to norm 1 and steps Adam."""
    if args.tail == "fused" and args.pnet == "fused":
        from ddr_amd.train import ClipAdam, daily_l1_loss

        return ClipAdam(model.net.flat, lr=1e-3, max_norm=1.0), daily_l1_loss

    def torch_l1(daily, obs, wd, inv_count):
        return torch.nn.functional.l1_loss(daily[:, wd:], obs[:, wd:], reduction="sum") * inv_count

    return TorchTail(model.parameters()), torch_l1


def denorm(un, uq, up):
    """utils.py:166-185 (torch, autograd reaches the unit-interval parameters)."""
    n = un * (RANGES["n"][1] - RANGES["n"][0]) + RANGES["n"][0]
    q = uq * (RANGES["q_spatial"][1] - RANGES["q_spatial"][0]) + RANGES["q_spatial"][0]
    lo, hi = math.log(RANGES["p_spatial"][0] + 1e-6), math.log(RANGES["p_spatial"][1])
    return n, q, torch.exp(up * (hi - lo) + lo)


def cpu_baseline(args, net_global, x_const):
    """The oracle port of the reference recipe, one core, on a bounded sample of the workload."""
    from oracle import mc_oracle as O

    os.environ.setdefault("OMP_NUM_THREADS", "1")
    w = args.workload
    if w == "c5":
        sample = synthetic.forest(synthetic.zipf_sizes(args.cpu_reaches, max(1, args.basins * args.cpu_reaches // args.reaches),
                                                       args.largest), seed=5, single_inflow=0.35)
    elif w == "c3":
        sample = synthetic.forest(synthetic.loguniform_sizes(12, 100, 20000, 3), seed=3, single_inflow=0.25)
    elif w == "c4":
        sample = synthetic.forest(synthetic.zipf_sizes(20_000, 60, 0.35), seed=4, single_inflow=0.15)
    else:
        sample = synthetic.hack_basin(5000, seed=2)
    T = args.cpu_T
    no = O.Network.from_coo(sample.n, sample.rows, sample.cols)
    no.solver = "scipy"
    at = synthetic.reach_attributes(sample.n, 7, x_const=x_const)
    u = synthetic.unit_parameters(sample.n, 7)
    r = O.Reaches(O.denormalize(u["n"], RANGES["n"]), O.denormalize(u["q_spatial"], RANGES["q_spatial"]),
                  O.denormalize(u["p_spatial"], RANGES["p_spatial"], True), at.length,
                  np.maximum(at.slope, np.float32(1e-3)), at.x)
    qp = synthetic.lateral_inflow(sample.n, T, 7)
    grad = WORKLOADS[w]["grad"]
    t0 = time.perf_counter()
    res = O.route(no, r, qp, O.Bounds(), dtype=np.float32)
    t_fwd = time.perf_counter() - t0
    if grad:
        W = np.random.default_rng(1).uniform(0, 1, (sample.n, T)).astype(np.float32)
        O.route_backward(no, r, qp, res["x"], W, O.Bounds())
    el = time.perf_counter() - t0
    what = ("fwd (fp32 + SciPy fp64 spsolve_triangular per step) + bwd (hand adjoint + SciPy transposed solve)"
            if grad else "fwd (fp32 + SciPy fp64 spsolve_triangular per step)")
    rs = sample.n * (T - 1)
    out = {"value": rs / el, "unit": "reach-timesteps/s", "cores": 1, "nproc": os.cpu_count(), "kind": "port",
           "sample": f"{sample.n} reaches x {T} h {w.upper()}-shaped sample, {what}, {el:.1f} s",
           "forward_only_value": rs / t_fwd}
    # basin-parallel: one single-threaded port process per core over disjoint C5-shaped basins (SURVEY §8(d)'s
    # stronger CPU figure); the process count is the GPU's share of this box's cores (at most 16 per GPU here)
    if w == "c5" and args.cpu_procs > 1:
        from oracle.cpu_bench import basin_parallel

        mp = basin_parallel(args.cpu_procs, args.cpu_reaches, max(1, args.basins * args.cpu_reaches // args.reaches),
                            args.largest, T, grad, x_const, RANGES)
        out["multi_process_value"] = mp["value"]
        out["multi_process"] = {"processes": mp["processes"], "cores": mp["processes"], "wall_s": round(mp["wall_s"], 1),
                                "per_process_value": mp["per_process_value"],
                                "sample": f"{mp['processes']} disjoint {args.cpu_reaches}-reach x {T} h C5-shaped "
                                          f"samples (seeds 100..), one single-threaded process each, {what}"}
    # the reference itself cannot travel to this box: its speed relative to the port was measured on the
    # same sample in the build container (tools/calibrate_cpu.py -> profiles/cpu_calibration.json, both on
    # one core); the reference-equivalent rate here is the port's rate divided by that ratio
    try:
        cal = json.loads((ROOT / "profiles" / "cpu_calibration.json").read_text())
    except (OSError, ValueError):
        cal = None
    if cal and w == "c5" and cal.get("reaches") == sample.n and cal.get("T") == T:
        key = "fwd_bwd" if grad else "fwd_only"
        ratio = cal["ratio_port_over_reference"][key]
        out["calibration"] = {"ratio_port_over_reference": ratio, "reference_equivalent_value": out["value" if grad else
                                                                                                      "forward_only_value"] / ratio,
                              "reference_in_build_container": cal["reference"][key], "port_in_build_container": cal["port"][key],
                              "source": "profiles/cpu_calibration.json (tools/calibrate_cpu.py, same sample, 1 core)"}
    return out


def split_factor() -> float:
    """The largest basin is split over a rank group when it exceeds this multiple of a rank's share
    (ddr_amd.split.plan_ranks; DDR_SPLIT_FACTOR overrides)."""
    return float(os.environ.get("DDR_SPLIT_FACTOR", "1.2"))


def shard_steps(T: int) -> int:
    """T for the depth-aware basin assignment (distributed.shard_network); DDR_SHARD_BY_DEPTH=0: reach count only."""
    return T if os.environ.get("DDR_SHARD_BY_DEPTH", "1") != "0" else 0


def setup_split(args, net, rank, world, dist, dev, T):
    """C5 at N > 1: the largest outlet basin routed by a group of ranks (ddr_amd.split) when it exceeds
    twice a rank's share, the other basins LPT-sharded over the remaining ranks.  A hand-shake
    launch checks the cross-rank path on this machine (against a whole-basin route of the same inputs); if any rank fails it, every rank falls back to
    whole-basin sharding (returns None; so does a plan without a split).  DDR_SPLIT_BASIN=0 disables, =force splits even at N = 2."""
    from ddr_amd.split import SplitBasin, block_edges, plan_block_ranks, plan_ranks, sub_network

    plan = plan_ranks(net.n, net.rows, net.cols, world, factor=split_factor(),
                      force=os.environ.get("DDR_SPLIT_BASIN") == "force", steps=shard_steps(T))
    ids_r, sp = plan[rank]
    any_split = any(s is not None for _, s in plan)
    if not any_split:
        args.split_handshake = "no split planned"
        return None
    n_loc, rows, cols, ids = sub_network(net.n, net.rows, net.cols, ids_r)
    g = split = None
    handle = None
    if sp is not None:
        group, idx = sp
        k = len(group)
        # k GPUs' worth of workgroups (one CU's share each); a one-GPU rehearsal (every rank on device 0)
        # keeps the group's blocks within the one device so that all of them can be resident at once
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        wg = cus if os.environ.get("DDR_BENCH_SAME_DEVICE") == "1" else k * cus
        g = RiverGraph(n_loc, rows, cols, steps_hint=T, target_blocks=wg, max_resident=wg)
        nloc, prod, cons = block_edges(g)
        br = plan_block_ranks(nloc, k, prod, cons)

        def exchange(obj):
            res = [None] * world
            dist.all_gather_object(res, (rank, obj))
            return [o for r_, o in res if r_ in group]

        ok = torch.ones(1, device=dev)
        try:
            split = SplitBasin(g, br, idx, k, T, exchange)
        except Exception as e:  # noqa: BLE001  (the peers then fail the hand-shake below too)
            log(f"[rank {rank}] split-basin setup failed ({e}); falling back to whole-basin sharding")
            ok.zero_()
    else:
        res = [None] * world
        dist.all_gather_object(res, (rank, handle))  # the split group's handle exchange (nothing to share)
        ok = torch.ones(1, device=dev)
    if split is not None:
        try:  # hand-shake on the split graph, every cross-rank edge exercised
            from ddr_amd.ops import check_status

            if os.environ.get("DDR_SPLIT_FAIL_RANK") == str(rank):  # rehearsal of the fallback path
                raise RuntimeError("simulated hand-shake failure (DDR_SPLIT_FAIL_RANK)")

            # a 720-step forward and backward: every cross-rank edge in both directions, over enough
            # chunks to catch an intermittent hand-off (~1 % of a training step's work); the owned rows
            # must equal a whole-basin route of the same inputs on this rank alone (partition-invariant)
            Th = min(T, 720)
            gen = torch.Generator().manual_seed(20240611)
            qp = (torch.rand((Th, n_loc), generator=gen) * 0.9 + 0.05).to(dev)
            un = torch.rand(n_loc, generator=gen).to(dev)
            z = torch.full((n_loc,), 0.5, device=dev)

            def trial(graph):
                zn = (un * 0.08 + 0.02).requires_grad_(True)
                ro, _, _, _ = route(graph, qp, zn, z, z * 10, z * 1000 + 1000, z * 0.01, z * 0.5, steps=Th,
                                    math=args.math)
                ro.backward(torch.ones_like(ro))
                check_status(True)
                return ro.detach(), zn.grad

            runoff, gn = trial(g)
            own = torch.from_numpy(split.owned_reaches).to(dev)  # the other ranks' rows are not this rank's
            runoff, gn = runoff[own], gn[own]
            if not bool(torch.isfinite(runoff).all()) or not bool(torch.isfinite(gn).all()):
                raise RuntimeError("non-finite hand-shake outputs")
            gw = RiverGraph(n_loc, rows, cols, steps_hint=Th)
            try:
                r_w, g_w = trial(gw)
            finally:
                gw.close()
            dr = float(((runoff - r_w[own]).abs() / r_w[own].abs().clamp_min(1e-30)).max())
            dg = float((gn - g_w[own]).abs().max() / g_w[own].abs().max().clamp_min(1e-30))
            log(f"[rank {rank}] split hand-shake vs whole-basin route: runoff max-rel {dr:.1e}, dL/dn {dg:.1e}")
            if not (dr <= 1e-6 and dg <= 1e-5):
                raise RuntimeError(f"hand-shake outputs differ from the whole-basin route ({dr:.1e}, {dg:.1e})")
            del runoff, gn, r_w, g_w, qp
        except Exception as e:  # noqa: BLE001
            log(f"[rank {rank}] split-basin hand-shake failed ({e}); falling back to whole-basin sharding")
            ok.zero_()
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if ok.item() < 1:
        args.split_handshake = "failed on some rank: whole-basin sharding"
        if g is not None:
            g.close()
        if split is not None:
            split.close()
        return None
    args.split_handshake = "passed on every rank (owned rows equal a whole-basin route)"
    return g, split, n_loc, rows, cols, ids


def counter_file(workload, T, lib_hash, reaches, world=1, split=None, root=ROOT):
    """PMC summary of this workload for the loaded library build (profiles/, made by tools/pmc.sh +
    tools/pmc_to_json.py); None when absent or stale: another build, T, or shard.  The counters describe
    one launch over the reaches ONE process routed: they apply to a line only when this rank's shard is
    the one measured -- the same reach count, world size and split role (``split`` = (index, k) of a
    split-basin rank, else None).  The files measured on one GPU (world 1, the whole network) therefore
    never label an N > 1 rank's line."""
    f = Path(root) / "profiles" / "counters" / f"{workload}.json"
    try:
        d = json.loads(f.read_text())
    except (OSError, ValueError):
        return None
    if d.get("build") != lib_hash or d.get("T") != T or d.get("reaches") != reaches:
        return None
    if int(d.get("world", 1)) != int(world) or d.get("split") != (None if split is None else list(split)):
        return None
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5", choices=sorted(WORKLOADS))
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reaches", type=int, default=800_000, help="C5 network size")
    ap.add_argument("--basins", type=int, default=3000)
    ap.add_argument("--largest", type=float, default=0.35)
    ap.add_argument("--T", type=int, default=0, help="override the workload's hours")
    ap.add_argument("--tau", type=int, default=3)
    ap.add_argument("--warmup-days", type=int, default=3)
    ap.add_argument("--cpu-reaches", type=int, default=40_000)
    ap.add_argument("--cpu-T", type=int, default=720)
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="C5: also time this many port processes in parallel over disjoint basins (0/1: off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dropin-steps", type=int, default=2, help="C5, 1 GPU: also time the drop-in dmc() path")
    ap.add_argument("--block-profile", default="", help="write a per-workgroup launch profile (JSON) here")
    ap.add_argument("--grad-qprime", action="store_true",
                    help="C5: q' requires grad, so the backward is the state-gradient adjoint (dL/dq' too)")
    ap.add_argument("--exact-adjoint", action="store_true",
                    help="fp32 backward as the exact adjoint of the fp32 trajectory (route(exact_adjoint=True), opt-in)")
    ap.add_argument("--stream", type=int, default=0,
                    help="C3, 1 GPU: also time K training steps over K different batches (a new gauge-union "
                         "adjacency per step, graphs built ahead on host threads by GraphPrefetcher)")
    ap.add_argument("--stream-workers", type=int, default=4, help="graph builder threads (each device builder on its own stream)")
    ap.add_argument("--stream-depth", type=int, default=3, help="graphs built ahead of use")
    ap.add_argument("--stream-builder", default="inline", choices=["inline", "device", "host"],
                    help="where the per-batch graph is built: on the device (ddr_graph_build_device, one builder "
                         "thread on its own stream) or on host threads (ddr_graph_build + upload)")
    ap.add_argument("--pnet", default="fused", choices=["fused", "torch"],
                    help="C3 parameter network: fused HIP kernels (ddr_amd.pnet) or the same network in PyTorch ops")
    ap.add_argument("--tail", default="fused", choices=["fused", "torch"],
                    help="C3 step tail (with --pnet fused): the daily L1 objective and clip + Adam as two HIP launches "
                         "(ddr_amd.train) or PyTorch's l1_loss / clip_grad_norm_ / fused Adam")
    ap.add_argument("--graph", action="store_true",
                    help="C3, no process group: capture the whole training step into one HIP graph (ddr_amd.capture) "
                         "and time its replays; kernel times come from eager steps before the capture")
    ap.add_argument("--fast-math", action="store_true",
                    help="forward coefficients in hardware-approximate fp32 math (route(math='fast'))")
    ap.add_argument("--math", default=None, choices=["exact", "faithful", "fast"],
                    help="forward coefficient arithmetic (default faithful, the drop-in dmc's default -- "
                         "MuskingumCunge(math) -- and what the trainer runs; --fast-math = fast)")
    args = ap.parse_args()
    args.math = args.math or ("fast" if args.fast_math else "faithful")
    spec = WORKLOADS[args.workload]
    T = args.T or spec["T"]
    args.T = T

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (a 1-GPU box): DDR_BENCH_SAME_DEVICE=1 puts every rank on device 0 and
    # DDR_DIST_BACKEND=gloo replaces RCCL, which refuses two ranks on one device
    local_dev = 0 if os.environ.get("DDR_BENCH_SAME_DEVICE") == "1" else local_rank
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    dist = None
    # DDR_BENCH_ALONE=1 (strong-scaling prediction on one GPU, tools/scale_alone.sh): run rank RANK's
    # shard of WORLD_SIZE alone, without a process group -- the shards share nothing on the data path,
    # so a rank's step time is its shard's time (plus the latency-bound gradient all-reduce)
    alone = os.environ.get("DDR_BENCH_ALONE") == "1"
    if world > 1 and not alone:
        import torch.distributed as dist

        backend = os.environ.get("DDR_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    t_setup = time.perf_counter()
    net, x_const = global_network(args)
    args.reaches_total = net.n
    # this rank's outlet basins (LPT by reach count refined by depth, distributed.shard_network; all of them at N = 1)
    n_loc, rows, cols, ids = shard_network(net.n, net.rows, net.cols, rank, world, steps=shard_steps(T)) if world > 1 else (
        net.n, net.rows, net.cols, np.arange(net.n))
    g, split = None, None
    if alone and os.environ.get("DDR_BENCH_SPLIT_PLAN") == "1":
        # prediction runs: a rank outside the split group, with the shard the split plan gives it
        from ddr_amd.split import plan_ranks, sub_network

        ids_r, sp = plan_ranks(net.n, net.rows, net.cols, world, factor=split_factor(), steps=shard_steps(T))[rank]
        if sp is not None:
            raise SystemExit("a split-group rank cannot run alone (its blocks wait for its peers)")
        n_loc, rows, cols, ids = sub_network(net.n, net.rows, net.cols, ids_r)
    if args.workload == "c5" and world > 1 and not alone and os.environ.get("DDR_SPLIT_BASIN", "1") != "0":
        plan = setup_split(args, net, rank, world, dist, dev, T)
        if plan is not None:
            g, split, n_loc, rows, cols, ids = plan
    if g is None:
        # DDR_BENCH_TARGET_BLOCKS (prediction runs): pack this rank's network into that many workgroups,
        # e.g. a split group's k x 256 blocks of the largest basin routed alone on one GPU as generations
        tb = int(os.environ.get("DDR_BENCH_TARGET_BLOCKS", "0"))
        g = RiverGraph(n_loc, rows, cols, steps_hint=T, target_blocks=tb, max_resident=tb)
    log(f"[rank {rank}] {g} built in {time.perf_counter() - t_setup:.1f}s"
        + (f", split basin rank {split.index}/{split.k} ({len(split.owned_reaches)} reaches, {split.n_x} cross-rank cut edges)"
           if split else ""))
    n_owned = n_loc if split is None else len(split.owned_reaches)
    at = synthetic.reach_attributes(net.n, 11, x_const=x_const)
    u = synthetic.unit_parameters(net.n, 11)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a)[ids])).to(dev)  # noqa: E731
    length, slope, xs = tt(at.length), tt(np.maximum(at.slope, np.float32(1e-3))), tt(at.x)
    # C3 trains from a DAILY q' store (the reference's default, configs.py:61-65 is_hourly=False):
    # (ceil(T / 24), N) rows indexed q'[t // 24] in the gather, the reader's repeat(24)
    # (readers.py:513-519); the other workloads route an hourly (T, N) field
    qp_hours = 24 if args.workload == "c3" else 1
    qprime = synthetic.lateral_inflow_torch(net.n, -(-T // qp_hours), seed=11, device=dev, ids=ids)
    consts = RouteConsts()
    lib = _lib.load()
    lib_hash = lib.ddr_version().decode().split()[-1]  # the routing kernels' hash (key of the counter files)
    # algorithmic bytes per reach-step, SURVEY §8(d): forward q' read + x_save write + runoff write; backward
    # dL/drunoff read + x_save read + q' read; gauge mode (C3) has no per-reach runoff / dL/drunoff (G x T
    # only).  These are the roofline's figures.  The fp32 adjoint itself never reads q' (the c4 term of the
    # VJP folds through the forward identity x = c1 Sx + c2 I + c3 Q + c4 qc, physics.h adjoint_step_fast):
    # what its kernel moves is 4 B less per reach-step (reported beside it as kernel_bytes_per_reach_step)
    fwd_bytes, bwd_bytes = (8, 8) if args.workload == "c3" else (12, 12)
    bwd_kernel_bytes = bwd_bytes - 4

    # ---- the step of each workload --------------------------------------------------------------------
    if args.workload == "c5":
        u_n, u_q, u_p = (tt(u[k]).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial"))
        gen = torch.Generator(device=dev).manual_seed(1234 + rank)
        W = torch.rand((n_loc, T), device=dev, dtype=torch.float32, generator=gen)  # dL/drunoff of sum(W * runoff)
        if args.grad_qprime:
            qprime.requires_grad_(True)

        def step():
            for t_ in (u_n, u_q, u_p, qprime):
                t_.grad = None
            n, q, p = denorm(u_n, u_q, u_p)
            runoff, _, _, _ = route(g, qprime, n, q, p, length, slope, xs, consts=consts, math=args.math,
                                     exact_adjoint=args.exact_adjoint)
            runoff.backward(W)

    elif args.workload == "c3":
        from ddr_amd.distributed import allreduce_gradients

        feats = tt(synthetic.reach_features(net.n, seed=11))
        model = FusedNet(args.pnet, dev)
        opt, loss_fn = make_tail(args, model)
        # one gauge per subnetwork outlet; observations indexed by the gauge's global number
        outlets_global = np.flatnonzero(net.down < 0)
        outlets = np.flatnonzero(np.isin(ids, outlets_global))
        gz = GaugeMap.build([np.array([o]) for o in outlets], n_loc, dev)
        window = DailyWindow.for_training(T, args.tau)
        G_global = len(outlets_global)
        obs = torch.from_numpy(np.random.default_rng(100).lognormal(np.log(5.0), 1.0, (G_global, window.D))
                               .astype(np.float32)[np.searchsorted(outlets_global, ids[outlets])]).to(dev)
        wd = args.warmup_days

        def step():
            opt.zero_grad(set_to_none=True)
            n, q, p = model(feats)
            daily, _, _, _ = route(g, qprime, n, q, p, length, slope, xs, gauges=gz, daily=window, consts=consts,
                                   math=args.math, steps=T, qprime_hours=qp_hours, exact_adjoint=args.exact_adjoint)
            # the global mean absolute error over all ranks' gauges (train.py:94-97): this rank's share
            loss = loss_fn(daily, obs, wd, 1.0 / (G_global * (window.D - wd)))
            loss.backward()
            allreduce_gradients(list(model.parameters()))  # RCCL, one flat bucket
            opt.step()  # clip_grad_norm_(max_norm=1) + Adam (train.py:99-100)

    else:
        from ddr_amd.geometry.statistics import geometry_statistics_from_inflow

        n, q, p = denorm(tt(u["n"]), tt(u["q_spatial"]), tt(u["p_spatial"]))

        def step():
            with torch.no_grad():
                if args.workload == "c4":  # first: the kernel timer reports the last forward launch
                    geometry_statistics_from_inflow(g, qprime[::24][:365], n, p, q, slope)
                route(g, qprime, n, q, p, length, slope, xs, consts=consts, save=False, math=args.math)

    ev = []
    kms = {"forward": [], "backward": []}  # main routing kernels, HIP events on the launch stream

    def timed_step():
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
        ev.append((e0, e1))
        if graph_mode:
            return
        for w_, key in ((0, "forward"), (1, "backward")):
            if key == "backward" and not spec["grad"]:
                continue
            ms = ctypes.c_float()
            _lib.check(lib.ddr_kernel_ms(w_, ctypes.byref(ms)))
            kms[key].append(ms.value)

    torch.cuda.synchronize()
    log(f"[rank {rank}] inputs resident ({torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB); warmup {args.warmup}")
    for _ in range(args.warmup):
        step()
    _lib.check(lib.ddr_set_kernel_timing(1))
    torch.cuda.synchronize()
    graph_mode = None
    if args.graph:
        if args.workload != "c3" or dist is not None or args.tail != "fused" or args.pnet != "fused":
            raise SystemExit("--graph: the C3 step with the fused network and tail, without a process group")
        from ddr_amd.capture import CapturedStep

        # the routing kernels' times from eager steps (the library's timers are off inside a capture)
        for _ in range(2):
            timed_step()
        ev.clear()
        step = CapturedStep(step, warmup=1, device=dev)
        graph_mode = "whole step captured into one HIP graph (ddr_amd.capture); kernel ms from 2 eager steps"
        torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        timed_step()
        log(f"[rank {rank}] step {i + 1}/{args.steps}")
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _lib.check(lib.ddr_set_kernel_timing(0))
    _lib.check(lib.ddr_status_check(1))  # any timed-out hand-off fails the run
    if args.block_profile and (rank == 0 or alone):
        block_profile(args.block_profile, g, step, lib)

    # ---- reductions over ranks ------------------------------------------------------------------------
    sizes = torch.zeros(max(world, 1), device=dev, dtype=torch.float64)
    sizes[rank] = n_owned
    # per rank: its routing kernels' mean ms (HIP events on the launch stream) and step ms
    per = torch.zeros((max(world, 1), 3), device=dev, dtype=torch.float64)
    per[rank, 0] = float(np.mean(kms["forward"])) if kms["forward"] else 0.0
    per[rank, 1] = float(np.mean(kms["backward"])) if kms["backward"] else 0.0
    per[rank, 2] = elapsed / args.steps * 1e3
    tmax = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    pg_world = 1
    if dist is not None:
        dist.all_reduce(sizes, op=dist.ReduceOp.SUM)
        dist.all_reduce(per, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        pg_world = dist.get_world_size()
    sizes = sizes.cpu().numpy()
    per = per.cpu().numpy()
    elapsed = float(tmax.item())
    total_reaches = int(sizes.sum())
    value = total_reaches * (T - 1) * args.steps / elapsed

    if rank == 0 or alone:
        step_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        reach_steps = n_owned * (T - 1)
        kern = {}
        for key, nb in (("forward", fwd_bytes), ("backward", bwd_bytes)):
            if kms[key]:
                k = float(np.mean(kms[key]))
                kern[key] = {"kernel_ms": k, "GB/s": nb * reach_steps / (k * 1e-3) / 1e9, "bytes_per_reach_step": nb,
                             "launches": len(kms[key])}
        if "backward" in kern:
            kern["backward"]["kernel_bytes_per_reach_step"] = bwd_kernel_bytes
        dom = max(kern, key=lambda k_: kern[k_]["kernel_ms"])
        achieved = kern[dom]["GB/s"]
        cf = counter_file(args.workload, args.T, lib_hash, n_owned, world,
                          None if split is None else (split.index, split.k))
        kc = (cf or {}).get("kernels", {}).get(f"route_{dom}_kernel", {})
        dropin = None
        if args.workload == "c5" and world == 1 and args.dropin_steps > 0:
            dropin = time_dropin(args, net, at, u, qprime, W, dev)
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(args, net, x_const)
        if cpu is not None:
            cpu["speedup_vs_port"] = value / cpu["value"]
            cal = cpu.get("calibration")
            if cal:
                cpu["speedup_vs_reference_equivalent"] = value / cal["reference_equivalent_value"]
        largest = int(net.basin_sizes.max())
        out = {
            "metric": spec["metric"],
            "value": value,
            "unit": "reach-timesteps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": spec["desc"] + (" + dL/dq' (state-gradient adjoint)" if args.grad_qprime else ""), "reaches": total_reaches, "T": T, "qprime_store": "daily" if qp_hours == 24 else "hourly",
                       "parameter_network": ({"fused": "fused HIP MLP 10-128-128-128-3 (ddr_amd.pnet, fp32 MFMA)",
                                              "torch": "PyTorch MLP 10-128-128-128-3"}[args.pnet]
                                             if args.workload == "c3" else None),
                       "step_graph": graph_mode,
                       "backward": "exact adjoint of the fp32 trajectory" if args.exact_adjoint else "default fp32 adjoint",
                       "step_tail": (("fused HIP daily L1 + clip/Adam (ddr_amd.train)" if args.tail == "fused" and args.pnet == "fused"
                                      else "PyTorch l1_loss + clip_grad_norm_ + fused Adam") if args.workload == "c3" else None),
                       "forward_math": {"exact": "exact (reference op order, correctly rounded pow)",
                                        "faithful": "faithful (reference op order, IEEE division, fp32 faithful-class pow)",
                                        "fast": "fast (hardware rcp/log/exp fp32)"}[args.math],
                       "basins": int(len(net.basin_sizes)), "largest_basin": largest,
                       "max_depth_rank0": g.info.max_depth, "blocks_rank0": g.info.n_blocks,
                       "cut_edges_rank0": g.info.n_cut, "generations_rank0": g.info.generations,
                       "parallelism": f"outlet basins LPT-sharded over {world} GPU(s)" + (
                           f"; the largest basin split over ranks 0..{split.k - 1} (ddr_amd.split)" if split else ""),
                       "split_basin": None if split is None else {"ranks": split.k, "cross_cut_edges": split.n_x,
                                                                  "receive_memory_kind": split.kind},
                       "reaches_per_rank": [int(s) for s in sizes],
                       "world_size_process_group": pg_world if dist is not None else None,
                       "per_rank_ms": None if dist is None else [
                           {"rank": r_, "reaches": int(sizes[r_]), "forward_kernel_ms": round(float(per[r_, 0]), 3),
                            "backward_kernel_ms": round(float(per[r_, 1]), 3) if spec["grad"] else None,
                            "step_ms": round(float(per[r_, 2]), 3)} for r_ in range(world)],
                       "split_handshake": getattr(args, "split_handshake", None),
                       "load_max_over_mean": float(sizes.max() / sizes.mean()),
                       "basin_bound_speedup": float(total_reaches / max(sizes.max(), largest))},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": kc.get("bytes_per_launch"),
                         "kernel": f"route_{dom}_kernel", "bytes_per_reach_step": kern[dom]["bytes_per_reach_step"],
                         "bytes_source": "SURVEY.md section 8(d) algorithmic bytes per reach-step x N (T - 1) / the kernel's "
                                         "mean duration (HIP events on its launch stream)",
                         "valu_frac": kc.get("valu_frac"), "counters": None if cf is None else cf.get("source"),
                         "note": "not HBM bound: VALU issue + per-tick barrier bound, see DESIGN.md section 4"},
            "kernels": kern,
            "step_gpu_ms": step_ms,
            "build": lib_hash,
            "cpu_baseline": cpu,
        }
        if dropin is not None:
            out["dropin_dmc"] = dropin
        if args.workload == "c3" and world == 1 and args.stream > 0:
            ts = time_training_stream(args, dev)
            # the stream's batches are larger on average than the fixed one (0.91-1.07M vs 0.90M reaches):
            # compared per reach-step, as throughput
            ts["throughput_vs_fixed_batch"] = ts["value"] / out["value"]
            out["training_stream"] = ts
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


BUILDERS = {"inline": "on the device, begun ahead on the training stream", "device": "on the device, builder threads",
            "host": "on host threads + upload"}


def time_training_stream(args, dev):
    """C3 as a training loop sees it: every step a new batch of 256 gauged subnetworks, i.e. a new
    adjacency, graph and gauge map per step (merit.py:197-223, scripts/train.py:54-104).  The graph of
    every step is built anew on host threads (GraphPrefetcher, ``--stream-workers``) while the device
    trains on the previous batch.  M = 4 distinct batches (inputs resident in HBM, generated before the
    timed loop) are cycled over K steps; each step's timed region is the wait for its graph + upload +
    the training step.  The first two steps are warm-up."""
    from ddr_amd.distributed import allreduce_gradients
    from ddr_amd.graph import GraphPrefetcher

    K, T, M = args.stream, args.T, 4
    t_gen = time.perf_counter()
    data = []
    window = DailyWindow.for_training(T, args.tau)
    for k in range(M):
        nt = synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 100 + k), seed=100 + k, single_inflow=0.25)
        at = synthetic.reach_attributes(nt.n, 200 + k)
        tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        outlets = np.flatnonzero(nt.down < 0)
        data.append(dict(net=nt, length=tt(at.length), slope=tt(np.maximum(at.slope, np.float32(1e-3))), xs=tt(at.x),
                         feats=tt(synthetic.reach_features(nt.n, seed=200 + k)),
                         qprime=synthetic.lateral_inflow_torch(nt.n, -(-T // 24), seed=200 + k, device=dev),
                         gz=GaugeMap.build([np.array([o]) for o in outlets], nt.n, dev),
                         obs=torch.from_numpy(np.random.default_rng(300 + k).lognormal(np.log(5.0), 1.0,
                                              (len(outlets), window.D)).astype(np.float32)).to(dev)))
    log(f"[stream] {M} batches resident in {time.perf_counter() - t_gen:.1f}s "
        f"({min(d['net'].n for d in data)}..{max(d['net'].n for d in data)} reaches)")
    model = FusedNet(args.pnet, dev)
    opt, loss_fn = make_tail(args, model)
    wd = args.warmup_days
    consts = RouteConsts()
    torch.cuda.synchronize()
    warm = 2
    # inline: device builds begun --stream-depth batches ahead on the training stream (PendingGraph);
    # device: device builds on builder threads' own streams; host: host builds on threads + upload
    on_dev = {"inline": "inline", "device": True, "host": False}[args.stream_builder]
    pf = GraphPrefetcher(((data[k % M]["net"].n, data[k % M]["net"].rows, data[k % M]["net"].cols, k % M)
                          for k in range(K + warm)), workers=args.stream_workers, steps_hint=T, on_device=on_dev,
                         depth=args.stream_depth)
    per = []
    evs = []
    t_start = None
    g = None
    for k in range(K + warm):
        if k == warm:
            torch.cuda.synchronize()
            t_start = time.perf_counter()
        t0 = time.perf_counter()
        if g is not None:
            g.close()  # the previous batch's graph: released stream-ordered after its launches
        g, m = next(pf)
        t_graph = time.perf_counter() - t0
        # the host is off the critical path when it enqueues this step before the device has finished the
        # previous one (the device then never waits for the host's graph)
        ahead = bool(evs) and not evs[-1][1].query() if k > warm else None
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        d = data[m]
        opt.zero_grad(set_to_none=True)
        n, q, p = model(d["feats"])
        daily, _, _, _ = route(g, d["qprime"], n, q, p, d["length"], d["slope"], d["xs"], gauges=d["gz"],
                               daily=window, consts=consts, steps=T, qprime_hours=24, math=args.math)
        loss = loss_fn(daily, d["obs"], wd, 1.0 / (daily.shape[0] * (window.D - wd)))
        loss.backward()
        allreduce_gradients(list(model.parameters()))
        opt.step()
        e1.record()
        if k >= warm:
            per.append({"reaches": int(d["net"].n), "generations": g.info.generations, "blocks": g.info.n_blocks,
                        "graph_wait_ms": round(t_graph * 1e3, 2), "host_ahead": ahead})
            evs.append((e0, e1))
    torch.cuda.synchronize()
    timed = time.perf_counter() - t_start
    for b, (e0, e1) in zip(per, evs):
        b["step_gpu_ms"] = round(e0.elapsed_time(e1), 2)
    g.close()
    pf.close()
    rs = sum(b["reaches"] for b in per) * (T - 1)
    waits = [b["graph_wait_ms"] for b in per]
    gpu = float(np.mean([b["step_gpu_ms"] for b in per]))
    return {"steps": K, "ms_per_step": timed / K * 1e3, "value": rs / timed, "unit": "reach-timesteps/s",
            "graph_builder": args.stream_builder, "graph_workers": args.stream_workers,
            "graph_wait_ms_mean": float(np.mean(waits)) if waits else None,
            "step_gpu_ms_mean": gpu,
            "host_ahead_steps": f"{sum(1 for b in per if b['host_ahead'])} of {sum(1 for b in per if b['host_ahead'] is not None)}"
                                " (steps enqueued while the device was still on the previous step)",
            # wall time per step not inside a training step's own GPU span: the next batches' device
            # builds (queued between steps on the training stream) and any device idle time
            "between_steps_ms": timed / K * 1e3 - gpu,
            "stream_over_gpu_step": timed / K * 1e3 / gpu,
            "graph_wait_note": "host time in next(prefetcher): the host runs ahead of the device and waits there "
                               "for its queue (device builds are stream-ordered between training steps); the "
                               "device-side cost of the builds is between_steps_ms",
            "ns_per_reach_step_gpu": float(np.mean([b["step_gpu_ms"] * 1e6 / (b["reaches"] * (T - 1)) for b in per])),
            "batches": per,
            "note": (f"new adjacency + graph build per step ({BUILDERS[args.stream_builder]}"
                     f", overlapped with training), {M} distinct batches cycled; graph_wait_ms is host time in "
                     "g.close() + next(prefetcher), i.e. it includes the host waiting for queued device work "
                     "(back-pressure), which costs nothing while the device is busy: between_steps_ms is the "
                     "device-side cost")}


def time_dropin(args, net, at, u, qprime, W, dev):
    """The trainer's own call path: ddr_amd.routing.dmc (torch_mc.py:144-223) on a RoutingDataclass with
    a torch sparse-CSR adjacency, forward + backward, including setup_inputs (graph cache lookup,
    hot start, PatternMapper) -- host work the kernel timings do not show."""
    from types import SimpleNamespace

    import scipy.sparse as sp

    from ddr_amd.routing import dmc

    params = SimpleNamespace(parameter_ranges=RANGES, log_space_parameters=["p_spatial"], defaults={"p_spatial": 21},
                             attribute_minimums={"discharge": 1e-4, "slope": 1e-3, "velocity": 0.01, "depth": 0.01,
                                                 "bottom_width": 0.01})
    a = sp.coo_matrix((np.ones(len(net.rows), np.float32), (net.rows, net.cols)), shape=(net.n, net.n)).tocsr()
    adj = torch.sparse_csr_tensor(torch.from_numpy(a.indptr.astype(np.int64)), torch.from_numpy(a.indices.astype(np.int64)),
                                  torch.from_numpy(a.data), size=(net.n, net.n))
    rd = SimpleNamespace(adjacency_matrix=adj, length=torch.from_numpy(at.length), slope=torch.from_numpy(at.slope),
                         x=torch.from_numpy(at.x), top_width=torch.empty(0), side_slope=torch.empty(0),
                         outflow_idx=None, gage_catchment=None, observations=None, flow_scale=None)
    model = dmc(SimpleNamespace(params=params), device=dev)
    sp_params = {k: torch.from_numpy(u[k]).to(dev).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial")}

    def one():
        out = model(routing_dataclass=rd, streamflow=qprime, spatial_parameters=sp_params)["runoff"]
        out.backward(W)

    one()  # builds and caches the river graph of this adjacency
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.dropin_steps):
        one()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.dropin_steps * 1e3
    # the BMI update (ddr_bmi.py:285-305): one route_timestep per hour under no_grad, state carried
    eng = model.routing_engine
    K = 24
    with torch.no_grad():
        for i in range(K + 2):
            if i == 2:
                torch.cuda.synchronize()
                t1 = time.perf_counter()
            qc = torch.clamp(qprime[i % qprime.shape[0]], min=1e-4)
            eng._discharge_t = eng.route_timestep(q_prime_clamp=qc)
        torch.cuda.synchronize()
    bmi_ms = (time.perf_counter() - t1) / K * 1e3
    return {"ms_per_step": ms, "steps": args.dropin_steps,
            "note": "dmc() forward + backward incl. setup_inputs (cached graph, hot start, PatternMapper)",
            "route_timestep_ms": bmi_ms,
            "route_timestep_note": f"BMI update: one MuskingumCunge.route_timestep (one hour, {net.n} reaches, no_grad), mean of {K}"}


def block_profile(path, g, step, lib):
    """One extra step with the per-workgroup profile on: start/end/import-wait per block (µs)."""
    nb = g.info.n_blocks
    # 16 words per block, then (phase-profile builds, -DDDR_PHASE_PROF=1) 8 phase counters per wave
    bufs = [torch.zeros(16 * nb + nb * 16 * 8, dtype=torch.int64, device=g.device) for _ in range(2)]
    for w in (0, 1):
        lib.ddr_set_block_profile(w, ctypes.c_void_p(bufs[w].data_ptr()))
    step()
    torch.cuda.synchronize()
    for w in (0, 1):
        lib.ddr_set_block_profile(w, None)
    s = g.structure()
    sizes = np.bincount(s["block"], minlength=nb)
    out = {}
    for w, key in ((0, "forward"), (1, "backward")):
        allw = bufs[w].cpu().numpy()
        p = allw[:16 * nb].reshape(nb, 16)
        ph = allw[16 * nb:].reshape(nb * 16, 8)
        ph = ph[ph.sum(1) > 0]
        if len(ph):
            tot = ph.sum(0).astype(np.float64)
            out[key + "_phase_frac"] = (tot / tot.sum()).tolist()
            out[key + "_phase_waves"] = ph.tolist()  # per wave (block-major, 16 waves), 8 phase counters
            log(f"[profile] {key} phases (cycle share over {len(ph)} waves): "
                + " ".join(f"{f:.3f}" for f in tot / tot.sum()))
        t0 = p[:, 0].min()
        out[key] = {"start_us": ((p[:, 0] - t0) / 100.0).tolist(), "end_us": ((p[:, 1] - t0) / 100.0).tolist(),
                    "wait_us": (p[:, 2] / 100.0).tolist(), "hwid": (p[:, 3] & 0xFFFFFFFF).tolist(),
                    "xcc": (p[:, 3] >> 32).tolist(),
                    "tick1024_us": np.where(p[:, 4:] > 0, (p[:, 4:] - t0) / 100.0, -1).tolist()}
        e = (p[:, 1] - t0) / 100.0
        log(f"[profile] {key}: end min/median/max {e.min():.0f}/{np.median(e):.0f}/{e.max():.0f} us, "
            f"wait max {p[:, 2].max() / 100:.0f} us")
    out["nloc"] = sizes.tolist()
    # per-block structure: cut edges in / out, basins, whether a basin spans blocks, depth span
    blk, down, basin, dist = s["block"], s["down"], s["basin"], s["dist"]
    has = down >= 0
    src, dst = np.flatnonzero(has), down[has]
    cut = blk[src] != blk[dst]
    out["cut_in"] = np.bincount(blk[dst[cut]], minlength=nb).tolist()
    out["cut_out"] = np.bincount(blk[src[cut]], minlength=nb).tolist()
    nblk_of_basin = np.bincount(np.unique(np.stack([basin, blk]), axis=1)[0])
    out["split"] = np.bincount(blk, weights=(nblk_of_basin[basin] > 1), minlength=nb).tolist()
    dmin = np.full(nb, np.iinfo(np.int64).max)
    np.minimum.at(dmin, blk, dist)
    dmx = np.zeros(nb, np.int64)
    np.maximum.at(dmx, blk, dist)
    out["dist_span"] = (dmx - dmin).tolist()
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    Path(path).write_text(json.dumps(out))


if __name__ == "__main__":
    main()
