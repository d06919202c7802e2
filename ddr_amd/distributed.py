"""Multi-GPU routing: one process per GPU, outlet basins sharded across ranks.

The solve needs no exchange (basins are independent); RCCL (``torch.distributed`` backend "nccl")
carries only what the training loop shares:
  * the parameter-network gradient all-reduce (KAN weights, ~200 KB: one flat bucket, latency-bound
    on xGMI -- a single all-reduce of the concatenated gradients, issued after ``loss.backward()``),
  * the gathered gauge / outlet discharge for the loss and metrics,
  * scalar loss / timing reductions.
"""

from __future__ import annotations

import numpy as np
import torch

from .partition import basin_depths, basin_labels, extract_basins, shard_basins


def rank_world():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_network(n: int, rows: np.ndarray, cols: np.ndarray, rank: int, world: int, steps: int = 0):
    """This rank's sub-network: whole outlet basins, LPT-balanced by reach count (``steps`` > 0: then refined
    against the rank time model (T + deepest basin) x reach count, partition.shard_basins).

    Returns (n_sub, rows_sub, cols_sub, reach_ids) with ``reach_ids`` the global reach index of each
    local reach (topological order preserved).
    """
    if steps > 0:
        lab, dep = basin_depths(n, rows, cols)
        outlets, first, inv, sizes = np.unique(lab, return_index=True, return_inverse=True, return_counts=True)
        shards = shard_basins(sizes, world, dep[first], steps)
    else:
        lab = basin_labels(n, rows, cols)
        outlets, inv, sizes = np.unique(lab, return_inverse=True, return_counts=True)
        shards = shard_basins(sizes, world)
    owner = np.empty(len(outlets), dtype=np.int64)
    for r, idx in enumerate(shards):
        owner[idx] = r
    keep = owner[inv] == rank
    return extract_basins(n, rows, cols, keep)


def allreduce_gradients(params, op_average: bool = False) -> None:
    """All-reduce the gradients of ``params`` as ONE flat bucket (sum; optional mean)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    if op_average:
        flat /= dist.get_world_size()
    off = 0
    for g in grads:
        k = g.numel()
        g.copy_(flat[off:off + k].view_as(g))
        off += k


def gather_rows(local: torch.Tensor, global_index: torch.Tensor, n_global: int) -> torch.Tensor:
    """Assemble a (n_global, ...) tensor from every rank's rows (e.g. gauge discharge (G_r, T) or the
    daily objective series (G_r, D)) on every rank.

    One all-gather of the row indices and one of the rows, each padded to the largest shard: the
    traffic is world x max_rows, not the world x n_global of an all-reduce over a zero-padded copy."""
    import torch.distributed as dist

    out = local.new_zeros((n_global,) + tuple(local.shape[1:]))
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        out[global_index] = local
        return out
    world = dist.get_world_size()
    idx = global_index.to(device=local.device, dtype=torch.int64)
    cnt = torch.tensor([idx.numel()], device=local.device, dtype=torch.int64)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    m = int(max(int(c.item()) for c in counts))
    pad_idx = torch.full((m,), -1, device=local.device, dtype=torch.int64)
    pad_idx[:idx.numel()] = idx
    pad_rows = local.new_zeros((m,) + tuple(local.shape[1:]))
    pad_rows[:idx.numel()] = local
    all_idx = [torch.empty_like(pad_idx) for _ in range(world)]
    all_rows = [torch.empty_like(pad_rows) for _ in range(world)]
    dist.all_gather(all_idx, pad_idx)
    dist.all_gather(all_rows, pad_rows)
    for i_, r_ in zip(all_idx, all_rows):
        keep = i_ >= 0
        out[i_[keep]] = r_[keep].detach()
    # this rank's rows once more from `local` itself: the all-gathered copies carry no gradient, so a
    # loss over the gathered series back-propagates into this rank's shard as it does with one process
    return out.index_put((idx,), local)
