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

from .partition import basin_labels, extract_basins, shard_basins


def rank_world():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_network(n: int, rows: np.ndarray, cols: np.ndarray, rank: int, world: int, depth_weight: float = 0.0):
    """This rank's sub-network: whole outlet basins, LPT-balanced by reach count.

    Returns (n_sub, rows_sub, cols_sub, reach_ids) with ``reach_ids`` the global reach index of each
    local reach (topological order preserved).
    """
    lab = basin_labels(n, rows, cols)
    outlets, inv, sizes = np.unique(lab, return_inverse=True, return_counts=True)
    owner = np.empty(len(outlets), dtype=np.int64)
    for r, idx in enumerate(shard_basins(sizes, world)):
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
    """Assemble a (n_global, ...) tensor from every rank's rows (e.g. gauge discharge (G_r, T))."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        out = local.new_zeros((n_global,) + tuple(local.shape[1:]))
        out[global_index] = local
        return out
    out = local.new_zeros((n_global,) + tuple(local.shape[1:]))
    out[global_index] = local
    dist.all_reduce(out, op=dist.ReduceOp.SUM)
    return out
