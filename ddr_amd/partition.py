"""Outlet-basin sharding of a river forest across ranks.

Outlet basins are independent for the whole solve (no edge crosses them), so a multi-GPU run
shards *basins* -- never reaches of one basin -- and needs no collective on the data path.  Cost
of a basin ~ reaches x T; assignment is LPT (longest-processing-time first) with a tie-break on
depth, so the largest basins are spread first.
"""

from __future__ import annotations

import heapq

import numpy as np


def basin_labels(n: int, rows: np.ndarray, cols: np.ndarray) -> np.ndarray:
    """Outlet reach id of every reach (rows = downstream, cols = upstream, lower triangular).

    Pointer jumping: every reach points at its downstream reach (an outlet at itself) and the pointers
    are squared until they stop moving -- ceil(log2(depth)) vectorised passes."""
    lab = np.arange(n, dtype=np.int64)
    lab[np.asarray(cols, dtype=np.int64)] = np.asarray(rows, dtype=np.int64)
    while True:
        nxt = lab[lab]
        if np.array_equal(nxt, lab):
            return lab
        lab = nxt


def lpt_assign(costs, n_bins: int, tiebreak=None) -> np.ndarray:
    """Bin of each item, largest cost first onto the least-loaded bin (deterministic)."""
    costs = np.asarray(costs, dtype=np.float64)
    tb = np.zeros_like(costs) if tiebreak is None else np.asarray(tiebreak, dtype=np.float64)
    order = np.lexsort((np.arange(len(costs)), -tb, -costs))
    heap = [(0.0, b) for b in range(n_bins)]
    heapq.heapify(heap)
    out = np.empty(len(costs), dtype=np.int64)
    for i in order:
        load, b = heapq.heappop(heap)
        out[i] = b
        heapq.heappush(heap, (load + costs[i], b))
    return out


def shard_basins(sizes, n_ranks: int, depths=None) -> list[np.ndarray]:
    """Indices of the basins owned by each rank."""
    owner = lpt_assign(sizes, n_ranks, depths)
    return [np.nonzero(owner == r)[0] for r in range(n_ranks)]


def extract_basins(n: int, rows: np.ndarray, cols: np.ndarray, keep_reach: np.ndarray):
    """Sub-network of the reaches with ``keep_reach`` True, renumbered in the original (topological)
    order.  Returns (n_sub, rows_sub, cols_sub, reach_ids) with reach_ids mapping back."""
    keep_reach = np.asarray(keep_reach, dtype=bool)
    ids = np.nonzero(keep_reach)[0]
    new = np.full(n, -1, dtype=np.int64)
    new[ids] = np.arange(len(ids))
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    m = keep_reach[rows] & keep_reach[cols]
    if np.any(keep_reach[rows] != keep_reach[cols]):
        raise ValueError("selection cuts an edge: shard whole basins only")
    return len(ids), new[rows[m]].astype(np.int32), new[cols[m]].astype(np.int32), ids
