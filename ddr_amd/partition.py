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


def basin_depths(n: int, rows: np.ndarray, cols: np.ndarray, lab: np.ndarray | None = None):
    """(outlet label of every reach, longest source-to-outlet path of every reach's basin, in reaches).

    Pointer jumping with distances: every reach points at its downstream reach at distance 1 (an outlet at
    itself, 0); the pointers and distances are doubled until every pointer is an outlet."""
    jump = np.arange(n, dtype=np.int64)
    jump[np.asarray(cols, dtype=np.int64)] = np.asarray(rows, dtype=np.int64)
    dist = (jump != np.arange(n)).astype(np.int64)
    while True:
        nxt = jump[jump]
        if np.array_equal(nxt, jump):
            break
        dist = dist + dist[jump]
        jump = nxt
    lab = jump if lab is None else lab
    depth = np.zeros(n, dtype=np.int64)
    np.maximum.at(depth, lab, dist + 1)
    return lab, depth[lab]


def shard_basins(sizes, n_ranks: int, depths=None, steps: int = 0) -> list[np.ndarray]:
    """Indices of the basins owned by each rank: LPT by reach count (ties: deeper first).

    With ``depths`` and ``steps`` (the window's T), the LPT result is then refined against the routing
    time model of a rank, (T + its deepest basin) ticks x a tick cost that grows with its reach count: a pass
    over a rank's blocks takes T + D ticks of the ALAP schedule, D its deepest basin (C5 shards: 2215-deep
    basin + 119k reaches 77.9 ms against 400k shallower reaches 64.6 ms, profiles/r06/n4_plan.txt).
    Single-basin moves from the slowest rank to the fastest are taken while they lower the slowest rank's
    modelled time by more than 1 %."""
    sizes = np.asarray(sizes, dtype=np.int64)
    owner = lpt_assign(sizes, n_ranks, depths)
    if depths is not None and steps > 0 and n_ranks > 1 and len(sizes) > n_ranks:
        depths = np.asarray(depths, dtype=np.int64)
        load = np.bincount(owner, weights=sizes, minlength=n_ranks).astype(np.float64)

        def deepest(r):
            d = depths[owner == r]
            return int(d.max()) if d.size else 0

        for _ in range(256):  # (a handful of moves in practice; bounded)
            dmax = np.array([deepest(r) for r in range(n_ranks)], dtype=np.float64)
            c = (steps + dmax) * load
            src, dst = int(np.argmax(c)), int(np.argmin(c))
            cand = np.nonzero(owner == src)[0]
            d_src = depths[cand]
            # the source rank's deepest basin once candidate i has left it
            top = d_src.max()
            second = np.sort(d_src)[-2] if len(d_src) > 1 else 0
            left_d = np.where((d_src == top) & (np.count_nonzero(d_src == top) == 1), second, top)
            c_src = (steps + left_d) * (load[src] - sizes[cand])
            c_dst = (steps + np.maximum(dmax[dst], d_src)) * (load[dst] + sizes[cand])
            m = np.maximum(c_src, c_dst)
            j = int(np.argmin(m))
            if m[j] > 0.99 * c[src]:
                break
            owner[cand[j]] = dst
            load[src] -= sizes[cand[j]]
            load[dst] += sizes[cand[j]]
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
