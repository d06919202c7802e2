"""One outlet basin routed by several GPUs (BASELINE.json north star item (5), SURVEY.md §8(e) "next").

Sharding by outlet basin (``distributed.shard_network``) leaves a basin that is larger than a rank's
share on one GPU: C5's 281k-reach basin (0.35 N) floors the 8-GPU step at its one-GPU time.  Here the
ranks of a *split group* all build the same graph of that basin (the builders are deterministic) with
k times the workgroups of one GPU, and each runs a contiguous range of its logical blocks (ticket
order = piece-height order, balanced by reaches).  The time-pipelined hand-off between blocks is the
same fp64 data-is-flag granule as inside one GPU; a cut edge whose two blocks belong to different
ranks writes its granules into the receive memory of the rank that reads them (system-scope stores
over xGMI into uncached memory exported by IPC handle, ``ddr_xmem_*``).  Before every routing launch
the ranks reset their receive rows and hand-shake on the device (``include/ddr_mc.h``), so the
training step needs no extra host synchronisation.

The reference has no counterpart (its solve runs a basin on one device, ``routing/utils.py:515-692``).
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .partition import basin_depths, basin_labels, extract_basins, shard_basins


def plan_block_ranks(nloc, k: int, prod=None, cons=None, tol: float = 0.05, sweeps: int = 8) -> np.ndarray:
    """Rank of each logical block: k contiguous ranges with equal reach counts -- of the ticket order,
    or (given the cut edges' producer / consumer blocks) of a depth-first order of the block graph from
    the outlet side when that crosses fewer edges -- then greedy moves of single blocks to the rank most
    of their cut edges lead to, while every rank stays within ``tol`` of the mean load: fewer
    cross-rank edges (each a system-scope hand-off over xGMI) for the same balance.  Deterministic,
    so every rank of a split computes the same plan.  Any assignment is deadlock-free: each rank takes
    its blocks in ticket (topological) order."""
    nloc = np.asarray(nloc, dtype=np.int64)
    if k < 1 or len(nloc) < k:
        raise ValueError("need at least one block per rank")

    def ranges(order):  # k contiguous ranges of `order` with equal reach counts
        w = nloc[order]
        mid = np.cumsum(w) - w / 2.0
        rr = np.minimum((mid * k / max(float(nloc.sum()), 1.0)).astype(np.int64), k - 1)
        for i in range(k):  # every rank gets at least one block (tiny graphs)
            if not np.any(rr == i):
                rr[min(i, len(rr) - 1)] = i
        out = np.empty(len(order), dtype=np.int64)
        out[order] = np.maximum.accumulate(rr)
        return out

    nb = len(nloc)
    r = ranges(np.arange(nb))
    if prod is None or cons is None or k == 1 or len(prod) == 0:
        return r.astype(np.int32)
    prod = np.asarray(prod, dtype=np.int64)
    cons = np.asarray(cons, dtype=np.int64)
    nbr = [[] for _ in range(nb)]
    for a, b in zip(prod.tolist(), cons.tolist()):
        nbr[a].append(b)
        nbr[b].append(a)
    # depth-first order of the block graph from the outlet side (the last tickets): contiguous ranges
    # of it are unions of whole upstream subtrees, crossed by few edges
    seen = np.zeros(nb, dtype=bool)
    order = []
    for root in range(nb - 1, -1, -1):
        if seen[root]:
            continue
        stack = [root]
        seen[root] = True
        while stack:
            b = stack.pop()
            order.append(b)
            for c in sorted(nbr[b], reverse=True):
                if not seen[c]:
                    seen[c] = True
                    stack.append(c)
    rd = ranges(np.asarray(order, dtype=np.int64))
    if np.count_nonzero(rd[prod] != rd[cons]) < np.count_nonzero(r[prod] != r[cons]):
        r = rd
    load = np.bincount(r, weights=nloc, minlength=k).astype(np.float64)
    mean = float(nloc.sum()) / k
    lo, hi = mean * (1.0 - tol), mean * (1.0 + tol)
    for _ in range(sweeps):
        moved = 0
        for b in range(nb):
            if not nbr[b]:
                continue
            cnt = np.bincount(r[nbr[b]], minlength=k)
            cur = r[b]
            best = int(np.argmax(cnt))
            if best == cur or cnt[best] <= cnt[cur]:
                continue
            if load[best] + nloc[b] > hi or load[cur] - nloc[b] < lo or np.count_nonzero(r == cur) == 1:
                continue
            r[b] = best
            load[best] += nloc[b]
            load[cur] -= nloc[b]
            moved += 1
        if moved == 0:
            break
    return r.astype(np.int32)


def block_edges(graph):
    """(nloc per logical block, producer block and consumer block of every cut edge) of a RiverGraph."""
    lib = _lib.load()
    info = graph.info
    nloc = np.zeros(info.n_blocks, dtype=np.int32)
    _lib.check(lib.ddr_graph_blocks(graph.handle, nloc.ctypes.data, len(nloc)))
    prod = np.empty(max(info.n_cut, 1), dtype=np.int32)
    cons = np.empty(max(info.n_cut, 1), dtype=np.int32)
    _lib.check(lib.ddr_graph_cut_blocks(graph.handle, prod.ctypes.data, cons.ctypes.data, int(info.n_cut)))
    return nloc, prod[:info.n_cut], cons[:info.n_cut]


def plan_ranks(n: int, rows, cols, world: int, factor: float = 1.2, force: bool = False, steps: int = 0):
    """Per rank: (reach_ids, split) where split is None (whole basins, LPT over the ranks outside the
    split group) or (group_ranks, index_in_group) for the ranks that route the largest basin together.

    The largest basin is split when it exceeds ``factor`` x the per-rank mean (or ``force``) and at
    least one rank remains for the other basins; its group has k = round(size / mean) ranks (at least 2).
    ``force`` with two ranks (a rehearsal) splits the largest basin over both and leaves the other basins out.
    factor 1.2: C5 at N = 4 (the 281k-reach basin is 1.4 x a rank's share) splits it over two ranks -- the
    basin alone on one rank took 55.5 ms, the two other ranks' 259k-reach shards 48.5-48.8 ms and the group
    (its 511 workgroups routed alone: 66.3 ms) about half that (profiles/r06/n4_plan.txt).
    ``steps`` > 0: whole basins are assigned by distributed.shard_network's depth-aware refinement."""
    lab, dep = basin_depths(n, rows, cols)
    outlets, first, inv, sizes = np.unique(lab, return_index=True, return_inverse=True, return_counts=True)
    bdep = dep[first] if steps > 0 else None
    mean = n / max(world, 1)
    big = int(np.argmax(sizes))
    k = int(round(sizes[big] / mean)) if world > 1 else 0
    k = min(max(k, 2), world - 1) if world > 2 else (2 if force and world == 2 else 0)
    split = world > 1 and k >= 2 and (force or sizes[big] > factor * mean) and (world - k >= 1 or force)
    out = []
    if not split:
        owner = np.empty(len(outlets), dtype=np.int64)
        for r, idx in enumerate(shard_basins(sizes, world, bdep, steps)):
            owner[idx] = r
        for r in range(world):
            out.append((np.nonzero(owner[inv] == r)[0], None))
        return out
    group = list(range(k))
    big_ids = np.nonzero(inv == big)[0]
    rest = [i for i in range(len(outlets)) if i != big]
    others = world - k
    owner = np.full(len(outlets), -1, dtype=np.int64)
    if others > 0 and rest:  # (none left: a forced 2-rank rehearsal routes only the split basin)
        for j, idx in enumerate(shard_basins(sizes[rest], others, None if bdep is None else bdep[rest], steps)):
            owner[np.asarray(rest)[idx]] = k + j
    for r in range(world):
        if r < k:
            out.append((big_ids, (group, r)))
        else:
            out.append((np.nonzero(owner[inv] == r)[0], None))
    return out


def sub_network(n: int, rows, cols, ids):
    keep = np.zeros(n, dtype=bool)
    keep[ids] = True
    return extract_basins(n, rows, cols, keep)


class SplitBasin:
    """Attach a split to ``graph`` (a RiverGraph built identically on every rank of the group).

    ``exchange(obj) -> list`` gathers one picklable object from every rank of the group, in group
    order (e.g. ``torch.distributed.all_gather_object`` restricted to the group)."""

    def __init__(self, graph, block_rank, index: int, k: int, t_cap: int, exchange):
        lib = _lib.load()
        self.graph, self.k, self.index = graph, k, index
        info = graph.info
        self.block_rank = np.ascontiguousarray(block_rank, dtype=np.int32)
        if len(self.block_rank) != info.n_blocks:
            raise ValueError("block_rank needs one entry per logical block")
        _, prod, cons = block_edges(graph)
        self.n_x = int(np.count_nonzero(self.block_rank[prod] != self.block_rank[cons]))
        nb = C.c_int64()
        _lib.check(lib.ddr_xmem_bytes(self.n_x, int(t_cap), C.byref(nb)))
        self.bytes = nb.value
        ptr = C.c_void_p()
        handle = (C.c_ubyte * 64)()
        kind = C.c_int32()
        self.local, self.peers, self._opened = None, [], []
        err = None
        try:
            _lib.check(lib.ddr_xmem_alloc(self.bytes, C.byref(ptr), handle, C.byref(kind)))
            self.local, self.kind = ptr.value, kind.value
        except Exception as e:  # noqa: BLE001  (still take part in the exchange: the peers wait for it)
            err = e
        handles = exchange(None if err else bytes(handle))
        self._attached = False
        try:
            if err is not None:
                raise err
            if len(handles) != k:
                raise ValueError("exchange must return one handle per rank of the group")
            if any(h is None for h in handles):
                raise RuntimeError("split basin: a peer could not allocate its receive memory")
            for r, h in enumerate(handles):
                if r == index:
                    self.peers.append(self.local)
                    continue
                p = C.c_void_p()
                _lib.check(lib.ddr_xmem_open((C.c_ubyte * 64).from_buffer_copy(h), C.byref(p)))
                self.peers.append(p.value)
                self._opened.append(p.value)
            arr = (C.c_void_p * k)(*self.peers)
            n_x = C.c_int64()
            _lib.check(lib.ddr_graph_set_split(graph.handle, index, k, self.block_rank.ctypes.data, self.local, arr,
                                               int(t_cap), C.byref(n_x)))
            self._attached = True
            if n_x.value != self.n_x:
                raise RuntimeError("cross-rank cut edges disagree between the host plan and the library")
        except Exception:
            self.close()  # neither opened handles nor the receive memory leak
            raise
        # the reaches this rank routes (their outputs and gradients are this rank's)
        blk = graph.structure()["block"] if hasattr(graph, "structure") else None
        self.owned_reaches = None if blk is None else np.nonzero(self.block_rank[blk] == index)[0]

    def close(self) -> None:
        """Release the receive memory (after the device is done with every launch of the split)."""
        import torch

        lib = _lib.load()
        torch.cuda.synchronize()
        if getattr(self, "_attached", False) and self.graph.handle is not None and self.graph.handle.value:
            _lib.check(lib.ddr_graph_clear_split(self.graph.handle))  # no later launch touches freed memory
        self._attached = False
        for p in self._opened:
            _lib.check(lib.ddr_xmem_close(p, 1))
        self._opened = []
        if self.local:
            _lib.check(lib.ddr_xmem_close(self.local, 0))
            self.local = None
