"""Seeded synthetic river forests for tests and benchmarks.

Every generator returns a topologically ordered, strictly lower-triangular, dendritic COO
(``rows`` = downstream reach, ``cols`` = upstream reach), the same contract as the reference's
engine output (``engine/src/ddr_engine/core/zarr_io.py:7-76``, ``merit/build.py:94,105``).

* ``random_binary_tree``  -- config C1: random attachment to a later reach with in-degree < 2.
* ``hack_basin``          -- one basin with a Hack's-law main stem (ceil(n**0.6) reaches), binary
  confluences and an explicit single-inflow fraction.
* ``forest``              -- a union of basins, each numbered contiguously in upstream-first order.
* ``zipf_sizes`` / ``loguniform_sizes`` -- basin-size laws for C3/C4/C5.

Reach attributes follow SURVEY §8(d) "Value distributions".
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


@dataclass
class SyntheticNetwork:
    n: int
    rows: np.ndarray  # int32 (E,), downstream reach
    cols: np.ndarray  # int32 (E,), upstream reach
    basin_sizes: np.ndarray  # int64 (B,), basins numbered contiguously in this order

    @property
    def down(self) -> np.ndarray:
        d = np.full(self.n, -1, dtype=np.int64)
        d[self.cols] = self.rows
        return d

    def dense(self) -> np.ndarray:
        a = np.zeros((self.n, self.n), dtype=np.float32)
        a[self.rows, self.cols] = 1.0
        return a


def _down_to_coo(down: np.ndarray):
    up = np.nonzero(down >= 0)[0]
    rows = down[up].astype(np.int32)
    cols = up.astype(np.int32)
    order = np.lexsort((cols, rows))
    return rows[order], cols[order]


def random_binary_tree(n: int, seed: int = 0) -> SyntheticNetwork:
    """C1: reach i drains into a uniformly chosen later reach whose in-degree is < 2."""
    rng = np.random.default_rng(seed)
    down = np.full(n, -1, dtype=np.int64)
    avail = [n - 1]
    indeg = np.zeros(n, dtype=np.int64)
    for i in range(n - 2, -1, -1):
        k = int(rng.integers(len(avail)))
        j = avail[k]
        down[i] = j
        indeg[j] += 1
        if indeg[j] == 2:
            avail[k] = avail[-1]
            avail.pop()
        avail.append(i)
    rows, cols = _down_to_coo(down)
    return SyntheticNetwork(n, rows, cols, np.array([n], dtype=np.int64))


def _hack_basin_down(n: int, rng: np.random.Generator, single_inflow: float, exponent: float) -> np.ndarray:
    """Parent pointers of one basin in creation order (a parent is always created first)."""
    # fraction f of spine joints left without a tributary so that the overall fraction of
    # single-inflow reaches is ~single_inflow (see DESIGN.md "synthetic networks")
    f = 2.0 * single_inflow / (1.0 + single_inflow)
    down = np.full(n, -1, dtype=np.int64)
    nxt = 0
    stack = [(n, -1)]
    while stack:
        m, parent = stack.pop()
        ls = min(m, max(1, math.ceil(m**exponent)))
        spine = np.arange(nxt, nxt + ls, dtype=np.int64)
        nxt += ls
        down[spine[0]] = parent
        down[spine[1:]] = spine[:-1]
        rest = m - ls
        if rest <= 0:
            continue
        k = int(round((1.0 - f) * (ls - 1)))
        k = max(1, min(k, rest, ls - 1))
        w = rng.pareto(1.2, size=k) + 0.05
        sizes = 1 + rng.multinomial(rest - k, w / w.sum())
        pos = rng.choice(ls - 1, size=k, replace=False)
        for s, p in zip(sizes.tolist(), pos.tolist()):
            stack.append((s, int(spine[p])))
    assert nxt == n
    return down


def hack_basin_down(n: int, rng: np.random.Generator, single_inflow: float = 0.25, exponent: float = 0.6):
    """Topologically numbered (upstream first) parent array of one Hack's-law basin."""
    local = _hack_basin_down(n, rng, single_inflow, exponent)
    # creation order is downstream-first; reversing it is a topological order
    new = (n - 1) - np.arange(n, dtype=np.int64)
    down = np.full(n, -1, dtype=np.int64)
    has = local >= 0
    down[new[has]] = new[local[has]]
    return down


def forest(sizes, seed: int = 0, single_inflow: float = 0.25, exponent: float = 0.6,
           shuffle_basins: bool = True) -> SyntheticNetwork:
    """Union of Hack's-law basins, each numbered contiguously (basin order shuffled)."""
    rng = np.random.default_rng(seed)
    sizes = np.asarray(sizes, dtype=np.int64)
    if shuffle_basins:
        sizes = sizes[rng.permutation(len(sizes))]
    n = int(sizes.sum())
    down = np.full(n, -1, dtype=np.int64)
    off = 0
    for s in sizes.tolist():
        d = hack_basin_down(int(s), rng, single_inflow, exponent)
        has = d >= 0
        seg = down[off : off + s]
        seg[has] = d[has] + off
        off += s
    rows, cols = _down_to_coo(down)
    return SyntheticNetwork(n, rows, cols, sizes)


def hack_basin(n: int, seed: int = 0, single_inflow: float = 0.25) -> SyntheticNetwork:
    return forest([n], seed=seed, single_inflow=single_inflow, shuffle_basins=False)


def zipf_sizes(total: int, n_basins: int, largest_frac: float) -> np.ndarray:
    """Basin sizes s_k ∝ k^-a (k = 1..B) with a chosen so that s_1 ≈ largest_frac · total."""
    k = np.arange(1, n_basins + 1, dtype=np.float64)
    lo, hi = 0.5, 4.0
    for _ in range(60):
        a = 0.5 * (lo + hi)
        w = k**-a
        if w[0] / w.sum() < largest_frac:
            lo = a
        else:
            hi = a
    w = k ** -(0.5 * (lo + hi))
    s = np.maximum(1, np.floor(total * w / w.sum())).astype(np.int64)
    s[0] += total - s.sum()
    return s


def loguniform_sizes(n_basins: int, lo: int, hi: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return np.round(np.exp(rng.uniform(math.log(lo), math.log(hi), size=n_basins))).astype(np.int64)


# ---------------------------------------------------------------------------------------------
# Attributes and forcing
# ---------------------------------------------------------------------------------------------


@dataclass
class ReachAttributes:
    length: np.ndarray
    slope: np.ndarray
    x: np.ndarray


def reach_attributes(n: int, seed: int = 0, x_const: float | None = None) -> ReachAttributes:
    rng = np.random.default_rng(seed + 1000)
    length = np.clip(rng.lognormal(math.log(3000.0), 0.6, n), 100.0, 50000.0).astype(np.float32)
    slope = rng.lognormal(math.log(1e-3), 1.0, n).astype(np.float32)
    if x_const is None:
        x = rng.uniform(0.1, 0.4, n).astype(np.float32)
    else:
        x = np.full(n, x_const, dtype=np.float32)
    return ReachAttributes(length, slope, x)


def lateral_inflow(n: int, T: int, seed: int = 0, t0: int = 0) -> np.ndarray:
    """q'[t, i] = a_i (1 + 0.5 sin(2π t/24 + φ_i)) s(t), (T, N) float32 (host)."""
    rng = np.random.default_rng(seed + 2000)
    a = rng.lognormal(math.log(0.5), 1.0, n).astype(np.float32)
    phi = rng.uniform(0, 2 * math.pi, n).astype(np.float32)
    t = np.arange(t0, t0 + T, dtype=np.float32)[:, None]
    season = (1.0 + 0.5 * np.sin(2 * math.pi * t / 8760.0)).astype(np.float32)
    return (a[None, :] * (1.0 + 0.5 * np.sin(2 * math.pi * t / 24.0 + phi[None, :])) * season).astype(np.float32)


def lateral_inflow_torch(n: int, T: int, seed: int = 0, device="cuda", chunk: int = 256, ids=None):
    """Same law as ``lateral_inflow`` generated on the device in time chunks (large T·N).  With ``ids``
    only those columns of the n-reach field (a rank's shard of a global network)."""
    import torch

    rng = np.random.default_rng(seed + 2000)
    a = rng.lognormal(math.log(0.5), 1.0, n).astype(np.float32)
    phi = rng.uniform(0, 2 * math.pi, n).astype(np.float32)
    if ids is not None:
        a, phi = a[ids], phi[ids]
        n = len(ids)
    a = torch.from_numpy(a).to(device)
    phi = torch.from_numpy(phi).to(device)
    out = torch.empty((T, n), dtype=torch.float32, device=device)
    for s in range(0, T, chunk):
        e = min(T, s + chunk)
        t = torch.arange(s, e, dtype=torch.float32, device=device)[:, None]
        season = 1.0 + 0.5 * torch.sin(2 * math.pi * t / 8760.0)
        out[s:e] = a[None, :] * (1.0 + 0.5 * torch.sin(2 * math.pi * t / 24.0 + phi[None, :])) * season
    return out


def unit_parameters(n: int, seed: int = 0):
    """KAN-like outputs in [0, 1] (fixed per seed): dict(n, q_spatial, p_spatial)."""
    rng = np.random.default_rng(seed + 3000)
    return {k: rng.uniform(0.0, 1.0, n).astype(np.float32) for k in ("n", "q_spatial", "p_spatial")}


def network_stats(net: SyntheticNetwork) -> dict:
    down = net.down
    n = net.n
    dist = np.zeros(n, dtype=np.int64)
    for i in range(n - 1, -1, -1):
        if down[i] >= 0:
            dist[i] = dist[down[i]] + 1
    indeg = np.bincount(net.rows, minlength=n)
    return dict(n=n, edges=len(net.rows), basins=len(net.basin_sizes), max_depth=int(dist.max()) + 1,
                largest_basin=int(net.basin_sizes.max()), single_inflow_frac=float((indeg == 1).mean()))


def reach_features(n: int, n_attr: int = 10, seed: int = 0) -> np.ndarray:
    """Normalised catchment attributes (N, n_attr) for a parameter network (the reference feeds the KAN
    ``routing_dataclass.normalized_spatial_attributes``, scripts/train.py:71)."""
    rng = np.random.default_rng(seed + 5000)
    return rng.standard_normal((n, n_attr)).astype(np.float32)
