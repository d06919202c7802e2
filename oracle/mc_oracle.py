"""CPU oracle for the Muskingum-Cunge routing hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the *checker* (or, in ``bench.py``, as the timed CPU baseline).  The
product path (``ddr_amd``) never imports it: the HIP library is the only implementation there.

This is a restatement, written from the equations, of the reference's routing algorithm
(taddyb/ddr).  Each function cites the reference lines it follows.

Parity pinning: the restatement is checked against golden vectors produced by running the
reference's own hot-path modules in the build container (``tests/golden/make_golden.py``,
fixtures ``tests/golden/*.npz``) and against the reference tests' known-answer vectors
(``tests/routing/test_routing_utils.py:138-151``, ``tests/routing/test_mmc.py:564-602``).

Two precisions are provided:

* ``np.float64`` -- every operation in double precision (the "fp64 oracle" of the north star).
* ``np.float32`` -- the reference recipe: element-wise math in fp32 in PyTorch's operation order
  (no FMA contraction, each op rounded), the triangular solve accumulated in fp64 and rounded to
  fp32 at the end (SciPy ``spsolve_triangular`` on fp64 copies, ``utils.py:587-600``).  ``pow`` is
  evaluated correctly rounded (fp64 pow rounded to fp32); the reference's ATen/Sleef ``powf`` is a
  1-ulp approximation, which is the documented source of residual fp32 drift.

Graph convention (reference ``dataclasses.py:197-200``): ``adjacency[i, j] = 1`` means reach j
drains into reach i; the matrix is strictly lower triangular (topological order) and dendritic
(each reach has at most one downstream reach).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# ---------------------------------------------------------------------------------------------
# Graph helpers
# ---------------------------------------------------------------------------------------------


@dataclass
class Network:
    """Dendritic, topologically ordered river network (oracle-side view).

    Built from the canonical CSR of the adjacency (row = downstream, col = upstream).
    """

    n: int
    crow: np.ndarray  # (n+1,) int64, CSR row pointers of N
    col: np.ndarray  # (nnz,) int64, ascending within a row
    down: np.ndarray = field(init=False)  # (n,) int64, -1 for outlets
    height: np.ndarray = field(init=False)  # longest upstream path length (0 = headwater)
    dist: np.ndarray = field(init=False)  # hops to the basin outlet (0 = outlet)
    solver: str = "levels"  # "levels" (vectorised sweep) or "scipy" (the reference recipe, for timing)

    def __post_init__(self) -> None:
        n = self.n
        self.crow = np.asarray(self.crow, dtype=np.int64)
        self.col = np.asarray(self.col, dtype=np.int64)
        rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(self.crow))
        if np.any(self.col >= rows):
            raise ValueError("adjacency is not strictly lower triangular (not topologically sorted)")
        down = np.full(n, -1, dtype=np.int64)
        if np.any(np.bincount(self.col, minlength=n) > 1):
            raise ValueError("adjacency is not dendritic (a reach has more than one downstream)")
        down[self.col] = rows
        self.down = down
        h = np.zeros(n, dtype=np.int64)
        for i in range(n):  # upstream-first order
            s, e = self.crow[i], self.crow[i + 1]
            if e > s:
                h[i] = h[self.col[s:e]].max() + 1
        self.height = h
        d = np.zeros(n, dtype=np.int64)
        for i in range(n - 1, -1, -1):  # downstream-first order
            if down[i] >= 0:
                d[i] = d[down[i]] + 1
        self.dist = d
        # level schedules for vectorised sweeps
        self._up_levels = _levels_with_slots(self.crow, self.col, h)
        order = np.argsort(d, kind="stable")
        bounds = np.searchsorted(d[order], np.arange(d.max() + 2 if n else 1))
        self._down_levels = [order[bounds[k] : bounds[k + 1]] for k in range(len(bounds) - 1)]

    @classmethod
    def from_dense(cls, adj: np.ndarray) -> "Network":
        adj = np.asarray(adj)
        n = adj.shape[0]
        crow = np.zeros(n + 1, dtype=np.int64)
        cols = []
        for i in range(n):
            nz = np.nonzero(adj[i])[0]
            cols.append(nz)
            crow[i + 1] = crow[i] + len(nz)
        col = np.concatenate(cols) if cols else np.zeros(0, dtype=np.int64)
        return cls(n, crow, col.astype(np.int64))

    @classmethod
    def from_coo(cls, n: int, rows: np.ndarray, cols: np.ndarray) -> "Network":
        crow, col, _ = coo_to_csr(n, rows, cols)
        return cls(n, crow, col)

    # ----- sweeps ---------------------------------------------------------------------------
    def spmv(self, v: np.ndarray) -> np.ndarray:
        """I = N @ v, summing upstream values in ascending column order (mmc.py:535)."""
        out = np.zeros(self.n, dtype=v.dtype)
        # level order is irrelevant for an SpMV; the slot decomposition keeps column order
        for nodes, ups in self._up_levels:
            acc = np.zeros(len(nodes), dtype=v.dtype)
            for k, (sel, src) in enumerate(ups):
                acc[sel] = acc[sel] + v[src]
            out[nodes] = acc
        return out

    def lower_solve(self, c1: np.ndarray, b: np.ndarray) -> np.ndarray:
        """Solve (I - diag(c1) N) x = b in fp64, upstream-first.

        Mirrors the SuperLU column sweep behind SciPy's ``spsolve_triangular`` used by the
        reference (``utils.py:587-600``): x_i = (b_i + c1_i*x_j1) + c1_i*x_j2 ... in ascending j.
        """
        c1 = c1.astype(np.float64)
        if self.solver == "scipy":
            return self._scipy_solve(c1, b, transpose=False)
        x = b.astype(np.float64).copy()
        for nodes, ups in self._up_levels:
            acc = x[nodes]
            cc = c1[nodes]
            for sel, src in ups:
                acc[sel] = acc[sel] + cc[sel] * x[src]
            x[nodes] = acc
        return x

    def upper_solve(self, c1: np.ndarray, g: np.ndarray) -> np.ndarray:
        """Solve (I - diag(c1) N)^T y = g in fp64, downstream-first (utils.py:188-242).

        Dendritic form: y_j = g_j + c1_down(j) * y_down(j).
        """
        c1 = c1.astype(np.float64)
        if self.solver == "scipy":
            return self._scipy_solve(c1, g, transpose=True)
        y = g.astype(np.float64).copy()
        for nodes in self._down_levels[1:]:
            d = self.down[nodes]
            y[nodes] = y[nodes] + c1[d] * y[d]
        return y


def _scipy_matrix(net: "Network", c1: np.ndarray):
    import scipy.sparse as sp

    rows = np.repeat(np.arange(net.n, dtype=np.int64), np.diff(net.crow))
    r = np.concatenate([rows, np.arange(net.n)])
    c = np.concatenate([net.col, np.arange(net.n)])
    v = np.concatenate([-c1[rows].astype(np.float32).astype(np.float64), np.ones(net.n)])
    return sp.csr_matrix((v, (r, c)), shape=(net.n, net.n))


def _scipy_solve(self, c1, b, transpose):
    """Reference recipe: SciPy spsolve_triangular on fp64 copies (utils.py:587-600, 188-242)."""
    from scipy.sparse.linalg import spsolve_triangular

    A = _scipy_matrix(self, c1)
    if transpose:
        return spsolve_triangular(A.T, np.asarray(b, np.float64), lower=False, unit_diagonal=False)
    return spsolve_triangular(A, np.asarray(b, np.float64), lower=True, unit_diagonal=False)


Network._scipy_solve = _scipy_solve


def _levels_with_slots(crow, col, height):
    """Group nodes by height; for each group, list (selector, upstream-index) per inflow slot."""
    n = len(crow) - 1
    levels = []
    if n == 0:
        return levels
    order = np.argsort(height, kind="stable")
    hb = np.searchsorted(height[order], np.arange(height.max() + 2))
    deg = np.diff(crow)
    for k in range(len(hb) - 1):
        nodes = order[hb[k] : hb[k + 1]]
        if k == 0:
            levels.append((nodes, []))
            continue
        dn = deg[nodes]
        ups = []
        for s in range(int(dn.max())):
            sel = dn > s
            ups.append((sel, col[crow[nodes[sel]] + s]))
        levels.append((nodes, ups))
    return levels


def coo_to_csr(n: int, rows: np.ndarray, cols: np.ndarray, vals: np.ndarray | None = None):
    """Canonical CSR (rows sorted, columns ascending, duplicates summed).

    Restates ``scipy.sparse.coo_matrix((vals, (rows, cols))).tocsr()`` used by the reference
    (``src/ddr/geodatazoo/merit.py:197-223``; SciPy 1.15.3).  Duplicates are summed in
    original COO order.
    """
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    vals = np.ones(len(rows), dtype=np.float32) if vals is None else np.asarray(vals)
    key = np.lexsort((np.arange(len(rows)), cols, rows))
    r, c, v = rows[key], cols[key], vals[key]
    if len(r):
        new = np.ones(len(r), dtype=bool)
        new[1:] = (r[1:] != r[:-1]) | (c[1:] != c[:-1])
        grp = np.cumsum(new) - 1
        vs = np.zeros(int(grp[-1]) + 1, dtype=v.dtype)
        np.add.at(vs, grp, v)
        r, c, v = r[new], c[new], vs
    crow = np.zeros(n + 1, dtype=np.int64)
    np.add.at(crow, r + 1, 1)
    crow = np.cumsum(crow)
    return crow, c, v


# ---------------------------------------------------------------------------------------------
# Element-wise physics
# ---------------------------------------------------------------------------------------------


@dataclass
class Bounds:
    """Lower bounds of the routing state (``mmc.py:203-208``, ``configs.py:86-95`` defaults)."""

    discharge: float = 1e-4
    velocity: float = 0.01
    depth: float = 0.01
    bottom_width: float = 0.01
    velocity_max: float = 15.0  # mmc.py:166
    side_slope_min: float = 0.5  # trapezoidal.py:79
    side_slope_max: float = 50.0


def _pow(a, b, dt):
    if dt == np.float32:
        return np.power(a.astype(np.float64), np.asarray(b, dtype=np.float32).astype(np.float64)).astype(
            np.float32
        )
    return np.power(a, b)


def denormalize(u, bounds, log_space=False, dtype=np.float32):
    """``utils.py:166-185`` (note the +1e-6 on the log-space lower bound only)."""
    u = np.asarray(u, dtype=dtype)
    if log_space:
        lo = np.log(dtype(bounds[0] + 1e-6))
        hi = np.log(dtype(bounds[1]))
        return np.exp(u * (hi - lo) + lo).astype(dtype)
    return ((u * dtype(bounds[1] - bounds[0])) + dtype(bounds[0])).astype(dtype)


def trapezoid_celerity(Q, n, q, p, slope, bd: Bounds, dtype=np.float32, full=False):
    """Manning celerity from the Leopold & Maddock power-law trapezoid.

    ``trapezoidal.py:62-97`` + ``mmc.py:150-167`` in PyTorch operation order.  Returns
    (celerity, top_width, side_slope) or, with ``full``, a dict of every intermediate.
    """
    f = dtype
    Q = Q.astype(f)
    qe = q + f(1e-6)
    num = (Q * n) * (qe + f(1.0))
    den = p * np.sqrt(slope)
    ratio = num / (den + f(1e-8))
    expo = f(3.0) / (f(5.0) + f(3.0) * qe)
    pw = _pow(ratio, expo, f)
    depth = np.maximum(pw, f(bd.depth))
    dq = _pow(depth, qe, f)
    tw = p * dq
    ss_raw = (tw * qe) / (f(2.0) * depth)
    ss = np.clip(ss_raw, f(bd.side_slope_min), f(bd.side_slope_max))
    bw_raw = tw - (f(2.0) * ss) * depth
    bw = np.maximum(bw_raw, f(bd.bottom_width))
    area = ((tw + bw) * depth) / f(2.0)
    sq = np.sqrt(f(1.0) + ss * ss)
    wp = bw + (f(2.0) * depth) * sq
    R = area / wp
    r23 = _pow(R, 2.0 / 3.0, f) if f == np.float32 else np.power(R, 2.0 / 3.0)
    v = ((f(1.0) / n) * r23) * np.sqrt(slope)
    vc = np.clip(v, f(bd.velocity), f(bd.velocity_max))
    c = (vc * f(5.0)) / f(3.0)
    if full:
        return dict(qe=qe, num=num, den=den, ratio=ratio, expo=expo, pw=pw, depth=depth, tw=tw,
                    ss_raw=ss_raw, ss=ss, bw_raw=bw_raw, bw=bw, area=area, sq=sq, wp=wp, R=R,
                    r23=r23, v=v, vc=vc, c=c)
    return c, tw, ss


def muskingum_coefficients(length, c, X, dt, dtype=np.float32):
    """``mmc.py:460-485``."""
    f = dtype
    dt = f(dt)
    k = length / c
    two_k = f(2.0) * k
    den = (two_k * (f(1.0) - X)) + dt
    c1 = (dt - two_k * X) / den
    c2 = (dt + two_k * X) / den
    c3 = ((two_k * (f(1.0) - X)) - dt) / den
    c4 = (f(2.0) * dt) / den
    return c1, c2, c3, c4


# ---------------------------------------------------------------------------------------------
# Forward routing
# ---------------------------------------------------------------------------------------------


@dataclass
class Reaches:
    """Static per-reach inputs of the routing step (already denormalised / clamped)."""

    n: np.ndarray
    q: np.ndarray
    p: np.ndarray  # (N,) or 0-d
    length: np.ndarray
    slope: np.ndarray  # clamped at the slope minimum (mmc.py:285-288)
    x: np.ndarray

    def astype(self, dtype):
        def cv(a):
            return np.asarray(a, dtype=dtype)

        p = cv(self.p)
        return Reaches(cv(self.n), cv(self.q), p, cv(self.length), cv(self.slope), cv(self.x))


def hotstart(net: Network, q0: np.ndarray, bd: Bounds, dtype=np.float32):
    """``compute_hotstart_discharge`` (mmc.py:25-66): clamp((I - N)^{-1} q'[0], q_lb)."""
    x = net.lower_solve(np.ones(net.n), np.asarray(q0, dtype=dtype)).astype(dtype)
    return np.maximum(x, dtype(bd.discharge))


def route(net: Network, r: Reaches, qprime: np.ndarray, bd: Bounds = Bounds(), dt=3600.0,
          q0: np.ndarray | None = None, dtype=np.float32, outflow_idx=None):
    """``MuskingumCunge.forward`` (mmc.py:365-443) with ``route_timestep`` (487-559).

    Returns dict(runoff (N,T) or (G,T), x (T,N) unclamped solve result (x[0]: the hot start's
    unclamped solve, or the carried Q0),
    q_last, top_width, side_slope).
    """
    f = dtype
    r = r.astype(f)
    qprime = np.asarray(qprime, dtype=f)
    T, N = qprime.shape
    qlb = f(bd.discharge)
    xs = np.zeros((T, N), dtype=f)
    if q0 is None:
        # the hot start's unclamped solve (its clamp's backward masks where it is below q_lb)
        xs[0] = net.lower_solve(np.ones(N), np.asarray(qprime[0], dtype=f)).astype(f)
        Q = np.maximum(xs[0], qlb)
    else:
        Q = np.asarray(q0, dtype=f).copy()
        xs[0] = Q
    tw = ss = np.zeros(0, dtype=f)
    for t in range(1, T):
        qc = np.maximum(qprime[t - 1], qlb)
        c, tw, ss = trapezoid_celerity(Q, r.n, r.q, r.p, r.slope, bd, f)
        c1, c2, c3, c4 = muskingum_coefficients(r.length, c, r.x, dt, f)
        I = net.spmv(Q)
        b = ((c2 * I) + (c3 * Q)) + (c4 * qc)
        x = net.lower_solve(c1, b).astype(f)
        xs[t] = x
        Q = np.maximum(x, qlb)
    Qall = np.maximum(xs, qlb)
    runoff = Qall.T.copy()
    if outflow_idx is not None and len(outflow_idx) != N:
        runoff = gauge_reduce(Qall, outflow_idx).T.copy()
    return dict(runoff=runoff, x=xs, q_last=Q, top_width=tw, side_slope=ss)


def gauge_reduce(Qall: np.ndarray, outflow_idx) -> np.ndarray:
    """out[g, t] = sum_{j in outflow_idx[g]} Q_t[j] (mmc.py:405-411, 433-439); (T, G)."""
    T, N = Qall.shape
    out = np.zeros((T, len(outflow_idx)), dtype=Qall.dtype)
    for g, idx in enumerate(outflow_idx):
        idx = np.asarray(idx, dtype=np.int64) % N  # Python-style negative indices
        acc = np.zeros(T, dtype=Qall.dtype)
        for j in idx:
            acc = acc + Qall[:, j]
        out[:, g] = acc
    return out


def area_downsample(x: np.ndarray, days: int) -> np.ndarray:
    """``functions.py:7-23`` ``F.interpolate(x.unsqueeze(1), size=(days,), mode="area")`` restated:
    adaptive average pooling, day d averages [floor(d L / D), ceil((d + 1) L / D)) -- summed in order,
    then divided by the window length (x: (G, L))."""
    G, L = x.shape
    out = np.zeros((G, days), dtype=x.dtype)
    for d in range(days):
        a, b = (d * L) // days, ((d + 1) * L + days - 1) // days
        acc = np.zeros(G, dtype=x.dtype)
        for h in range(a, b):
            acc = acc + x[:, h]
        out[:, d] = acc / x.dtype.type(b - a)
    return out


def daily_l1_objective(gauge_runoff: np.ndarray, obs: np.ndarray, tau: int = 3, warmup: int = 3):
    """``scripts/train.py:78-97``: trim [13 : -11 + tau], pool to len // 24 days, drop gauges whose
    observations have a NaN, L1 against obs (already cut to the routed days), skipping ``warmup``
    days.  Returns (loss, daily (G, D), dloss/d(gauge_runoff) (G, T)) -- the last by the chain rule of
    the mean absolute error through the pooling, fp64."""
    G, T = gauge_runoff.shape
    trimmed = gauge_runoff[:, 13:(-11 + tau) if (-11 + tau) < 0 else (-11 + tau)]
    L = trimmed.shape[1]
    D = L // 24
    daily = area_downsample(trimmed, D)
    keep = ~np.isnan(obs).any(axis=1)
    pred = daily[keep][:, warmup:].astype(np.float64)
    target = obs[keep][:, warmup:].astype(np.float64)
    diff = pred - target
    loss = float(np.abs(diff).mean())
    gd = np.zeros((G, D), dtype=np.float64)
    gd[np.flatnonzero(keep)[:, None], np.arange(warmup, D)[None, :]] = np.sign(diff) / diff.size
    gh = np.zeros((G, T), dtype=np.float64)
    for d in range(D):
        a, b = (d * L) // D, ((d + 1) * L + D - 1) // D
        gh[:, 13 + a:13 + b] += gd[:, d:d + 1] / (b - a)
    return loss, daily, gh


def accumulate_daily(net: Network, q_daily: np.ndarray, bd: Bounds = Bounds()) -> np.ndarray:
    """``scripts/geometry_predictor.py:193-212``: per day d, Q_d = compute_hotstart_discharge(
    max(q'_d, q_lb)) = max((I - N)^{-1} max(q'_d, q_lb), q_lb) -- (n_days, N) float32."""
    f = np.float32
    out = np.zeros(q_daily.shape, dtype=f)
    for d in range(q_daily.shape[0]):
        out[d] = hotstart(net, np.maximum(np.asarray(q_daily[d], f), f(bd.discharge)), bd, f)
    return out


def geometry_statistics(n, p, q, slope, daily_q: np.ndarray, bd: Bounds = Bounds()) -> dict:
    """``src/ddr/geometry/statistics.py:20-83``: per-day trapezoid geometry (trapezoidal.py:62-97, fp32
    reference order, correctly rounded pow) and per-reach nanmin / nanmax / nanmedian / nanmean over
    the days, for depth, top_width, bottom_width, side_slope, hydraulic_radius and discharge."""
    f = np.float32
    D, N = daily_q.shape
    geo = {k: np.empty((D, N), dtype=f) for k in ("depth", "top_width", "bottom_width", "side_slope",
                                                    "hydraulic_radius")}
    for d in range(D):
        g = trapezoid_celerity(np.asarray(daily_q[d], f), np.asarray(n, f), np.asarray(q, f), np.asarray(p, f),
                               np.asarray(slope, f), bd, f, full=True)
        geo["depth"][d], geo["top_width"][d], geo["bottom_width"][d] = g["depth"], g["tw"], g["bw"]
        geo["side_slope"][d], geo["hydraulic_radius"][d] = g["ss"], g["R"]
    out = {}
    with np.errstate(all="ignore"):
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            for name, arr in [*geo.items(), ("discharge", np.asarray(daily_q, f))]:
                out[f"{name}_min"] = np.nanmin(arr, axis=0).astype(f)
                out[f"{name}_max"] = np.nanmax(arr, axis=0).astype(f)
                out[f"{name}_median"] = np.nanmedian(arr, axis=0).astype(f)
                out[f"{name}_mean"] = np.nanmean(arr, axis=0).astype(f)
    return out


# ---------------------------------------------------------------------------------------------
# Adjoint (hand derived) -- fp64
# ---------------------------------------------------------------------------------------------


def _celerity_vjp(Q, n, q, p, slope, bd: Bounds, g_c):
    """VJP of c = trapezoid_celerity(Q, n, q, p, S) -> (gQ, gn, gq, gp); fp64.

    Clamp gradients are inclusive at the bounds (torch.clamp backward passes grad where
    lo <= x <= hi), matching the reference's autograd.
    """
    d = trapezoid_celerity(Q, n, q, p, slope, bd, np.float64, full=True)
    sS = np.sqrt(slope)
    g_vc = g_c * 5.0 / 3.0
    g_v = g_vc * ((d["v"] >= bd.velocity) & (d["v"] <= bd.velocity_max))
    inv_n = 1.0 / n
    # v = inv_n * R^(2/3) * sS
    g_R = g_v * inv_n * sS * (2.0 / 3.0) * np.power(d["R"], -1.0 / 3.0)
    g_n = g_v * d["r23"] * sS * (-inv_n * inv_n)
    # R = area / wp
    g_area = g_R / d["wp"]
    g_wp = -g_R * d["area"] / (d["wp"] * d["wp"])
    # wp = bw + 2 depth sq ; sq = sqrt(1 + ss^2)
    g_bw = g_wp.copy()
    g_depth = g_wp * 2.0 * d["sq"]
    g_ss = g_wp * 2.0 * d["depth"] * d["ss"] / d["sq"]
    # area = (tw + bw) depth / 2
    g_tw = g_area * d["depth"] / 2.0
    g_bw = g_bw + g_area * d["depth"] / 2.0
    g_depth = g_depth + g_area * (d["tw"] + d["bw"]) / 2.0
    # bw = max(tw - 2 ss depth, bw_lb)
    g_bwr = g_bw * (d["bw_raw"] >= bd.bottom_width)
    g_tw = g_tw + g_bwr
    g_ss = g_ss - 2.0 * d["depth"] * g_bwr
    g_depth = g_depth - 2.0 * d["ss"] * g_bwr
    # ss = clamp(tw qe / (2 depth), 0.5, 50)
    g_ssr = g_ss * ((d["ss_raw"] >= bd.side_slope_min) & (d["ss_raw"] <= bd.side_slope_max))
    qe = d["qe"]
    g_tw = g_tw + g_ssr * qe / (2.0 * d["depth"])
    g_qe = g_ssr * d["tw"] / (2.0 * d["depth"])
    g_depth = g_depth - g_ssr * d["ss_raw"] / d["depth"]
    # tw = p depth^qe
    dq = np.power(d["depth"], qe)
    g_p = g_tw * dq
    g_depth = g_depth + g_tw * p * qe * np.power(d["depth"], qe - 1.0)
    g_qe = g_qe + g_tw * p * dq * np.log(d["depth"])
    # depth = max(pw, d_lb)
    g_pw = g_depth * (d["pw"] >= bd.depth)
    # pw = ratio^e
    e = d["expo"]
    g_ratio = g_pw * e * np.power(d["ratio"], e - 1.0)
    g_e = g_pw * d["pw"] * np.log(d["ratio"])
    # e = 3 / (5 + 3 qe)
    g_qe = g_qe + g_e * (-9.0) / ((5.0 + 3.0 * qe) ** 2)
    # ratio = num / (p sS + 1e-8)
    dd = d["den"] + 1e-8
    g_num = g_ratio / dd
    g_p = g_p - g_ratio * d["num"] / (dd * dd) * sS
    # num = Q n (qe + 1)
    g_Q = g_num * n * (qe + 1.0)
    g_n = g_n + g_num * Q * (qe + 1.0)
    g_qe = g_qe + g_num * Q * n
    return g_Q, g_n, g_qe, g_p


def geometry_vjp(Q, n, q, p, slope, bd: Bounds, g_tw, g_ss):
    """VJP of the reported geometry (trapezoidal.py:62-79 -> mmc.py:161-162: top_width = p depth^qe,
    side_slope = clamp(top_width qe / (2 depth), 0.5, 50)) w.r.t. (Q, n, q_spatial, p_spatial), fp64; torch's
    clamp backward is inclusive at both bounds.  g_tw / g_ss may be None."""
    f = np.float64
    Q, n, q, p, S = (np.asarray(a, f) for a in (Q, n, q, p, slope))
    p = np.broadcast_to(p, Q.shape)
    g_tw = np.zeros_like(Q) if g_tw is None else np.asarray(g_tw, f)
    g_ss = np.zeros_like(Q) if g_ss is None else np.asarray(g_ss, f)
    qe = q + 1e-6
    num = Q * n * (qe + 1.0)
    den = p * np.sqrt(S) + 1e-8
    base = num / den
    e = 3.0 / (5.0 + 3.0 * qe)
    d0 = base ** e
    depth = np.maximum(d0, bd.depth)
    tw = p * depth ** qe
    ss_raw = tw * qe / (2.0 * depth)
    m_ss = (ss_raw >= 0.5) & (ss_raw <= 50.0)
    gs = g_ss * m_ss
    g_twt = g_tw + gs * qe / (2.0 * depth)
    g_depth = g_twt * p * qe * depth ** (qe - 1.0) - gs * tw * qe / (2.0 * depth * depth)
    g_p = g_twt * depth ** qe
    g_qe = g_twt * tw * np.log(depth) + gs * tw / (2.0 * depth)
    g_d0 = g_depth * (d0 >= bd.depth)
    g_base = g_d0 * e * d0 / base
    g_qe = g_qe + g_d0 * d0 * np.log(base) * (-9.0 / (5.0 + 3.0 * qe) ** 2)
    g_num = g_base / den
    g_p = g_p - g_base * num / (den * den) * np.sqrt(S)
    g_Q = g_num * n * (qe + 1.0)
    g_n = g_num * Q * (qe + 1.0)
    g_qe = g_qe + g_num * Q * n
    return g_Q, g_n, g_qe, g_p


def route_backward(net: Network, r: Reaches, qprime: np.ndarray, xs: np.ndarray, grad_runoff: np.ndarray,
                   bd: Bounds = Bounds(), dt=3600.0, outflow_idx=None, want_qprime=False, carry=False,
                   state_seed=None):
    """Adjoint of ``route`` w.r.t. (n, q_spatial, p_spatial) (and optionally q' and the state), fp64.

    ``xs`` is the (T, N) unclamped solve output of the forward (``xs[0]`` = Q0).
    ``grad_runoff`` is dL/d runoff, (N, T) or (G, T) in gauge mode.
    The hot start has no parameter dependence (mmc.py:337-342) so the parameter sweep stops at t = 1;
    with ``want_qprime`` step 0 adds the hot start's transposed solve (mmc.py:25-66) to dL/dq'[0].
    ``carry``: the forward carried Q0 = ``xs[0]`` (``route(q0=...)``), which step 1 uses unclamped
    (mmc.py:330-342, 487-559); ``q0`` of the result is then dL/dQ0.
    ``state_seed`` (2, N): per-reach dL/dQ_{T-1} (the final ``_discharge_t``, mmc.py:441) and dL/dQ_{T-2} (the
    state of the reported geometry, mmc.py:161-162; ``geometry_vjp``), added to those steps' dL/dQ.
    """
    f = np.float64
    r = r.astype(f)
    xs = np.asarray(xs, dtype=f)
    qprime = np.asarray(qprime, dtype=f)
    T, N = xs.shape
    qlb = bd.discharge
    G = np.asarray(grad_runoff, dtype=f)
    gauge = outflow_idx is not None and len(outflow_idx) != N
    Qall = np.maximum(xs, qlb)
    Q0 = xs[0] if carry else Qall[0]  # the state step 1 reads
    if gauge:
        g_all = np.zeros((T, N))
        for g, idx in enumerate(outflow_idx):
            idx = np.asarray(idx, dtype=np.int64) % N
            # output[:, 0] = clamp(sum of the gauge's initial states) (mmc.py:398-412)
            m0 = float(np.sum(Q0[idx], dtype=np.float64) >= qlb)
            for j in idx:
                g_all[:, j] += G[g]
                g_all[0, j] += G[g, 0] * (m0 - 1.0)
    else:
        g_all = G.T.copy()
    if state_seed is not None:
        sd = np.asarray(state_seed, dtype=f)
        g_all[T - 1] += sd[0]
        if T >= 2:
            g_all[T - 2] += sd[1]
    lam = np.zeros(N)
    gn = np.zeros(N)
    gq = np.zeros(N)
    gp = np.zeros(N)
    gqp = np.zeros((T, N)) if want_qprime else None
    p_full = np.broadcast_to(r.p, (N,)).astype(f)
    for t in range(T - 1, 0, -1):
        lam = lam + g_all[t]
        gx = lam * (xs[t] >= qlb)
        Qp = Qall[t - 1]
        if t == 1:
            Qp = Q0
        c, _, _ = trapezoid_celerity(Qp, r.n, r.q, p_full, r.slope, bd, f)
        c1, c2, c3, c4 = muskingum_coefficients(r.length, c, r.x, dt, f)
        gb = net.upper_solve(c1, gx)
        qc = np.maximum(qprime[t - 1], qlb)
        Sx = net.spmv(xs[t])
        I = net.spmv(Qp)
        gc1 = gb * Sx
        gc2 = gb * I
        gc3 = gb * Qp
        gc4 = gb * qc
        # coefficients -> k -> c
        X = r.x
        two_k = 2.0 * (r.length / c)
        den = two_k * (1.0 - X) + dt
        g_twok = (gc1 * (-X - c1 * (1.0 - X)) + gc2 * (X - c2 * (1.0 - X))
                  + gc3 * (1.0 - X) * (1.0 - c3) - gc4 * c4 * (1.0 - X)) / den
        g_k = 2.0 * g_twok
        g_c = -g_k * (r.length / c) / c
        gQc, gn_t, gq_t, gp_t = _celerity_vjp(Qp, r.n, r.q, p_full, r.slope, bd, g_c)
        gn += gn_t
        gq += gq_t
        gp += gp_t
        up_push = np.zeros(N)
        has_down = net.down >= 0
        dn = net.down[has_down]
        up_push[has_down] = gb[dn] * c2[dn]
        if want_qprime:
            gqp[t - 1] += gb * c4 * (qprime[t - 1] >= qlb)
        lam = up_push + gb * c3 + gQc
    g0 = None
    if carry:
        # runoff[:, 0] = clamp(Q0) per reach (the gauge sums' clamp is already in g_all[0])
        g0 = lam + g_all[0] * (1.0 if gauge else (xs[0] >= qlb))
    lam = lam + g_all[0]
    if want_qprime and not carry:
        # hot start: Q0 = clamp(solve(I - N, q'[0]))
        gx0 = lam * (xs[0] >= qlb)
        gqp[0] += net.upper_solve(np.ones(N), gx0)
    p_is_scalar = np.ndim(r.p) == 0
    return dict(n=gn, q_spatial=gq, p_spatial=(gp.sum() if p_is_scalar else gp), qprime=gqp, lam0=lam, q0=g0)


def param_grads_from_unit(gn, gq, gp, u_n, u_q, u_p, ranges, log_space=("p_spatial",)):
    """Chain the denormalize VJP (utils.py:166-185) onto physical-parameter gradients."""
    out = {}
    for name, g, u in (("n", gn, u_n), ("q_spatial", gq, u_q), ("p_spatial", gp, u_p)):
        if u is None:
            continue
        lo, hi = ranges[name]
        if name in log_space:
            llo, lhi = np.log(lo + 1e-6), np.log(hi)
            val = np.exp(np.asarray(u, np.float64) * (lhi - llo) + llo)
            out[name] = g * val * (lhi - llo)
        else:
            out[name] = g * (hi - lo)
    return out
