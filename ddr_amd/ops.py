"""PyTorch custom ops over the HIP routing library (``torch.library`` ``ddrx::*``).

``ddrx::mc_route``          fused forward over all T steps     (mmc.py:365-443 + 487-559)
``ddrx::mc_route_backward`` reverse-time adjoint               (autograd of the above)

``mc_route`` is registered with ``register_autograd`` so the denormalised parameters
(``n``, ``q_spatial``, ``p_spatial``) receive gradients exactly where the reference's autograd
delivers them; everything upstream (``denormalize``, the KAN) stays PyTorch.

The op takes the graph as an integer id into a registry of live :class:`RiverGraph` objects, raw
device pointers go to the C ABI, and all work is enqueued on ``torch.cuda.current_stream()``.
"""

from __future__ import annotations

import ctypes as C
import os
import weakref
from dataclasses import dataclass

import torch

from . import _lib
from .graph import RiverGraph

_GRAPHS: "weakref.WeakValueDictionary[int, RiverGraph]" = weakref.WeakValueDictionary()
_CHECK_STATUS = os.environ.get("DDR_CHECK_STATUS", "0") == "1"


def register_graph(g: RiverGraph) -> int:
    gid = id(g)
    _GRAPHS[gid] = g
    return gid


def _graph(gid: int) -> RiverGraph:
    g = _GRAPHS.get(gid)
    if g is None:
        raise RuntimeError("routing graph was garbage-collected before use")
    return g


@dataclass(frozen=True)
class RouteConsts:
    """Physical constants (mmc.py:192-208; trapezoidal.py:79; mmc.py:166)."""

    dt: float = 3600.0
    discharge_lb: float = 1e-4
    velocity_lb: float = 0.01
    velocity_ub: float = 15.0
    depth_lb: float = 0.01
    bottom_width_lb: float = 0.01
    side_slope_lb: float = 0.5
    side_slope_ub: float = 50.0

    def as_list(self) -> list[float]:
        return [self.dt, self.discharge_lb, self.velocity_lb, self.velocity_ub, self.depth_lb, self.bottom_width_lb,
                self.side_slope_lb, self.side_slope_ub]


def _consts(c: list[float]) -> _lib.Consts:
    return _lib.Consts(*[float(v) for v in c])


def _reaches(n, q, p, length, slope, x_storage, flow_scale, qp_hours: int = 1, qp_valid=None) -> _lib.Reaches:
    return _lib.Reaches(n.data_ptr(), q.data_ptr(), p.data_ptr(), 1 if p.numel() > 1 else 0, length.data_ptr(),
                        slope.data_ptr(), x_storage.data_ptr(), flow_scale.data_ptr() if flow_scale is not None else None,
                        int(qp_hours), qp_valid.data_ptr() if qp_valid is not None else None)


def _gauges(G, g_off, g_idx, r_off, r_g) -> _lib.Gauges | None:
    if g_off is None:
        return None
    return _lib.Gauges(G, g_off.data_ptr(), g_idx.data_ptr(), r_off.data_ptr() if r_off is not None else None,
                       r_g.data_ptr() if r_g is not None else None)


def _check_inputs(qprime, tensors, p=None):
    """dtype/device/contiguity, and per-reach lengths: the kernels index every per-reach array by
    reach id, so a short one would be read out of bounds instead of raising (the reference's
    broadcasting raises a shape error)."""
    if qprime.dim() != 2:
        raise ValueError("streamflow must be (T, N)")
    if not qprime.is_cuda:
        raise RuntimeError("ddrx::mc_route runs on the HIP device only (no CPU fallback); move inputs to cuda")
    dt = qprime.dtype
    if dt not in (torch.float32, torch.float64):
        raise TypeError("routing supports float32 and float64")
    N = qprime.shape[1]
    for name, t in tensors:
        if t is None:
            continue
        if t.dtype != dt or t.device != qprime.device or not t.is_contiguous():
            raise ValueError("all routing inputs must share dtype/device and be contiguous")
        if t.numel() != N:
            raise ValueError(f"{name} has {t.numel()} elements, the network has {N} reaches")
    if p is not None and p.numel() not in (1, N):
        raise ValueError(f"p_spatial has {p.numel()} elements: expected 1 or {N}")


def qprime_has_nan() -> bool:
    """Whether the calling thread's last ``route(..., check_qprime=True)`` saw a NaN in its q' (waits for
    that launch's q' gather, not for its routing kernel)."""
    v = C.c_int32()
    _lib.check(_lib.load().ddr_qprime_nan_wait(C.byref(v)))
    return bool(v.value)


def check_status(wait: bool = True) -> None:
    """Raise ``DDRError(DDR_ERR_TIMEOUT)`` if an earlier routing launch had a timed-out
    inter-workgroup hand-off (its outputs hold NaN).  Without ``wait`` only launches that have
    already completed are inspected; every routing call does that implicitly."""
    _lib.check(_lib.load().ddr_status_check(1 if wait else 0))


@torch.library.custom_op("ddrx::mc_route", mutates_args=())
def mc_route(qprime: torch.Tensor, n: torch.Tensor, q: torch.Tensor, p: torch.Tensor, length: torch.Tensor,
             slope: torch.Tensor, x_storage: torch.Tensor, flow_scale: torch.Tensor | None, q0: torch.Tensor | None,
             g_off: torch.Tensor | None, g_idx: torch.Tensor | None, r_off: torch.Tensor | None,
             r_g: torch.Tensor | None, qp_valid: torch.Tensor | None, graph_id: int, consts: list[float], flags: int,
             steps: int, qp_hours: int, daily: list[int]
             ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """Returns (runoff, q_last, top_width_last, side_slope_last, x_save, bnd).

    ``steps`` = T routing steps; ``qprime`` is (T, N), or (ceil(T / 24), N) daily rows with
    ``qp_hours`` = 24.  Gauge mode (``g_off``/``g_idx``): runoff is (G, T), or with ``daily`` =
    [t0, L, D] the fused daily objective series (G, D).  ``r_off``/``r_g`` (reach -> gauge map) are
    only consumed by the backward."""
    _check_inputs(qprime, (("n", n), ("q_spatial", q), ("length", length), ("slope", slope),
                           ("x_storage", x_storage), ("flow_scale", flow_scale), ("q0", q0)), p)
    if p.dtype != qprime.dtype or p.device != qprime.device or not p.is_contiguous():
        raise ValueError("all routing inputs must share dtype/device and be contiguous")
    g = _graph(graph_id)
    T, N = int(steps), qprime.shape[1]
    rows = -(-T // max(1, qp_hours))
    if qprime.shape[0] < rows:
        # a daily store may hold more rows than the window routes (the reader keeps the first
        # (rho - 1) * 24 hours of rho days, readers.py:513-519)
        raise ValueError(f"streamflow has {qprime.shape[0]} rows, {T} steps at {qp_hours} h per row need {rows}")
    if N != g.n:
        raise ValueError(f"streamflow has {N} reaches, network has {g.n}")
    if qp_valid is not None and (qp_valid.dtype != torch.uint8 or qp_valid.numel() != N):
        raise ValueError("qprime_valid must be a uint8 mask of N reaches")
    dev, dt = qprime.device, qprime.dtype
    gauge = g_off is not None
    if daily and not gauge:
        raise ValueError("the fused daily objective needs gauge mode (outflow_idx)")
    G = g_off.numel() - 1 if gauge else N
    save = bool(flags & _lib.DDR_FWD_SAVE_X) or gauge
    fflags = flags | (_lib.DDR_FWD_SAVE_X if save else 0) | (_lib.DDR_FWD_NO_RUNOFF if gauge else 0)
    runoff = torch.empty((G, daily[2] if daily else T), device=dev, dtype=dt)
    x_save = torch.empty(g.save_numel(T), device=dev, dtype=dt)  # always written (runoff is staged here)
    bnd = torch.empty(g.bnd_numel(T), device=dev, dtype=torch.float64)
    status = torch.empty(g.info.status_bytes, device=dev, dtype=torch.uint8)
    q_last = torch.empty(N, device=dev, dtype=dt)
    tw = torch.zeros(N, device=dev, dtype=dt)
    ss = torch.zeros(N, device=dev, dtype=dt)
    lib = _lib.load()
    f32 = dt == torch.float32
    fwd = lib.ddr_mc_forward_f32 if f32 else lib.ddr_mc_forward_f64
    stream = _lib.stream_ptr(dev)
    r = _reaches(n, q, p, length, slope, x_storage, flow_scale, qp_hours, qp_valid)
    c = _consts(consts)
    _lib.check(fwd(g.handle, C.byref(c), C.byref(r), qprime.data_ptr(), T, _lib.ptr(q0), runoff.data_ptr(),
                   x_save.data_ptr(), bnd.data_ptr() if bnd.numel() else None, status.data_ptr(),
                   q_last.data_ptr(), tw.data_ptr(), ss.data_ptr(), int(fflags), stream))
    if gauge:
        gz = _gauges(G, g_off, g_idx, None, None)
        if daily:
            red = lib.ddr_gauge_daily_f32 if f32 else lib.ddr_gauge_daily_f64
            _lib.check(red(g.handle, x_save.data_ptr(), T, C.byref(gz), float(consts[1]), int(fflags), int(daily[0]),
                           int(daily[1]), int(daily[2]), runoff.data_ptr(), stream))
        else:
            red = lib.ddr_gauge_reduce_f32 if f32 else lib.ddr_gauge_reduce_f64
            _lib.check(red(g.handle, x_save.data_ptr(), T, C.byref(gz), float(consts[1]), int(fflags),
                           runoff.data_ptr(), stream))
    if _CHECK_STATUS:
        _lib.check(lib.ddr_status_check(1))
    return runoff, q_last, tw, ss, x_save, bnd


@mc_route.register_fake
def _(qprime, n, q, p, length, slope, x_storage, flow_scale, q0, g_off, g_idx, r_off, r_g, qp_valid, graph_id, consts,
      flags, steps, qp_hours, daily):
    T, N = int(steps), qprime.shape[1]
    G = g_off.shape[0] - 1 if g_off is not None else N
    g = _graph(graph_id)
    return (qprime.new_empty((G, daily[2] if daily else T)), qprime.new_empty(N), qprime.new_empty(N),
            qprime.new_empty(N), qprime.new_empty(g.save_numel(T)), qprime.new_empty(g.bnd_numel(T), dtype=torch.float64))


@torch.library.custom_op("ddrx::mc_route_backward", mutates_args=())
def mc_route_backward(grad_runoff: torch.Tensor, qprime: torch.Tensor, n: torch.Tensor, q: torch.Tensor,
                      p: torch.Tensor, length: torch.Tensor, slope: torch.Tensor, x_storage: torch.Tensor,
                      flow_scale: torch.Tensor | None, x_save: torch.Tensor, bnd: torch.Tensor,
                      g_off: torch.Tensor | None, g_idx: torch.Tensor | None, r_off: torch.Tensor | None,
                      r_g: torch.Tensor | None, qp_valid: torch.Tensor | None, gseed: torch.Tensor | None,
                      graph_id: int, consts: list[float], flags: int, steps: int, qp_hours: int, daily: list[int],
                      want_qprime: bool, want_q0: bool
                      ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """Returns per-reach (dL/dn, dL/dq_spatial, dL/dp_spatial), dL/dq' (shape of ``qprime``, or empty)
    and dL/dQ0 (N, carried state, or empty).  With ``daily`` the incoming gradient is dL/d(daily
    series) (G, D): its pooling adjoint seeds the gauge-mode routing adjoint.  ``gseed`` (2, N): per-reach
    gradients into the states Q_{T-1} (``_discharge_t``) and Q_{T-2} (the reported geometry's), or None."""
    g = _graph(graph_id)
    T, N = int(steps), qprime.shape[1]
    dev, dt = qprime.device, qprime.dtype
    f32 = dt == torch.float32
    lib = _lib.load()
    stream = _lib.stream_ptr(dev)
    grad_runoff = grad_runoff.to(dtype=dt).contiguous()
    if daily:
        G = grad_runoff.shape[0]
        if grad_runoff.shape[1] != daily[2]:
            raise ValueError("daily-series gradient must be (G, D)")
        hourly = torch.empty((G, T), device=dev, dtype=dt)
        seed = lib.ddr_gauge_daily_seed_f32 if f32 else lib.ddr_gauge_daily_seed_f64
        _lib.check(seed(G, T, int(daily[0]), int(daily[1]), int(daily[2]), grad_runoff.data_ptr(), hourly.data_ptr(),
                        stream))
        grad_runoff = hourly
    if grad_runoff.shape[1] != T:
        raise ValueError("runoff gradient must be (N or G, T)")
    gn = torch.empty(N, device=dev, dtype=dt)
    gq = torch.empty(N, device=dev, dtype=dt)
    gp = torch.empty(N, device=dev, dtype=dt)
    bwd_bnd = torch.empty(g.bwd_numel(T), device=dev, dtype=torch.float64)
    status = torch.empty(g.info.status_bytes, device=dev, dtype=torch.uint8)
    r = _reaches(n, q, p, length, slope, x_storage, flow_scale, qp_hours, qp_valid)
    c = _consts(consts)
    gz = None
    if r_off is not None:
        gz = _lib.Gauges(grad_runoff.shape[0], g_off.data_ptr() if g_off is not None else None,
                         g_idx.data_ptr() if g_idx is not None else None, r_off.data_ptr(), r_g.data_ptr())
    want_q0 = want_q0 and bool(flags & _lib.DDR_FWD_CARRY)
    gqp = torch.empty(qprime.shape if want_qprime else (0,), device=dev, dtype=dt)
    gq0 = torch.empty(N if want_q0 else 0, device=dev, dtype=dt)
    if gseed is not None:
        gseed = gseed.to(dtype=dt).contiguous()
        if gseed.shape != (2, N):
            raise ValueError("state seed must be (2, N)")
    if want_qprime or want_q0 or gseed is not None:
        # the general adjoint: state gradients (route_backward_kernel<GS>: also the step-0 sweep and dL/dq')
        # and / or the per-reach state seeds
        work = None
        if want_qprime or want_q0:
            G = grad_runoff.shape[0] if gz is not None else 0
            work = torch.empty(int(lib.ddr_state_work_bytes(g.handle, T, G, 4 if f32 else 8)), device=dev,
                               dtype=torch.uint8)
        bwd = lib.ddr_mc_backward_ex_f32 if f32 else lib.ddr_mc_backward_ex_f64
        _lib.check(bwd(g.handle, C.byref(c), C.byref(r), qprime.data_ptr(), int(qprime.shape[0]), T, x_save.data_ptr(),
                       bnd.data_ptr() if bnd.numel() else None, grad_runoff.data_ptr(),
                       C.byref(gz) if gz is not None else None, _lib.ptr(gseed), bwd_bnd.data_ptr(),
                       status.data_ptr(), gn.data_ptr(), gq.data_ptr(), gp.data_ptr(),
                       gqp.data_ptr() if want_qprime else None, gq0.data_ptr() if want_q0 else None,
                       _lib.ptr(work), int(flags), stream))
    else:
        bwd = lib.ddr_mc_backward_f32 if f32 else lib.ddr_mc_backward_f64
        _lib.check(bwd(g.handle, C.byref(c), C.byref(r), qprime.data_ptr(), T, x_save.data_ptr(),
                       bnd.data_ptr() if bnd.numel() else None, grad_runoff.data_ptr(),
                       C.byref(gz) if gz is not None else None, bwd_bnd.data_ptr(),
                       status.data_ptr(), gn.data_ptr(), gq.data_ptr(), gp.data_ptr(), int(flags), stream))
    if _CHECK_STATUS:
        _lib.check(lib.ddr_status_check(1))
    return gn, gq, gp, gqp, gq0


@mc_route_backward.register_fake
def _(grad_runoff, qprime, n, q, p, length, slope, x_storage, flow_scale, x_save, bnd, g_off, g_idx, r_off, r_g,
      qp_valid, gseed, graph_id, consts, flags, steps, qp_hours, daily, want_qprime, want_q0):
    N = qprime.shape[1]
    want_q0 = want_q0 and bool(flags & _lib.DDR_FWD_CARRY)
    return (qprime.new_empty(N), qprime.new_empty(N), qprime.new_empty(N),
            qprime.new_empty(qprime.shape if want_qprime else (0,)), qprime.new_empty(N if want_q0 else 0))


def _setup_context(ctx, inputs, output):
    (qprime, n, q, p, length, slope, x_storage, flow_scale, q0, g_off, g_idx, r_off, r_g, qp_valid, graph_id, consts,
     flags, steps, qp_hours, daily) = inputs
    runoff, q_last, tw, ss, x_save, bnd = output
    ctx.graph_id = graph_id
    # strong reference: the registry is weak, and the saved x_save / bnd layouts belong to this
    # graph's schedule, so it must outlive the backward (a reused id() would pick another graph)
    ctx.graph = _graph(graph_id)
    ctx.consts = consts
    ctx.flags = flags
    ctx.steps = steps
    ctx.daily = list(daily)
    ctx.gauge = g_off is not None
    ctx.p_scalar = p.numel() == 1
    ctx.p_shape = p.shape
    ctx.qp_hours = qp_hours
    ctx.save_for_backward(qprime, n, q, p, length, slope, x_storage, flow_scale, x_save, bnd, g_off, g_idx, r_off, r_g,
                          qp_valid)
    ctx.set_materialize_grads(False)


def state_at(graph: RiverGraph, x_save: torch.Tensor, steps: int, t: int, discharge_lb: float, flags: int
             ) -> torch.Tensor:
    """Q_t (N, reference order) from a forward's saved states (``ddr_state_f32``): max(x(t), q_lb), the
    carried state at t = 0 unclamped -- the reference's ``_discharge_t`` after step t (mmc.py:441, 557)."""
    out = torch.empty(graph.n, device=x_save.device, dtype=x_save.dtype)
    lib = _lib.load()
    fn = lib.ddr_state_f32 if x_save.dtype == torch.float32 else lib.ddr_state_f64
    _lib.check(fn(graph.handle, x_save.data_ptr(), int(steps), int(t), float(discharge_lb), int(flags), out.data_ptr(),
                  _lib.stream_ptr(x_save.device)))
    return out


def _geometry_vjp(ctx, n, q, p, slope, x_save, g_tw, g_ss):
    """VJP of the reported top width / side slope (mmc.py:161-162): the power-law geometry of the last step,
    computed from Q_{T-2} (trapezoidal.py:62-79), differentiated by PyTorch's autograd like the reference's.
    Returns dL/dQ_{T-2} (the adjoint's second state seed) and the geometry's own (dL/dn, dL/dq, dL/dp)."""
    from .geometry.trapezoidal import compute_trapezoidal_geometry

    T = ctx.steps
    if T < 2 or ctx.flags & _lib.DDR_FWD_ACCUMULATE:
        raise NotImplementedError("this launch reports no geometry (T < 2 or an accumulation launch)")
    # (a carried 2-step window, route_timestep's: Q_{T-2} is the carried state itself, unclamped)
    qprev = state_at(ctx.graph, x_save, T, T - 2, ctx.consts[1], ctx.flags)
    with torch.enable_grad():
        Qv = qprev.detach().requires_grad_(True)
        nv, qv, pv = (t.detach().requires_grad_(True) for t in (n, q, p))
        geo = compute_trapezoidal_geometry(nv, pv, qv, Qv, slope, depth_lb=ctx.consts[4],
                                           bottom_width_lb=ctx.consts[5], side_slope_lb=ctx.consts[6],
                                           side_slope_ub=ctx.consts[7])
        outs, gouts = [], []
        for key, gv in (("top_width", g_tw), ("side_slope", g_ss)):
            if gv is not None:
                outs.append(geo[key].expand_as(gv))
                gouts.append(gv)
        gQ, gn, gq, gp = torch.autograd.grad(outs, (Qv, nv, qv, pv), gouts, allow_unused=True)
    z = lambda g_, like: torch.zeros_like(like) if g_ is None else g_  # noqa: E731
    return z(gQ, Qv), z(gn, n), z(gq, q), z(gp, p)


def _backward(ctx, g_runoff, g_qlast, g_tw, g_ss, g_xsave, g_bnd):
    (qprime, n, q, p, length, slope, x_storage, flow_scale, x_save, bnd, g_off, g_idx, r_off, r_g,
     qp_valid) = ctx.saved_tensors
    T = ctx.steps
    N = qprime.shape[1]
    nz = lambda g_: g_ is not None and bool(g_.ne(0).any())  # noqa: E731
    geo = nz(g_tw) or nz(g_ss)
    # per-reach state seeds (ddr_mc_backward_ex): row 0 dL/dQ_{T-1} = dL/d_discharge_t (an autograd tensor in
    # the reference in gauge mode too, mmc.py:433-441), row 1 dL/dQ_{T-2} from the reported geometry's VJP
    # A carried 2-step window (route_timestep, mmc.py:487-559): Q_{T-2} = Q_0 is the carried state, which the
    # geometry reads unclamped -- its VJP goes straight into dL/dQ0, not through the adjoint's step-0 seed
    # (which is runoff[:, 0]'s clamp)
    geo_q0 = geo and T == 2 and bool(ctx.flags & _lib.DDR_FWD_CARRY)
    gseed = None
    if g_qlast is not None or (geo and not geo_q0):
        gseed = torch.zeros((2, N), device=qprime.device, dtype=qprime.dtype)
        if g_qlast is not None:
            gseed[0] = g_qlast
    extra, gQ_geo = None, None
    if geo:
        gQ, gn2, gq2, gp2 = _geometry_vjp(ctx, n, q, p, slope, x_save, g_tw if nz(g_tw) else None,
                                          g_ss if nz(g_ss) else None)
        if geo_q0:
            gQ_geo = gQ
        else:
            gseed[1] = gQ
        extra = (gn2, gq2, gp2)
    if g_runoff is None:
        G = g_off.numel() - 1 if ctx.gauge else N
        g_runoff = torch.zeros((G, ctx.daily[2] if ctx.daily else T), device=qprime.device, dtype=qprime.dtype)
    # dL/dq' and dL/dQ0 (the carried state) when the caller's graph asks for them: route_timestep is
    # differentiable w.r.t. both in the reference (mmc.py:487-559), the hot start w.r.t. q'[0]
    want_qp = bool(ctx.needs_input_grad[0])
    want_q0 = bool(ctx.needs_input_grad[8])
    gn, gq, gp, gqp, gq0 = mc_route_backward(g_runoff, qprime, n, q, p, length, slope, x_storage, flow_scale, x_save,
                                             bnd, g_off, g_idx, r_off, r_g, qp_valid, gseed, ctx.graph_id, ctx.consts,
                                             ctx.flags, T, ctx.qp_hours, ctx.daily, want_qp, want_q0)
    if ctx.p_scalar:
        gp = gp.sum().reshape(ctx.p_shape)
    if extra is not None:
        gn = gn + extra[0]
        gq = gq + extra[1]
        gp = gp + extra[2].reshape(gp.shape)
    if want_q0 and gQ_geo is not None:
        gq0 = gq0 + gQ_geo
    return ((gqp if want_qp else None), gn, gq, gp) + (None,) * 4 + ((gq0 if want_q0 else None),) + (None,) * 11


mc_route.register_autograd(_backward, setup_context=_setup_context)


# -------------------------------------------------------------------------------------------------
# Convenience wrapper used by the drop-in routing engine
# -------------------------------------------------------------------------------------------------


@dataclass
class GaugeMap:
    """outflow_idx (mmc.py:344-363) as device arrays in both directions."""

    n_gauges: int
    offsets: torch.Tensor
    index: torch.Tensor
    reach_offsets: torch.Tensor
    reach_gauges: torch.Tensor

    @classmethod
    def build(cls, outflow_idx, n_reaches: int, device) -> "GaugeMap":
        import numpy as np

        idx = [np.asarray(i, dtype=np.int64).reshape(-1) for i in outflow_idx]
        flat = np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)
        if flat.size and (flat.max() >= n_reaches or flat.min() < -n_reaches):
            raise AssertionError(f"Output index {flat.max()} out of bounds for discharge tensor of size {n_reaches}.")
        flat = np.where(flat < 0, flat + n_reaches, flat)  # Python-style negative indices
        offs = np.zeros(len(idx) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(i) for i in idx])
        gid = np.repeat(np.arange(len(idx), dtype=np.int64), [len(i) for i in idx])
        order = np.argsort(flat, kind="stable")
        roff = np.zeros(n_reaches + 1, dtype=np.int64)
        np.add.at(roff, flat + 1, 1)
        roff = np.cumsum(roff)
        rg = gid[order]
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        return cls(len(idx), t(offs), t(flat), t(roff), t(rg))


@dataclass(frozen=True)
class DailyWindow:
    """The gauge-mode training objective's window (scripts/train.py:78-82): hours [t0, t0 + L) of the
    hourly series, area-pooled to D days."""

    t0: int
    L: int
    D: int

    @classmethod
    def for_training(cls, T: int, tau: int = 3) -> "DailyWindow":
        """runoff[:, 13 : -11 + tau] pooled to len // 24 days (train.py:78-82; tau default 3,
        configs.py:116-119)."""
        end = T + (-11 + tau) if (-11 + tau) < 0 else min(T, -11 + tau)
        L = end - 13
        if L < 24:
            raise ValueError(f"T = {T} hours leaves no whole day after the [13 : -11 + tau] trim")
        return cls(13, L, L // 24)


def route(graph: RiverGraph, qprime: torch.Tensor, n: torch.Tensor, q: torch.Tensor, p: torch.Tensor,
          length: torch.Tensor, slope: torch.Tensor, x_storage: torch.Tensor, *, flow_scale: torch.Tensor | None = None,
          q0: torch.Tensor | None = None, gauges: GaugeMap | None = None, consts: RouteConsts = RouteConsts(),
          save: bool | None = None, steps: int | None = None, qprime_hours: int = 1,
          qprime_valid: torch.Tensor | None = None, daily: DailyWindow | None = None, accumulate: bool = False,
          fast_math: bool = False, math: str | None = None, check_qprime: bool = False, exact_adjoint: bool = False):
    """Fused differentiable routing.  Returns (runoff, q_last, top_width_last, side_slope_last).

    ``math`` (fp32 forward): ``"exact"`` (default) -- the reference's operation order, IEEE division,
    correctly rounded pow: bit-identical to the oracle; ``"faithful"`` -- the same order and IEEE
    divisions with the pows in fp32 faithful-class arithmetic (the accuracy class of the reference's
    own Sleef ``powf``; no fp64 on the dependency chain); ``"fast"`` (= ``fast_math=True``).

    ``fast_math`` (fp32): the forward's Muskingum coefficients in hardware-approximate fp32 math
    (v_rcp / v_log / v_exp, the adjoint's operation set) instead of the reference's exact operation
    sequence: ~1e-6 relative per coefficient, discharge within the stated 1e-4 of the reference
    (tests/test_gpu_fastmath.py), no longer bit-identical to the oracle.  The backward is the same
    either way.

    ``qprime_hours`` = 24 with ``steps`` = T routes a daily store (ceil(T / 24), N) indexed in-kernel
    (readers.py:513-519); ``qprime_valid`` (N, bool) marks divides present in the store, the others get
    0.001 (readers.py:523-530).  ``daily`` (gauge mode) returns the fused daily objective series
    (G, D).  ``accumulate`` makes every step a hot start (geometry_predictor.py:193-212).

    ``check_qprime``: the q' gather also tests the window's flow-scaled q' for NaN (the reference's
    cold-start assertion, mmc.py:335); :func:`qprime_has_nan` then returns the verdict, waiting for the
    gather only.

    ``exact_adjoint`` (fp32 backward): the gradients are the exact adjoint of the fp32 trajectory the forward
    computed (~1e-7 norm-relative on any depth; the fp32 default is ~1e-3 on a 2215-deep basin, ~1e-7 on
    shallow ones) at ~30 % more backward time (q' re-read, fp64 upstream sums: DDR_BWD_EXACT_ADJOINT).  The
    fp64 model's own gradient differs from both by the fp32 states' rounding (~1e-3 there); route in fp64 for
    that."""
    dt = qprime.dtype
    dev = qprime.device

    def prep(t):
        return None if t is None else t.to(device=dev, dtype=dt).contiguous()

    n, q, p, length, slope, x_storage, flow_scale, q0 = map(prep, (n, q, p, length, slope, x_storage, flow_scale, q0))
    p = p.reshape(-1) if p.numel() > 1 else p.reshape(1)
    if steps is None:
        steps = qprime.shape[0] * max(1, qprime_hours)
    if save is None:
        save = (not accumulate) and torch.is_grad_enabled() and any(
            t is not None and t.requires_grad for t in (n, q, p, qprime, q0))
    math = math or ("fast" if fast_math else "exact")
    if math not in ("exact", "faithful", "fast"):
        raise ValueError(f"math must be 'exact', 'faithful' or 'fast', not {math!r}")
    flags = ((_lib.DDR_FWD_SAVE_X if save else 0) | (_lib.DDR_FWD_CARRY if q0 is not None else 0)
             | (_lib.DDR_FWD_ACCUMULATE if accumulate else 0) | (_lib.DDR_FWD_FAST_MATH if math == "fast" else 0)
             | (_lib.DDR_FWD_FAITHFUL_MATH if math == "faithful" else 0)
             | (_lib.DDR_FWD_CHECK_QPRIME if check_qprime else 0)
             | (_lib.DDR_BWD_EXACT_ADJOINT if exact_adjoint else 0))
    valid = None if qprime_valid is None else qprime_valid.to(device=dev, dtype=torch.uint8).contiguous()
    gid = register_graph(graph)
    gz = gauges
    out = mc_route(qprime.contiguous(), n, q, p, length, slope, x_storage, flow_scale, q0,
                   gz.offsets if gz else None, gz.index if gz else None, gz.reach_offsets if gz else None,
                   gz.reach_gauges if gz else None, valid, gid, consts.as_list(), flags, int(steps), int(qprime_hours),
                   [daily.t0, daily.L, daily.D] if daily is not None else [])
    runoff, q_last, tw, ss, _, _ = out
    return runoff, q_last, tw, ss
