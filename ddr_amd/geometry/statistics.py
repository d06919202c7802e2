"""Drop-in for ``ddr.geometry.statistics`` (reference ``src/ddr/geometry/statistics.py:20-83``) on the
HIP geometry-statistics kernel (``csrc/geometry.hip``), plus the fused C4 pipeline of
``scripts/geometry_predictor.py:176-212``: per-day discharge accumulation for every day of a water
year in ONE routing launch (``DDR_FWD_ACCUMULATE``: each step a hot start, ``mmc.py:25-66``), then
per-reach min / max / median / mean of the trapezoid geometry over the days, without the
(days, N) discharge ever leaving the device.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .. import _lib

GEOMETRY_VARS = ("depth", "top_width", "bottom_width", "side_slope", "hydraulic_radius", "discharge")
STATS = ("min", "max", "median", "mean")


def _stats_device(qd: torch.Tensor, reach_stride: int, day_stride: int, n_reach: int, n_days: int, n, p, q, slope,
                  depth_lb: float, bw_lb: float) -> torch.Tensor:
    dev = qd.device
    f = lambda t: torch.as_tensor(t, dtype=torch.float32).to(dev).reshape(-1).contiguous()  # noqa: E731
    n, p, q, slope = f(n), f(p), f(q), f(slope)
    for name, t in (("n", n), ("q_spatial", q), ("slope", slope)):
        if t.numel() != n_reach:
            raise ValueError(f"{name} has {t.numel()} elements, expected {n_reach}")
    if p.numel() not in (1, n_reach):
        raise ValueError(f"p_spatial has {p.numel()} elements, expected 1 or {n_reach}")
    out = torch.empty((len(GEOMETRY_VARS) * len(STATS), n_reach), device=dev, dtype=torch.float32)
    _lib.check(_lib.load().ddr_geometry_stats_f32(
        qd.data_ptr(), int(reach_stride), int(day_stride), int(n_reach), int(n_days), n.data_ptr(), p.data_ptr(),
        1 if p.numel() > 1 else 0, q.data_ptr(), slope.data_ptr(), C.c_double(depth_lb), C.c_double(bw_lb),
        out.data_ptr(), _lib.stream_ptr(dev)))
    return out


def _as_dict(out: torch.Tensor) -> dict[str, np.ndarray]:
    host = out.cpu().numpy()
    return {f"{v}_{s}": host[i * len(STATS) + j] for i, v in enumerate(GEOMETRY_VARS) for j, s in enumerate(STATS)}


def compute_geometry_statistics(n: torch.Tensor, p_spatial: torch.Tensor, q_spatial: torch.Tensor, slope: torch.Tensor,
                                daily_accumulated_discharge, attribute_minimums: dict[str, float] | None = None,
                                device=None) -> dict[str, np.ndarray]:
    """Per-reach temporal statistics (``statistics.py:20-83``): keys ``{var}_{min,max,median,mean}`` for
    depth, top_width, bottom_width, side_slope, hydraulic_radius and discharge, each (N,) float32.

    ``daily_accumulated_discharge`` is (n_days, N) (numpy or tensor), up to 32768 days (~89 years) per
    call: windows beyond 512 days sort each reach's values in LDS (one workgroup per reach).
    Runs on the HIP device (``device``, default the current one); no CPU fallback."""
    if not torch.cuda.is_available():
        raise RuntimeError("compute_geometry_statistics runs on the HIP device only (no CPU fallback)")
    mins = attribute_minimums or {}
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    qd = torch.as_tensor(np.asarray(daily_accumulated_discharge) if not torch.is_tensor(daily_accumulated_discharge)
                         else daily_accumulated_discharge, dtype=torch.float32).to(dev).contiguous()
    if qd.dim() != 2:
        raise ValueError("daily_accumulated_discharge must be (n_days, N)")
    n_days, n_reach = qd.shape
    out = _stats_device(qd, 1, n_reach, n_reach, n_days, n, p_spatial, q_spatial, slope, mins.get("depth", 0.01),
                        mins.get("bottom_width", 0.01))
    return _as_dict(out)


def daily_accumulated_discharge(graph, q_prime_daily: torch.Tensor, discharge_lb: float = 1e-4) -> torch.Tensor:
    """``geometry_predictor.py:193-212`` for all days at once: Q_d = max((I - N)^-1 max(q'_d, q_lb), q_lb),
    returned reach-major (N, n_days).  ``q_prime_daily`` is (n_days, N): q' at the first hour of
    each day."""
    from ..ops import RouteConsts, route

    qd = torch.clamp(q_prime_daily.to(torch.float32), min=discharge_lb).contiguous()
    N = qd.shape[1]
    one = torch.ones(N, device=qd.device, dtype=torch.float32)
    with torch.no_grad():
        acc, _, _, _ = route(graph, qd, one, one, one, one, one, one, consts=RouteConsts(discharge_lb=discharge_lb),
                             save=False, accumulate=True)
    return acc


def geometry_statistics_from_inflow(graph, q_prime_daily: torch.Tensor, n, p_spatial, q_spatial, slope,
                                    attribute_minimums: dict[str, float] | None = None) -> dict[str, np.ndarray]:
    """The fused C4 geometry pipeline: daily accumulation (one routing launch) + statistics kernel."""
    mins = attribute_minimums or {}
    acc = daily_accumulated_discharge(graph, q_prime_daily, mins.get("discharge", 1e-4))
    N, D = acc.shape
    out = _stats_device(acc, D, 1, N, D, n, p_spatial, q_spatial, slope, mins.get("depth", 0.01),
                        mins.get("bottom_width", 0.01))
    return _as_dict(out)
