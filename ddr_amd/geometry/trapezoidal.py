"""Drop-in for ``ddr.geometry.trapezoidal`` (reference ``src/ddr/geometry/trapezoidal.py:14-108``).

Stand-alone trapezoid geometry for the callers outside the routing loop (BMI output cache, the
geometry predictor).  Inside the fused routing kernels the same expressions are evaluated per reach
and step in registers (``ddr_amd/csrc/physics.h``); this PyTorch version keeps the reference
operation order so both agree bit-for-bit where PyTorch's ``pow`` is correctly rounded.
"""

from __future__ import annotations

import torch


def compute_trapezoidal_geometry(n: torch.Tensor, p_spatial: torch.Tensor, q_spatial: torch.Tensor,
                                 discharge: torch.Tensor, slope: torch.Tensor, depth_lb: float = 0.01,
                                 bottom_width_lb: float = 0.01, side_slope_lb: float = 0.5,
                                 side_slope_ub: float = 50.0) -> dict[str, torch.Tensor]:
    """Invert Manning for depth under the Leopold & Maddock power law, then derive the trapezoid.

    ``side_slope_lb`` / ``side_slope_ub`` default to the reference's fixed clamp (trapezoidal.py:79); the routing
    kernels take them from ``RouteConsts``, and the geometry VJP (``ops._geometry_vjp``) passes those."""
    qe = q_spatial + 1e-6
    numerator = discharge * n * (qe + 1)
    denominator = p_spatial * torch.pow(slope, 0.5)
    expo = torch.div(3.0, 5.0 + 3.0 * qe)
    depth = torch.clamp(torch.pow(torch.div(numerator, denominator + 1e-8), expo), min=depth_lb)
    top_width = p_spatial * torch.pow(depth, qe)
    side_slope = torch.clamp(top_width * qe / (2 * depth), min=side_slope_lb, max=side_slope_ub)
    bottom_width = torch.clamp(top_width - (2 * side_slope * depth), min=bottom_width_lb)
    area = (top_width + bottom_width) * depth / 2
    wetted_perimeter = bottom_width + 2 * depth * torch.sqrt(1 + side_slope**2)
    hydraulic_radius = area / wetted_perimeter
    velocity = torch.div(1, n) * torch.pow(hydraulic_radius, (2 / 3)) * torch.pow(slope, (1 / 2))
    return {"depth": depth, "top_width": top_width, "bottom_width": bottom_width, "side_slope": side_slope,
            "cross_sectional_area": area, "wetted_perimeter": wetted_perimeter,
            "hydraulic_radius": hydraulic_radius, "velocity": velocity}
