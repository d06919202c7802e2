"""The drop-in trapezoid geometry (ddr_amd.geometry.trapezoidal) against the reference's property tests
(tests/geometry/test_trapezoidal.py:12-148), on the CPU (the drop-in is PyTorch; the kernels evaluate the same
expressions in registers and are checked against the reference goldens in the GPU tests)."""

import numpy as np
import pytest
import torch

from ddr_amd.geometry.trapezoidal import compute_trapezoidal_geometry


def geo(**kw):
    base = dict(n=torch.tensor([0.035]), p_spatial=torch.tensor([21.0]), q_spatial=torch.tensor([0.5]),
                discharge=torch.tensor([10.0]), slope=torch.tensor([0.001]))
    base.update(kw)
    return compute_trapezoidal_geometry(**base)


def test_keys_shapes_and_positive_values():
    keys = {"depth", "top_width", "bottom_width", "side_slope", "cross_sectional_area", "wetted_perimeter",
            "hydraulic_radius", "velocity"}
    assert set(geo().keys()) == keys
    r = geo(n=torch.full((100,), 0.035), p_spatial=torch.full((100,), 21.0), q_spatial=torch.full((100,), 0.5),
            discharge=torch.full((100,), 10.0), slope=torch.full((100,), 0.001))
    assert all(v.shape == (100,) for v in r.values())
    r = geo(n=torch.tensor([0.035, 0.05, 0.1]), p_spatial=torch.tensor([21.0, 50.0, 10.0]),
            q_spatial=torch.tensor([0.5, 0.3, 0.8]), discharge=torch.tensor([10.0, 100.0, 1.0]),
            slope=torch.tensor([0.001, 0.01, 0.0001]))
    assert all((v > 0).all() for v in r.values())


def test_monotone_in_discharge_roughness_and_slope():
    two = lambda v: torch.tensor(v)  # noqa: E731
    r = geo(n=two([0.035, 0.035]), p_spatial=two([21.0, 21.0]), q_spatial=two([0.5, 0.5]),
            discharge=two([10.0, 100.0]), slope=two([0.001, 0.001]))
    assert r["depth"][1] > r["depth"][0] and r["top_width"][1] > r["top_width"][0]
    r = geo(n=two([0.02, 0.15]), p_spatial=two([21.0, 21.0]), q_spatial=two([0.5, 0.5]),
            discharge=two([50.0, 50.0]), slope=two([0.001, 0.001]))
    assert r["depth"][1] > r["depth"][0]
    r = geo(n=two([0.035, 0.035]), p_spatial=two([21.0, 21.0]), q_spatial=two([0.5, 0.5]),
            discharge=two([50.0, 50.0]), slope=two([0.0001, 0.01]))
    assert r["depth"][0] > r["depth"][1]


def test_lower_bounds_and_rectangular_limit():
    assert geo(discharge=torch.tensor([1e-8]), depth_lb=0.05)["depth"].item() >= 0.05
    assert geo(q_spatial=torch.tensor([0.99]), discharge=torch.tensor([0.01]),
               bottom_width_lb=0.1)["bottom_width"].item() >= 0.1
    assert geo(q_spatial=torch.tensor([0.0]))["side_slope"].item() == pytest.approx(0.5, abs=0.01)


def test_area_and_hydraulic_radius_identities():
    r = geo(discharge=torch.tensor([50.0]))
    area = (r["top_width"] + r["bottom_width"]) * r["depth"] / 2
    assert r["cross_sectional_area"].item() == pytest.approx(area.item(), rel=1e-5)
    assert r["hydraulic_radius"].item() == pytest.approx((r["cross_sectional_area"] / r["wetted_perimeter"]).item(),
                                                         rel=1e-5)


def test_side_slope_bounds_are_parameters():
    """The routing kernels take the side-slope clamp from RouteConsts (the drop-in passes it here for the
    geometry VJP); the reference's fixed [0.5, 50] is the default."""
    q = torch.tensor([0.0, 0.5, 0.99])
    d = geo(n=torch.full((3,), 0.035), p_spatial=torch.full((3,), 21.0), q_spatial=q,
            discharge=torch.full((3,), 10.0), slope=torch.full((3,), 0.001))
    c = geo(n=torch.full((3,), 0.035), p_spatial=torch.full((3,), 21.0), q_spatial=q,
            discharge=torch.full((3,), 10.0), slope=torch.full((3,), 0.001), side_slope_lb=1.0, side_slope_ub=2.0)
    assert np.all(c["side_slope"].numpy() >= 1.0) and np.all(c["side_slope"].numpy() <= 2.0)
    assert d["side_slope"][0].item() == pytest.approx(0.5)
