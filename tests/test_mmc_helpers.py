"""MuskingumCunge helpers kept for API compatibility (reference tests/routing/test_mmc.py:127-232), on the CPU:
_sparse_eye, _sparse_diag and calculate_muskingum_coefficients (mmc.py:460-485, 561-630)."""

import torch

from conftest import PARAMS_MOCK, cfg_of
from ddr_amd.routing import MuskingumCunge


def test_sparse_eye_and_diag():
    mc = MuskingumCunge(cfg_of(PARAMS_MOCK), device="cpu")
    eye = mc._sparse_eye(5)
    assert eye.shape == (5, 5) and eye.layout in (torch.sparse_coo, torch.sparse_csr)
    assert torch.equal(eye.to_dense(), torch.eye(5))
    d = torch.tensor([1.0, 2.0, 3.0, 4.0])
    dm = mc._sparse_diag(d)
    assert dm.shape == (4, 4) and dm.layout in (torch.sparse_coo, torch.sparse_csr)
    assert torch.equal(dm.to_dense(), torch.diag(d))


def test_muskingum_coefficients():
    """Shapes, finiteness, c4 > 0, and the scheme's identities c1 + c2 = c4 and c1 + c2 + c3 = 1; a very small
    velocity (0.01 m/s) stays finite."""
    mc = MuskingumCunge(cfg_of(PARAMS_MOCK), device="cpu")
    c1, c2, c3, c4 = mc.calculate_muskingum_coefficients(torch.tensor([1000.0, 1500.0, 2000.0]),
                                                         torch.tensor([1.0, 1.5, 2.0]), torch.tensor([0.2, 0.25, 0.3]))
    for c in (c1, c2, c3, c4):
        assert c.shape == (3,) and torch.isfinite(c).all()
    assert (c4 > 0).all()
    torch.testing.assert_close(c1 + c2, c4, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(c1 + c2 + c3, torch.ones(3), rtol=1e-6, atol=1e-6)
    # the reference formula, mmc.py:479-485 (k = L / v, denominator 2k(1 - X) + dt)
    k = torch.tensor([1000.0, 1000.0, 1000.0])
    den = 2 * k * (1 - torch.tensor([0.2, 0.25, 0.3])) + mc.t
    torch.testing.assert_close(c4, 2 * mc.t / den)
    out = mc.calculate_muskingum_coefficients(torch.tensor([1000.0]), torch.tensor([0.01]), torch.tensor([0.2]))
    assert all(torch.isfinite(c).all() for c in out)
