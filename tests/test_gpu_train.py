"""GPU parity of the fused C3 step tail (ddr_amd.train, csrc/train.hip) against the PyTorch ops it replaces:
the daily L1 objective + gradient (scripts/train.py:91-94) and clip_grad_norm_ + Adam (train.py:99-100).
Tolerances: the loss to 1e-6 relative (fp64 vs fp32 summation order), its gradient bitwise (sign x 1/count),
the parameters after five clipped Adam steps to 1e-6 relative (fused vs torch's operation order)."""

import numpy as np
import pytest
import torch

from ddr_amd.train import ClipAdam, daily_l1_loss

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wd", [0, 5])
def test_daily_l1_matches_torch(cuda, wd):
    g = torch.Generator(device=cuda).manual_seed(3)
    daily = torch.rand((256, 89), device=cuda, generator=g).requires_grad_(True)
    obs = torch.rand((256, 89), device=cuda, generator=g)
    obs[3, 40] = daily[3, 40].detach()  # a zero difference: sign 0, as torch's abs backward
    loss = daily_l1_loss(daily, obs, wd)
    (loss * 2.0).backward()
    ref_in = daily.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.l1_loss(ref_in[:, wd:], obs[:, wd:])
    (ref * 2.0).backward()
    assert abs(loss.item() - ref.item()) <= 1e-6 * abs(ref.item())
    torch.testing.assert_close(daily.grad, ref_in.grad, rtol=0, atol=0)
    assert float(daily.grad[:, :wd].abs().sum()) == 0.0


def test_daily_l1_rejects_cpu_and_bad_shapes(cuda):
    with pytest.raises(RuntimeError):
        daily_l1_loss(torch.zeros(2, 3), torch.zeros(2, 3), 0)
    with pytest.raises(ValueError):
        daily_l1_loss(torch.zeros(2, 3, device=cuda), torch.zeros(2, 4, device=cuda), 0)


@pytest.mark.parametrize("scale", [1e-3, 10.0], ids=["unclipped", "clipped"])
def test_clip_adam_matches_torch(cuda, scale):
    torch.manual_seed(0)
    p0 = torch.randn(34179, device=cuda)
    ours = p0.clone()
    ref = torch.nn.Parameter(p0.clone())
    opt = ClipAdam(ours, lr=1e-3, max_norm=1.0)
    topt = torch.optim.Adam([ref], lr=1e-3)
    for k in range(5):
        grad = torch.randn(p0.shape, device=cuda, generator=torch.Generator(device=cuda).manual_seed(k)) * scale
        ours.grad = grad.clone()
        ref.grad = grad.clone()
        opt.step()
        norm = torch.nn.utils.clip_grad_norm_([ref], max_norm=1.0)
        topt.step()
        assert abs(opt.last_norm.item() - norm.item()) <= 1e-6 * norm.item()
    err = (ours - ref.detach()).abs().max().item()
    assert err <= 1e-6 * ref.detach().abs().max().item(), err
    np.testing.assert_array_equal(opt.m.cpu().numpy() != 0, np.ones(p0.shape, bool))
