"""The fused parameter network (csrc/pnet.hip; C3's stand-in for the reference's KAN, src/ddr/nn/kan.py:11-62)
against the same network in PyTorch ops (fp32, hipBLASLt GEMMs + autograd).

Tolerances: outputs max-rel 1e-5 (fp32 GEMMs summed in another order: ~1e-7 per product chain, amplified at most
by the log-space denormalisation's exp); parameter gradients norm-relative 1e-5.
"""

import numpy as np
import pytest
import torch

from conftest import normrel
from ddr_amd.pnet import ParamNet, TorchParamNet, param_count

pytestmark = pytest.mark.gpu

RANGES = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}


@pytest.mark.parametrize("N,F", [(1, 10), (63, 10), (1000, 7), (70001, 10), (300000, 10)])
def test_fused_network_matches_torch(cuda, N, F):
    gen = torch.Generator().manual_seed(N + F)
    x = torch.randn((N, F), generator=gen).to(cuda)
    fused = ParamNet(F, RANGES, seed=3).to(cuda)
    ref = TorchParamNet(F, RANGES, seed=3).to(cuda)
    with torch.no_grad():  # non-zero biases, so their gradients and the bias paths are exercised
        b = torch.randn(param_count(F), generator=gen).to(cuda) * 0.1
        fused.flat.add_(b)
        ref.flat.add_(b)
    outs = fused(x)
    routs = ref(x)
    gs = [torch.randn(N, generator=gen).to(cuda) for _ in range(3)]
    for o, r in zip(outs, routs):
        assert o.shape == (N,)
        assert float(((o - r).abs() / r.abs().clamp_min(1e-6)).max()) <= 1e-5
    sum((o * g).sum() for o, g in zip(outs, gs)).backward()
    sum((o * g).sum() for o, g in zip(routs, gs)).backward()
    assert normrel(fused.flat.grad.cpu().numpy(), ref.flat.grad.cpu().numpy()) <= 1e-5


def test_fused_network_backward_is_deterministic(cuda):
    F, N = 10, 50000
    x = torch.randn((N, F), generator=torch.Generator().manual_seed(1)).to(cuda)
    net = ParamNet(F, RANGES).to(cuda)
    grads = []
    for _ in range(2):
        net.flat.grad = None
        n, q, p = net(x)
        (n.sum() + 2 * q.sum() + p.mean()).backward()
        grads.append(net.flat.grad.clone())
    assert torch.equal(grads[0], grads[1])
    assert np.isfinite(grads[0].cpu().numpy()).all()


def test_fused_network_rejects_misplaced_parameters(cuda):
    """The C ABI takes raw pointers: parameters left on the host, cast to fp64 or on another device must raise
    (a ValueError), not reach the kernel as fp32 device memory."""
    ranges = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}
    x = torch.rand((1000, 10), device=cuda)
    net = ParamNet(10, ranges)
    with pytest.raises(ValueError):
        net(x)  # parameters still on the host
    net = net.to(cuda).double()
    with pytest.raises(ValueError):
        net(x)  # fp64 parameters
    net = net.float()
    outs = net(x)
    assert all(o.shape == (1000,) for o in outs)
