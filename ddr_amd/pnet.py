"""Fused parameter network of the C3 training step (``bench.py --workload c3``), on the fp32 matrix cores.

The reference trains a KAN (``src/ddr/nn/kan.py:11-62``: Linear -> pykan KAN layers -> Linear -> sigmoid,
outputs ``n``, ``q_spatial``, ``p_spatial`` in [0, 1]) whose outputs the routing engine denormalises
(``routing/utils.py:166-185``).  pykan is not installed here, so the training step uses a stand-in of the same
contract and comparable cost: attributes (N, F) -> 3 x [Linear(., 128) + SiLU] -> Linear(128, 3) -> sigmoid ->
denormalize.  ``ParamNet`` runs it (forward and backward) as two persistent HIP launches
(``ddr_pnet_forward_f32`` / ``ddr_pnet_backward_f32``, ``csrc/pnet.hip``) instead of ~60 PyTorch launches;
``TorchParamNet`` is the same network in PyTorch ops (the numerics reference of ``tests/test_gpu_pnet.py``).

The parameters are one flat tensor (torch.nn.Linear's (out, in) weight layout, ``views()``), so the
multi-GPU gradient all-reduce, the clipping norm and Adam each touch one buffer.
"""

from __future__ import annotations

import ctypes as C
import math

import torch

from . import _lib

HIDDEN = 128
OUT = 3


def param_count(n_features: int) -> int:
    return (HIDDEN * n_features + HIDDEN) + 2 * (HIDDEN * HIDDEN + HIDDEN) + (OUT * HIDDEN + OUT)


def views(flat: torch.Tensor, n_features: int) -> dict[str, torch.Tensor]:
    """W1 (128, F), b1, W2 (128, 128), b2, W3, b3, W4 (3, 128), b4 of the flat parameter vector."""
    shapes = [("w1", (HIDDEN, n_features)), ("b1", (HIDDEN,)), ("w2", (HIDDEN, HIDDEN)), ("b2", (HIDDEN,)),
              ("w3", (HIDDEN, HIDDEN)), ("b3", (HIDDEN,)), ("w4", (OUT, HIDDEN)), ("b4", (OUT,))]
    out, o = {}, 0
    for name, shp in shapes:
        k = math.prod(shp)
        out[name] = flat[o:o + k].view(shp)
        o += k
    return out


def init_params(n_features: int, seed: int = 0) -> torch.Tensor:
    """randn / sqrt(fan_in) weights, zero biases (bench.py's ParamNet initialisation, identical on every rank)."""
    g = torch.Generator().manual_seed(seed)
    flat = torch.zeros(param_count(n_features))
    v = views(flat, n_features)
    for w in ("w1", "w2", "w3", "w4"):
        v[w].copy_(torch.randn(v[w].shape, generator=g) / math.sqrt(v[w].shape[1]))
    return flat


def denorm_table(ranges: dict, log_space=("p_spatial",)) -> list[float]:
    """[3][3] (scale, offset, log flag) for outputs (n, q_spatial, p_spatial): utils.py:166-185 -- linear
    u (hi - lo) + lo, or exp(u (ln hi - ln(lo + 1e-6)) + ln(lo + 1e-6)) in log space."""
    rows = []
    for name in ("n", "q_spatial", "p_spatial"):
        lo, hi = ranges[name]
        if name in log_space:
            llo, lhi = math.log(lo + 1e-6), math.log(hi)
            rows += [lhi - llo, llo, 1.0]
        else:
            rows += [hi - lo, lo, 0.0]
    return rows


def _check_device_f32(t: torch.Tensor, dev: torch.device, what: str, shape=None) -> None:
    """The C ABI takes raw device pointers: a host, fp64, strided or other-device tensor would be read as
    fp32 device memory (a GPU memory fault, not a Python error), so reject it here."""
    if not (t.is_cuda and t.device == dev):
        raise ValueError(f"the fused parameter network's {what} must be on {dev} (got {t.device})")
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError(f"the fused parameter network's {what} must be contiguous float32")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"the fused parameter network's {what} must have shape {tuple(shape)}, got {tuple(t.shape)}")


class _PnetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, flat, table):
        lib = _lib.load()
        N, F = x.shape
        dev = x.device
        z = torch.empty((3, N, HIDDEN), device=dev, dtype=torch.float32)
        u = torch.empty((N, OUT), device=dev, dtype=torch.float32)
        outs = [torch.empty(N, device=dev, dtype=torch.float32) for _ in range(OUT)]
        tab = (C.c_float * 9)(*table)
        _lib.check(lib.ddr_pnet_forward_f32(N, F, x.data_ptr(), flat.data_ptr(), tab, z.data_ptr(), u.data_ptr(),
                                            outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(),
                                            _lib.stream_ptr(dev)))
        ctx.save_for_backward(x, flat, z, u)
        ctx.table = table
        return tuple(outs)

    @staticmethod
    def backward(ctx, gn, gq, gp):
        x, flat, z, u = ctx.saved_tensors
        lib = _lib.load()
        N, F = x.shape
        dev = x.device
        g = [t.to(torch.float32).contiguous() if t is not None else torch.zeros(N, device=dev) for t in (gn, gq, gp)]
        for t in g:
            _check_device_f32(t, dev, "output gradient", (N,))
        grad = torch.empty_like(flat)
        work = torch.empty(max(int(lib.ddr_pnet_work_bytes(N, F)), 4), device=dev, dtype=torch.uint8)
        tab = (C.c_float * 9)(*ctx.table)
        _lib.check(lib.ddr_pnet_backward_f32(N, F, x.data_ptr(), flat.data_ptr(), tab, z.data_ptr(), u.data_ptr(),
                                             g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(), grad.data_ptr(),
                                             work.data_ptr(), _lib.stream_ptr(dev)))
        return None, grad, None


class ParamNet(torch.nn.Module):
    """attributes (N, F) -> (n, q_spatial, p_spatial), each (N,), denormalised; fused HIP forward/backward."""

    def __init__(self, n_features: int, ranges: dict, log_space=("p_spatial",), seed: int = 0):
        super().__init__()
        if not 1 <= n_features <= 12:
            raise ValueError("the fused network takes 1..12 input features")
        self.n_features = n_features
        self.flat = torch.nn.Parameter(init_params(n_features, seed))
        self.table = denorm_table(ranges, log_space)

    def forward(self, x: torch.Tensor):
        if not x.is_cuda:
            raise RuntimeError("the fused parameter network runs on the HIP device only (no CPU fallback)")
        x = x.to(torch.float32).contiguous()
        if x.dim() != 2 or x.shape[1] != self.n_features:
            raise ValueError(f"attributes must be (N, {self.n_features})")
        # the parameters as the kernels read them: fp32, contiguous, on x's device (not after .double() or
        # without .to(device))
        _check_device_f32(self.flat, x.device, "parameters", (param_count(self.n_features),))
        return _PnetFn.apply(x, self.flat, self.table)


class TorchParamNet(torch.nn.Module):
    """The same network in PyTorch ops (numerics reference; shares the flat parameter layout)."""

    def __init__(self, n_features: int, ranges: dict, log_space=("p_spatial",), seed: int = 0):
        super().__init__()
        self.n_features = n_features
        self.flat = torch.nn.Parameter(init_params(n_features, seed))
        self.table = denorm_table(ranges, log_space)

    def forward(self, x: torch.Tensor):
        v = views(self.flat, self.n_features)
        h = x
        for l in ("1", "2", "3"):
            h = torch.nn.functional.silu(torch.nn.functional.linear(h, v["w" + l], v["b" + l]))
        u = torch.sigmoid(torch.nn.functional.linear(h, v["w4"], v["b4"]))
        outs = []
        for j in range(OUT):
            s, o, lg = self.table[3 * j: 3 * j + 3]
            y = u[:, j] * s + o
            outs.append(torch.exp(y) if lg else y)
        return tuple(outs)
