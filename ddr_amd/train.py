"""The tail of the C3 training step on the device in three launches (``csrc/train.hip``).

The reference's loop (``scripts/train.py:91-100``) ends each mini-batch with ``l1_loss`` over the gauges'
daily series after the warm-up, ``loss.backward()``, ``clip_grad_norm_(max_norm=1.0)`` and ``optimizer.step()``
(Adam).  In PyTorch ops that is ~15 small launches per step (slice, subtract, abs, sum, scale and their
backward; the norm, the clip factor, the scaling; Adam's moment updates).  Here:

* :func:`daily_l1_loss` -- the objective and its gradient in one pass (``ddr_daily_l1_f32``); the backward is
  one multiply by the incoming scalar;
* :class:`ClipAdam` -- clip + Adam over one flat parameter vector (``ddr_clip_adam_f32``), e.g.
  :class:`ddr_amd.pnet.ParamNet`'s ``flat``.

Both are deterministic (fixed slices and reduction order) and run on the HIP device only.
"""

from __future__ import annotations

import ctypes as C

import torch

from . import _lib


class _DailyL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, daily, obs, warmup, inv_count):
        G, D = daily.shape
        loss = torch.empty((), device=daily.device, dtype=torch.float32)
        grad = torch.empty_like(daily) if ctx.needs_input_grad[0] else None
        _lib.check(_lib.load().ddr_daily_l1_f32(G, D, int(warmup), daily.data_ptr(), obs.data_ptr(), C.c_float(inv_count),
                                                loss.data_ptr(), grad.data_ptr() if grad is not None else None,
                                                _lib.stream_ptr(daily.device)))
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g, None, None, None


def daily_l1_loss(daily: torch.Tensor, obs: torch.Tensor, warmup: int, inv_count: float | None = None) -> torch.Tensor:
    """``inv_count * sum |daily[:, warmup:] - obs[:, warmup:]|`` (G, D) -> scalar; ``inv_count`` defaults to the
    mean's 1 / (G (D - warmup)) -- ``torch.nn.functional.l1_loss(daily[:, warmup:], obs[:, warmup:])``."""
    if not daily.is_cuda:
        raise RuntimeError("daily_l1_loss runs on the HIP device only (no CPU fallback)")
    if daily.dim() != 2 or obs.shape != daily.shape:
        raise ValueError("daily and obs must be the same (G, D) shape")
    G, D = daily.shape
    if not 0 <= warmup < D:
        raise ValueError("warmup must be in [0, D)")
    if inv_count is None:
        inv_count = 1.0 / (G * (D - warmup))
    daily = daily.to(torch.float32).contiguous()
    obs = obs.to(device=daily.device, dtype=torch.float32).contiguous()
    return _DailyL1.apply(daily, obs, warmup, float(inv_count))


class ClipAdam:
    """``clip_grad_norm_(max_norm)`` then ``torch.optim.Adam(lr, betas, eps)`` (no weight decay) on one flat
    fp32 parameter tensor, in two launches per step (64 workgroups).  ``max_norm`` <= 0 disables clipping.  ``last_norm`` holds the
    gradient norm of the last step (a device scalar, clip_grad_norm_'s return value).

    Unlike ``torch.nn.utils.clip_grad_norm_``, the clip is applied inside the update only: ``param.grad`` keeps
    the unclipped gradient after :meth:`step` (code that reads or accumulates ``.grad`` afterwards sees the raw
    gradient, not the reference loop's clipped one, ``scripts/train.py:99-100``)."""

    def __init__(self, param: torch.Tensor, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 max_norm: float = 1.0):
        if not param.is_cuda or param.dtype != torch.float32 or not param.is_contiguous():
            raise ValueError("ClipAdam takes one contiguous fp32 HIP parameter tensor")
        self.param = param
        self.lr, self.betas, self.eps, self.max_norm = float(lr), tuple(map(float, betas)), float(eps), float(max_norm)
        self.m = torch.zeros_like(param)
        self.v = torch.zeros_like(param)
        self.last_norm = torch.zeros((), device=param.device, dtype=torch.float32)
        self.work = torch.empty(int(_lib.load().ddr_clip_adam_work_bytes()), device=param.device, dtype=torch.uint8)
        # the step counter lives on the device (as torch's capturable Adam): a captured step replays correctly
        self.step_count = torch.zeros((), device=param.device, dtype=torch.float32)

    def zero_grad(self, set_to_none: bool = True) -> None:
        if set_to_none:
            self.param.grad = None
        elif self.param.grad is not None:
            self.param.grad.zero_()

    @torch.no_grad()
    def step(self) -> None:
        g = self.param.grad
        if g is None:
            return
        g = g.contiguous()
        b1, b2 = self.betas
        _lib.check(_lib.load().ddr_clip_adam_f32(self.param.numel(), self.param.data_ptr(), g.data_ptr(),
                                                 self.m.data_ptr(), self.v.data_ptr(), C.c_float(self.lr), C.c_float(b1),
                                                 C.c_float(b2), C.c_float(self.eps), self.step_count.data_ptr(),
                                                 C.c_float(self.max_norm), self.last_norm.data_ptr(),
                                                 self.work.data_ptr(), _lib.stream_ptr(self.param.device)))
