"""Drop-in for ``ddr.routing.torch_mc`` (reference ``src/ddr/routing/torch_mc.py``).

``dmc`` is the ``nn.Module`` façade the trainer, tester, router and BMI call:
``dmc(cfg, device)(routing_dataclass=..., streamflow=(T, N), spatial_parameters={...},
carry_state=False, retain_grads=False) -> {"runoff": (N, T) | (G, T)}``.
It owns no learnable parameters; the routing engine is :class:`~ddr_amd.routing.mmc.MuskingumCunge`
on the fused HIP kernels.
"""

from __future__ import annotations

from typing import Any

import torch

from .mmc import MuskingumCunge

_MIRRORED = ("t", "parameter_bounds", "p_spatial", "velocity_lb", "depth_lb", "discharge_lb", "bottom_width_lb")


class dmc(torch.nn.Module):  # noqa: N801  (reference class name)
    """Differentiable Muskingum-Cunge routing module (torch_mc.py:18-339)."""

    def __init__(self, cfg: Any, device: str | torch.device | None = "cpu") -> None:
        super().__init__()
        self.cfg = cfg
        self.device_num: str | torch.device = device if device is not None else "cpu"
        self.routing_engine = MuskingumCunge(cfg, self.device_num)
        self._mirror_engine_constants()
        self._discharge_t: torch.Tensor = torch.empty(0)
        self.network: torch.Tensor = torch.empty(0)
        self.n: torch.Tensor = torch.empty(0)
        self.q_spatial: torch.Tensor = torch.empty(0)
        self.top_width: torch.Tensor = torch.empty(0)
        self.side_slope: torch.Tensor = torch.empty(0)
        self.epoch = 0
        self.mini_batch = 0

    def _mirror_engine_constants(self) -> None:
        for name in _MIRRORED:
            setattr(self, name, getattr(self.routing_engine, name))

    # ---- device moves rebuild the engine on the new device (torch_mc.py:63-128) -------------
    def to(self, device: torch.device | str) -> "dmc":  # type: ignore[override]
        super().to(device)
        self.device_num = device if isinstance(device, str) else str(device)
        self.routing_engine = MuskingumCunge(self.cfg, self.device_num)
        self._mirror_engine_constants()
        return self

    def cuda(self, device: int | torch.device | None = None) -> "dmc":  # type: ignore[override]
        if device is None:
            return self.to("cuda")
        return self.to(f"cuda:{device}" if isinstance(device, int) else str(device))

    def cpu(self) -> "dmc":  # type: ignore[override]
        return self.to("cpu")

    def set_progress_info(self, epoch: int, mini_batch: int) -> None:
        self.epoch = epoch
        self.mini_batch = mini_batch
        self.routing_engine.set_progress_info(epoch, mini_batch)

    def forward(self, **kwargs: Any) -> dict[str, torch.Tensor]:
        """Route ``streamflow`` through the network (torch_mc.py:144-223)."""
        eng = self.routing_engine
        eng.setup_inputs(routing_dataclass=kwargs["routing_dataclass"],
                         streamflow=kwargs["streamflow"].to(self.device_num),
                         spatial_parameters=kwargs["spatial_parameters"],
                         carry_state=kwargs.get("carry_state", False))
        self.network, self.n, self.q_spatial, self.p_spatial = eng.network, eng.n, eng.q_spatial, eng.p_spatial
        # (the reference mirrors _discharge_t here too, overwritten below before the caller can see it: not
        # read here, so a cold start's hot start runs inside forward's launch)
        output = eng.forward()
        self.top_width, self.side_slope = eng.top_width, eng.side_slope
        self._discharge_t = eng._discharge_t
        if kwargs.get("retain_grads", False):
            for t in (self.n, self.q_spatial, self._discharge_t):
                if t is not None and t.requires_grad:
                    t.retain_grad()
            if self.p_spatial is not None and self.p_spatial.requires_grad:
                self.p_spatial.retain_grad()
            for v in (eng.spatial_parameters or {}).values():
                if v.requires_grad:
                    v.retain_grad()
            if output.requires_grad:
                output.retain_grad()
        return {"runoff": output}

    # ---- compatibility pass-throughs (torch_mc.py:225-295) -----------------------------------
    def fill_op(self, data_vector: torch.Tensor) -> torch.Tensor:
        return self.routing_engine.fill_op(data_vector)

    def _sparse_eye(self, n: int) -> torch.Tensor:
        return self.routing_engine._sparse_eye(n)

    def _sparse_diag(self, data: torch.Tensor) -> torch.Tensor:
        return self.routing_engine._sparse_diag(data)

    def route_timestep(self, q_prime_clamp: torch.Tensor, mapper: Any) -> torch.Tensor:
        return self.routing_engine.route_timestep(q_prime_clamp=q_prime_clamp, mapper=mapper)

    # ---- checkpoint extras (torch_mc.py:297-339) ---------------------------------------------
    def state_dict(self, *args: Any, **kwargs: Any) -> dict[str, Any]:  # type: ignore[override]
        state: dict[str, Any] = super().state_dict(*args, **kwargs)
        state.update(cfg=self.cfg, device_num=self.device_num, epoch=self.epoch, mini_batch=self.mini_batch)
        return state

    def load_state_dict(self, state_dict: dict[str, Any], strict: bool = True) -> None:  # type: ignore[override]
        state_dict = dict(state_dict)
        self.cfg = state_dict.pop("cfg", self.cfg)
        self.device_num = state_dict.pop("device_num", self.device_num)
        self.epoch = state_dict.pop("epoch", 0)
        self.mini_batch = state_dict.pop("mini_batch", 0)
        super().load_state_dict(state_dict, strict)
        self.routing_engine = MuskingumCunge(self.cfg, self.device_num)
        self.routing_engine.set_progress_info(self.epoch, self.mini_batch)
        self._mirror_engine_constants()
