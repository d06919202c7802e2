"""Drop-in for ``ddr.routing.mmc`` (reference ``src/ddr/routing/mmc.py``).

``MuskingumCunge`` keeps the reference's constructor, attributes and methods; ``forward`` runs the
whole T-step window as one fused HIP launch (``ddrx::mc_route``) instead of T-1 Python iterations of
``route_timestep`` + SciPy/CuPy solves, and its backward is the fused adjoint launch.  Everything
before the op -- slope clamp, flow scaling, ``denormalize`` -- stays PyTorch, exactly as in the
reference, so autograd reaches the KAN unchanged.

The hot start (``compute_hotstart_discharge``, mmc.py:25-66) and the single-step ``route_timestep``
(mmc.py:487-559, used by the BMI coupling) reuse the same kernels (T = 1 and T = 2 windows).
"""

from __future__ import annotations

import os

import logging
import weakref
from typing import Any

import torch

from ..graph import RiverGraph, adjacency_to_coo
from ..ops import GaugeMap, RouteConsts, qprime_has_nan, route
from .utils import PatternMapper, denormalize, get_network_idx, triangular_sparse_solve

log = logging.getLogger(__name__)

# id(adjacency) -> (weakref to the adjacency object, graph); identity-checked (tensors compare
# element-wise, so they cannot be WeakKeyDictionary keys)
_GRAPH_CACHE: dict[int, tuple[Any, RiverGraph]] = {}


def graph_for(adjacency, device) -> RiverGraph:
    """Build (once per adjacency object) the device river graph of a RoutingDataclass adjacency."""
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    hit = _GRAPH_CACHE.get(id(adjacency))
    if hit is not None:
        ref, g = hit
        if ref() is adjacency and g.device == dev:
            return g
    n, rows, cols = adjacency_to_coo(adjacency)
    g = RiverGraph(n, rows, cols, device=dev)
    try:
        ref = weakref.ref(adjacency)
    except TypeError:
        return g
    for k in [k for k, (r, _) in _GRAPH_CACHE.items() if r() is None]:
        del _GRAPH_CACHE[k]
    _GRAPH_CACHE[id(adjacency)] = (ref, g)
    return g


def compute_hotstart_discharge(q_prime_t0: torch.Tensor, mapper: PatternMapper, discharge_lb: torch.Tensor,
                               device: str | torch.device) -> torch.Tensor:
    """Topological accumulation (I - N) Q = q'_0, then clamp (mmc.py:25-66).

    With a mapper built from a network (it carries the RiverGraph) this is the fused kernel's
    hot-start sweep; otherwise the general HIP triangular solve on ``mapper.map(-1)``.
    """
    lb = float(discharge_lb)
    g = getattr(mapper, "graph", None)
    if g is not None:
        dev = q_prime_t0.device
        n = q_prime_t0.shape[0]
        one = torch.ones(n, device=dev, dtype=q_prime_t0.dtype)
        # differentiable w.r.t. q'[0] like the reference's solve (the adjoint's step-0 sweep)
        _, q_last, _, _ = route(g, q_prime_t0.reshape(1, n), one, one, one, one, one, one,
                                consts=RouteConsts(discharge_lb=lb))
        return q_last
    num_segments = q_prime_t0.shape[0]
    neg_ones = -torch.ones(num_segments, device=q_prime_t0.device)
    neg_ones[0] = 1.0  # diagonal maps to datvec[0]; keeps identity
    A_values = mapper.map(neg_ones)
    discharge = triangular_sparse_solve(A_values, mapper.crow_indices, mapper.col_indices, q_prime_t0, True, False,
                                        device)
    return torch.clamp(discharge, min=discharge_lb)


def _assert_no_nan(q_prime: torch.Tensor) -> None:
    """mmc.py:335 on the host: one reduction pass (a NaN makes the sum NaN); the elementwise check only
    decides the rare NaN-sum case (+inf and -inf)."""
    if bool(torch.isnan(q_prime.sum())):
        assert ~torch.any(torch.isnan(q_prime)), "q_prime has NaN flows"


def _apply_data_override(derived: torch.Tensor, data: torch.Tensor | None) -> torch.Tensor:
    """Observed geometry replaces the power-law one where available (mmc.py:74-99)."""
    if data is None or data.numel() == 0:
        return derived
    nan_mask = torch.isnan(data)
    if not nan_mask.any():
        return data
    return torch.where(~nan_mask, data, derived)


class MuskingumCunge:
    """Muskingum-Cunge routing engine (mmc.py:171-630) on the fused HIP kernels.

    The cold start's hot-start state (mmc.py:330-342) is materialised lazily: ``forward`` runs it as
    step 0 of its own fused launch (the kernel's t = 0 branch: the same accumulation, the same bits), so a
    training step makes one routing launch, not a separate T = 1 launch first; reading ``_discharge_t``
    before ``forward`` (tests, BMI ``initialize``) runs that launch then, with the same result.
    """

    @property
    def _discharge_t(self) -> torch.Tensor | None:
        if self._hot_pending is not None:
            qp = self._hot_pending  # (the q' of the setup_inputs that made the cold start)
            self._hot_pending = None
            _assert_no_nan(qp)
            mapper, _, _ = self.create_pattern_mapper()
            self._state = compute_hotstart_discharge(qp[0].to(self.device), mapper, self.discharge_lb, self.device)
        return self._state

    @_discharge_t.setter
    def _discharge_t(self, value: torch.Tensor | None) -> None:
        self._hot_pending = None
        self._state = value

    def __init__(self, cfg: Any, device: str | torch.device = "cpu") -> None:
        self.cfg = cfg
        self.device = device
        # forward coefficient arithmetic of the fused kernel: "faithful" (default: the reference's
        # operation order and IEEE divisions, the three pows in fp32 faithful-class arithmetic -- at most
        # 1 ulp, the accuracy class of the reference's own Sleef powf; <= 4.6e-7 from the reference's
        # goldens, tests/test_gpu_fastmath.py; what bench.py times), "exact" (correctly rounded pow:
        # bit-identical to the oracle, ops.route's default) or "fast"; cfg.params.routing_math or
        # DDR_ROUTING_MATH select another
        self.math = (getattr(cfg.params, "routing_math", None) or os.environ.get("DDR_ROUTING_MATH") or "faithful")
        if self.math not in ("exact", "faithful", "fast"):
            raise ValueError(f"routing_math must be 'exact', 'faithful' or 'fast', not {self.math!r}")
        self._eager_nan_check = bool(getattr(cfg.params, "eager_nan_check", False)) or \
            os.environ.get("DDR_EAGER_NAN_CHECK") == "1"
        # the fp32 backward as the exact adjoint of the fp32 trajectory (ops.route exact_adjoint; ~30 % more
        # backward time): cfg.params.exact_adjoint or DDR_EXACT_ADJOINT=1
        self._exact_adjoint = bool(getattr(cfg.params, "exact_adjoint", False)) or \
            os.environ.get("DDR_EXACT_ADJOINT") == "1"
        self.t = torch.tensor(3600.0, device=self.device)
        self.n: torch.Tensor | None = None
        self.q_spatial: torch.Tensor | None = None
        self._hot_pending: torch.Tensor | None = None  # the q' of a cold start whose hot start has not run yet
        self._state: torch.Tensor | None = None
        self._discharge_t = None
        self.network: torch.Tensor | None = None
        self.parameter_bounds = self.cfg.params.parameter_ranges
        self.p_spatial = torch.tensor(self.cfg.params.defaults["p_spatial"], device=self.device)
        mins = self.cfg.params.attribute_minimums
        self.velocity_lb = torch.tensor(mins["velocity"], device=self.device)
        self.depth_lb = torch.tensor(mins["depth"], device=self.device)
        self.discharge_lb = torch.tensor(mins["discharge"], device=self.device)
        self.bottom_width_lb = torch.tensor(mins["bottom_width"], device=self.device)
        self.routing_dataclass: Any = None
        self.length: torch.Tensor | None = None
        self.slope: torch.Tensor | None = None
        self.top_width: torch.Tensor | None = None
        self.side_slope: torch.Tensor | None = None
        self._data_top_width: torch.Tensor | None = None
        self._data_side_slope: torch.Tensor | None = None
        self.x_storage: torch.Tensor | None = None
        self.observations: Any = None
        self.output_indices: list[Any] | None = None
        self.gage_catchment: list[str] | None = None
        self.q_prime: torch.Tensor | None = None
        self.spatial_parameters: dict[str, torch.Tensor] | None = None
        self.epoch = 0
        self.mini_batch = 0
        self._flat_indices: torch.Tensor | None = None
        self._group_ids: torch.Tensor | None = None
        self._num_outputs: int | None = None
        self._scatter_input: torch.Tensor | None = None
        self._graph: RiverGraph | None = None
        self._gauges: GaugeMap | None = None

    # ------------------------------------------------------------------------------------------
    def set_progress_info(self, epoch: int, mini_batch: int) -> None:
        self.epoch = epoch
        self.mini_batch = mini_batch

    def _consts(self) -> RouteConsts:
        return RouteConsts(dt=float(self.t), discharge_lb=float(self.discharge_lb),
                           velocity_lb=float(self.velocity_lb), depth_lb=float(self.depth_lb),
                           bottom_width_lb=float(self.bottom_width_lb))

    def setup_inputs(self, routing_dataclass: Any, streamflow: torch.Tensor, spatial_parameters: dict[str, torch.Tensor],
                     carry_state: bool = False) -> None:
        """mmc.py:250-269."""
        self._set_network_context(routing_dataclass, streamflow)
        self._denormalize_spatial_parameters(spatial_parameters)
        self._init_discharge_state(carry_state)
        self._precompute_scatter_indices()

    def _set_network_context(self, routing_dataclass: Any, streamflow: torch.Tensor) -> None:
        """mmc.py:271-304."""
        self.routing_dataclass = routing_dataclass
        self.output_indices = routing_dataclass.outflow_idx
        self.gage_catchment = routing_dataclass.gage_catchment
        obs = getattr(routing_dataclass, "observations", None)
        self.observations = obs.gage_id if obs is not None else None
        self.network = routing_dataclass.adjacency_matrix
        self.length = routing_dataclass.length.to(self.device).to(torch.float32)
        self.slope = torch.clamp(routing_dataclass.slope.to(self.device).to(torch.float32),
                                 min=self.cfg.params.attribute_minimums["slope"])
        self.x_storage = routing_dataclass.x.to(self.device).to(torch.float32)
        tw = getattr(routing_dataclass, "top_width", None)
        ss = getattr(routing_dataclass, "side_slope", None)
        self._data_top_width = tw.to(self.device).to(torch.float32) if tw is not None and tw.numel() > 0 else None
        self._data_side_slope = ss.to(self.device).to(torch.float32) if ss is not None and ss.numel() > 0 else None
        self.q_prime = streamflow.to(self.device)
        fs = getattr(routing_dataclass, "flow_scale", None)
        if fs is not None:
            self.q_prime = self.q_prime * fs.unsqueeze(0).to(self.device)
        if torch.device(self.device).type == "cuda":
            self._graph = graph_for(self.network, self.device)

    def _denormalize_spatial_parameters(self, spatial_parameters: dict[str, torch.Tensor]) -> None:
        """mmc.py:306-328."""
        self.spatial_parameters = spatial_parameters
        log_space = self.cfg.params.log_space_parameters
        self.n = denormalize(spatial_parameters["n"], self.parameter_bounds["n"], "n" in log_space)
        self.q_spatial = denormalize(spatial_parameters["q_spatial"], self.parameter_bounds["q_spatial"],
                                     "q_spatial" in log_space)
        if "p_spatial" in spatial_parameters and "p_spatial" in self.parameter_bounds:
            self.p_spatial = denormalize(spatial_parameters["p_spatial"], self.parameter_bounds["p_spatial"],
                                         "p_spatial" in log_space)

    def _init_discharge_state(self, carry_state: bool) -> None:
        """Cold start via topological accumulation, or carry (mmc.py:330-342)."""
        if carry_state and (self._state is not None or self._hot_pending is not None):
            return
        assert self.q_prime is not None, "q_prime must be set before initializing discharge state"
        if self._graph is not None:
            # forward's launch runs the hot start as its step 0 and the NaN assertion of mmc.py:335 inside
            # its q' gather (no separate pass over q'); reading _discharge_t first runs both here.  So a NaN
            # q' raises at forward() (or at that first read), not here as in the reference -- unless the
            # eager check is asked for (cfg.params.eager_nan_check or DDR_EAGER_NAN_CHECK=1: one host-synced
            # reduction over q' per cold start, the reference's timing of the AssertionError)
            if self._eager_nan_check:
                _assert_no_nan(self.q_prime)
            self._state = None
            self._hot_pending = self.q_prime
        else:
            _assert_no_nan(self.q_prime)
            mapper, _, _ = self.create_pattern_mapper()
            self._discharge_t = compute_hotstart_discharge(self.q_prime[0].to(self.device), mapper,
                                                           self.discharge_lb, self.device)

    def _precompute_scatter_indices(self) -> None:
        """Gauge mode when len(outflow_idx) != N (mmc.py:344-363)."""
        assert self._state is not None or self._hot_pending is not None, \
            "discharge state must be initialized before scatter indices"
        n = self.q_prime.shape[1]
        if self.output_indices is not None and len(self.output_indices) != n:
            self._gauges = GaugeMap.build(self.output_indices, n, self.device)
            self._flat_indices = self._gauges.index
            self._group_ids = torch.repeat_interleave(
                torch.arange(self._gauges.n_gauges, device=self._gauges.offsets.device),
                self._gauges.offsets[1:] - self._gauges.offsets[:-1])
            self._num_outputs = self._gauges.n_gauges
            self._scatter_input = torch.zeros(self._num_outputs, device=self.device, dtype=torch.float32)
        else:
            self._gauges = None
            self._flat_indices = self._group_ids = self._num_outputs = self._scatter_input = None

    def _p_tensor(self, like: torch.Tensor) -> torch.Tensor:
        p = self.p_spatial
        if not torch.is_tensor(p):
            p = torch.tensor(p)
        return p.to(device=like.device, dtype=like.dtype)

    def forward(self) -> torch.Tensor:
        """Fused forward over the whole window (mmc.py:365-443)."""
        if self.routing_dataclass is None:
            raise ValueError("routing_dataclass not set. Call setup_inputs() first.")
        if self.q_prime is None or (self._state is None and self._hot_pending is None):
            raise ValueError("Streamflow not set. Call setup_inputs() first.")
        if self._graph is None:
            raise RuntimeError("MuskingumCunge.forward runs on the HIP device only (no CPU fallback); "
                               "construct it with a cuda device")
        qp = self.q_prime.to(torch.float32)
        # a pending cold start of this q': the launch's own step 0 is the hot start (mmc.py:25-66, 385, 412)
        own = self._hot_pending is not None and self._hot_pending is self.q_prime
        q0 = None if own else self._discharge_t
        runoff, q_last, tw, ss = route(self._graph, qp, self.n, self.q_spatial, self._p_tensor(qp), self.length,
                                       self.slope, self.x_storage, q0=q0, gauges=self._gauges,
                                       consts=self._consts(), math=self.math, check_qprime=own,
                                       exact_adjoint=self._exact_adjoint)
        # mmc.py:335 (the cold start's assertion), decided by the launch's q' gather: this waits for the
        # gather only -- the routing kernel queued behind it keeps running while the host goes on
        assert not (own and qprime_has_nan()), "q_prime has NaN flows"
        self._discharge_t = q_last  # (also clears the pending cold start)
        if qp.shape[0] > 1:
            self.top_width = _apply_data_override(tw, self._data_top_width)
            self.side_slope = _apply_data_override(ss, self._data_side_slope)
        return runoff

    def create_pattern_mapper(self) -> tuple[PatternMapper, torch.Tensor, torch.Tensor]:
        """mmc.py:445-458 (the mapper carries the device graph)."""
        if self.network is None:
            raise ValueError("Network not set. Call setup_inputs() first.")
        g = self._graph
        mapper = PatternMapper(self.fill_op, self.network.shape[0], device=self.device, graph=g)
        rows, cols = get_network_idx(mapper)
        return mapper, rows, cols

    def calculate_muskingum_coefficients(self, length: torch.Tensor, velocity: torch.Tensor,
                                         x_storage: torch.Tensor):
        """mmc.py:460-485 (PyTorch; the fused kernel computes the same in-register)."""
        k = torch.div(length, velocity)
        denom = (2.0 * k * (1.0 - x_storage)) + self.t
        c_1 = (self.t - (2.0 * k * x_storage)) / denom
        c_2 = (self.t + (2.0 * k * x_storage)) / denom
        c_3 = ((2.0 * k * (1.0 - x_storage)) - self.t) / denom
        c_4 = (2.0 * self.t) / denom
        return c_1, c_2, c_3, c_4

    def route_timestep(self, q_prime_clamp: torch.Tensor, mapper: PatternMapper | None = None) -> torch.Tensor:
        """One step from ``_discharge_t`` with lateral inflow ``q_prime_clamp`` (mmc.py:487-559).

        Runs the fused kernel over a 2-step window (carried state + this step); differentiable.
        Updates ``top_width``/``side_slope`` like the reference; the caller assigns ``_discharge_t``.
        """
        if self._discharge_t is None or self.n is None or self.length is None or self.network is None:
            raise ValueError("Required attributes not set. Call setup_inputs() first.")
        if self._graph is None:
            raise RuntimeError("route_timestep runs on the HIP device only (no CPU fallback)")
        q = q_prime_clamp.to(torch.float32).reshape(1, -1)
        qp = torch.cat([q, q], 0)
        runoff, q_last, tw, ss = route(self._graph, qp, self.n, self.q_spatial, self._p_tensor(qp), self.length,
                                       self.slope, self.x_storage, q0=self._discharge_t, consts=self._consts(),
                                       math=self.math, exact_adjoint=self._exact_adjoint)
        self.top_width = _apply_data_override(tw, self._data_top_width)
        self.side_slope = _apply_data_override(ss, self._data_side_slope)
        return q_last

    # ---- sparse helpers kept for API compatibility (mmc.py:561-630) ------------------------------
    def fill_op(self, data_vector: torch.Tensor) -> torch.Tensor:
        if self.network is None:
            raise ValueError("Network not set. Call setup_inputs() first.")
        identity_matrix = self._sparse_eye(self.network.shape[0])
        vec_diag = self._sparse_diag(data_vector)
        net = self.network if self.network.layout != torch.strided else self.network.to_sparse_csr()
        vec_filled = torch.matmul(vec_diag.cpu(), net.cpu().to(vec_diag.dtype)).to(self.device)
        return identity_matrix.to(self.device) + vec_filled

    def _sparse_eye(self, n: int) -> torch.Tensor:
        idx = torch.arange(n, dtype=torch.int64)
        return torch.sparse_coo_tensor(torch.vstack([idx, idx]), torch.ones(n), size=(n, n)).to_sparse_csr().to(
            self.device)

    def _sparse_diag(self, data: torch.Tensor) -> torch.Tensor:
        n = len(data)
        idx = torch.arange(n, dtype=torch.int64)
        return torch.sparse_coo_tensor(torch.vstack([idx, idx]), data.cpu(), size=(n, n)).to_sparse_csr()
