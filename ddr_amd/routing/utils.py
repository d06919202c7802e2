"""Drop-in for ``ddr.routing.utils`` (reference ``src/ddr/routing/utils.py``).

Same public names and argument meaning.  The triangular solve runs on the HIP library
(``ddr_tri_solve``); there is no SciPy/CuPy path and no CPU fallback -- a CPU tensor raises.

``PatternMapper`` keeps the reference's value-index layout (``utils.py:25-129``: each CSR row's
columns ascend with the diagonal last; diagonal slots map to ``datvec[0]``, row i's off-diagonal
slots to ``datvec[i]``) and additionally carries the :class:`RiverGraph` when it was built from a
network, so callers that pass a mapper (``compute_hotstart_discharge``) reach the fused kernels.
"""

from __future__ import annotations

import logging
from collections.abc import Callable
from typing import Any

import numpy as np
import torch

from .. import _lib

log = logging.getLogger(__name__)


class PatternMapper:
    """Map data vectors to the non-zeros of a sparse matrix (utils.py:25-129)."""

    def __init__(
        self,
        fillOp: Callable[[torch.Tensor], torch.Tensor],
        matrix_dim: int,
        constant_diags: list[float] | None = None,
        constant_offsets: list[int] | None = None,
        aux: Any = None,
        indShift: int = 0,
        device: str | torch.device | None = None,
        graph: Any = None,
    ) -> None:
        # value -> index trick of the reference; indices are exact in int64 (the reference's fp32
        # index vector limits it to < 2^24 reaches, utils.py:65-79; this version computes the
        # pattern in float64 so the limit is 2^53)
        offset = 1
        ind = torch.arange(offset, matrix_dim + offset, dtype=torch.float64)
        A = fillOp(ind.to(torch.float32)) if graph is None else None
        if A is not None:
            if not A.is_sparse_csr:
                A = A.to_sparse_csr()
            A = A.cpu()
            crow = A.crow_indices().to(torch.int64)
            col = A.col_indices().to(torch.int64)
            src = (A.values().to(torch.float64).round().to(torch.int64) - offset)
        else:
            # the graph caches its layout (per device): one build per adjacency, not per forward
            crow, col, src = graph.pattern_mapper_tensors(device)
        self.crow_indices = crow.to(device) if device is not None else crow
        self.col_indices = col.to(device) if device is not None else col
        self.src_index = src.to(self.crow_indices.device)
        self._matrix_dim = matrix_dim
        self._ind_shift = indShift
        self._M_csr = None
        self.graph = graph

    @property
    def M_csr(self) -> torch.Tensor:
        """The (N, nnz) selection matrix of the reference's ``map`` (utils.py:83-102), built on first
        use: the fused routing path never needs it (``map`` here is a gather)."""
        if self._M_csr is None:
            src = self.src_index.cpu()
            n_vals = len(src)
            cidx = torch.arange(0, n_vals, dtype=torch.int64) + self._ind_shift
            M_coo = torch.sparse_coo_tensor(torch.stack((src, cidx), 0), torch.ones(n_vals),
                                            size=(self._matrix_dim, n_vals))
            self._M_csr = M_coo.to_sparse_csr().to(self.crow_indices.device)
        return self._M_csr

    def map(self, datvec: torch.Tensor) -> torch.Tensor:
        """A_values[k] = datvec[src(k)] (utils.py:89-102); differentiable gather."""
        return datvec[self.src_index.to(datvec.device)]

    def getSparseIndices(self) -> tuple[torch.Tensor, torch.Tensor]:
        return self.crow_indices, self.col_indices


def get_network_idx(mapper: PatternMapper) -> tuple[torch.Tensor, torch.Tensor]:
    """Row/column index of every stored entry (utils.py:140-163), vectorised."""
    crow = mapper.crow_indices.cpu().to(torch.int64)
    counts = crow[1:] - crow[:-1]
    rows = torch.repeat_interleave(torch.arange(len(counts), dtype=torch.int64), counts)
    return rows, mapper.col_indices.cpu().to(torch.int64)


def denormalize(value: torch.Tensor, bounds: list[float], log_space: bool = False) -> torch.Tensor:
    """NN output in [0, 1] -> physical bounds (utils.py:166-185; +1e-6 on the log lower bound)."""
    if log_space:
        log_min = torch.log(torch.tensor(bounds[0] + 1e-6, device=value.device, dtype=value.dtype))
        log_max = torch.log(torch.tensor(bounds[1], device=value.device, dtype=value.dtype))
        return torch.exp(value * (log_max - log_min) + log_min)
    return (value * (bounds[1] - bounds[0])) + bounds[0]


def _fill_row_indices_vectorized(crow_indices: torch.Tensor, row_indices: torch.Tensor) -> None:
    """Row index of each stored entry (utils.py:392-428), in place, vectorised."""
    crow = crow_indices.cpu().to(torch.int64)
    counts = crow[1:] - crow[:-1]
    row_indices.copy_(torch.repeat_interleave(torch.arange(len(counts), dtype=torch.int64), counts))


def _compute_row_indices_gpu(crow_indices: torch.Tensor, nnz: int) -> torch.Tensor:
    counts = crow_indices[1:] - crow_indices[:-1]
    return torch.repeat_interleave(torch.arange(len(counts), device=crow_indices.device, dtype=torch.long), counts)


def _tri_solve(A_values, crow_host, col_host, rhs, lower: bool, transpose: bool, unit: bool = False) -> torch.Tensor:
    if not rhs.is_cuda:
        raise RuntimeError("triangular_sparse_solve runs on the HIP device only (no CPU fallback); use cuda tensors")
    n = crow_host.numel() - 1
    vals = A_values.detach().to(torch.float32).contiguous()
    b = rhs.detach().to(torch.float32).contiguous()
    x = torch.empty_like(b)
    crow = np.ascontiguousarray(crow_host.numpy().astype(np.int64))
    col = np.ascontiguousarray(col_host.numpy().astype(np.int64))
    lib = _lib.load()
    _lib.check(lib.ddr_tri_solve_ex(n, len(col), crow.ctypes.data, col.ctypes.data, vals.data_ptr(), b.data_ptr(),
                                    x.data_ptr(), int(lower), int(transpose), int(unit), _lib.stream_ptr(rhs.device)))
    return x.to(rhs.dtype)


class TriangularSparseSolver(torch.autograd.Function):
    """Sparse triangular solve A x = b with gradients for A's values and b (utils.py:515-692).

    Forward and the transposed backward solve accumulate in fp64 from fp32 values (the reference's
    SciPy semantics, utils.py:587-600, 188-242) on the HIP device.  ``unit_diagonal`` as SciPy / CuPy
    (utils.py:596, 611; backward 239, 307): every diagonal entry is taken as 1 and never read, in both
    directions; the value gradient still covers every stored entry (utils.py:321-389).
    """

    @staticmethod
    def forward(ctx, A_values, crow_indices, col_indices, b, lower, unit_diagonal, device):
        crow_h = crow_indices.detach().cpu().to(torch.int64)
        col_h = col_indices.detach().cpu().to(torch.int64)
        try:
            x = _tri_solve(A_values, crow_h, col_h, b, bool(lower), False, bool(unit_diagonal))
        except _lib.DDRError as e:
            log.error(f"HIP triangular sparse solve failed: {e}")
            raise ValueError(f"HIP triangular sparse solver failed: {e}") from e
        ctx.save_for_backward(A_values, crow_indices, col_indices, x, b)
        ctx.crow_h, ctx.col_h = crow_h, col_h
        ctx.lower = lower
        ctx.unit_diagonal = bool(unit_diagonal)
        return x

    @staticmethod
    def backward(ctx, grad_output):
        A_values, crow_indices, col_indices, x, b = ctx.saved_tensors
        gradb = _tri_solve(A_values, ctx.crow_h, ctx.col_h, grad_output.contiguous(), bool(ctx.lower), True,
                           ctx.unit_diagonal)
        gradA = None
        if A_values.requires_grad:
            gradA = torch.empty(A_values.shape, device=A_values.device, dtype=torch.float32)
            crow_d = crow_indices.to(device=A_values.device, dtype=torch.int64).contiguous()
            col_d = col_indices.to(device=A_values.device, dtype=torch.int64).contiguous()
            gb = gradb.to(torch.float32).contiguous()
            xx = x.to(torch.float32).contiguous()
            _lib.check(_lib.load().ddr_tri_grad_values(crow_d.numel() - 1, col_d.numel(), crow_d.data_ptr(),
                                                       col_d.data_ptr(), gb.data_ptr(), xx.data_ptr(),
                                                       gradA.data_ptr(), _lib.stream_ptr(A_values.device)))
            gradA = gradA.to(A_values.dtype)
        return gradA, None, None, gradb, None, None, None


triangular_sparse_solve = TriangularSparseSolver.apply

__all__ = [
    "PatternMapper", "denormalize", "get_network_idx", "triangular_sparse_solve", "TriangularSparseSolver",
    "_fill_row_indices_vectorized", "_compute_row_indices_gpu",
]

