"""Drop-in replacement of ``ddr.routing`` on the MI355X routing kernels."""

from .mmc import MuskingumCunge, compute_hotstart_discharge
from .torch_mc import dmc
from .utils import PatternMapper, denormalize, get_network_idx, triangular_sparse_solve

__all__ = ["MuskingumCunge", "compute_hotstart_discharge", "dmc", "PatternMapper", "denormalize",
           "get_network_idx", "triangular_sparse_solve"]
