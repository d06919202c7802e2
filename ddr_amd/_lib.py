"""ctypes binding of ``libddr_mc.so`` (the C ABI declared in ``include/ddr_mc.h``).

The library is loaded from ``ddr_amd/lib/libddr_mc.so`` (built in-tree by
``__graft_entry__.build()`` / ``make -C ddr_amd/csrc``).  There is no fallback: if the library is
missing every routing entry point raises ``RuntimeError``.

``torch`` is imported first on purpose: PyTorch-ROCm ships its own ``libamdhip64.so`` (soname
``libamdhip64.so.7``), so the dynamic linker binds this library to the HIP runtime that owns the
caller's device memory and streams.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the library load, see module docstring)

LIB_PATH = Path(os.environ.get("DDR_LIB") or Path(__file__).resolve().parent / "lib" / "libddr_mc.so")

# status codes (include/ddr_mc.h)
DDR_OK = 0
DDR_ERR_ARG = -1
DDR_ERR_NOT_LOWER = -2
DDR_ERR_NOT_DENDRITIC = -3
DDR_ERR_DUPLICATE = -4
DDR_ERR_HIP = -5
DDR_ERR_CAPACITY = -6
DDR_ERR_TIMEOUT = -7
DDR_ERR_SINGULAR = -8

DDR_BUILD_HOST_ONLY = 1

DDR_FWD_SAVE_X = 1
DDR_FWD_CARRY = 2
DDR_FWD_NO_RUNOFF = 4
DDR_FWD_ACCUMULATE = 8
DDR_FWD_FAST_MATH = 16
DDR_FWD_FAITHFUL_MATH = 32
DDR_FWD_CHECK_QPRIME = 64
DDR_BWD_EXACT_ADJOINT = 128

DDR_DEBUG_FORCE_TIMEOUT = 1
DDR_DEBUG_NO_STEADY = 2
DDR_DEBUG_NO_STORER = 4
DDR_DEBUG_NO_PLAIN = 8


class BuildOpts(C.Structure):
    _fields_ = [("flags", C.c_int32), ("max_block_reaches", C.c_int32), ("target_blocks", C.c_int32),
                ("max_resident", C.c_int32), ("steps_hint", C.c_int32)]


class GraphInfo(C.Structure):
    _fields_ = [(name, C.c_int64) for name in (
        "n", "nnz", "n_basins", "n_pieces", "n_blocks", "n_cut", "max_depth", "max_block_depth",
        "reaches_per_thread", "save_elems_per_t", "save_elems_fixed", "bnd_elems_per_t", "bwd_elems_per_t",
        "bwd_elems_fixed", "status_bytes", "generations")]


class Consts(C.Structure):
    _fields_ = [(name, C.c_double) for name in (
        "dt", "discharge_lb", "velocity_lb", "velocity_ub", "depth_lb", "bottom_width_lb", "side_slope_lb",
        "side_slope_ub")]


class Reaches(C.Structure):
    _fields_ = [("n", C.c_void_p), ("q_spatial", C.c_void_p), ("p_spatial", C.c_void_p), ("p_stride", C.c_int64),
                ("length", C.c_void_p), ("slope", C.c_void_p), ("x_storage", C.c_void_p),
                ("flow_scale", C.c_void_p), ("qprime_hours", C.c_int64), ("qprime_valid", C.c_void_p)]


class Gauges(C.Structure):
    _fields_ = [("n_gauges", C.c_int64), ("offsets", C.c_void_p), ("index", C.c_void_p),
                ("reach_offsets", C.c_void_p), ("reach_gauges", C.c_void_p)]


_P = C.c_void_p
_I64 = C.c_int64
_I32 = C.c_int32
_SIGS = {
    "ddr_graph_build": (C.c_int, [_I64, _I64, _P, _P, C.POINTER(BuildOpts), C.POINTER(C.c_void_p)]),
    "ddr_graph_build_device": (C.c_int, [_I64, _I64, _P, _P, C.POINTER(BuildOpts), _P, C.POINTER(C.c_void_p)]),
    "ddr_graph_fingerprint": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "ddr_graph_build_device_begin": (C.c_int, [_I64, _I64, _P, _P, C.POINTER(BuildOpts), _P,
                                               C.POINTER(C.c_void_p)]),
    "ddr_graph_build_device_finish": (C.c_int, [_P, C.POINTER(C.c_void_p)]),
    "ddr_graph_build_device_cancel": (C.c_int, [_P]),
    "ddr_graph_destroy": (C.c_int, [_P]),
    "ddr_graph_destroy_async": (C.c_int, [_P, _P]),
    "ddr_graph_upload": (C.c_int, [_P]),
    "ddr_graph_upload_async": (C.c_int, [_P, _P]),
    "ddr_graph_build_async": (C.c_int, [_I64, _I64, _P, _P, C.POINTER(BuildOpts), _P, C.POINTER(C.c_void_p)]),
    "ddr_pool_trim": (C.c_int, [C.POINTER(C.c_int64)]),
    "ddr_qprime_nan_wait": (C.c_int, [C.POINTER(C.c_int32)]),
    "ddr_collate_gauges": (C.c_int, [_I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "ddr_collate_gauges_device": (C.c_int, [_I64, _I64, _I64, _P, _P, _P, _P, _I64, C.POINTER(C.c_int64), _P, _P,
                                            C.POINTER(C.c_int64), _P, _P, _P, _P, _I64, _P, _P]),
    "ddr_graph_get_info": (C.c_int, [_P, C.POINTER(GraphInfo)]),
    "ddr_graph_csr": (C.c_int, [_P, _P, _P]),
    "ddr_graph_structure": (C.c_int, [_P, _P, _P, _P, _P]),
    "ddr_mc_forward_f32": (C.c_int, [_P, C.POINTER(Consts), C.POINTER(Reaches), _P, _I64, _P, _P, _P, _P, _P, _P,
                                     _P, _P, _I32, _P]),
    "ddr_mc_forward_f64": (C.c_int, [_P, C.POINTER(Consts), C.POINTER(Reaches), _P, _I64, _P, _P, _P, _P, _P, _P,
                                     _P, _P, _I32, _P]),
    "ddr_mc_backward_f32": (C.c_int, [_P, C.POINTER(Consts), C.POINTER(Reaches), _P, _I64, _P, _P, _P,
                                      C.POINTER(Gauges), _P, _P, _P, _P, _P, _I32, _P]),
    "ddr_mc_backward_f64": (C.c_int, [_P, C.POINTER(Consts), C.POINTER(Reaches), _P, _I64, _P, _P, _P,
                                      C.POINTER(Gauges), _P, _P, _P, _P, _P, _I32, _P]),
    "ddr_hotstart_f32": (C.c_int, [_P, _P, C.c_double, _P, _P]),
    "ddr_state_work_bytes": (_I64, [_P, _I64, _I64, _I32]),
    "ddr_mc_backward_state_f32": (C.c_int, [_P, C.POINTER(Consts), C.POINTER(Reaches), _P, _I64, _I64, _P, _P, _P,
                                            C.POINTER(Gauges), _P, _P, _P, _P, _P, _P, _P, _P, _I32, _P]),
    "ddr_mc_backward_state_f64": (C.c_int, [_P, C.POINTER(Consts), C.POINTER(Reaches), _P, _I64, _I64, _P, _P, _P,
                                            C.POINTER(Gauges), _P, _P, _P, _P, _P, _P, _P, _P, _I32, _P]),
    "ddr_mc_backward_ex_f32": (C.c_int, [_P, C.POINTER(Consts), C.POINTER(Reaches), _P, _I64, _I64, _P, _P, _P,
                                         C.POINTER(Gauges), _P, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _P]),
    "ddr_mc_backward_ex_f64": (C.c_int, [_P, C.POINTER(Consts), C.POINTER(Reaches), _P, _I64, _I64, _P, _P, _P,
                                         C.POINTER(Gauges), _P, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _P]),
    "ddr_pnet_param_count": (_I64, [_I32]),
    "ddr_pnet_work_bytes": (_I64, [_I64, _I32]),
    "ddr_pnet_forward_f32": (C.c_int, [_I64, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "ddr_pnet_backward_f32": (C.c_int, [_I64, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "ddr_daily_l1_f32": (C.c_int, [_I64, _I64, _I64, _P, _P, C.c_float, _P, _P, _P]),
    "ddr_clip_adam_work_bytes": (_I64, []),
    "ddr_clip_adam_f32": (C.c_int, [_I64, _P, _P, _P, _P, C.c_float, C.c_float, C.c_float, C.c_float, _P,
                                    C.c_float, _P, _P, _P]),
    "ddr_state_f32": (C.c_int, [_P, _P, _I64, _I64, C.c_double, _I32, _P, _P]),
    "ddr_state_f64": (C.c_int, [_P, _P, _I64, _I64, C.c_double, _I32, _P, _P]),
    "ddr_gauge_reduce_f32": (C.c_int, [_P, _P, _I64, C.POINTER(Gauges), C.c_double, _I32, _P, _P]),
    "ddr_gauge_reduce_f64": (C.c_int, [_P, _P, _I64, C.POINTER(Gauges), C.c_double, _I32, _P, _P]),
    "ddr_gauge_daily_f32": (C.c_int, [_P, _P, _I64, C.POINTER(Gauges), C.c_double, _I32, _I64, _I64, _I64, _P, _P]),
    "ddr_gauge_daily_f64": (C.c_int, [_P, _P, _I64, C.POINTER(Gauges), C.c_double, _I32, _I64, _I64, _I64, _P, _P]),
    "ddr_gauge_daily_seed_f32": (C.c_int, [_I64, _I64, _I64, _I64, _I64, _P, _P, _P]),
    "ddr_gauge_daily_seed_f64": (C.c_int, [_I64, _I64, _I64, _I64, _I64, _P, _P, _P]),
    "ddr_geometry_stats_f32": (C.c_int, [_P, _I64, _I64, _I64, _I64, _P, _P, _I64, _P, _P, C.c_double, C.c_double,
                                         _P, _P]),
    "ddr_graph_status": (C.c_int, [_P, _P]),
    "ddr_xmem_alloc": (C.c_int, [_I64, C.POINTER(C.c_void_p), _P, C.POINTER(C.c_int32)]),
    "ddr_xmem_open": (C.c_int, [_P, C.POINTER(C.c_void_p)]),
    "ddr_xmem_close": (C.c_int, [_P, _I32]),
    "ddr_xmem_bytes": (C.c_int, [_I64, _I64, C.POINTER(C.c_int64)]),
    "ddr_graph_blocks": (C.c_int, [_P, _P, _I64]),
    "ddr_graph_cut_blocks": (C.c_int, [_P, _P, _P, _I64]),
    "ddr_graph_set_split": (C.c_int, [_P, _I32, _I32, _P, _P, _P, _I64, C.POINTER(C.c_int64)]),
    "ddr_graph_clear_split": (C.c_int, [_P]),
    "ddr_status_check": (C.c_int, [_I32]),
    "ddr_set_debug_flags": (C.c_int, [_I32]),
    "ddr_tri_solve": (C.c_int, [_I64, _I64, _P, _P, _P, _P, _P, _I32, _I32, _P]),
    "ddr_tri_solve_ex": (C.c_int, [_I64, _I64, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P]),
    "ddr_tri_grad_values": (C.c_int, [_I64, _I64, _P, _P, _P, _P, _P, _P]),
    "ddr_set_kernel_timing": (C.c_int, [_I32]),
    "ddr_kernel_ms": (C.c_int, [_I32, C.POINTER(C.c_float)]),
    "ddr_set_block_profile": (C.c_int, [_I32, _P]),
    "ddr_device_info": (C.c_int, [C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "ddr_last_error": (C.c_char_p, []),
    "ddr_version": (C.c_char_p, []),
}
EXPORTED = tuple(_SIGS)

_lib = None


def load() -> C.CDLL:
    """Load (once) and return the routing library; raise if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("DDR_MC_LIB", LIB_PATH))
    if not path.exists():
        raise RuntimeError(
            f"libddr_mc.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C ddr_amd/csrc` (there is no CPU fallback)")
    lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
    # an explicitly chosen library (DDR_LIB / DDR_MC_LIB: an A/B variant of an earlier build) may lack
    # entry points added since; the default in-tree library must export every one
    variant = bool(os.environ.get("DDR_LIB") or os.environ.get("DDR_MC_LIB"))
    for name, (res, args) in _SIGS.items():
        if variant and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


class DDRError(ValueError):
    """Error returned by the routing library (a ValueError, like the reference solver's)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"ddr_mc error {code}: {msg}")
        self.code = code


def check(code: int) -> None:
    if code != DDR_OK:
        msg = load().ddr_last_error()
        raise DDRError(code, msg.decode() if msg else "")


def ptr(t) -> int | None:
    """Raw data pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
