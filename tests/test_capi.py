"""The C-ABI library loads and exports every entry point include/ddr_mc.h declares (no GPU needed)."""

import re
from pathlib import Path

import pytest

from ddr_amd import _lib

HEADER = Path(__file__).resolve().parents[1] / "include" / "ddr_mc.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ddr_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "ddr_mc_forward_f32" in names and "ddr_mc_backward_f32" in names and "ddr_graph_build" in names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    assert set(declared_functions()) == set(_lib.EXPORTED)


def test_version_and_error_plumbing():
    lib = _lib.load()
    assert b"gfx950" in lib.ddr_version()
    # a bad call returns a status code and a thread-local message; no exception crosses the ABI
    import ctypes as C

    code = lib.ddr_graph_build(0, 0, None, None, None, C.byref(C.c_void_p()))
    assert code == _lib.DDR_ERR_ARG
    assert b"at least one reach" in lib.ddr_last_error()


def test_pnet_param_count_matches_python():
    from ddr_amd import _lib
    from ddr_amd.pnet import param_count

    lib = _lib.load()
    for F in (1, 7, 10, 12):
        assert int(lib.ddr_pnet_param_count(F)) == param_count(F)
    assert int(lib.ddr_pnet_param_count(13)) == -1


def test_training_tail_refuses_host_tensors():
    """ddr_amd.train runs on the HIP device only: host tensors raise before any library call."""
    import torch

    from ddr_amd.train import ClipAdam, daily_l1_loss

    with pytest.raises(RuntimeError):
        daily_l1_loss(torch.zeros(2, 3), torch.zeros(2, 3), 0)
    with pytest.raises(ValueError):
        ClipAdam(torch.zeros(8))
