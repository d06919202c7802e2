"""The routing kernels' steady-tick path (every reach of a block runs a step in [1, T - 1]: no activity
tests, no hot-start or carried-state case) is the general tick with those branches removed: outputs and
gradients are bitwise those of the general path (DDR_DEBUG_NO_STEADY), for every forward arithmetic,
carried state, gauge mode and partition."""

import numpy as np
import pytest
import torch

from conftest import synthetic_case
from ddr_amd import _lib, synthetic
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import GaugeMap, route

pytestmark = pytest.mark.gpu


def _run(case, dev, g, math, q0=None, gauges=None, no_steady=False, flags=None):
    lib = _lib.load()
    _lib.check(lib.ddr_set_debug_flags(flags if flags is not None else (_lib.DDR_DEBUG_NO_STEADY if no_steady else 0)))
    try:
        tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, torch.float32)  # noqa: E731
        u = {k: tt(case.u[k]).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial")}
        n = u["n"] * 0.2 + 0.02
        q = u["q_spatial"]
        p = torch.exp(u["p_spatial"] * 5.0)
        runoff, q_last, tw, ss = route(g, tt(case.qprime), n, q, p, tt(case.length), tt(np.maximum(case.slope, 1e-3)),
                                       tt(case.x), gauges=gauges, q0=None if q0 is None else tt(q0), math=math)
        W = torch.from_numpy(np.random.default_rng(5).uniform(0, 1, tuple(runoff.shape)).astype(np.float32)).to(dev)
        (runoff * W).sum().backward()
        torch.cuda.synchronize()
        out = {"runoff": runoff.detach().cpu().numpy(), "q_last": q_last.detach().cpu().numpy(),
               "tw": tw.detach().cpu().numpy(), "ss": ss.detach().cpu().numpy()}
        out.update({f"g_{k}": v.grad.cpu().numpy() for k, v in u.items()})
        return out
    finally:
        _lib.check(lib.ddr_set_debug_flags(0))


@pytest.mark.parametrize("math", ["exact", "faithful", "fast"])
@pytest.mark.parametrize("part", ["whole", "cut"])
@pytest.mark.parametrize("carry", [False, True], ids=["hot", "carry"])
def test_steady_path_is_bitwise_the_general_path(cuda, math, part, carry):
    net = synthetic.forest(synthetic.loguniform_sizes(12, 50, 3000, 7), seed=7)
    T = 300
    case = synthetic_case(net, T, 7)
    gkw = {} if part == "whole" else {"max_block_reaches": 256, "target_blocks": 1 << 20}
    g = RiverGraph(net.n, net.rows, net.cols, **gkw)
    assert g.info.max_depth + 2 < T  # steady ticks exist
    q0 = np.random.default_rng(8).uniform(0.1, 5.0, net.n).astype(np.float32) if carry else None
    a = _run(case, cuda, g, math, q0=q0)
    b = _run(case, cuda, g, math, q0=q0, no_steady=True)
    for k in a:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


def test_steady_path_gauge_mode(cuda):
    net = synthetic.forest(synthetic.loguniform_sizes(10, 50, 2000, 9), seed=9)
    case = synthetic_case(net, 240, 9)
    g = RiverGraph(net.n, net.rows, net.cols, max_block_reaches=256, target_blocks=1 << 20)
    outlets = np.flatnonzero(net.down < 0)
    gz = GaugeMap.build([np.array([o]) for o in outlets], net.n, cuda)
    a = _run(case, cuda, g, "faithful", gauges=gz)
    b = _run(case, cuda, g, "faithful", gauges=gz, no_steady=True)
    for k in a:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


@pytest.mark.parametrize("T", [300, 302], ids=["rows16B", "ragged"])
def test_storer_waves_are_bitwise_the_compute_wave_stores(cuda, T):
    """Light blocks (<= 512 reaches, one per thread) store x_save / runoff from their idle upper waves in
    the forward, and import the cut-outs' (A, B) granules on them in the backward (requested ahead of the
    chunk boundary) and publish each reach's x(t - 4) from x_save ahead of time; outputs and gradients equal
    the compute-wave stores, imports and x loads bit for bit (T % 4 != 0: per-step runoff stores)."""
    net = synthetic.forest(synthetic.loguniform_sizes(12, 50, 3000, 11), seed=11)
    case = synthetic_case(net, T, 11)
    g = RiverGraph(net.n, net.rows, net.cols, max_block_reaches=256, target_blocks=1 << 20)
    assert g.info.reaches_per_thread == 1
    assert g.info.n_cut > 0  # cut edges: the backward imports run
    q0 = np.random.default_rng(12).uniform(0.1, 5.0, net.n).astype(np.float32)
    outlets = np.flatnonzero(net.down < 0)
    gz = GaugeMap.build([np.array([o]) for o in outlets], net.n, cuda)
    for kw in ({}, {"q0": q0}, {"gauges": gz}):
        a = _run(case, cuda, g, "faithful", flags=0, **kw)
        b = _run(case, cuda, g, "faithful", flags=_lib.DDR_DEBUG_NO_STORER, **kw)
        for k in a:
            assert np.array_equal(a[k], b[k], equal_nan=True), k


@pytest.mark.parametrize("cap", [256, 1536, 4096], ids=["kr1", "kr2", "kr4"])
def test_plain_instances_are_bitwise_the_general_ones(cuda, cap):
    """Launches without the rare options (split basin, block profile, state seeds, daily accumulation) run
    kernel instances compiled without them (route.hip, PL); outputs and gradients equal the general
    instances' (DDR_DEBUG_NO_PLAIN) bit for bit, per-reach runoff and gauge mode, at one, two and four reaches
    per thread."""
    net = synthetic.forest(synthetic.loguniform_sizes(10, 200, 12000, 13), seed=13)
    T = 200
    case = synthetic_case(net, T, 13)
    g = RiverGraph(net.n, net.rows, net.cols, max_block_reaches=cap, target_blocks=16)
    assert g.info.reaches_per_thread == {256: 1, 1536: 2, 4096: 4}[cap]
    outlets = np.flatnonzero(net.down < 0)
    gz = GaugeMap.build([np.array([o]) for o in outlets], net.n, cuda)
    for kw in ({}, {"gauges": gz}):
        a = _run(case, cuda, g, "faithful", flags=0, **kw)
        b = _run(case, cuda, g, "faithful", flags=_lib.DDR_DEBUG_NO_PLAIN, **kw)
        for k in a:
            assert np.array_equal(a[k], b[k], equal_nan=True), k

