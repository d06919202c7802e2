"""A whole C3-shaped training step captured into one HIP graph (ddr_amd.capture.CapturedStep) replays the
same computation as the eager step: parameter network, daily q' gather, routing forward, daily objective,
routing backward, network backward, clip + Adam -- every piece deterministic, so K replays after the
warm-up leave the parameters bit-identical to K eager steps."""

import numpy as np
import pytest
import torch

from ddr_amd import synthetic
from ddr_amd.capture import CapturedStep
from ddr_amd.graph import RiverGraph
from ddr_amd.ops import DailyWindow, GaugeMap, RouteConsts, route
from ddr_amd.pnet import ParamNet
from ddr_amd.train import ClipAdam, daily_l1_loss

pytestmark = pytest.mark.gpu

RANGES = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}


def _setup(dev):
    net = synthetic.forest(synthetic.zipf_sizes(20000, 40, 0.2), seed=7, single_inflow=0.3)
    T = 24 * 6
    at = synthetic.reach_attributes(net.n, 7)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    length, slope, xs = tt(at.length), tt(np.maximum(at.slope, np.float32(1e-3))), tt(at.x)
    feats = tt(synthetic.reach_features(net.n, seed=7))
    qprime = tt(synthetic.lateral_inflow(net.n, T // 24, 7))
    outlets = np.flatnonzero(net.down < 0)
    gz = GaugeMap.build([np.array([o]) for o in outlets], net.n, dev)
    window = DailyWindow.for_training(T)
    obs = tt(np.random.default_rng(8).lognormal(np.log(5.0), 1.0, (len(outlets), window.D)).astype(np.float32))
    g = RiverGraph(net.n, net.rows, net.cols, steps_hint=T)
    model = ParamNet(10, RANGES).to(dev)
    opt = ClipAdam(model.flat, lr=1e-3, max_norm=1.0)

    def step():
        opt.zero_grad(set_to_none=True)
        n, q, p = model(feats)
        daily, _, _, _ = route(g, qprime, n, q, p, length, slope, xs, gauges=gz, daily=window, consts=RouteConsts(),
                               math="faithful", steps=T, qprime_hours=24)
        daily_l1_loss(daily, obs, 1).backward()
        opt.step()

    return model, opt, step


def test_captured_c3_step_replays_the_eager_step(cuda):
    K = 4
    model_e, opt_e, step_e = _setup(cuda)
    for _ in range(K):
        step_e()
    torch.cuda.synchronize()
    model_g, opt_g, step_g = _setup(cuda)
    cap = CapturedStep(step_g, warmup=1, device=cuda)  # one eager step, then the capture (which runs nothing)
    for _ in range(K - 1):
        cap()
    torch.cuda.synchronize()
    assert float(opt_g.step_count.item()) == K
    np.testing.assert_array_equal(model_g.flat.detach().cpu().numpy(), model_e.flat.detach().cpu().numpy())
    np.testing.assert_array_equal(opt_g.m.cpu().numpy(), opt_e.m.cpu().numpy())
    assert not np.array_equal(model_g.flat.detach().cpu().numpy(),
                              ParamNet(10, RANGES).flat.detach().numpy())  # the steps did train
