"""dmc module plumbing on the CPU (reference tests/routing/test_torch_mc.py:30-122, 280-337): construction,
device moves (.to / .cpu / .cuda route through .to), progress info, state_dict extras.  No routing runs here:
the routing itself is HIP-only (a CPU forward raises, as tested on the device)."""

from unittest.mock import patch

import torch

from conftest import PARAMS_MOCK, cfg_of
from ddr_amd.routing import MuskingumCunge, dmc


def test_init_and_routing_engine():
    cfg = cfg_of(PARAMS_MOCK)
    assert dmc(cfg, device=None).device_num == "cpu"
    model = dmc(cfg, device="cpu")
    assert isinstance(model.routing_engine, MuskingumCunge)
    assert model.routing_engine.device == "cpu" and model.routing_engine.cfg == cfg


def test_device_moves():
    model = dmc(cfg_of(PARAMS_MOCK), device="cpu")
    assert model.to("cpu") is model and model.device_num == "cpu" and model.routing_engine.device == "cpu"
    assert model.t.device.type == "cpu"
    assert model.to(torch.device("cpu")) is model and model.device_num == "cpu"
    assert model.cpu() is model and model.routing_engine.device == "cpu"
    for arg, want in ((None, "cuda"), (0, "cuda:0"), (torch.device("cpu"), "cpu")):
        with patch.object(model, "to") as to:
            to.return_value = model
            assert (model.cuda() if arg is None else model.cuda(arg)) is model
            to.assert_called_once_with(want)


def test_progress_info_and_state_dict_extras():
    model = dmc(cfg_of(PARAMS_MOCK), device="cpu")
    model.set_progress_info(epoch=4, mini_batch=9)
    assert model.epoch == 4 and model.mini_batch == 9
    assert model.routing_engine.epoch == 4 and model.routing_engine.mini_batch == 9
    sd = model.state_dict()
    assert sd["epoch"] == 4 and sd["mini_batch"] == 9 and "cfg" in sd
    m2 = dmc(cfg_of(PARAMS_MOCK), device="cpu")
    m2.load_state_dict(sd)
    assert m2.epoch == 4 and m2.mini_batch == 9
