"""Where the drop-in dmc() step's time goes at C5: the trainer's call path
(torch_mc.forward -> setup_inputs -> forward, then backward) timed piece by piece against the bench's
direct ops.route step.  Usage: python tools/dropin_breakdown.py [--reaches N] [--T T] > out.json"""

import argparse
import json
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import scipy.sparse as sp  # noqa: E402

from ddr_amd import synthetic  # noqa: E402
from ddr_amd.routing import dmc  # noqa: E402

RANGES = {"n": [0.015, 0.25], "q_spatial": [0.0, 1.0], "p_spatial": [1.0, 200.0]}


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reaches", type=int, default=800_000)
    ap.add_argument("--T", type=int, default=8760)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    net = synthetic.forest(synthetic.zipf_sizes(args.reaches, max(1, 3000 * args.reaches // 800_000), 0.35), seed=5,
                           single_inflow=0.35)
    at = synthetic.reach_attributes(net.n, 11)
    u = synthetic.unit_parameters(net.n, 11)
    qprime = synthetic.lateral_inflow_torch(net.n, args.T, seed=11, device=dev)
    W = torch.rand((net.n, args.T), device=dev)
    a = sp.coo_matrix((np.ones(len(net.rows), np.float32), (net.rows, net.cols)), shape=(net.n, net.n)).tocsr()
    adj = torch.sparse_csr_tensor(torch.from_numpy(a.indptr.astype(np.int64)), torch.from_numpy(a.indices.astype(np.int64)),
                                  torch.from_numpy(a.data), size=(net.n, net.n))
    rd = SimpleNamespace(adjacency_matrix=adj, length=torch.from_numpy(at.length), slope=torch.from_numpy(at.slope),
                         x=torch.from_numpy(at.x), top_width=torch.empty(0), side_slope=torch.empty(0), outflow_idx=None,
                         gage_catchment=None, observations=None, flow_scale=None)
    out = {"reaches": net.n, "T": args.T}
    for math in ("exact", "faithful"):
        params = SimpleNamespace(parameter_ranges=RANGES, log_space_parameters=["p_spatial"], defaults={"p_spatial": 21},
                                 attribute_minimums={"discharge": 1e-4, "slope": 1e-3, "velocity": 0.01, "depth": 0.01,
                                                     "bottom_width": 0.01}, routing_math=math)
        model = dmc(SimpleNamespace(params=params), device=dev)
        spp = {k: torch.from_numpy(u[k]).to(dev).requires_grad_(True) for k in ("n", "q_spatial", "p_spatial")}
        eng = model.routing_engine

        def one():
            o = model(routing_dataclass=rd, streamflow=qprime, spatial_parameters=spp)["runoff"]
            o.backward(W)

        def setup():
            eng.setup_inputs(routing_dataclass=rd, streamflow=qprime, spatial_parameters=spp)

        def fwd():
            with torch.no_grad():
                eng.forward()

        def nan_check():
            bool(torch.isnan(eng.q_prime.sum()))

        def mapper():
            eng.create_pattern_mapper()

        r = {"dmc_fwd_bwd_ms": timed(one), "setup_inputs_ms": timed(setup), "nan_check_ms": timed(nan_check),
             "pattern_mapper_ms": timed(mapper)}
        setup()
        r["forward_nograd_ms"] = timed(fwd)
        from ddr_amd.routing.mmc import compute_hotstart_discharge

        m, _, _ = eng.create_pattern_mapper()
        r["hotstart_ms"] = timed(lambda: compute_hotstart_discharge(eng.q_prime[0], m, eng.discharge_lb, dev))
        out[math] = r
        print(json.dumps({math: r}), file=sys.stderr, flush=True)
        del model, eng
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
