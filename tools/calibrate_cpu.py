"""Calibrate bench.py's cpu_baseline: the reference itself vs the oracle port on the SAME sample.

BUILD-CONTAINER ONLY (the reference never travels to the GPU box).  Loads the reference's routing
modules with tests/golden/make_golden.py's stub loader, and times on one core, on the bench's C5-shaped
CPU sample (40k reaches, 150 outlet basins, Zipf sizes with the largest 0.35, seed 5, T = 720 h):
  * the reference MuskingumCunge forward + autograd backward (loss = sum(W * runoff)), and its forward
    under torch.no_grad();
  * the oracle port (oracle/mc_oracle.py: fp32 step + SciPy fp64 spsolve_triangular per step, hand
    adjoint with the transposed SciPy solve per step), forward + backward and forward only.
Writes profiles/cpu_calibration.json (read by bench.py on the GPU box); bench.py divides the port's rate measured on the GPU box by
the fwd+bwd (or forward-only) ratio to report the reference-equivalent CPU rate beside it.

Run:  OMP_NUM_THREADS=1 python tools/calibrate_cpu.py [reaches] [T]
"""
import json
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("OMP_NUM_THREADS", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
torch.set_num_threads(1)

from make_golden import PARAMS_DEFAULT, cfg_of, load_reference, routing_dc  # noqa: E402

from ddr_amd import synthetic  # noqa: E402
from oracle import mc_oracle as O  # noqa: E402

reaches = int(sys.argv[1]) if len(sys.argv) > 1 else 40_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 720
RANGES = PARAMS_DEFAULT["parameter_ranges"]
sample = synthetic.forest(synthetic.zipf_sizes(reaches, max(1, 3000 * reaches // 800_000), 0.35), seed=5,
                          single_inflow=0.35)
at = synthetic.reach_attributes(sample.n, 7)
u = synthetic.unit_parameters(sample.n, 7)
qp = synthetic.lateral_inflow(sample.n, T, 7)
W = np.random.default_rng(1).uniform(0, 1, (sample.n, T)).astype(np.float32)
rs = sample.n * (T - 1)
out = {"sample": f"{sample.n} reaches x {T} h, C5-shaped (bench.py cpu_baseline sample)", "reaches": sample.n,
       "T": T, "threads": 1, "nproc": os.cpu_count()}

# ---- the oracle port (what bench.py times on the GPU box) ----
no = O.Network.from_coo(sample.n, sample.rows, sample.cols)
no.solver = "scipy"
r = O.Reaches(O.denormalize(u["n"], RANGES["n"]), O.denormalize(u["q_spatial"], RANGES["q_spatial"]),
              O.denormalize(u["p_spatial"], RANGES["p_spatial"], True), at.length,
              np.maximum(at.slope, np.float32(1e-3)), at.x)
t0 = time.perf_counter()
res = O.route(no, r, qp, O.Bounds(), dtype=np.float32)
t_fwd = time.perf_counter() - t0
O.route_backward(no, r, qp, res["x"], W, O.Bounds())
t_all = time.perf_counter() - t0
out["port"] = {"fwd_bwd": rs / t_all, "fwd_only": rs / t_fwd, "seconds": t_all}
print("port", out["port"], flush=True)

# ---- the reference itself ----
utils, mmc = load_reference()
dc = routing_dc(sample.n, sample.rows, sample.cols, at)
params = cfg_of(PARAMS_DEFAULT)
with torch.no_grad():
    mc = mmc.MuskingumCunge(params, device="cpu")
    spp = {k: torch.from_numpy(v).clone() for k, v in u.items()}
    t0 = time.perf_counter()
    mc.setup_inputs(dc, torch.from_numpy(qp), spp)
    mc.forward()
    t_ref_fwd = time.perf_counter() - t0
print("reference fwd (no_grad)", rs / t_ref_fwd, flush=True)
mc = mmc.MuskingumCunge(params, device="cpu")
spp = {k: torch.from_numpy(v).clone().requires_grad_(True) for k, v in u.items()}
t0 = time.perf_counter()
mc.setup_inputs(dc, torch.from_numpy(qp), spp)
o = mc.forward()
(o * torch.from_numpy(W)).sum().backward()
t_ref = time.perf_counter() - t0
out["reference"] = {"fwd_bwd": rs / t_ref, "fwd_only": rs / t_ref_fwd, "seconds": t_ref + t_ref_fwd}
out["ratio_port_over_reference"] = {"fwd_bwd": out["port"]["fwd_bwd"] / out["reference"]["fwd_bwd"],
                                    "fwd_only": out["port"]["fwd_only"] / out["reference"]["fwd_only"]}
print(json.dumps(out, indent=1), flush=True)
(ROOT / "profiles" / "r03").mkdir(parents=True, exist_ok=True)
(ROOT / "profiles" / "cpu_calibration.json").write_text(json.dumps(out, indent=1) + "\n")
