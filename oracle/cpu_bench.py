"""Basin-parallel CPU baseline: one oracle-port process per core over disjoint basins.  TEST INFRASTRUCTURE.

Used only by ``bench.py``'s ``cpu_baseline`` leg (never by the product path).  Each worker routes its own
C5-shaped sub-forest (a different seed: disjoint basins of the same size law) through the oracle port of the
reference recipe -- per step fp32 element-wise physics and SciPy's fp64 ``spsolve_triangular``, then the hand
adjoint with the transposed solve per step (``mc_oracle.route`` / ``route_backward``) -- on one thread.  This is
the "N processes (one per core) on disjoint basins" figure of SURVEY.md section 8(d): outlet basins share nothing,
so the reference's single-process routing parallelises across processes this way.
"""

from __future__ import annotations

import os
import time


def run_sample(seed: int, reaches: int, basins: int, largest: float, T: int, grad: bool, x_const=None,
               ranges=None) -> tuple[int, float, float]:
    """Route one C5-shaped sample forward (+ backward); returns (reach-steps, seconds, wall-clock start)."""
    os.environ["OMP_NUM_THREADS"] = "1"
    import numpy as np

    from ddr_amd import synthetic
    from oracle import mc_oracle as O

    sample = synthetic.forest(synthetic.zipf_sizes(reaches, basins, largest), seed=seed, single_inflow=0.35)
    no = O.Network.from_coo(sample.n, sample.rows, sample.cols)
    no.solver = "scipy"
    at = synthetic.reach_attributes(sample.n, seed, x_const=x_const)
    u = synthetic.unit_parameters(sample.n, seed)
    r = O.Reaches(O.denormalize(u["n"], ranges["n"]), O.denormalize(u["q_spatial"], ranges["q_spatial"]),
                  O.denormalize(u["p_spatial"], ranges["p_spatial"], True), at.length,
                  np.maximum(at.slope, np.float32(1e-3)), at.x)
    qp = synthetic.lateral_inflow(sample.n, T, seed)
    W = np.random.default_rng(seed).uniform(0, 1, (sample.n, T)).astype(np.float32) if grad else None
    wall0 = time.time()
    t0 = time.perf_counter()
    res = O.route(no, r, qp, O.Bounds(), dtype=np.float32)
    if grad:
        O.route_backward(no, r, qp, res["x"], W, O.Bounds())
    return sample.n * (T - 1), time.perf_counter() - t0, wall0


def basin_parallel(procs: int, reaches: int, basins: int, largest: float, T: int, grad: bool, x_const, ranges,
                   seed0: int = 100) -> dict:
    """`procs` single-threaded worker processes (``python -m oracle.cpu_bench``: fresh interpreters, no GPU
    state), one disjoint sample each.  The rate is the sum of the workers' reach-steps over the wall time from
    the first worker's start of routing to the last one's end (wall clocks; imports excluded)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parent.parent)
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1",
               PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    spec = json.dumps({"reaches": reaches, "basins": basins, "largest": largest, "T": T, "grad": grad,
                       "x_const": x_const, "ranges": ranges})
    ps = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_bench", str(seed0 + i), spec], cwd=root, env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for i in range(procs)]
    res = []
    for p in ps:
        out, err = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"cpu_bench worker failed: {err[-400:]}")
        res.append(json.loads(out.strip().splitlines()[-1]))
    wall = max(r["end"] for r in res) - min(r["start"] for r in res)
    rs = sum(r["reach_steps"] for r in res)
    return {"value": rs / wall, "processes": procs, "wall_s": wall,
            "per_process_value": [round(r["reach_steps"] / r["seconds"]) for r in res]}


if __name__ == "__main__":
    import json
    import sys

    seed, spec = int(sys.argv[1]), json.loads(sys.argv[2])
    rs, sec, start = run_sample(seed, spec["reaches"], spec["basins"], spec["largest"], spec["T"], spec["grad"],
                                spec["x_const"], spec["ranges"])
    print(json.dumps({"reach_steps": rs, "seconds": sec, "start": start, "end": time.time()}))
