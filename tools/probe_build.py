"""Graph build latency on an idle device: the on-device builder vs the host builder + upload, for the C3
training-stream batches (~0.9-1.07M reaches) and the C5 forest."""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from ddr_amd import synthetic  # noqa: E402
from ddr_amd.graph import RiverGraph  # noqa: E402

out = []
nets = [(f"c3_stream_{k}", synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 100 + k), seed=100 + k,
                                             single_inflow=0.25), 2136) for k in range(4)]
nets.append(("c5", synthetic.forest(synthetic.zipf_sizes(800_000, 3000, 0.35), seed=5, single_inflow=0.35), 8760))
dev = torch.device("cuda:0")
for name, net, T in nets:
    rows = torch.from_numpy(net.rows).to(dev)
    cols = torch.from_numpy(net.cols).to(dev)
    rec = {"name": name, "reaches": net.n}
    for mode in ("device", "host"):
        ts = []
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "device":
                g = RiverGraph(net.n, rows, cols, steps_hint=T)
            else:
                g = RiverGraph(net.n, net.rows, net.cols, steps_hint=T)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            fp = g.fingerprint()
            g.close()
        rec[mode + "_ms"] = [round(t, 2) for t in ts]
        rec[mode + "_fp"] = hex(fp)
    out.append(rec)
    print(json.dumps(rec), flush=True)
