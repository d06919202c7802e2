"""Device copy rate for the q' gather's byte count (the gather reads q' and writes the same bytes once):
a plain D2D copy of a (T, N) fp32 array and a torch clone, timed with HIP events.  Usage: python tools/copy_bw.py [N] [T]"""
import sys

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 800_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 8760
a = torch.rand((T, N), device="cuda", dtype=torch.float32)
b = torch.empty_like(a)
for name, fn in (("copy_", lambda: b.copy_(a)), ("add_", lambda: torch.add(a, 0.0, out=b))):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"{name}: {ms:.2f} ms for {2 * a.numel() * 4 / 1e9:.1f} GB moved = {2 * a.numel() * 4 / ms / 1e9:.2f} TB/s", flush=True)
