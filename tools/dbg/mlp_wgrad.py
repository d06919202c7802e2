"""Micro-benchmark: the C3 parameter network's weight gradients (K = 896k rows) -- hipBLASLt's
default GEMM vs a batched split-K form."""
import time
import torch

dev = torch.device("cuda:0")
N = 896201
for fin, fout in ((10, 128), (128, 128), (128, 3)):
    x = torch.randn(N, fin, device=dev)
    gy = torch.randn(N, fout, device=dev)
    def ref():
        return gy.t() @ x
    def split(B=128):
        k = N // B
        m = B * k
        w = torch.bmm(gy[:m].view(B, k, fout).transpose(1, 2), x[:m].view(B, k, fin)).sum(0)
        if m < N:
            w = w + gy[m:].t() @ x[m:]
        return w
    for f, name in ((ref, "mm"), (split, "bmm-split")):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            w = f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20 * 1e3
        err = (w - ref()).abs().max().item() / ref().abs().max().item()
        print(f"{fin}x{fout} {name}: {dt:.3f} ms  rel err {err:.2e}")
