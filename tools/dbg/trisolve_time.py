"""Per-call time of the per-step triangular solve API at 800k reaches (cached plan after call 1)."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, ".")
from ddr_amd import synthetic
from ddr_amd.routing.utils import triangular_sparse_solve
import scipy.sparse as sp
dev = torch.device("cuda:0")
net = synthetic.forest(synthetic.zipf_sizes(800_000, 3000, 0.35), seed=5, single_inflow=0.35)
n = net.n
A = sp.coo_matrix((-0.3 * np.ones(len(net.rows)), (net.rows, net.cols)), shape=(n, n)) + sp.identity(n)
A = A.tocsr(); A.sort_indices()
crow = torch.from_numpy(A.indptr.astype(np.int64)); col = torch.from_numpy(A.indices.astype(np.int64))
vals = torch.from_numpy(A.data.astype(np.float32)).to(dev)
b = torch.rand(n, device=dev)
for i in range(4):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    x = triangular_sparse_solve(vals, crow, col, b, True, False, dev)
    torch.cuda.synchronize(); print(f"call {i}: {1e3 * (time.perf_counter() - t0):.1f} ms")
