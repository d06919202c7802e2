"""Per-batch gauge union: a training batch's gauge subset adjacencies -> one compressed network.

Mirrors the reference's batch collation (``src/ddr/io/builders.py:55-109`` ``construct_network_matrix``
and the compression steps of ``Merit._collate_gages``, ``src/ddr/geodatazoo/merit.py:197-238``; the
Lynker twin ``lynker_hydrofabric.py:198-266``): union of the subsets' (row, col) pairs,
``active = unique(rows | cols | gauges)`` in CONUS order, the compressed CSR, each gauge's
``outflow_idx`` (the compressed upstream reaches of its reach, or the reach itself for a headwater
gauge) and its compressed index.  The union runs in the C library (``ddr_collate_gauges``:
O(E + n_conus) passes instead of a Python set and dict remaps) and hands the routing graph builder
its COO directly.  The one output that differs in form: each ``outflow_idx`` list is ascending; the
reference lists them in Python ``set`` iteration order (the sum over a gauge's reaches is the same
set of terms).
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass
class CollatedBatch:
    n_conus: int
    active: np.ndarray          # (n,) int64 CONUS ids of the batch's reaches, ascending (merit.py:205-208)
    crow: np.ndarray            # (n + 1,) int64 canonical CSR of the compressed union (merit.py:221-222)
    col: np.ndarray             # (nnz,) int64
    outflow_idx: list           # per gauge: int64 compressed indices (merit.py:227-235)
    gage_compressed_indices: list  # per gauge (merit.py:237)
    gage_idx: list              # per gauge, CONUS index (builders.py:93)
    gage_catchment: list        # per gauge (builders.py:94)

    @property
    def n(self) -> int:
        return int(len(self.active))

    def coo(self) -> tuple[int, np.ndarray, np.ndarray]:
        """(n, rows, cols) int32 of the compressed union, the routing graph builder's input."""
        rows = np.repeat(np.arange(self.n, dtype=np.int32), np.diff(self.crow))
        return self.n, rows, self.col.astype(np.int32)

    def adjacency(self, device=None):
        """``RoutingDataclass.adjacency_matrix``: torch sparse CSR, fp32 values 1 (merit.py:271-279)."""
        import torch

        return torch.sparse_csr_tensor(torch.from_numpy(self.crow), torch.from_numpy(self.col),
                                       torch.ones(len(self.col), dtype=torch.float32), size=(self.n, self.n),
                                       device=device)

    def graph(self, **kw):
        from .graph import RiverGraph

        n, rows, cols = self.coo()
        return RiverGraph(n, rows, cols, **kw)


def collate_gauges(n_conus: int, subsets, gage_catchment=None) -> CollatedBatch:
    """Union of gauge subsets.  ``subsets``: sequence of ``(rows, cols, gage_idx)`` in CONUS numbering
    (rows = downstream reach)."""
    subsets = list(subsets)
    G = len(subsets)
    lens = [len(np.asarray(r)) for r, _, _ in subsets]
    off = np.zeros(G + 1, dtype=np.int64)
    off[1:] = np.cumsum(lens)
    E = int(off[-1])
    rows = np.ascontiguousarray(np.concatenate([np.asarray(r, np.int32).reshape(-1) for r, _, _ in subsets])
                                if G else np.zeros(0, np.int32))
    cols = np.ascontiguousarray(np.concatenate([np.asarray(c, np.int32).reshape(-1) for _, c, _ in subsets])
                                if G else np.zeros(0, np.int32))
    if len(cols) != E:
        raise ValueError("every subset needs as many cols as rows")
    gidx = np.ascontiguousarray(np.array([int(g) for _, _, g in subsets], dtype=np.int32))
    cap = int(min(n_conus, 2 * E + G))
    active = np.empty(max(cap, 1), np.int32)
    crow = np.empty(cap + 1, np.int64)
    col = np.empty(max(E, 1), np.int32)
    out_off = np.empty(G + 1, np.int64)
    out_idx = np.empty(max(E + G, 1), np.int32)
    gage_c = np.empty(max(G, 1), np.int32)
    na = C.c_int64()
    nnz = C.c_int64()
    _lib.check(_lib.load().ddr_collate_gauges(int(n_conus), G, off.ctypes.data, rows.ctypes.data, cols.ctypes.data,
                                              gidx.ctypes.data, active.ctypes.data, C.byref(na), crow.ctypes.data,
                                              col.ctypes.data, C.byref(nnz), out_off.ctypes.data, out_idx.ctypes.data,
                                              len(out_idx), gage_c.ctypes.data))
    n = na.value
    outflow = [out_idx[out_off[g]:out_off[g + 1]].astype(np.int64) for g in range(G)]
    return CollatedBatch(int(n_conus), active[:n].astype(np.int64), crow[:n + 1].copy(), col[:nnz.value].astype(np.int64),
                         outflow, [int(x) for x in gage_c[:G]], [int(x) for x in gidx],
                         list(gage_catchment) if gage_catchment is not None else [None] * G)


def collate_batch(batch, gages_adjacency) -> CollatedBatch:
    """``Merit._collate_gages``' network half (merit.py:197-238): keep the batch's gauges present in
    the gages-adjacency store (``np.isin(batch, keys)``, :199-200), read their subsets
    (builders.py:79-97) and form the union."""
    keys = set(gages_adjacency.keys())
    batch = [b for b in np.asarray(batch).tolist() if b in keys]
    subsets, cats, n_conus = [], [], None
    for gid in batch:
        root = gages_adjacency[gid]
        attrs = dict(root.attrs)
        subsets.append((root["indices_0"][:], root["indices_1"][:], attrs["gage_idx"]))
        cats.append(attrs.get("gage_catchment"))
        n_conus = int(attrs["shape"][0])
    if n_conus is None:
        raise ValueError("no gauge of the batch is in the gages-adjacency store")
    return collate_gauges(n_conus, subsets, cats)


def construct_network_matrix(batch, subsets):
    """``builders.construct_network_matrix`` (builders.py:55-109) API: (coo_matrix in CONUS numbering,
    gage_idx list, gage_catchment list).  The union's entries come out in canonical (row, col) order."""
    import scipy.sparse as sp

    cb = collate_batch(batch, subsets)
    n, rows, cols = cb.coo()
    r = cb.active[rows]
    c = cb.active[cols]
    coo = sp.coo_matrix((np.ones(len(r)), (r, c)), shape=(cb.n_conus, cb.n_conus))
    return coo, cb.gage_idx, cb.gage_catchment


@dataclass
class DeviceBatch:
    """The gauge union computed on the device (``ddr_collate_gauges_device``): every array a device
    tensor; ``graph()`` builds the routing schedule on the device from the compressed COO, so nothing
    per reach leaves the device between the zarr subsets and the routing launch."""
    n_conus: int
    active: "torch.Tensor"       # (n,) int32 CONUS ids, ascending
    rows: "torch.Tensor"         # (nnz,) int32 compressed COO (downstream)
    cols: "torch.Tensor"         # (nnz,) int32 (upstream, ascending)
    crow: "torch.Tensor"         # (n + 1,) int64 canonical CSR
    col: "torch.Tensor"          # (nnz,) int32
    out_off: "torch.Tensor"      # (G + 1,) int64
    out_idx: "torch.Tensor"      # int32
    gage_c: "torch.Tensor"       # (G,) int32
    gage_idx: list

    @property
    def n(self) -> int:
        return int(self.active.numel())

    def graph(self, **kw):
        from .graph import RiverGraph

        return RiverGraph(self.n, self.rows, self.cols, **kw)

    def outflow_idx(self) -> list:
        off = self.out_off.cpu().numpy()
        idx = self.out_idx.cpu().numpy().astype(np.int64)
        return [idx[off[g]:off[g + 1]] for g in range(len(off) - 1)]

    def to_host(self) -> CollatedBatch:
        return CollatedBatch(self.n_conus, self.active.cpu().numpy().astype(np.int64), self.crow.cpu().numpy(),
                             self.col.cpu().numpy().astype(np.int64), self.outflow_idx(),
                             [int(x) for x in self.gage_c.cpu().numpy()], list(self.gage_idx), [None] * len(self.gage_idx))


def collate_gauges_device(n_conus: int, subsets, device=None, stream=None) -> DeviceBatch:
    """:func:`collate_gauges` on the device.  ``subsets``: ``(rows, cols, gage_idx)`` in CONUS numbering,
    host arrays or device tensors; they are concatenated on the device."""
    import torch

    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    subsets = list(subsets)
    G = len(subsets)
    with torch.cuda.device(dev):
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        with torch.cuda.stream(st):
            t = lambda a: torch.as_tensor(a).reshape(-1).to(dev, torch.int32)  # noqa: E731
            rows = torch.cat([t(r) for r, _, _ in subsets]) if G else torch.zeros(0, dtype=torch.int32, device=dev)
            cols = torch.cat([t(c) for _, c, _ in subsets]) if G else torch.zeros(0, dtype=torch.int32, device=dev)
            if rows.shape != cols.shape:
                raise ValueError("every subset needs as many cols as rows")
            gidx_list = [int(g) for _, _, g in subsets]
            gidx = torch.tensor(gidx_list, dtype=torch.int32, device=dev)
            E = rows.numel()
            cap = int(min(n_conus, 2 * E + G))
            i32 = dict(dtype=torch.int32, device=dev)
            active = torch.empty(max(cap, 1), **i32)
            rows_c, cols_c, col = (torch.empty(max(E, 1), **i32) for _ in range(3))
            crow = torch.empty(cap + 1, dtype=torch.int64, device=dev)
            out_off = torch.empty(G + 1, dtype=torch.int64, device=dev)
            out_idx = torch.empty(max(E + G, 1), **i32)
            gage_c = torch.empty(max(G, 1), **i32)
        na, nnz = C.c_int64(), C.c_int64()
        _lib.check(_lib.load().ddr_collate_gauges_device(
            int(n_conus), G, E, rows.data_ptr(), cols.data_ptr(), gidx.data_ptr(), active.data_ptr(), cap, C.byref(na),
            rows_c.data_ptr(), cols_c.data_ptr(), C.byref(nnz), crow.data_ptr(), col.data_ptr(), out_off.data_ptr(),
            out_idx.data_ptr(), out_idx.numel(), gage_c.data_ptr(), st.cuda_stream))
    n, k = na.value, nnz.value
    return DeviceBatch(int(n_conus), active[:n], rows_c[:k], cols_c[:k], crow[:n + 1], col[:k], out_off,
                       out_idx[:int(out_off[-1].item()) if G else 0], gage_c[:G], gidx_list)
