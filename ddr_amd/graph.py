"""River graph handle: the device-resident schedule the routing kernels run on.

Replaces the reference's per-forward ``PatternMapper`` construction (``routing/utils.py:25-163``,
``mmc.py:445-458``; rebuilt twice per forward there) with one validated, partitioned graph built
once per adjacency and cached.

Input is the ddr-engine COO contract (``engine/src/ddr_engine/core/zarr_io.py:7-76``): row =
downstream reach, column = upstream reach, strictly lower triangular (topological order), dendritic.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass(frozen=True)
class GraphInfo:
    n: int
    nnz: int
    n_basins: int
    n_pieces: int
    n_blocks: int
    n_cut: int
    max_depth: int
    max_block_depth: int
    reaches_per_thread: int
    save_elems_per_t: int
    save_elems_fixed: int
    bnd_elems_per_t: int
    bwd_elems_per_t: int
    bwd_elems_fixed: int
    status_bytes: int
    generations: int


def adjacency_to_coo(adj) -> tuple[int, np.ndarray, np.ndarray]:
    """(n, rows, cols) of an adjacency given as torch sparse CSR/COO, dense torch/numpy or SciPy sparse.

    Accepts the layouts the reference's ``RoutingDataclass.adjacency_matrix`` takes: sparse CSR in
    production (``merit.py:280-287``), dense in the reference tests (``tests/routing/test_utils.py:81-83``).
    """
    import torch

    if isinstance(adj, torch.Tensor):
        n = int(adj.shape[0])
        if adj.layout == torch.sparse_csr:
            crow = adj.crow_indices().cpu().numpy().astype(np.int64)
            col = adj.col_indices().cpu().numpy().astype(np.int64)
            vals = adj.values().detach().cpu().numpy()
            rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(crow))
            keep = _unit_values(vals)
            return n, rows[keep].astype(np.int32), col[keep].astype(np.int32)
        if adj.layout == torch.sparse_coo:
            a = adj.coalesce()
            idx = a.indices().cpu().numpy()
            vals = a.values().detach().cpu().numpy()
            keep = _unit_values(vals)
            return n, idx[0][keep].astype(np.int32), idx[1][keep].astype(np.int32)
        dense = adj.detach().cpu().numpy()
    else:
        try:
            import scipy.sparse as sp

            if sp.issparse(adj):
                a = adj.tocoo()
                a.sum_duplicates()
                keep = _unit_values(a.data)
                return int(a.shape[0]), a.row[keep].astype(np.int32), a.col[keep].astype(np.int32)
        except ImportError:  # pragma: no cover
            pass
        dense = np.asarray(adj)
    r, c = np.nonzero(dense)
    _unit_values(dense[r, c])
    return int(dense.shape[0]), r.astype(np.int32), c.astype(np.int32)


def _unit_values(vals) -> np.ndarray:
    """Mask of the stored entries that are edges; every edge must have weight 1.

    The routing kernels sum upstream discharge unweighted (the reference's ``torch.matmul(network,
    Q)``, ``mmc.py:535``, with the engine's 0/1 adjacency, ``zarr_io.py:7-76``); a weighted adjacency
    would silently route differently, so it is rejected.
    """
    vals = np.asarray(vals)
    keep = vals != 0
    if np.any(vals[keep] != 1):
        raise ValueError("adjacency values must be 0 or 1 (weighted networks are not supported by the "
                         "fused routing kernels)")
    return keep


def pool_trim() -> int:
    """Release the library's idle pooled blocks (device blocks of device-built / stream-ordered graphs,
    pinned staging): the pools keep freed blocks for reuse (hipFree / hipHostFree synchronise with the
    device), so a trainer whose batch sizes change can return the peak to HIP (``ddr_pool_trim``).
    Returns the bytes released."""
    freed = C.c_int64()
    _lib.check(_lib.load().ddr_pool_trim(C.byref(freed)))
    return int(freed.value)


class RiverGraph:
    """Validated, partitioned river network uploaded to the current HIP device.

    ``rows`` / ``cols`` (the COO, row = downstream reach) may be host arrays -- the host builder
    (``ddr_graph_build``), or ``host_only=True`` for a build that touches no device -- or device
    tensors, or ``on_device=True``: then the whole build runs on the device (``ddr_graph_build_device``,
    north star (1)) on ``stream`` (default: the current stream) and the schedule never leaves it.  Both
    builders emit the same schedule for the same COO (:meth:`fingerprint`).  A host build given a
    ``stream`` uploads its schedule stream-ordered on it (``ddr_graph_build_async``: one pinned staging
    block, one pooled device block, no device-wide synchronisation); its memory is then released
    stream-ordered too (:meth:`close`)."""

    def __init__(self, n: int, rows, cols, *, max_block_reaches: int = 0, target_blocks: int = 0,
                 max_resident: int = 0, steps_hint: int = 0, host_only: bool = False, device=None,
                 on_device: bool | None = None, stream=None):
        lib = _lib.load()
        import torch

        dev_tensor = isinstance(rows, torch.Tensor) and rows.is_cuda
        on_device = dev_tensor if on_device is None else bool(on_device)
        if on_device and host_only:
            raise ValueError("a device build cannot be host-only")
        opts = _lib.BuildOpts(_lib.DDR_BUILD_HOST_ONLY if host_only else 0, int(max_block_reaches),
                              int(target_blocks), int(max_resident), int(steps_hint))
        handle = C.c_void_p()
        self._handle = None
        self.host_only = host_only
        self.device = None
        self.device_built = on_device
        self._stream_ordered = on_device
        if on_device:
            if dev_tensor:
                dev = rows.device
            else:
                dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
            with torch.cuda.device(dev):
                st = stream if stream is not None else torch.cuda.current_stream(dev)
                with torch.cuda.stream(st):
                    r = torch.as_tensor(rows).to(dev, torch.int32).contiguous()
                    c = torch.as_tensor(cols).to(dev, torch.int32).contiguous()
                if r.shape != c.shape:
                    raise ValueError("rows and cols must have the same length")
                _lib.check(lib.ddr_graph_build_device(int(n), r.numel(), r.data_ptr(), c.data_ptr(), C.byref(opts),
                                                      st.cuda_stream, C.byref(handle)))
                # the build may still be running on `st` (the schedule's last kernels): keep the COO alive
                # for the caching allocator until then
                r.record_stream(st)
                c.record_stream(st)
            self.device = dev
        else:
            rows = np.ascontiguousarray(np.asarray(rows, dtype=np.int32))
            cols = np.ascontiguousarray(np.asarray(cols, dtype=np.int32))
            if rows.shape != cols.shape:
                raise ValueError("rows and cols must have the same length")
            if not host_only:
                dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
                self.device = dev
                with torch.cuda.device(dev):
                    if stream is not None:
                        _lib.check(lib.ddr_graph_build_async(int(n), len(rows), rows.ctypes.data, cols.ctypes.data,
                                                             C.byref(opts), stream.cuda_stream, C.byref(handle)))
                        self._stream_ordered = True
                    else:
                        _lib.check(lib.ddr_graph_build(int(n), len(rows), rows.ctypes.data, cols.ctypes.data,
                                                       C.byref(opts), C.byref(handle)))
            else:
                _lib.check(lib.ddr_graph_build(int(n), len(rows), rows.ctypes.data, cols.ctypes.data, C.byref(opts),
                                               C.byref(handle)))
        self._handle = handle
        info = _lib.GraphInfo()
        _lib.check(lib.ddr_graph_get_info(handle, C.byref(info)))
        self.info = GraphInfo(**{f: int(getattr(info, f)) for f, _ in _lib.GraphInfo._fields_})
        self.n = self.info.n

    @classmethod
    def _adopt(cls, handle: C.c_void_p, device, device_built: bool) -> "RiverGraph":
        """Wrap a finished C handle (ddr_graph_build_device_finish)."""
        g = cls.__new__(cls)
        g._handle = handle
        g.host_only = False
        g.device = device
        g.device_built = device_built
        g._stream_ordered = device_built
        info = _lib.GraphInfo()
        _lib.check(_lib.load().ddr_graph_get_info(handle, C.byref(info)))
        g.info = GraphInfo(**{f: int(getattr(info, f)) for f, _ in _lib.GraphInfo._fields_})
        g.n = g.info.n
        return g

    def fingerprint(self) -> int:
        """Hash of the whole schedule (equal for a host and a device build of the same COO)."""
        fp = C.c_uint64()
        _lib.check(_lib.load().ddr_graph_fingerprint(self._handle, C.byref(fp)))
        return int(fp.value)

    # ------------------------------------------------------------------------------------------
    @classmethod
    def from_adjacency(cls, adj, **kw) -> "RiverGraph":
        n, r, c = adjacency_to_coo(adj)
        return cls(n, r, c, **kw)

    def upload(self, device=None, stream=None) -> "RiverGraph":
        """Upload a host-only build to ``device`` (default: the current HIP device); returns self.

        The host build (``host_only=True``) touches no device and releases the GIL inside the C
        call, so it can run on a worker thread while the device routes another batch
        (:class:`GraphPrefetcher`); only this step is on the device's thread.  With ``stream`` the
        upload is stream-ordered on it (``ddr_graph_upload_async``: no host wait)."""
        if not self.host_only:
            return self
        import torch

        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        with torch.cuda.device(dev):
            if stream is not None:
                _lib.check(_lib.load().ddr_graph_upload_async(self._handle, stream.cuda_stream))
                self._stream_ordered = True
            else:
                _lib.check(_lib.load().ddr_graph_upload(self._handle))
        self.device = dev
        self.host_only = False
        return self

    @property
    def handle(self) -> C.c_void_p:
        return self._handle

    def csr(self) -> tuple[np.ndarray, np.ndarray]:
        """Canonical CSR (crow, col) int64 -- bit-exact with ``scipy.sparse...tocsr()``."""
        crow = np.zeros(self.n + 1, dtype=np.int64)
        col = np.zeros(max(self.info.nnz, 1), dtype=np.int64)
        _lib.check(_lib.load().ddr_graph_csr(self._handle, crow.ctypes.data, col.ctypes.data))
        return crow, col[: self.info.nnz]

    def pattern_mapper_layout(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(crow, col, src) of A = I + diag(d) N in the reference PatternMapper layout.

        ``mmc.py:561-584`` + ``utils.py:65-87``: row i holds N's columns ascending, then the diagonal
        (the largest column of a lower-triangular row); off-diagonal slots read ``datvec[i]``, the
        diagonal slot ``datvec[0]``.
        """
        crow, col = self.csr()
        n = self.n
        deg = np.diff(crow)
        crow_a = crow + np.arange(n + 1, dtype=np.int64)
        nnz = int(crow_a[-1])
        col_a = np.empty(nnz, dtype=np.int64)
        src = np.empty(nnz, dtype=np.int64)
        rows = np.repeat(np.arange(n, dtype=np.int64), deg)
        pos_off = crow_a[:-1][rows] + (np.arange(len(col)) - crow[:-1][rows])
        col_a[pos_off] = col
        src[pos_off] = rows
        diag_pos = crow_a[1:] - 1
        col_a[diag_pos] = np.arange(n)
        src[diag_pos] = 0
        return crow_a, col_a, src

    def pattern_mapper_tensors(self, device=None):
        """:meth:`pattern_mapper_layout` as int64 tensors on ``device``, cached per device."""
        import torch

        key = str(torch.device(device)) if device is not None else "cpu"
        cache = self.__dict__.setdefault("_pm_cache", {})
        if key not in cache:
            crow, col, src = (torch.from_numpy(v) for v in self.pattern_mapper_layout())
            cache[key] = tuple(t.to(device) if device is not None else t for t in (crow, col, src))
        return cache[key]

    def structure(self) -> dict[str, np.ndarray]:
        out = {k: np.zeros(self.n, dtype=np.int64) for k in ("down", "dist", "basin", "block")}
        _lib.check(_lib.load().ddr_graph_structure(self._handle, *(out[k].ctypes.data for k in
                                                                   ("down", "dist", "basin", "block"))))
        return out

    def save_numel(self, T: int) -> int:
        """Forward workspace (reals): routing states, then q' in the same schedule layout."""
        return self.info.save_elems_per_t * T + self.info.save_elems_fixed

    def state_numel(self, T: int) -> int:
        """Reals of one schedule-layout (T, N) array (half of :meth:`save_numel`)."""
        return self.save_numel(T) // 2

    def bnd_numel(self, T: int) -> int:
        return self.info.bnd_elems_per_t * T

    def bwd_numel(self, T: int) -> int:
        """Backward workspace in doubles: cut-edge boundary granules + fp64 gradient accumulators."""
        return self.info.bwd_elems_per_t * T + self.info.bwd_elems_fixed

    def close(self) -> None:
        if self._handle is not None and self._handle.value:
            if getattr(self, "_stream_ordered", False):
                # stream-ordered release after the work queued on the current stream (the routing launches
                # that used this graph): no device-wide synchronisation per training batch
                import torch

                _lib.load().ddr_graph_destroy_async(self._handle, torch.cuda.current_stream(self.device).cuda_stream)
            else:
                _lib.load().ddr_graph_destroy(self._handle)
        self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self) -> str:
        i = self.info
        return (f"RiverGraph(n={i.n}, edges={i.nnz}, basins={i.n_basins}, pieces={i.n_pieces}, blocks={i.n_blocks}, "
                f"cut={i.n_cut}, depth={i.max_depth}, kr={i.reaches_per_thread}, generations={i.generations})")


class PendingGraph:
    """A device build begun on a stream (``ddr_graph_build_device_begin``): every device pass up to the
    piece table is enqueued and nothing waits; :meth:`finish` (later, typically a training step on)
    packs the pieces on the host, enqueues the schedule emission on the same stream and returns the
    :class:`RiverGraph`.  Host COO arrays go up through pinned memory, so beginning never blocks."""

    def __init__(self, n: int, rows, cols, *, device=None, stream=None, max_block_reaches: int = 0,
                 target_blocks: int = 0, max_resident: int = 0, steps_hint: int = 0):
        import torch

        if isinstance(rows, torch.Tensor) and rows.is_cuda:
            dev = rows.device
        else:
            dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.device = dev
        self.stream = stream if stream is not None else torch.cuda.current_stream(dev)
        opts = _lib.BuildOpts(0, int(max_block_reaches), int(target_blocks), int(max_resident), int(steps_hint))

        def up(a):
            if isinstance(a, torch.Tensor) and a.is_cuda:
                return a.to(dev, torch.int32).contiguous()
            h = torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).pin_memory()
            return h.to(dev, non_blocking=True)

        with torch.cuda.device(dev), torch.cuda.stream(self.stream):
            # (the pinned host copies are released only after the device copies: the caching host
            # allocator records the stream)
            self._rows, self._cols = up(rows), up(cols)
        if self._rows.shape != self._cols.shape:
            raise ValueError("rows and cols must have the same length")
        h = C.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(_lib.load().ddr_graph_build_device_begin(int(n), self._rows.numel(), self._rows.data_ptr(),
                                                                 self._cols.data_ptr(), C.byref(opts),
                                                                 self.stream.cuda_stream, C.byref(h)))
        self._pending = h

    def finish(self) -> RiverGraph:
        import torch

        if self._pending is None:
            raise RuntimeError("build already finished")
        out = C.c_void_p()
        p, self._pending = self._pending, None
        with torch.cuda.device(self.device):
            _lib.check(_lib.load().ddr_graph_build_device_finish(p, C.byref(out)))
        # the COO tensors were allocated on the build stream: their memory is reused only in its order
        self._rows = self._cols = None
        return RiverGraph._adopt(out, self.device, True)

    def cancel(self) -> None:
        if self._pending is not None:
            _lib.load().ddr_graph_build_device_cancel(self._pending)
            self._pending = None

    def __del__(self):
        try:
            self.cancel()
        except Exception:
            pass


class GraphPrefetcher:
    """Builds the routing graphs of upcoming batches on host threads, ahead of their use.

    In training every batch is a new gauge union (``merit.py:197-223``: one adjacency per batch), so
    the host build (validation, basin split, workgroup packing: ~0.2-0.3 s at 900k reaches) would
    otherwise sit on the critical path of each step.  ``GraphPrefetcher(coo_iter, workers=k)``
    keeps up to ``depth`` builds in flight on ``workers`` threads (the C build releases the GIL) and
    yields uploaded :class:`RiverGraph` objects in order; the upload (~10 ms) runs on the consumer's
    thread.  ``on_device=True`` builds on the device instead (``ddr_graph_build_device``: each builder
    thread on its own high-priority stream; nothing per reach runs on the host).  ``on_device="inline"``
    (the training loop's choice): :class:`PendingGraph` builds begun ``depth`` batches ahead on the
    consumer's stream, finished when taken -- no threads, and the build's short kernels never wait
    behind the training step's persistent routing launches.  ``coo_iter`` yields ``(n, rows, cols)`` or ``(n, rows, cols, payload)``; the payload
    (e.g. the batch's RoutingDataclass) is returned alongside the graph.  ``upload=False`` yields the
    host-only builds (upload them with :meth:`RiverGraph.upload`).
    """

    def __init__(self, coo_iter, *, workers: int = 4, depth: int | None = None, device=None, upload: bool = True,
                 on_device: bool | str = False, **build_kw):
        from concurrent.futures import ThreadPoolExecutor

        self._it = iter(coo_iter)
        self._inline = on_device == "inline"
        if self._inline:
            # device builds begun on the consumer's own stream, ``depth`` batches ahead: each next()
            # finishes the oldest (host packing, emission enqueued) and begins the next one -- no
            # threads, no host waits, nothing competing with the training kernels for the device
            self._kw = dict(build_kw)
            self._device = device
            self._depth = max(1, int(depth if depth is not None else 2))
            self._q = []
            self._fill_inline()
            return
        self._on_device = bool(on_device)
        if self._on_device:
            import threading

            import torch

            self._dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
            self._tls = threading.local()  # one build stream per builder thread
        self._pool = ThreadPoolExecutor(max_workers=max(1, int(workers)), thread_name_prefix="ddr-graph")
        self._depth = max(1, int(depth if depth is not None else workers + 1))
        self._kw = dict(build_kw)
        self._device = device
        self._upload = upload
        self._q = []
        self._fill()

    def _build(self, item):
        n, rows, cols, *rest = item
        if self._on_device:
            # the COO goes up on the builder thread's stream and the whole build runs there, beside the
            # training stream (high priority: the build's short kernels are dispatched first in the gaps
            # between the training step's persistent routing launches); the build reads its stream once
            # per split pass and returns with the schedule still in flight -- routing launches wait for
            # it on their own stream
            import torch

            st = getattr(self._tls, "stream", None)
            if st is None:
                st = self._tls.stream = torch.cuda.Stream(self._dev, priority=-1)
            g = RiverGraph(n, rows, cols, on_device=True, device=self._dev, stream=st, **self._kw)
            return g, (rest[0] if rest else None)
        return RiverGraph(n, rows, cols, host_only=True, **self._kw), (rest[0] if rest else None)

    def _fill_inline(self):
        while len(self._q) < self._depth:
            try:
                item = next(self._it)
            except StopIteration:
                break
            n, rows, cols, *rest = item
            self._q.append((PendingGraph(n, rows, cols, device=self._device, **self._kw), rest[0] if rest else None))

    def _fill(self):
        while len(self._q) < self._depth:
            try:
                item = next(self._it)
            except StopIteration:
                break
            self._q.append(self._pool.submit(self._build, item))

    def __iter__(self):
        return self

    def __next__(self):
        if self._inline:
            if not self._q:
                raise StopIteration
            pg, payload = self._q.pop(0)
            g = pg.finish()
            self._fill_inline()
            return g, payload
        if not self._q:
            self._pool.shutdown(wait=False)
            raise StopIteration
        fut = self._q.pop(0)
        self._fill()
        g, payload = fut.result()
        if self._upload:
            g.upload(self._device)
        return g, payload

    def close(self):
        if self._inline:
            for pg, _ in self._q:
                pg.cancel()
            self._q.clear()
            return
        for f in self._q:
            f.cancel()
        self._q.clear()
        self._pool.shutdown(wait=True)
