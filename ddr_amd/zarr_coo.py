"""Minimal zarr (v3, and v2) reader/writer for the ddr-engine COO adjacency stores.

The engine writes its CONUS adjacency and the per-gauge subset adjacencies as zarr groups holding
1-D arrays ``indices_0`` (downstream reach, int32), ``indices_1`` (upstream reach, int32), ``values``
(uint8) and ``order`` (int32), with the attributes ``format``, ``shape``, ``geodataset`` and, for a
gauge subset, ``gage_idx`` / ``gage_catchment`` (``engine/src/ddr_engine/core/zarr_io.py:7-76,
85-140``; read back by ``coo_from_zarr`` ``:198-245`` and ``ddr.io.readers.read_zarr``
``src/ddr/io/readers.py:58-80``).  zarr-python is not installed in this image, so this module reads
and writes exactly that subset of the format from the published zarr v3 specification: ``zarr.json``
metadata, regular chunk grid, ``default`` (``c/0``) or ``v2`` chunk keys, the ``bytes`` codec with
either endianness and the ``zstd`` / ``gzip`` bytes-to-bytes codecs (zarr-python 3's default array
codec chain is ``bytes`` + ``zstd``); zarr v2 groups (``.zgroup`` / ``.zarray`` / ``.zattrs``) with
``zstd`` / ``zlib`` / ``gzip`` / no compressor are read too.  zstd comes from the system
``libzstd.so.1`` through ctypes.

Parity: unpinned -- the reference ships no zarr fixture and zarr-python cannot run here; the tests
check round trips through this module's writer and hand-built v2/v3 stores against the spec.
"""

from __future__ import annotations

import ctypes as C
import ctypes.util
import gzip
import json
import math
import zlib
from pathlib import Path

import numpy as np

_ZSTD = None


def _zstd():
    global _ZSTD
    if _ZSTD is None:
        name = ctypes.util.find_library("zstd") or "libzstd.so.1"
        lib = C.CDLL(name)
        lib.ZSTD_decompress.restype = C.c_size_t
        lib.ZSTD_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        lib.ZSTD_compress.restype = C.c_size_t
        lib.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
        lib.ZSTD_compressBound.restype = C.c_size_t
        lib.ZSTD_compressBound.argtypes = [C.c_size_t]
        lib.ZSTD_isError.restype = C.c_uint
        lib.ZSTD_isError.argtypes = [C.c_size_t]
        lib.ZSTD_getFrameContentSize.restype = C.c_ulonglong
        lib.ZSTD_getFrameContentSize.argtypes = [C.c_void_p, C.c_size_t]
        _ZSTD = lib
    return _ZSTD


def zstd_decompress(buf: bytes, size_hint: int) -> bytes:
    lib = _zstd()
    n = lib.ZSTD_getFrameContentSize(buf, len(buf))
    # the chunk's size is known from the array metadata: a frame declaring more is corrupt (or hostile)
    # and is refused before anything is allocated for it; an undeclared size decompresses into
    # size_hint bytes at most (ZSTD_decompress fails if the content does not fit)
    if n < (1 << 62) and int(n) > int(size_hint):
        raise ValueError(f"corrupt zstd chunk: declares {int(n)} bytes, the chunk holds at most {int(size_hint)}")
    cap = int(n) if n < (1 << 62) else int(size_hint)
    out = C.create_string_buffer(max(cap, 1))
    r = lib.ZSTD_decompress(out, cap, buf, len(buf))
    if lib.ZSTD_isError(r):
        raise ValueError("corrupt zstd chunk")
    return out.raw[:r]


def zstd_compress(buf: bytes, level: int = 0) -> bytes:
    lib = _zstd()
    cap = lib.ZSTD_compressBound(len(buf))
    out = C.create_string_buffer(cap)
    r = lib.ZSTD_compress(out, cap, buf, len(buf), int(level))
    if lib.ZSTD_isError(r):
        raise ValueError("zstd compression failed")
    return out.raw[:r]


_V3_DTYPES = {"bool": "?", "int8": "i1", "int16": "i2", "int32": "i4", "int64": "i8", "uint8": "u1", "uint16": "u2",
              "uint32": "u4", "uint64": "u8", "float32": "f4", "float64": "f8"}


class Array:
    """A 1-D (or n-D, C order) zarr array read whole: ``arr[:]`` returns a NumPy array."""

    def __init__(self, path: Path):
        self.path = Path(path)
        if (self.path / "zarr.json").exists():
            m = json.loads((self.path / "zarr.json").read_text())
            if m.get("node_type") != "array":
                raise ValueError(f"{path} is not a zarr array")
            self.v = 3
            self.shape = tuple(m["shape"])
            self.dtype = np.dtype(_V3_DTYPES[m["data_type"]])
            if m["chunk_grid"]["name"] != "regular":
                raise ValueError("only regular chunk grids are supported")
            self.chunks = tuple(m["chunk_grid"]["configuration"]["chunk_shape"])
            enc = m.get("chunk_key_encoding", {"name": "default"})
            self.sep = enc.get("configuration", {}).get("separator", "/" if enc["name"] == "default" else ".")
            self.prefix = "c" if enc["name"] == "default" else None
            self.fill = m.get("fill_value", 0)
            self.codecs = m["codecs"]
            self.attrs = m.get("attributes", {})
        elif (self.path / ".zarray").exists():
            m = json.loads((self.path / ".zarray").read_text())
            self.v = 2
            self.shape = tuple(m["shape"])
            self.dtype = np.dtype(m["dtype"])
            self.chunks = tuple(m["chunks"])
            self.sep = m.get("dimension_separator", ".")
            self.prefix = None
            self.fill = m.get("fill_value", 0) or 0
            if m.get("order", "C") != "C" or m.get("filters"):
                raise ValueError("only C-order zarr v2 arrays without filters are supported")
            self.compressor = m.get("compressor")
            za = self.path / ".zattrs"
            self.attrs = json.loads(za.read_text()) if za.exists() else {}
        else:
            raise FileNotFoundError(f"no zarr array at {path}")

    def _decode(self, raw: bytes, n_items: int) -> np.ndarray:
        dt = self.dtype
        if self.v == 2:
            c = self.compressor
            if c is not None:
                cid = c["id"]
                if cid == "zstd":
                    raw = zstd_decompress(raw, n_items * dt.itemsize)
                elif cid == "zlib":
                    raw = zlib.decompress(raw)
                elif cid == "gzip":
                    raw = gzip.decompress(raw)
                else:
                    raise ValueError(f"unsupported zarr v2 compressor {cid!r}")
            return np.frombuffer(raw, dtype=dt).astype(dt.newbyteorder("="), copy=False)
        for codec in reversed(self.codecs):  # decode runs the chain backwards
            name = codec["name"]
            if name == "zstd":
                raw = zstd_decompress(raw, n_items * dt.itemsize)
            elif name == "gzip":
                raw = gzip.decompress(raw)
            elif name == "bytes":
                endian = codec.get("configuration", {}).get("endian", "little")
                dt = dt.newbyteorder("<" if endian == "little" else ">") if dt.itemsize > 1 else dt
            elif name == "crc32c":
                raw = raw[:-4]  # checksum not verified (no crc32c in the standard library)
            else:
                raise ValueError(f"unsupported zarr v3 codec {name!r}")
        return np.frombuffer(raw, dtype=dt).astype(self.dtype.newbyteorder("="), copy=False)

    def _key(self, idx) -> Path:
        parts = [str(i) for i in idx]
        if self.prefix is not None:
            return self.path / self.sep.join([self.prefix] + parts)
        return self.path / self.sep.join(parts)

    def __getitem__(self, sl) -> np.ndarray:
        if sl != slice(None):
            raise IndexError("only whole-array reads ([:]) are supported")
        out = np.full(self.shape, self.fill, dtype=self.dtype.newbyteorder("="))
        if out.size == 0:
            return out
        grid = [max(1, math.ceil(s / c)) for s, c in zip(self.shape, self.chunks)]
        for idx in np.ndindex(*grid):
            f = self._key(idx)
            if not f.exists():
                continue  # missing chunk: fill value
            block = self._decode(f.read_bytes(), int(np.prod(self.chunks))).reshape(self.chunks)
            dst = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, self.chunks, self.shape))
            out[dst] = block[tuple(slice(0, d.stop - d.start) for d in dst)]
        return out


class Group:
    """A zarr group: ``group[name]`` is a child :class:`Group` or :class:`Array`; ``attrs`` a dict."""

    def __init__(self, path: Path):
        self.path = Path(path)
        if (self.path / "zarr.json").exists():
            m = json.loads((self.path / "zarr.json").read_text())
            if m.get("node_type") != "group":
                raise ValueError(f"{path} is not a zarr group")
            self.attrs = m.get("attributes", {})
        elif (self.path / ".zgroup").exists():
            za = self.path / ".zattrs"
            self.attrs = json.loads(za.read_text()) if za.exists() else {}
        else:
            raise FileNotFoundError(f"no zarr group at {path}")

    def __getitem__(self, name: str):
        p = self.path / str(name)
        if (p / "zarr.json").exists():
            kind = json.loads((p / "zarr.json").read_text()).get("node_type")
            return Group(p) if kind == "group" else Array(p)
        if (p / ".zgroup").exists():
            return Group(p)
        if (p / ".zarray").exists():
            return Array(p)
        raise KeyError(name)

    def __contains__(self, name) -> bool:
        p = self.path / str(name)
        return any((p / f).exists() for f in ("zarr.json", ".zgroup", ".zarray"))

    def keys(self) -> list[str]:
        return sorted(c.name for c in self.path.iterdir() if c.is_dir() and str(c.name) in self)


def read_zarr(path) -> Group:
    """``ddr.io.readers.read_zarr`` (readers.py:58-80): open a store read-only."""
    path = Path(path)
    if not path.exists():
        raise FileNotFoundError(f"Cannot find file: {path}")
    return Group(path)


def coo_from_zarr(path) -> tuple[int, np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """``coo_from_zarr`` (zarr_io.py:198-245) without SciPy objects: (n, rows, cols, values, order)."""
    g = read_zarr(path)
    shape = g.attrs["shape"]
    return (int(shape[0]), g["indices_0"][:].astype(np.int32), g["indices_1"][:].astype(np.int32),
            g["values"][:], g["order"][:])


# ---------------------------------------------------------------------------------------------------
# writer (zarr v3, bytes + zstd: zarr-python 3's default codec chain) -- used to build test stores
# ---------------------------------------------------------------------------------------------------

def _write_array(path: Path, data: np.ndarray, chunk: int, level: int = 0) -> None:
    path.mkdir(parents=True, exist_ok=True)
    data = np.ascontiguousarray(data)
    dt = {v: k for k, v in _V3_DTYPES.items()}[data.dtype.str.lstrip("<>|=")]
    chunk = max(1, int(chunk))
    meta = {"zarr_format": 3, "node_type": "array", "shape": list(data.shape), "data_type": dt,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": [chunk]}},
            "chunk_key_encoding": {"name": "default", "configuration": {"separator": "/"}},
            "fill_value": 0, "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                                        {"name": "zstd", "configuration": {"level": level, "checksum": False}}],
            "attributes": {}, "dimension_names": None, "storage_transformers": []}
    (path / "zarr.json").write_text(json.dumps(meta))
    for i in range(max(1, math.ceil(data.shape[0] / chunk)) if data.size else 0):
        blk = np.zeros(chunk, dtype=data.dtype.newbyteorder("<"))
        part = data[i * chunk:(i + 1) * chunk]
        blk[:len(part)] = part
        f = path / "c" / str(i)
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_bytes(zstd_compress(blk.tobytes(), level))


def _write_group(path: Path, attrs: dict) -> None:
    path.mkdir(parents=True, exist_ok=True)
    (path / "zarr.json").write_text(json.dumps({"zarr_format": 3, "node_type": "group", "attributes": attrs}))


def coo_to_zarr(path, n: int, rows, cols, order=None, attrs: dict | None = None, chunk: int = 1 << 16) -> None:
    """The engine's COO group layout (zarr_io.py:85-140): indices_0/1 int32, values uint8, order int32."""
    path = Path(path)
    rows = np.asarray(rows, np.int32)
    cols = np.asarray(cols, np.int32)
    a = {"format": "COO", "shape": [int(n), int(n)],
         "data_types": {"indices_0": "int32", "indices_1": "int32", "values": "uint8"}}
    a.update(attrs or {})
    _write_group(path, a)
    _write_array(path / "indices_0", rows, chunk)
    _write_array(path / "indices_1", cols, chunk)
    _write_array(path / "values", np.ones(len(rows), np.uint8), chunk)
    _write_array(path / "order", np.asarray(order if order is not None else np.arange(n), np.int32), chunk)


def gauge_subsets_to_zarr(path, n_conus: int, subsets: dict, chunk: int = 1 << 16) -> None:
    """A gages-adjacency store: one COO subgroup per gauge id, attrs gage_idx / gage_catchment / shape
    (the engine's gauge subsets, read by builders.py:55-109).  ``subsets[id] = (rows, cols, gage_idx,
    gage_catchment)``."""
    path = Path(path)
    _write_group(path, {"format": "gages_adjacency"})
    for gid, (rows, cols, gidx, gcat) in subsets.items():
        coo_to_zarr(path / str(gid), n_conus, rows, cols, order=np.zeros(0, np.int32),
                    attrs={"gage_idx": int(gidx), "gage_catchment": gcat}, chunk=chunk)
