"""Per-batch gauge union (ddr_collate_gauges) and the zarr COO stores it reads.

Pinned by tests/golden/collate.npz: the reference's own ``construct_network_matrix``
(builders.py:55-109) and ``Merit._collate_gages`` (merit.py:197-238) run on synthetic gauge subsets
(make_golden.py make_collate).  The zarr reader/writer has no reference fixture (parity unpinned):
round trips and a hand-built zarr v2 store.
"""

import json
import zlib

import numpy as np
import pytest

from conftest import load_golden
from ddr_amd import _lib, synthetic
from ddr_amd.batching import collate_batch, collate_gauges, construct_network_matrix
from ddr_amd.zarr_coo import Array, coo_from_zarr, coo_to_zarr, gauge_subsets_to_zarr, read_zarr


def subsets_of(d):
    off = d["sub_off"]
    return [(d["sub_rows"][off[g]:off[g + 1]], d["sub_cols"][off[g]:off[g + 1]], int(d["gage_idx"][g]))
            for g in range(len(off) - 1)]


def check_against_reference(cb, d):
    np.testing.assert_array_equal(cb.active, d["ref_divide_ids"] - 500000)  # merit_ids[active]
    np.testing.assert_array_equal(cb.crow, d["ref_crow"])
    np.testing.assert_array_equal(cb.col, d["ref_col"])
    assert cb.gage_idx == d["ref_gage_idx"].tolist()
    assert cb.gage_compressed_indices == np.searchsorted(cb.active, d["ref_gage_idx"]).tolist()
    roff = d["ref_outflow_off"]
    for g, o in enumerate(cb.outflow_idx):
        ref = d["ref_outflow_flat"][roff[g]:roff[g + 1]]
        np.testing.assert_array_equal(o, np.sort(ref))  # reference lists are in set iteration order


def test_collate_matches_reference_golden():
    d = load_golden("collate")
    batch = d["batch"].tolist()
    keep = [i for i, b in enumerate(d["gage_ids"].tolist()) if b in batch]
    subs = subsets_of(d)
    cb = collate_gauges(int(d["n_conus"]), [subs[i] for i in keep])
    check_against_reference(cb, d)


def test_construct_network_matrix_and_store_round_trip(tmp_path):
    d = load_golden("collate")
    n = int(d["n_conus"])
    subs = subsets_of(d)
    store = {gid: (r, c, gi, 70000 + k) for k, (gid, (r, c, gi)) in enumerate(zip(d["gage_ids"].tolist(), subs))}
    gauge_subsets_to_zarr(tmp_path / "gages.zarr", n, store, chunk=500)
    g = read_zarr(tmp_path / "gages.zarr")
    assert sorted(g.keys()) == sorted(store)
    cb = collate_batch(d["batch"], g)  # the batch holds one gauge missing from the store
    check_against_reference(cb, d)
    assert cb.gage_catchment == d["ref_gage_catchment_batch"].tolist()
    coo, idx, wb = construct_network_matrix(d["batch"], g)
    pairs = np.array(sorted(zip(coo.row.tolist(), coo.col.tolist()))).reshape(-1, 2)
    np.testing.assert_array_equal(pairs, d["ref_union_pairs"])
    assert idx == d["ref_gage_idx"].tolist() and wb == d["ref_gage_catchment"].tolist()
    # the collated network feeds the graph builder directly; its CSR is the reference's
    from ddr_amd.graph import RiverGraph

    nb, rows, cols = cb.coo()
    crow, col = RiverGraph(nb, rows, cols, host_only=True).csr()
    np.testing.assert_array_equal(crow, d["ref_crow"])
    np.testing.assert_array_equal(col, d["ref_col"])


def test_conus_coo_round_trip(tmp_path):
    net = synthetic.forest(synthetic.zipf_sizes(5000, 30, 0.35), seed=3)
    order = np.arange(net.n, dtype=np.int32) * 7 + 11
    coo_to_zarr(tmp_path / "conus.zarr", net.n, net.rows, net.cols, order=order, attrs={"geodataset": "merit"},
                chunk=1024)
    n, rows, cols, vals, ordr = coo_from_zarr(tmp_path / "conus.zarr")
    assert n == net.n and read_zarr(tmp_path / "conus.zarr").attrs["geodataset"] == "merit"
    np.testing.assert_array_equal(rows, net.rows)
    np.testing.assert_array_equal(cols, net.cols)
    np.testing.assert_array_equal(vals, np.ones(len(net.rows), np.uint8))
    np.testing.assert_array_equal(ordr, order)


def test_zarr_v2_and_missing_chunks(tmp_path):
    """A zarr v2 array (zlib, '.' keys, big-endian) with a missing chunk reads as the fill value."""
    p = tmp_path / "a"
    p.mkdir()
    data = np.arange(10, dtype=">i4")
    (p / ".zarray").write_text(json.dumps({"zarr_format": 2, "shape": [10], "chunks": [4], "dtype": ">i4",
                                           "compressor": {"id": "zlib", "level": 1}, "fill_value": -1,
                                           "order": "C", "filters": None}))
    (p / "0").write_bytes(zlib.compress(data[:4].tobytes()))
    (p / "2").write_bytes(zlib.compress(np.array([8, 9, 0, 0], dtype=">i4").tobytes()))
    got = Array(p)[:]
    assert got.dtype == np.int32 and got.dtype.isnative
    np.testing.assert_array_equal(got, [0, 1, 2, 3, -1, -1, -1, -1, 8, 9])


def test_collate_rejects_bad_unions():
    # reach 0 drains into 1 in one subset and into 2 in another: not a dendritic union
    with pytest.raises(_lib.DDRError) as e:
        collate_gauges(5, [(np.array([1]), np.array([0]), 1), (np.array([2]), np.array([0]), 2)])
    assert e.value.code == _lib.DDR_ERR_NOT_DENDRITIC
    with pytest.raises(_lib.DDRError) as e:
        collate_gauges(5, [(np.array([1]), np.array([3]), 1)])
    assert e.value.code == _lib.DDR_ERR_NOT_LOWER
    # a lone headwater gauge: one reach, outflow_idx = itself
    cb = collate_gauges(5, [(np.zeros(0, np.int32), np.zeros(0, np.int32), 3)])
    assert cb.active.tolist() == [3] and cb.outflow_idx[0].tolist() == [0] and cb.col.size == 0
    # inconsistent subsets: three gauges on reach 3, whose three inflow edges only the
    # first subset holds, need 9 outflow entries against E + G = 6: refused, not written past the end
    empty = (np.zeros(0, np.int32), np.zeros(0, np.int32), 3)
    with pytest.raises(_lib.DDRError) as e:
        collate_gauges(5, [(np.array([3, 3, 3]), np.array([0, 1, 2]), 3), empty, empty])
    assert e.value.code == _lib.DDR_ERR_ARG and "out_idx_cap" in str(e.value)


def test_collate_conus_scale_union_matches_numpy():
    """64 random gauges over a 200k-reach CONUS: the C union equals a NumPy restatement of
    merit.py:204-222 (np.unique + searchsorted remap + scipy tocsr)."""
    import scipy.sparse as sp

    net = synthetic.forest(synthetic.zipf_sizes(200_000, 400, 0.2), seed=5)
    down = net.down
    rng = np.random.default_rng(5)
    gauges = rng.choice(np.flatnonzero(down >= 0), 64, replace=False)
    # each gauge's subset: the edges of its upstream closure (a descending sweep over topological ids)
    subs = []
    for x in gauges:
        inside = np.zeros(net.n, bool)
        inside[x] = True
        for j in range(x - 1, max(-1, x - 20000), -1):
            if down[j] >= 0 and inside[down[j]]:
                inside[j] = True
        inside[x] = False
        ups = np.flatnonzero(inside)
        subs.append((down[ups].astype(np.int32), ups.astype(np.int32), int(x)))
    cb = collate_gauges(net.n, subs)
    r = np.concatenate([s[0] for s in subs]).astype(np.int64)
    c = np.concatenate([s[1] for s in subs]).astype(np.int64)
    key = np.unique(r * net.n + c)
    r, c = key // net.n, key % net.n
    active = np.unique(np.concatenate([r, c, gauges]))
    np.testing.assert_array_equal(cb.active, active)
    a = sp.coo_matrix((np.ones(len(r)), (np.searchsorted(active, r), np.searchsorted(active, c))),
                      shape=(len(active), len(active))).tocsr()
    np.testing.assert_array_equal(cb.crow, a.indptr)
    np.testing.assert_array_equal(cb.col, a.indices)


def test_zstd_frame_larger_than_chunk_is_refused():
    """A frame whose header declares more bytes than the chunk can hold raises before any
    allocation of that size; a well-formed frame decodes."""
    from ddr_amd.zarr_coo import zstd_compress, zstd_decompress

    frame = zstd_compress(np.arange(64, dtype=np.int32).tobytes())
    assert np.array_equal(np.frombuffer(zstd_decompress(frame, 256), np.int32), np.arange(64))
    with pytest.raises(ValueError, match="declares 256 bytes"):
        zstd_decompress(frame, 16)
