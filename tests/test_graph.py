"""Graph construction (host side of ddr_graph_build): bit-exact CSR, dendritic structure, partition.

Runs on CPU (DDR_BUILD_HOST_ONLY: validation + partition without device upload).
Reference targets: scipy ``coo_matrix(...).tocsr()`` (merit.py:197-223) and the PatternMapper layout
(utils.py:25-129, mmc.py:561-584) recorded in tests/golden/csr.npz.
"""

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_golden
from ddr_amd import _lib, synthetic
from ddr_amd.graph import RiverGraph, adjacency_to_coo
from oracle import mc_oracle as O


def host_graph(n, rows, cols, **kw):
    return RiverGraph(n, rows, cols, host_only=True, **kw)


@pytest.mark.parametrize("net", [synthetic.random_binary_tree(2000, 0), synthetic.random_binary_tree(300, 3),
                                 synthetic.forest(synthetic.zipf_sizes(20000, 200, 0.35), seed=1),
                                 synthetic.hack_basin(5000, seed=2)], ids=["c1", "t300", "forest", "hack"])
def test_csr_bit_exact_vs_scipy(net):
    g = host_graph(net.n, net.rows, net.cols)
    crow, col = g.csr()
    a = sp.coo_matrix((np.ones(len(net.rows), np.float32), (net.rows, net.cols)), shape=(net.n, net.n)).tocsr()
    np.testing.assert_array_equal(crow, a.indptr)
    np.testing.assert_array_equal(col, a.indices)


def test_csr_and_pattern_mapper_vs_reference_golden():
    d = load_golden("csr")
    for tag, net in (("t300", synthetic.random_binary_tree(300, 3)), ("c1", synthetic.random_binary_tree(2000, 0))):
        g = host_graph(net.n, net.rows, net.cols)
        crow, col = g.csr()
        np.testing.assert_array_equal(crow, d[f"{tag}_crow"])
        np.testing.assert_array_equal(col, d[f"{tag}_col"])
        mcrow, mcol, src = g.pattern_mapper_layout()
        np.testing.assert_array_equal(mcrow, d[f"{tag}_mcrow"])
        np.testing.assert_array_equal(mcol, d[f"{tag}_mcol"])
        np.testing.assert_array_equal(src, d[f"{tag}_mapidx"])


def test_unsorted_coo_order_is_canonicalised():
    net = synthetic.random_binary_tree(500, 1)
    perm = np.random.default_rng(0).permutation(len(net.rows))
    g1 = host_graph(net.n, net.rows, net.cols)
    g2 = host_graph(net.n, net.rows[perm], net.cols[perm])
    for a, b in zip(g1.csr(), g2.csr()):
        np.testing.assert_array_equal(a, b)


def test_structure_matches_oracle():
    net = synthetic.forest(synthetic.zipf_sizes(5000, 50, 0.35), seed=4)
    g = host_graph(net.n, net.rows, net.cols)
    s = g.structure()
    o = O.Network.from_coo(net.n, net.rows, net.cols)
    np.testing.assert_array_equal(s["down"], o.down)
    np.testing.assert_array_equal(s["dist"], o.dist)
    assert g.info.n_basins == len(net.basin_sizes)
    assert g.info.max_depth == o.dist.max() + 1


@pytest.mark.parametrize("rows,cols,code", [
    ([0], [1], _lib.DDR_ERR_NOT_LOWER),          # upstream index above downstream: unsorted network
    ([2, 2], [1, 1], _lib.DDR_ERR_DUPLICATE),    # duplicate edge
    ([1, 2], [0, 0], _lib.DDR_ERR_NOT_DENDRITIC),  # reach 0 drains into two reaches
    ([5], [0], _lib.DDR_ERR_ARG),                # index out of range
    ([1], [1], _lib.DDR_ERR_NOT_LOWER),          # self loop
])
def test_invalid_networks_rejected(rows, cols, code):
    with pytest.raises(_lib.DDRError) as e:
        host_graph(3, np.array(rows), np.array(cols))
    assert e.value.code == code
    assert isinstance(e.value, ValueError)


def test_empty_and_single_reach():
    g = host_graph(1, np.zeros(0, np.int32), np.zeros(0, np.int32))
    assert g.info.n_basins == 1 and g.info.n_blocks == 1 and g.info.max_depth == 1
    crow, col = g.csr()
    np.testing.assert_array_equal(crow, [0, 0])
    assert col.size == 0
    g = host_graph(4, np.zeros(0, np.int32), np.zeros(0, np.int32))  # isolated reaches
    assert g.info.n_basins == 4


@pytest.mark.parametrize("cap", [64, 200, 1024])
def test_partition_invariants(cap):
    net = synthetic.forest(synthetic.zipf_sizes(20000, 40, 0.5), seed=7, single_inflow=0.35)
    g = host_graph(net.n, net.rows, net.cols, max_block_reaches=cap, target_blocks=1 << 20, max_resident=1 << 20)
    s = g.structure()
    blk = s["block"]
    counts = np.bincount(blk)
    assert counts.max() <= cap
    assert g.info.n_blocks == len(counts) and counts.min() > 0
    # cut edges = edges whose endpoints live in different blocks
    cut = int(np.sum(blk[net.rows] != blk[net.cols]))
    assert cut == g.info.n_cut
    # block-level dependency graph must be acyclic (deadlock freedom of the persistent launch)
    edges = {(int(a), int(b)) for a, b in zip(blk[net.cols], blk[net.rows]) if a != b}
    indeg = np.zeros(len(counts), np.int64)
    adj = [[] for _ in counts]
    for a, b in edges:
        adj[a].append(b)
        indeg[b] += 1
    stack = [i for i in range(len(counts)) if indeg[i] == 0]
    seen = 0
    while stack:
        v = stack.pop()
        seen += 1
        for w in adj[v]:
            indeg[w] -= 1
            if indeg[w] == 0:
                stack.append(w)
    assert seen == len(counts), "block dependency graph has a cycle"
    # ticket order (route.hip take_ticket): every producer block precedes its consumers
    assert all(a < b for a, b in edges), "a cut edge runs from a later block to an earlier one"
    # save buffer sizes
    assert g.save_numel(10) == 2 * net.n * 10 + g.info.save_elems_fixed
    assert g.state_numel(10) * 2 == g.save_numel(10)


def test_more_blocks_than_resident_workgroups_build_in_generations():
    """No co-residency ceiling: a graph needing more workgroups than the device holds packs into
    several generations of ticket-ordered blocks (round-1 raised DDR_ERR_CAPACITY here)."""
    net = synthetic.hack_basin(20000, seed=1)
    g = host_graph(net.n, net.rows, net.cols, max_block_reaches=64, max_resident=16)
    assert g.info.n_blocks > 16 and g.info.n_cut > 0
    assert g.info.generations >= -(-g.info.n_blocks // 16)
    s = g.structure()
    blk = s["block"]
    assert np.bincount(blk).max() <= 64
    assert all(a < b for a, b in zip(blk[net.cols], blk[net.rows]) if a != b)


def test_weighted_adjacency_rejected():
    net = synthetic.random_binary_tree(16, 2)
    dense = net.dense()
    dense[net.rows[0], net.cols[0]] = 0.5
    with pytest.raises(ValueError):
        adjacency_to_coo(dense)
    with pytest.raises(ValueError):
        adjacency_to_coo(sp.csr_matrix(dense))


def test_adjacency_layouts_agree():
    import torch

    net = synthetic.random_binary_tree(64, 5)
    dense = net.dense()
    ref = adjacency_to_coo(dense)
    for adj in (torch.from_numpy(dense), torch.from_numpy(dense).to_sparse_csr(), torch.from_numpy(dense).to_sparse(),
                sp.csr_matrix(dense)):
        n, r, c = adjacency_to_coo(adj)
        order = np.lexsort((c, r))
        assert n == ref[0]
        np.testing.assert_array_equal(r[order], ref[1])
        np.testing.assert_array_equal(c[order], ref[2])


def test_prefetcher_builds_match_serial_builds():
    """GraphPrefetcher's worker-thread builds are the same schedules as serial builds, in order."""
    from ddr_amd.graph import GraphPrefetcher

    nets = [synthetic.forest(synthetic.loguniform_sizes(12, 50, 2000, s), seed=s) for s in range(5)]
    pf = GraphPrefetcher(((nt.n, nt.rows, nt.cols, k) for k, nt in enumerate(nets)), workers=3, depth=2,
                         upload=False, max_block_reaches=256, target_blocks=16)
    got = list(pf)
    assert [k for _, k in got] == list(range(5))
    for (g, k), nt in zip(got, nets):
        ref = host_graph(nt.n, nt.rows, nt.cols, max_block_reaches=256, target_blocks=16)
        assert g.info == ref.info
        for key in ("down", "dist", "basin", "block"):
            np.testing.assert_array_equal(g.structure()[key], ref.structure()[key])


def test_generation_fallback_builds_fast():
    """A batch just over the one-generation capacity goes straight to two generations (no futile
    capacity shrinking), and the capacity search stays a handful of packing passes."""
    import time

    net = synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 1), seed=1, single_inflow=0.25)
    t = time.perf_counter()
    # ~1M reaches in 256 mid-size basins: pieces at the full capacity (no dominant basin) fit 256
    # workgroups in one generation; 180 resident workgroups force the two-generation fallback
    g = host_graph(net.n, net.rows, net.cols, steps_hint=2136, max_resident=256, target_blocks=256)
    assert time.perf_counter() - t < 5.0
    assert g.info.generations == 1 and g.info.n_blocks <= 256
    t = time.perf_counter()
    g2 = host_graph(net.n, net.rows, net.cols, steps_hint=2136, max_resident=180, target_blocks=180)
    assert time.perf_counter() - t < 5.0
    assert g2.info.generations == 2 and g2.info.n_blocks <= 360


def test_light_load_blocks_keep_half_a_workgroup(monkeypatch):
    """At light load (block capacity <= 512 reaches, one per thread) no block exceeds 512 reaches: a larger
    one loses the idle helper waves and runs three routing waves per SIMD (route.hip).  C3 8-way shard 3
    packed five ~700-reach blocks before the rule (graph.cpp light_clamp; profiles/r04/ab_r04.txt item 24);
    DDR_PACK_NO_LIGHT_CLAMP restores the previous packing, which the last assertion checks is still the
    case that needs the rule."""
    from ddr_amd.distributed import shard_network

    net = synthetic.forest(synthetic.loguniform_sizes(256, 100, 20000, 3), seed=3, single_inflow=0.25)
    for r in (1, 3):
        n, rows, cols, _ = shard_network(net.n, net.rows, net.cols, r, 8)
        g = host_graph(n, rows, cols, steps_hint=2136)
        nl = np.bincount(g.structure()["block"], minlength=g.info.n_blocks)
        assert g.info.reaches_per_thread == 1 and g.info.generations == 1
        assert nl.max() <= 512, (r, int(nl.max()))
        assert g.info.n_blocks <= 256
    monkeypatch.setenv("DDR_PACK_NO_LIGHT_CLAMP", "1")
    g = host_graph(n, rows, cols, steps_hint=2136)
    assert np.bincount(g.structure()["block"]).max() > 512
