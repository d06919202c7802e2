"""Host planning of a basin split across ranks (ddr_amd.split): contiguous, balanced block ranges and
the rank plan (the largest basin's group, the other basins LPT over the remaining ranks)."""

import numpy as np

from ddr_amd import synthetic
from ddr_amd.partition import basin_labels
from ddr_amd.split import plan_block_ranks, plan_ranks


def test_block_ranks_contiguous_and_balanced():
    rng = np.random.default_rng(0)
    nloc = rng.integers(100, 400, 768)
    for k in (2, 3, 4, 8):
        r = plan_block_ranks(nloc, k)
        assert r[0] == 0 and r[-1] == k - 1
        assert np.all(np.diff(r) >= 0) and np.all(np.diff(r) <= 1)  # contiguous ticket ranges
        load = np.bincount(r, weights=nloc, minlength=k)
        assert load.max() <= nloc.sum() / k + nloc.max()
    assert list(plan_block_ranks([1, 1], 2)) == [0, 1]


def test_rank_plan_splits_only_a_dominant_basin():
    net = synthetic.forest(synthetic.zipf_sizes(80000, 300, 0.35), seed=5, single_inflow=0.35)
    lab = basin_labels(net.n, net.rows, net.cols)
    big = np.bincount(lab).argmax()
    for world in (1, 2):
        plan = plan_ranks(net.n, net.rows, net.cols, world)
        assert all(s is None for _, s in plan)
        ids = np.concatenate([i for i, _ in plan])
        assert np.array_equal(np.sort(ids), np.arange(net.n))  # every reach exactly once
    # the largest basin (0.35 N) is 1.4 x a rank's share at N = 4 (split over 2 ranks; not with factor 2)
    # and 2.8 x at N = 8 (3 ranks)
    assert all(s is None for _, s in plan_ranks(net.n, net.rows, net.cols, 4, factor=2.0))
    for world, kk in ((4, 2), (8, 3)):
        plan = plan_ranks(net.n, net.rows, net.cols, world)
        groups = [s for _, s in plan if s is not None]
        k = len(groups)
        assert k == max(2, round(np.count_nonzero(lab == big) / (net.n / world))) == kk
        assert [s[1] for s in groups] == list(range(k)) and all(s[0] == list(range(k)) for s in groups)
        for i, _ in plan[:k]:
            assert np.all(lab[i] == big) and len(i) == np.count_nonzero(lab == big)  # the whole basin, on each
        rest = np.concatenate([i for i, _ in plan[k:]])
        assert np.array_equal(np.sort(np.concatenate([plan[0][0], rest])), np.arange(net.n))
    sizes = [len(i) for i, _ in plan[k:]]
    assert max(sizes) < np.count_nonzero(lab == big) / 2  # the others are balanced below the basin's share
    forced = plan_ranks(net.n, net.rows, net.cols, 2, force=True)
    assert all(s is not None for _, s in forced)


def test_block_rank_refinement_cuts_fewer_edges_within_balance():
    # a chain of 4 trees of blocks: each tree's blocks interleaved in ticket order (as piece heights do)
    rng = np.random.default_rng(3)
    nb, k = 400, 4
    tree = np.arange(nb) % 4
    nloc = rng.integers(200, 300, nb)
    prod, cons = [], []
    for t in range(4):
        ids = np.nonzero(tree == t)[0]
        for i in range(1, len(ids)):  # each block feeds the next block of its tree
            prod.append(ids[i - 1])
            cons.append(ids[i])
    prod, cons = np.array(prod), np.array(cons)
    r0 = plan_block_ranks(nloc, k)
    r1 = plan_block_ranks(nloc, k, prod, cons, tol=0.05)
    x0 = np.count_nonzero(r0[prod] != r0[cons])
    x1 = np.count_nonzero(r1[prod] != r1[cons])
    assert x1 < x0
    load = np.bincount(r1, weights=nloc, minlength=k)
    assert load.max() <= nloc.sum() / k * 1.05 + 1 and load.min() >= nloc.sum() / k * 0.95 - 1
    assert np.array_equal(r1, plan_block_ranks(nloc, k, prod, cons, tol=0.05))  # deterministic
