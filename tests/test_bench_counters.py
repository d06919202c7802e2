"""bench.counter_file labels a bench line with PMC counters only when they were measured on the same
shard: the same build, T, reach count, world size and split role (an N > 1 or split
rank's line must not carry the one-GPU whole-network counters)."""

import json

import bench


def _write(tmp_path, **kw):
    d = {"build": "abc", "T": 8760, "reaches": 800_000, "kernels": {}, **kw}
    (tmp_path / "profiles" / "counters").mkdir(parents=True, exist_ok=True)
    (tmp_path / "profiles" / "counters" / "c5.json").write_text(json.dumps(d))


def test_counters_key_on_the_rank_shard(tmp_path):
    _write(tmp_path)
    cf = lambda **kw: bench.counter_file(**{"workload": "c5", "T": 8760, "lib_hash": "abc", "reaches": 800_000,  # noqa: E731
                                            "world": 1, "split": None, "root": tmp_path, **kw})
    assert cf() is not None
    assert cf(lib_hash="other") is None
    assert cf(T=720) is None
    assert cf(reaches=134_000) is None            # a split rank's owned reaches
    assert cf(world=8) is None                    # the same count on another world size
    assert cf(split=(0, 3)) is None               # a split-group rank
    assert bench.counter_file("c3", 2136, "abc", 800_000, root=tmp_path) is None  # no file


def test_counters_measured_on_a_split_rank_match_only_that_rank(tmp_path):
    _write(tmp_path, reaches=94_000, world=8, split=[1, 3])
    assert bench.counter_file("c5", 8760, "abc", 94_000, 8, (1, 3), root=tmp_path) is not None
    assert bench.counter_file("c5", 8760, "abc", 94_000, 8, (2, 3), root=tmp_path) is None
    assert bench.counter_file("c5", 8760, "abc", 94_000, 8, None, root=tmp_path) is None
