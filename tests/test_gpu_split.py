"""A basin split across ranks (ddr_amd.split) routes bitwise like the same graph on one rank: two or
three processes share cuda:0 (the one-GPU rehearsal; the receive memory goes through IPC handles and
system-scope granules exactly as between GPUs), each runs its range of the logical blocks, and the
reaches each owns match the single-process launch bit for bit, forward and gradients, over two
consecutive launches (the device hand-shake's epochs advance)."""

import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import split_worker as W

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("math,world", [("exact", 2), ("faithful", 2), ("exact", 3)])
def test_split_basin_processes_bitwise(cuda, tmp_path, math, world):
    from ddr_amd.graph import RiverGraph

    net, at, u, qp, Wt = W.case()
    g = RiverGraph(net.n, net.rows, net.cols, **W.GRAPH_KW)
    assert g.info.n_blocks >= 4 and g.info.n_cut > 0
    ref = W.route_once(g, net, at, u, qp, Wt, math, cuda)
    ref_b = W.route_once(g, net, at, u, W.second_inputs(qp), Wt, math, cuda)
    port = _free_port()
    outs = [str(tmp_path / f"r{r}.npz") for r in range(world)]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "split_worker.py"), str(r), str(world), str(port),
                               outs[r], math], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=150)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("split workers timed out")
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-3000:] for l in logs)
    got = [np.load(o) for o in outs]
    assert all(int(d["fp"]) == g.fingerprint() for d in got)  # the same graph on every rank
    assert int(got[0]["n_x"]) > 0  # the split really crosses ranks
    owned = [d["owned"] for d in got]
    assert np.array_equal(np.sort(np.concatenate(owned)), np.arange(net.n))  # a partition of the reaches
    for d, own in zip(got, owned):
        # launches 0, 1: forward + backward each; 2, 3: forward A, forward B, backward A, backward B
        for i, r in ((0, ref), (1, ref), (2, ref), (3, ref_b)):
            assert np.array_equal(d[f"{i}_runoff"][own], r["runoff"][own]), i
            for k in ("g_n", "g_q_spatial", "g_p_spatial"):
                assert np.array_equal(d[f"{i}_{k}"][own], r[k][own]), (i, k)
        assert d["nan_col0"] and d["nan_qlast"] and d["own_finite"]
        assert d["gauge_refused"]
