"""Data-parallel direct deep-tree levels (engine._direct_dp): two ranks sharing
the one GPU grow, from their row shards, the forest one rank grows from all
rows - bit for bit."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, out):
    env = dict(os.environ, H2OMX_DIST_BACKEND="gloo", OMP_NUM_THREADS="2", H2OMX_TREE_ENGINE="seg")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "_dp_direct_worker.py"), str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    i = r.stdout.find('{"rank"')
    assert i >= 0, r.stdout
    return json.JSONDecoder().raw_decode(r.stdout, i)[0]


@pytest.mark.gpu
def test_direct_levels_two_ranks_reproduce_one_rank(tmp_path):
    from test_bench_contract import _assert_same_trees

    one, two = tmp_path / "one.npy", tmp_path / "two.npy"
    o1 = _run(1, one)
    o2 = _run(2, two)
    assert o1["segmented"] and o2["segmented"]
    assert o1["direct_dp_levels"] == 0 and o2["direct_dp_levels"] > 0, (o1, o2)
    _assert_same_trees(np.load(one), np.load(two), exact_values=True)
