"""Multi-rank GPU training equals single-rank training bit for bit.

Two ranks share the box's single MI355X (collectives over gloo; RCCL needs
one GPU per rank).  Histograms and leaf sums are exact integers and the
stochastic-rounding dither / bagging hash use global row ids, so the trees
grown from two row shards must be identical to the trees grown from all rows
on one rank."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("dist,depth,sr,n,split", [
    ("bernoulli", 5, 1.0, 30001, 0.5),
    ("gaussian", 6, 0.7, 30001, 0.5),
    # 200k + 400k rows: on their own the two shards would pick different
    # fixed-point scales (2^15 vs 2^14 per max|g|); the ranks must agree on one
    ("bernoulli", 4, 1.0, 600000, 1 / 3),
])
def test_two_ranks_equal_one_rank(cuda_dev, tmp_path, dist, depth, sr, n, split):
    worker = os.path.join(HERE, "_multirank_worker.py")
    one = tmp_path / "one.npy"
    extra = [str(n), str(split)]
    subprocess.run([sys.executable, worker, str(one), dist, str(depth), str(sr), *extra], check=True, timeout=300)
    two = tmp_path / "two.npy"
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), H2OMX_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, worker, str(two), dist, str(depth), str(sr), *extra],
                                      env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    a, b = np.load(one), np.load(two)
    assert a.shape == b.shape
    for t in range(a.shape[0]):
        keep, stack = [], [0]
        while stack:
            i = stack.pop()
            keep.append(i)
            if a[t][i]["feat"] >= 0:
                stack += [int(a[t][i]["left"]), int(a[t][i]["left"]) + 1]
        for f in ("feat", "bin", "na_left", "value"):
            np.testing.assert_array_equal(a[t][keep][f], b[t][keep][f], err_msg=f"tree {t} field {f}")
