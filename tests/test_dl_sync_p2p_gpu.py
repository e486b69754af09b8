"""Synchronous-gradient DeepLearning over the device P2P path (GPU).

Two ranks share the development box's one MI355X (gloo bootstrap, IPC-mapped
P2P buffers - the code path xGMI peers take on an 8-GPU node).  With
``sync_gradients=True`` the per-layer gradient buckets are all-reduced by P2P
kernels on a side stream (``Comm.all_reduce_bucket_``), so after the first
eager step every update is ONE HIP-graph replay with no host-issued
collective; the replicas must be bit-identical (rank-order sums) and match the
1-rank run on the concatenated mini-batches to fp32 rounding (the sums of the
2 x 256 rows are associated differently, so not bit for bit)."""
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


def _run(nproc, out_dir):
    env = dict(os.environ, H2OMX_DIST_BACKEND="gloo", H2OMX_P2P="1", OMP_NUM_THREADS="2", H2OMX_P2P_TIMEOUT_S="20")
    out_dir.mkdir()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "_dl_sync_worker.py"),
           str(out_dir)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return [json.load(open(out_dir / f"rank{k}.json")) for k in range(nproc)]


@pytest.mark.gpu
def test_sync_gradients_p2p_one_graph_bit_identical_replicas(tmp_path):
    two = _run(2, tmp_path / "two")
    one = _run(1, tmp_path / "one")[0]
    a, b = two
    assert a["p2p"] and b["p2p"]
    assert a["tspi"] == 2 * 256
    # replicas agree bit for bit
    assert a["digest"] == b["digest"]
    # the first step runs eagerly (P2P kernels launched from Python, no host-issued
    # RCCL / gloo call), the second is captured; every later step is one graph
    # replay that issues no collective at all
    assert all(s["host"] == 0 for s in a["steps"]), a["steps"]
    assert a["steps"][0]["p2p"] > 0
    assert all(s["graph"] for s in a["steps"][1:]), a["steps"]
    assert len(a["steps"]) > 10 and all(s["p2p"] == 0 for s in a["steps"][2:]), a["steps"]
    # vs one rank on the concatenated batches: the same training up to fp32 rounding
    wa, w1 = np.asarray(a["w"]), np.asarray(one["w"])
    assert wa.shape == w1.shape
    rel = np.abs(wa - w1).max() / np.abs(w1).max()
    assert rel < 2e-4, rel
