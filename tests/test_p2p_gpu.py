"""One-shot P2P all-reduce (h2omx/parallel/p2p.py, csrc/p2p_kernels.hip).

GPU: two ranks share the one MI355X of the development box and map each
other's symmetric buffers through IPC (the same code path as xGMI peers on an
8-GPU node); results are checked against exact host sums, eagerly and from a
replayed HIP graph, and a strong-scaled 2-rank GBM run with the collectives
inside ONE step graph must reproduce the 1-rank trees bit for bit.
CPU: the availability agreement (any rank failing disables P2P everywhere)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeComm:
    def __init__(self, rank, world, errs):
        import torch

        self.rank, self.world_size, self.device = rank, world, torch.device("cpu")
        self._errs = errs
        self.p2p_error = None

    def all_gather_object(self, obj):
        out = list(self._errs)
        out[self.rank] = obj
        return out


def test_p2p_setup_disabled_everywhere_when_one_rank_fails():
    from h2omx.parallel.p2p import P2PUnavailable, setup

    # this rank (CPU device) cannot set up P2P either; the peer reports its own error
    c = _FakeComm(0, 2, [None, "P2PUnavailable: hipIpcOpenMemHandle failed"])
    assert setup(c) is None
    assert "rank 1" in c.p2p_error and "rank 0" in c.p2p_error
    with pytest.raises(P2PUnavailable):
        setup(_FakeComm(0, 2, [None, None]), required=True)


def test_comm_routes_to_rccl_without_p2p():
    from h2omx.parallel.comm import Comm

    c = Comm(0, 1)
    assert c.p2p is None and not c.graph_collectives
    assert "p2p_calls" in c.collective_stats()


@pytest.mark.gpu
def test_p2p_allreduce_two_ranks_one_gpu():
    env = dict(os.environ, H2OMX_DIST_BACKEND="gloo", H2OMX_P2P="1", OMP_NUM_THREADS="2",
               H2OMX_P2P_TIMEOUT_S="10")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "_p2p_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    # the two ranks share stdout: their JSON objects may land on one line
    dec, outs, txt, i = json.JSONDecoder(), [], r.stdout, 0
    while True:
        i = txt.find('{"rank"', i)
        if i < 0:
            break
        obj, i = dec.raw_decode(txt, i)
        outs.append(obj)
    assert len(outs) == 2, r.stdout
    for o in outs:
        assert o["p2p"], o
        bad = {k: v for k, v in o["checks"].items() if v is False}
        assert not bad, (o["rank"], bad)
    # float results are identical on both ranks (rank-order summation)
    for k in ("torch.float64_digest", "torch.float32_digest"):
        assert outs[0]["checks"][k] == outs[1]["checks"][k]


def _bench(nproc, extra, env_extra, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="2", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--steps", "3", "--warmup", "1"] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
def test_gbm_two_ranks_p2p_one_graph_reproduces_one_rank(tmp_path):
    """Strong scaling with the P2P collectives captured in the step graph: zero
    host-issued collectives per timed tree, trees bit-identical to one rank."""
    import numpy as np

    from test_bench_contract import _assert_same_trees

    extra = ["--rows", "300000", "--scaling", "strong", "--instrument-steps", "2", "--fit-trees", "0"]
    one, two = tmp_path / "one.npy", tmp_path / "two.npy"
    o1 = _bench(1, extra + ["--dump-trees", str(one)], {})
    o2 = _bench(2, extra + ["--dump-trees", str(two)], {"H2OMX_DIST_BACKEND": "gloo", "H2OMX_P2P": "1"})
    assert o2["collective_transport"].startswith("p2p"), o2["collective_transport"]
    assert o1["graph_replay"] and o2["graph_replay"]
    assert o2["collectives_host_issued_per_tree"] == 0
    # device-side exchanges, each inside a kernel the 1-rank step also runs:
    # 5 fused level reduce + split scans and the leaf finalisation
    assert o2["allreduce_calls_per_tree"] == 6
    _assert_same_trees(np.load(one), np.load(two), exact_values=True)
    assert o1["train_auc"] == o2["train_auc"]


def _ranks(txt):
    dec, outs, i = json.JSONDecoder(), [], 0
    while True:
        i = txt.find('{"rank"', i)
        if i < 0:
            return outs
        obj, i = dec.raw_decode(txt, i)
        outs.append(obj)


@pytest.mark.gpu
def test_p2p_timeout_fails_the_fit():
    """Rank 1 stalls past the P2P timeout before tree 6: the survivor's exchanges
    time out on the device, abort every rank's exchanges, and BOTH ranks' GBM
    jobs end FAILED with PeerLost - no model is returned from timed-out sums."""
    env = dict(os.environ, H2OMX_DIST_BACKEND="gloo", H2OMX_P2P="1", OMP_NUM_THREADS="2",
               H2OMX_P2P_TIMEOUT_S="2", H2OMX_FAULT_STALL="1:6:5")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "_p2p_fault_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    outs = _ranks(r.stdout)
    assert len(outs) == 2, r.stdout + r.stderr[-2000:]
    for o in outs:
        assert o["p2p"], o
        assert o["job_status"] == "FAILED", o
        assert o["job_exception"].startswith("PeerLost"), o
        assert not o["model_returned"], o


@pytest.mark.gpu
def test_loopback_proxy_runs_the_n_rank_sequence():
    """bench.py --loopback-ranks 4: one GPU runs the 4-rank step (fused P2P level
    exchanges and leaf exchange against its own buffers) as one graph replay."""
    out = _bench(1, ["--rows", "200000", "--loopback-ranks", "4", "--instrument-steps", "2", "--fit-trees", "0"],
                 {})
    assert out["loopback"]["ranks"] == 4
    assert out["collective_transport"].startswith("p2p loopback")
    assert out["graph_replay"]
    assert out["collectives_host_issued_per_tree"] == 0
    assert out["allreduce_calls_per_tree"] == 6
    assert out["ms_per_step"] > 0
