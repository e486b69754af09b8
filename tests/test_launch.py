"""One rank per GPU: the local-rank launcher (h2omx/runtime/launch.py), the
node entry point's ranks-per-pod contract and bench.py's own spawning.

CPU tests run the ranks over gloo; the RCCL test needs >= 2 GPUs (skipped on
the one-GPU box, run by the driver's multi-GPU node)."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
WORKER = os.path.join(HERE, "_launch_worker.py")


def _cpu_env(**kw):
    return dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2", **kw)


def _reachable(tr):
    keep, stack = [], [0]
    while stack:
        i = stack.pop()
        keep.append(i)
        if tr[i]["feat"] >= 0:
            stack += [int(tr[i]["left"]), int(tr[i]["left"]) + 1]
    return sorted(keep)


def _same_trees(a, b, exact_values):
    assert a.shape[0] == b.shape[0]
    for t in range(a.shape[0]):
        keep = _reachable(a[t])
        assert keep == _reachable(b[t]), f"tree {t} shape"
        for f in ("feat", "bin", "na_left"):
            np.testing.assert_array_equal(a[t][keep][f], b[t][keep][f], err_msg=f"tree {t} {f}")
        if exact_values:
            np.testing.assert_array_equal(a[t][keep]["value"], b[t][keep]["value"])
        else:
            np.testing.assert_allclose(a[t][keep]["value"], b[t][keep]["value"], rtol=1e-5, atol=1e-7)


def test_launcher_two_ranks_equal_one_rank_cpu(tmp_path):
    one, two = tmp_path / "one.npy", tmp_path / "two.npy"
    subprocess.run([sys.executable, WORKER, str(one)], env=_cpu_env(), check=True, timeout=300)
    r = subprocess.run([sys.executable, "-m", "h2omx.runtime.launch", "--nproc", "2", "--", sys.executable, WORKER,
                        str(two)], env=_cpu_env(), cwd=ROOT, timeout=300)
    assert r.returncode == 0
    _same_trees(np.load(one), np.load(two), exact_values=False)


def test_launcher_stops_peers_when_a_rank_dies():
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-m", "h2omx.runtime.launch", "--nproc", "3", "--", sys.executable, WORKER,
                        "fail:1"], env=_cpu_env(), cwd=ROOT, timeout=120, capture_output=True, text=True)
    assert r.returncode == 3
    assert "local rank 1 exited with 3" in r.stderr
    assert time.monotonic() - t0 < 60          # peers (sleeping 120 s) were terminated


def test_rank_env_contract():
    from h2omx.runtime.launch import rank_env

    e = rank_env({"X": "1"}, 2, 4, 8, 16, "10.0.0.1", 1234)
    assert (e["LOCAL_RANK"], e["RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == ("2", "10", "16", "4")
    assert (e["MASTER_ADDR"], e["MASTER_PORT"], e["X"]) == ("10.0.0.1", "1234", "1")
    k = rank_env({"MASTER_ADDR": "keep"}, 1, 8, 0, 8, None, None)
    assert k["H2OMX_LOCAL_RANK"] == "1" and k["MASTER_ADDR"] == "keep" and "RANK" not in k


def test_statefulset_contract_ranks_per_pod():
    from h2omx.runtime.cluster import config_from_env

    env = {"H2O_KUBERNETES_SERVICE_DNS": "h2o-x-service.ns.svc.cluster.local", "H2O_NODE_EXPECTED_COUNT": "2",
           "H2OMX_GPUS_PER_NODE": "4", "H2OMX_LOCAL_RANK": "3", "POD_NAME": "h2o-x-stateful-set-1"}
    cfg = config_from_env(env)
    assert (cfg.rank, cfg.world_size, cfg.local_rank, cfg.gpus_per_node) == (7, 8, 3, 4)
    assert cfg.master_addr == "h2o-x-stateful-set-0.h2o-x-service.ns.svc.cluster.local"
    # single pod, eight GPUs: ranks 0..7 of one pod
    env.update(H2O_NODE_EXPECTED_COUNT="1", H2OMX_GPUS_PER_NODE="8", H2OMX_LOCAL_RANK="5",
               POD_NAME="h2o-x-stateful-set-0")
    cfg = config_from_env(env)
    assert (cfg.rank, cfg.world_size) == (5, 8)
    env["H2OMX_LOCAL_RANK"] = "8"
    with pytest.raises(ValueError):
        config_from_env(env)


def test_wait_for_peers_counts_pods_not_ranks():
    from h2omx.runtime.cluster import ClusterConfig, wait_for_peers

    cfg = ClusterConfig(rank=0, world_size=8, service_dns="svc", gpus_per_node=4, lookup_timeout_s=1)
    calls = []

    def resolver(*a):
        calls.append(a)
        return [(None, None, None, None, ("10.0.0.1", 0)), (None, None, None, None, ("10.0.0.2", 0))]

    assert wait_for_peers(cfg, resolver=resolver, sleep=lambda s: None) == ["10.0.0.1", "10.0.0.2"]
    # one pod with all the ranks: nothing to wait for
    cfg1 = ClusterConfig(rank=0, world_size=8, service_dns="svc", gpus_per_node=8)
    assert wait_for_peers(cfg1, resolver=lambda *a: pytest.fail("no lookup")) == []


def test_bench_spawns_its_own_ranks_cpu():
    """``bench.py --gpus 2`` outside torchrun starts one child rank per GPU."""
    env = _cpu_env()
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--rows",
                        "4000", "--steps", "2", "--warmup", "1"], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 4000 and out["scaling"] == "strong"   # 4000 rows over 2 ranks


@pytest.mark.gpu
def test_launcher_rccl_two_gpus(tmp_path):
    """RCCL (backend "nccl") between two GPUs of one node, ranks started by the
    launcher: the HIP tree engine's multi-rank model equals the one-rank model
    bit for bit.  Needs >= 2 GPUs: the driver's multi-GPU node runs it."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 GPUs (RCCL between ranks)")
    one, two = tmp_path / "one.npy", tmp_path / "two.npy"
    env = dict(os.environ, H2OMX_WORKER_DEVICE="cuda")
    env.pop("H2OMX_DIST_BACKEND", None)
    subprocess.run([sys.executable, WORKER, str(one)], env=env, check=True, timeout=300)
    r = subprocess.run([sys.executable, "-m", "h2omx.runtime.launch", "--nproc", "2", "--", sys.executable, WORKER,
                        str(two)], env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 0
    _same_trees(np.load(one), np.load(two), exact_values=True)
