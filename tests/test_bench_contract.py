"""bench.py contract: one JSON line from rank 0 with the driver's fields, under
``torch.distributed.run`` with several ranks (gloo on the CPU; two ranks
sharing the one GPU over gloo on a GPU box — the 8-GPU RCCL run is the
driver's).  Rows are scaled down; the code path is the timed one."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, extra, env_extra=None, timeout=600):
    env = dict(os.environ, OMP_NUM_THREADS="2", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--steps", "2", "--warmup", "1"] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == nproc and out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["config"]["parallelism"].startswith(f"dp{nproc}")
    return out


@pytest.mark.parametrize("model,extra", [
    ("gbm-higgs", ["--rows", "6000"]),
    ("dl-mlp", ["--rows", "2048", "--batch", "256"]),
])
def test_bench_two_ranks_cpu(model, extra):
    out = _run(2, ["--device", "cpu", "--model", model] + extra)
    if model == "gbm-higgs":
        assert out["config"]["global_batch"] == 12000
        assert 0.6 < out["train_auc"] <= 1.0
    else:
        assert out["config"]["global_batch"] == 512


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu():
    """Two ranks on the one GPU (gloo carries the collectives): the weak-scaling
    GBM path of the driver's N>1 run, HIP kernels included."""
    out = _run(2, ["--model", "gbm-higgs", "--rows", "200000"], {"H2OMX_DIST_BACKEND": "gloo"}, timeout=300)
    assert out["config"]["global_batch"] == 400000
    assert 0.6 < out["train_auc"] <= 1.0
