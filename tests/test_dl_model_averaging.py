"""DeepLearning replica synchronisation on 2 gloo ranks (models/deeplearning.py
_DLTrainer): H2O-style model averaging per train_samples_per_iteration (the
default, auto-tuned at -2) and per-step gradient all-reduce
(sync_gradients=True).  Every mode must end with identical replicas and a
model as good as the single-rank one."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, tmp_path):
    port = _port()
    procs, outs = [], []
    for r in range(world):
        out = tmp_path / f"dl{world}_{r}.json"
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dl_worker.py"), str(out)], env=env))
        outs.append(out)
    for p in procs:
        assert p.wait(timeout=300) == 0
    return [json.load(open(o)) for o in outs]


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    t = tmp_path_factory.mktemp("dl")
    return _run(1, t)[0], _run(2, t)


def test_replicas_identical_and_accurate(results):
    one, two = results
    for mode in ("auto", "fixed", "epoch", "grad"):
        a, b = two[0][mode], two[1][mode]
        assert a["w0"] == b["w0"] and a["wsum"] == b["wsum"], mode      # replicas agree bit for bit
        assert a["auc"] == b["auc"]
        assert a["auc"] > one[mode]["auc"] - 0.02, (mode, a["auc"], one[mode]["auc"])
        assert a["auc"] > 0.8


def test_iteration_lengths(results):
    one, two = results
    assert one["auto"]["tspi"] == 0                        # single GPU: nothing to synchronise
    r = two[0]
    assert r["grad"]["tspi"] == 2 * 256                   # one gradient all-reduce per mini-batch
    assert r["fixed"]["tspi"] == 5120                      # 2 ranks x 256 rows x 10 steps
    assert r["epoch"]["tspi"] == 2 * 256 * (20000 // 256)  # one local epoch
    assert r["auto"]["tspi"] >= 2 * 256 and r["auto"]["tspi"] % 512 == 0
