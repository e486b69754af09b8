"""AutoML schedulers on a two-rank gloo world (CPU).

parallelism="task" replicates the frame and deals the model plan to the ranks;
every rank ends with the same leaderboard, and because each base model sees
the full replicated frame, its metrics equal the one-rank run's.  The default
data-parallel scheduler trains each model across both shards (row-sharded
trees equal one-rank trees bit for bit, GLM to solver tolerance)."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
WORKER = os.path.join(HERE, "_automl_worker.py")


def _run(world, mode, tmp, explo=0.0):
    out = str(tmp / f"lb_{mode}_{world}_{explo}")
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    if world == 1:
        subprocess.run([sys.executable, WORKER, out, mode, str(explo)], env=env, check=True, timeout=600)
    else:
        r = subprocess.run([sys.executable, "-m", "h2omx.runtime.launch", "--nproc", str(world), "--", sys.executable,
                            WORKER, out, mode, str(explo)], env=env, cwd=ROOT, timeout=600)
        assert r.returncode == 0
    return [json.load(open(f"{out}.{r}")) for r in range(world)]


@pytest.fixture(scope="module")
def runs(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("aml")
    return {"one": _run(1, "data", tmp)[0], "task": _run(2, "task", tmp), "data": _run(2, "data", tmp)}


def _by_id(lb):
    return {r["model_id"].replace("p_task", "P").replace("p_data", "P"): r for r in lb}


def test_task_parallel_leaderboard_identical_on_ranks(runs):
    a, b = runs["task"]
    assert [r["model_id"] for r in a["leaderboard"]] == [r["model_id"] for r in b["leaderboard"]]
    for ra, rb in zip(a["leaderboard"], b["leaderboard"]):
        for k, v in ra.items():
            if isinstance(v, float):      # NaN-aware; the metalearner runs on each rank (fp64 BLAS order)
                assert (v != v and rb[k] != rb[k]) or abs(v - rb[k]) <= 1e-6 * max(1.0, abs(v)), (ra["model_id"], k)
            else:
                assert v == rb[k], (ra["model_id"], k)
    # both ranks trained base models (round-robin), then exchanged them
    trained_on = {e["msg"].split(" trained on rank ")[1] for e in a["events"] if " trained on rank " in e["msg"]}
    assert trained_on == {"0", "1"}
    assert sum(r["algo"] == "stackedensemble" for r in a["leaderboard"]) == 2


def test_task_parallel_base_models_equal_one_rank(runs):
    one, task = _by_id(runs["one"]["leaderboard"]), _by_id(runs["task"][0]["leaderboard"])
    assert set(one) == set(task)
    for k, r in one.items():
        if r["algo"] == "stackedensemble":
            continue
        assert abs(task[k]["auc"] - r["auc"]) < 1e-9, k
        assert abs(task[k]["logloss"] - r["logloss"]) < 1e-9, k


def test_data_parallel_matches_one_rank(runs):
    one, dp = _by_id(runs["one"]["leaderboard"]), _by_id(runs["data"][0]["leaderboard"])
    assert set(one) == set(dp)
    for k, r in one.items():
        assert abs(dp[k]["auc"] - r["auc"]) < 2e-3, k


def test_task_parallel_exploitation_phase(tmp_path):
    """exploitation_ratio > 0 under parallelism="task": the exploration round
    keeps its share of max_models, then the exploitation plan (built from the
    exchanged leaderboard) is dealt over the ranks - the same exploitation models
    with the same metrics as the one-rank sequential run."""
    one = _by_id(_run(1, "data", tmp_path, 0.4)[0]["leaderboard"])
    a, b = _run(2, "task", tmp_path, 0.4)
    assert [r["model_id"] for r in a["leaderboard"]] == [r["model_id"] for r in b["leaderboard"]]
    task = _by_id(a["leaderboard"])
    sel = [k for k in one if "_selection_AutoML" in k]
    assert sel, sorted(one)
    for name in sel:
        assert name in task, (sorted(one), sorted(task))
        assert abs(task[name]["auc"] - one[name]["auc"]) < 1e-9, name
    assert set(one) == set(task)
