"""AutoML: presets + round-robin grids under a model budget, leaderboard
ordering and extra columns, get_best_model, modeling_plan, project
continuation, per-model runtime caps (tree models stop adding trees)."""
import time

import numpy as np
import pandas as pd

from h2omx.automl import H2OAutoML, get_automl
from h2omx.frame import Frame
from h2omx.models import H2OGradientBoostingEstimator


def _frame(n=800, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    df = pd.DataFrame(X, columns=list("abcd"))
    df["y"] = pd.Categorical(np.where(X[:, 0] - X[:, 1] + 0.3 * rng.normal(size=n) > 0, "yes", "no"))
    return Frame.from_pandas(df)


def test_automl_budget_leaderboard_and_helpers():
    fr = _frame()
    aml = H2OAutoML(max_models=6, nfolds=3, seed=1, project_name="t_aml",
                    exclude_algos=["DeepLearning"]).train(y="y", training_frame=fr)
    lb = aml.leaderboard
    base = [r for r in lb if r["algo"] != "stackedensemble"]
    assert len(base) == 6
    aucs = [r["auc"] for r in lb]
    assert aucs == sorted(aucs, reverse=True)
    assert aml.leader.model_id == lb[0]["model_id"]
    ext = aml.get_leaderboard("ALL")
    assert all(r["training_time_ms"] >= 0 and r["predict_time_per_row_ms"] > 0 for r in ext)
    best_gbm = aml.get_best_model(algorithm="gbm")
    assert best_gbm is not None and best_gbm.algo == "gbm"
    worst = aml.get_best_model(criterion="logloss")
    assert worst is not None
    assert get_automl("t_aml") is aml
    assert aml.event_log.nrows >= 6
    assert aml.training_info["models"] == len(aml.models)
    # same project_name: the leaderboard grows
    aml2 = H2OAutoML(max_models=2, nfolds=3, seed=2, project_name="t_aml", include_algos=["GLM", "DRF"]).train(
        y="y", training_frame=fr)
    assert len(aml2.models) > len(aml.models)


def test_modeling_plan_and_grids():
    fr = _frame(500)
    aml = H2OAutoML(max_models=4, nfolds=0, seed=3, modeling_plan=[("XGBoost", "grids"), ("GBM", "grids")]).train(
        y="y", training_frame=fr)
    ids = [m.model_id for m in aml.models]
    assert all("_grid_1_model_" in i for i in ids)
    assert {m.algo for m in aml.models} == {"xgboost", "gbm"}


def test_max_runtime_secs_stops_trees():
    fr = _frame(3000)
    t = time.time()
    m = H2OGradientBoostingEstimator(ntrees=100000, max_depth=3, max_runtime_secs=1.0, seed=1).train(
        y="y", training_frame=fr)
    assert time.time() - t < 30
    assert 0 < m.ens.ntrees < 100000


def test_exploitation_phase_lr_annealing():
    """exploitation_ratio > 0 reserves part of the model budget for the
    exploitation step: the best explored GBM retrained with learning-rate
    annealing (H2O's GBM_lr_annealing_selection)."""
    fr = _frame(seed=4)
    aml = H2OAutoML(max_models=8, nfolds=3, seed=1, project_name="t_aml_exploit", exploitation_ratio=0.2,
                    include_algos=["GBM", "StackedEnsemble"]).train(y="y", training_frame=fr)
    ids = [m.model_id for m in aml.models]
    ex = [m for m in aml.models if m.model_id.startswith("GBM_lr_annealing_selection")]
    assert len(ex) == 1 and ex[0].params["learn_rate_annealing"] == 0.99
    base = [m for m in aml.models if m.algo == "gbm"]
    assert len(base) == 8 and ids.index(ex[0].model_id) == len(base) - 1
    off = H2OAutoML(max_models=3, nfolds=0, seed=1, project_name="t_aml_noexploit",
                    include_algos=["GBM"]).train(y="y", training_frame=fr)
    assert not any(m.model_id.startswith("GBM_lr_annealing") for m in off.models)


def test_exploitation_xgboost_lr_search():
    fr = _frame(seed=5)
    aml = H2OAutoML(max_models=6, nfolds=3, seed=2, project_name="t_aml_exploit_xgb", exploitation_ratio=0.3,
                    include_algos=["GBM", "XGBoost"]).train(y="y", training_frame=fr)
    ids = [m.model_id for m in aml.models]
    assert len(ids) == 6
    assert any(i.startswith("XGBoost_lr_search_selection") for i in ids)
    assert any(i.startswith("GBM_lr_annealing_selection") for i in ids)
    xs = [m for m in aml.models if m.model_id.startswith("XGBoost_lr_search_selection")][0]
    assert xs.algo == "xgboost" and "failed" not in " ".join(str(e) for e in aml.event_log.to_pandas().values.ravel())


def _hicard_frame(n=3000, seed=5):
    rng = np.random.default_rng(seed)
    city = rng.integers(0, 40, n)
    effect = rng.normal(scale=1.5, size=40)
    a = rng.normal(size=n)
    logit = effect[city] + 0.8 * a
    df = pd.DataFrame({"city": pd.Categorical([f"c{v}" for v in city]), "color": pd.Categorical(
        rng.choice(["r", "g", "b"], n)), "a": a})
    df["y"] = pd.Categorical(np.where(logit + rng.logistic(size=n) > 0, "yes", "no"))
    return df


def test_automl_target_encoding_preprocessing():
    """preprocessing=["target_encoding"]: the 40-level predictor is replaced by its
    out-of-fold blended target mean for the tree algos (the 3-level one is left
    alone); the encoder travels with each model, so raw frames score as-is."""
    df = _hicard_frame()
    fr = Frame.from_pandas(df)
    aml = H2OAutoML(max_models=3, nfolds=3, seed=1, include_algos=["GLM", "GBM", "DRF"],
                    preprocessing=["target_encoding"]).train(y="y", training_frame=fr)
    by = {m.algo: m for m in aml.models}
    assert {"glm", "gbm", "drf"} <= set(by)
    for algo in ("gbm", "drf"):
        m = by[algo]
        assert len(m.preprocessors) == 1 and "city_te" in m.x and "city" not in m.x and "color" in m.x
        assert m.training_metrics["AUC"] > 0.7
    assert not by["glm"].preprocessors and "city" in by["glm"].x
    assert any("target_encoding" in e["msg"] for e in aml.events)
    # scoring the raw frame goes through the encoder (no *_te columns needed)
    p = by["gbm"].predict(Frame.from_pandas(df.head(50)))
    assert p.nrows == 50
    perf = by["gbm"].model_performance(fr)
    assert perf["AUC"] > 0.7
    import pytest

    from h2omx.mojo import mojo_bytes
    with pytest.raises(ValueError, match="preprocessing"):
        mojo_bytes(by["gbm"])


def test_automl_target_encoding_skips_low_cardinality():
    fr = _frame(400)
    aml = H2OAutoML(max_models=1, nfolds=0, seed=1, include_algos=["GBM"],
                    preprocessing=["target_encoding"]).train(y="y", training_frame=fr)
    assert not aml.models[0].preprocessors
    assert any("step skipped" in e["msg"] for e in aml.events)


def test_automl_auto_scheduler_choice():
    """parallelism="auto": task-parallel while the replicated frame fits a share
    of one device's memory, data-parallel otherwise / when asked / on one rank."""

    class _Comm:
        world_size, rank = 2, 0

        def all_reduce_numpy(self, a):
            return a * 2

    fr = _frame(300)
    aml = H2OAutoML(max_models=1, seed=1)
    assert aml.parallelism == "auto"
    assert aml._scheduler(fr, None) == "data"
    assert aml._scheduler(fr, _Comm()) == "task"
    aml.TASK_MEM_FRACTION = 1e-12
    assert aml._scheduler(fr, _Comm()) == "data"
    assert H2OAutoML(max_models=1, parallelism="data")._scheduler(fr, _Comm()) == "data"
    assert any("parallelism auto" in e["msg"] for e in aml.events)
