"""Grid search (H2OGridSearch): Cartesian / RandomDiscrete walks, budgets,
early stopping, failures and sorting (CPU)."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.frame.frame import DKV
from h2omx.grid import H2OGridSearch
from h2omx.models import H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator, H2OKMeansEstimator


@pytest.fixture(scope="module")
def frame():
    rng = np.random.default_rng(0)
    n = 4000
    X = rng.normal(size=(n, 4)).astype(np.float32)
    y = rng.random(n) < 1 / (1 + np.exp(-(X[:, 0] - X[:, 1] + 0.5 * X[:, 2] * X[:, 3])))
    df = pd.DataFrame(X, columns=list("abcd"))
    df["y"] = pd.Categorical(np.where(y, "t", "f"))
    return Frame.from_pandas(df)


def test_cartesian_grid_sorted(frame):
    g = H2OGridSearch(H2OGradientBoostingEstimator, {"max_depth": [1, 3], "learn_rate": [0.05, 0.3]},
                      grid_id="g_cart", ntrees=8, seed=1)
    g.train(y="y", training_frame=frame)
    assert len(g.models) == 4 and not g.failed_params
    combos = [(m.params["max_depth"], m.params["learn_rate"]) for m in g.models]
    assert combos == [(1, 0.05), (1, 0.3), (3, 0.05), (3, 0.3)]
    g.get_grid(sort_by="auc", decreasing=True)
    aucs = [m.training_metrics["AUC"] for m in g.models]
    assert aucs == sorted(aucs, reverse=True)
    assert g.models[0].params["max_depth"] == 3          # deeper trees fit the interaction
    assert DKV.get("g_cart") is g
    t = g.summary_table()
    assert set(t[0]) == {"max_depth", "learn_rate", "model_ids", "auc"}


def test_random_discrete_budget_and_seed(frame):
    hp = {"alpha": [0.0, 0.25, 0.5, 0.75, 1.0], "lambda_": [1e-4, 1e-2]}
    a = H2OGridSearch(H2OGeneralizedLinearEstimator, hp, search_criteria={"strategy": "RandomDiscrete",
                                                                           "max_models": 3, "seed": 7})
    a.train(y="y", training_frame=frame)
    b = H2OGridSearch(H2OGeneralizedLinearEstimator, hp, search_criteria={"strategy": "RandomDiscrete",
                                                                           "max_models": 3, "seed": 7})
    b.train(y="y", training_frame=frame)
    assert len(a.models) == 3
    assert [m.grid_hyper_params for m in a.models] == [m.grid_hyper_params for m in b.models]


def test_grid_early_stopping_and_failures(frame):
    # every model is identical -> the best-so-far metric never improves
    g = H2OGridSearch(H2OGradientBoostingEstimator, {"seed": list(range(1, 30))}, ntrees=3, max_depth=2,
                      sample_rate=1.0, search_criteria={"strategy": "RandomDiscrete", "stopping_rounds": 2,
                                                        "stopping_metric": "logloss", "seed": 1})
    g.train(y="y", training_frame=frame)
    assert 4 <= len(g.models) < 29
    bad = H2OGridSearch(H2OGradientBoostingEstimator, {"distribution": ["bernoulli", "no_such_dist"]}, ntrees=2)
    bad.train(y="y", training_frame=frame)
    assert len(bad.models) == 1 and bad.failed_params == [{"distribution": "no_such_dist"}]
    assert bad.failure_details and "no_such_dist" in bad.failure_details[0]


def test_clustering_grid(frame):
    g = H2OGridSearch(H2OKMeansEstimator, {"k": [2, 4, 6]}, seed=1, max_iterations=10)
    g.train(x=list("abcd"), training_frame=frame)
    g.get_grid()          # default: tot_withinss ascending
    ws = [m.stats["tot_withinss"] for m in g.models]
    assert ws == sorted(ws) and g.models[0].params["k"] == 6
