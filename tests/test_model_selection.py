"""ModelSelection (maxr / forward / backward / allsubsets) vs exhaustive NumPy
least squares; ANOVA GLM type-III tests."""
import itertools

import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models.model_selection import H2OANOVAGLMEstimator, H2OModelSelectionEstimator


def _df(n=1500, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 6))
    X[:, 3] = X[:, 0] * 0.6 + 0.8 * X[:, 3]          # correlated pair
    y = 2 * X[:, 0] - 1.5 * X[:, 2] + 0.8 * X[:, 4] + rng.normal(size=n)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
    df["y"] = y
    return df


def _best_r2(df, k):
    X = df[[f"x{i}" for i in range(6)]].to_numpy()
    y = df.y.to_numpy()
    tss = ((y - y.mean()) ** 2).sum()
    best = (-1, None)
    for s in itertools.combinations(range(6), k):
        A = np.c_[X[:, s], np.ones(len(y))]
        r = y - A @ np.linalg.lstsq(A, y, rcond=None)[0]
        best = max(best, (1 - (r ** 2).sum() / tss, s))
    return best


@pytest.mark.parametrize("mode", ["maxr", "allsubsets", "forward"])
def test_model_selection_finds_best_subsets(mode):
    df = _df()
    fr = Frame.from_pandas(df)
    m = H2OModelSelectionEstimator(mode=mode, max_predictor_number=3).train(y="y", training_frame=fr)
    res = m.result()
    assert [r["size"] for r in res] == [1, 2, 3]
    for r in res:
        r2, s = _best_r2(df, r["size"])
        assert abs(r["best_r2_value"] - r2) < 1e-6
        assert sorted(r["predictors"]) == sorted(f"x{i}" for i in s)
    assert abs(m.coef(3)["x0"] - 2) < 0.15
    pred = m.predict(fr).to_pandas()["predict"]
    assert np.corrcoef(pred, df.y)[0, 1] > 0.9


def test_model_selection_backward():
    df = _df(seed=1)
    m = H2OModelSelectionEstimator(mode="backward", min_predictor_number=2).train(
        y="y", training_frame=Frame.from_pandas(df))
    sizes = [r["size"] for r in m.result()]
    assert sizes[0] == 2 and sizes[-1] == 6
    two = [r for r in m.result() if r["size"] == 3][0]
    assert set(two["predictors"]) == {"x0", "x2", "x4"}


def test_anova_glm_type3():
    rng = np.random.default_rng(2)
    n = 2000
    a, b, c = rng.normal(size=(3, n))
    y = 1.0 * a + 0.5 * a * b + rng.normal(size=n)
    df = pd.DataFrame({"a": a, "b": b, "c": c, "y": y})
    m = H2OANOVAGLMEstimator(family="gaussian", highest_interaction_term=2).train(
        y="y", training_frame=Frame.from_pandas(df))
    tab = {r["term"]: r for r in m.result()}
    assert tab["a"]["p_value"] < 1e-10 and tab["a:b"]["p_value"] < 1e-10
    assert tab["c"]["p_value"] > 1e-3 and tab["b:c"]["p_value"] > 1e-3
    assert tab["a"]["statistic_type"] == "F"
