"""RuleFit: recovers a planted rule + linear term (CPU tree + lasso path)."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models.rulefit import H2ORuleFitEstimator, _cd_lasso


def _df(n=4000, seed=0, binary=False):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-1, 1, size=(n, 4))
    f = 2.0 * ((X[:, 0] > 0.3) & (X[:, 1] < 0)) + 0.8 * X[:, 2]
    df = pd.DataFrame(X, columns=["a", "b", "c", "d"])
    if binary:
        y = (rng.random(n) < 1 / (1 + np.exp(-(3 * f - 1.5)))).astype(int)
        df["y"] = pd.Categorical(np.where(y == 1, "1", "0"))
    else:
        df["y"] = f + 0.1 * rng.normal(size=n)
    return df


def test_cd_lasso_matches_closed_form_when_unpenalised():
    rng = np.random.default_rng(1)
    X = rng.normal(size=(200, 5))
    y = X @ np.array([1.0, -2, 0, 0.5, 0]) + 0.01 * rng.normal(size=200)
    G, b = X.T @ X / 200, X.T @ y / 200
    np.testing.assert_allclose(_cd_lasso(G, b, 0.0, np.zeros(5), iters=5000, tol=1e-12), np.linalg.solve(G, b),
                               rtol=1e-6, atol=1e-8)
    assert np.count_nonzero(_cd_lasso(G, b, 10.0, np.zeros(5))) == 0


def test_rulefit_regression_finds_planted_rule():
    df = _df()
    fr = Frame.from_pandas(df)
    m = H2ORuleFitEstimator(min_rule_length=1, max_rule_length=3, rule_generation_ntrees=20, seed=3).train(
        y="y", training_frame=fr)
    pred = m.predict(fr).to_pandas()["predict"].to_numpy()
    r2 = 1 - np.mean((pred - df.y) ** 2) / np.var(df.y)
    assert r2 > 0.9, r2
    imp = m.rule_importance()
    top = " ".join(r["variable"] for r in imp[:5])
    assert "(a " in top and "(b " in top
    assert any(r["variable"] == "linear.c" for r in imp)
    vi = dict((v, s) for v, _, s, _ in m.varimp())
    assert vi["d"] < 0.2


def test_rulefit_binomial_and_rule_cap():
    df = _df(binary=True, seed=2)
    fr = Frame.from_pandas(df)
    m = H2ORuleFitEstimator(max_rule_length=2, min_rule_length=2, rule_generation_ntrees=10, max_num_rules=8,
                            model_type="RULES", seed=1).train(y="y", training_frame=fr)
    assert m.training_metrics["AUC"] > 0.8
    assert 0 < np.count_nonzero(m.beta) <= 8
    with pytest.raises(ValueError):
        H2ORuleFitEstimator(model_type="TREES").train(y="y", training_frame=fr)
