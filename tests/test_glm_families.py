"""GLM negative binomial / fractional binomial / ordinal families and
interaction columns, against fp64 maximum-likelihood references (scipy);
GPU IRLS kernel parity for the new family codes."""
import numpy as np
import pandas as pd
import pytest
import torch
from scipy.optimize import minimize

from h2omx.frame import Frame
from h2omx.models import H2OGeneralizedLinearEstimator


def _nb_data(n=4000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 2))
    mu = np.exp(0.5 + 0.4 * X[:, 0] - 0.3 * X[:, 1])
    theta = 0.5
    y = rng.negative_binomial(1 / theta, 1 / (1 + theta * mu))
    return pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "y": y.astype(float)}), theta


def test_negative_binomial_mle():
    df, theta = _nb_data()
    fr = Frame.from_pandas(df)
    m = H2OGeneralizedLinearEstimator(family="negativebinomial", theta=theta, lambda_=0.0).train(
        x=["a", "b"], y="y", training_frame=fr)
    X = np.c_[df[["a", "b"]].values, np.ones(len(df))]
    y = df.y.values

    def nll(b):
        mu = np.exp(X @ b)
        return -(y * np.log(theta * mu / (1 + theta * mu)) - np.log(1 + theta * mu) / theta).sum()

    ref = minimize(nll, np.zeros(3), method="BFGS").x
    c = m.coef()
    np.testing.assert_allclose([c["a"], c["b"], c["Intercept"]], ref, atol=2e-3)


def test_fractional_binomial():
    rng = np.random.default_rng(1)
    n = 3000
    x = rng.normal(size=n)
    y = 1 / (1 + np.exp(-(0.3 + 0.8 * x)))
    y = np.clip(y + rng.normal(scale=0.05, size=n), 0, 1)
    fr = Frame.from_pandas(pd.DataFrame({"x": x, "y": y}))
    m = H2OGeneralizedLinearEstimator(family="fractionalbinomial", lambda_=0.0).train(x=["x"], y="y", training_frame=fr)
    X = np.c_[x, np.ones(n)]

    def nll(b):
        p = 1 / (1 + np.exp(-(X @ b)))
        return -(y * np.log(p) + (1 - y) * np.log(1 - p)).sum()

    ref = minimize(nll, np.zeros(2), method="BFGS").x
    np.testing.assert_allclose([m.coef()["x"], m.coef()["Intercept"]], ref, atol=2e-3)
    P = m.predict(fr).vec("predict").data.numpy()
    assert 0 <= P.min() and P.max() <= 1


def test_ordinal():
    rng = np.random.default_rng(2)
    n = 5000
    X = rng.normal(size=(n, 2))
    eta = 1.0 * X[:, 0] - 0.5 * X[:, 1]
    th = np.array([-1.0, 0.5, 1.5])
    u = rng.logistic(size=n)
    yi = (eta + u > th[:, None]).sum(0)
    df = pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "y": pd.Categorical([f"L{k}" for k in yi])})
    fr = Frame.from_pandas(df)
    m = H2OGeneralizedLinearEstimator(family="ordinal", lambda_=0.0, standardize=False).train(
        x=["a", "b"], y="y", training_frame=fr)
    c = m.coef()
    np.testing.assert_allclose([c["a"], c["b"]], [1.0, -0.5], atol=0.08)
    np.testing.assert_allclose(m.stats["ordinal_thresholds"], th, atol=0.1)
    P = m.predict_raw(fr)
    assert P.shape == (4, n)
    np.testing.assert_allclose(P.sum(0).numpy(), 1.0, atol=1e-5)
    freq = np.bincount(yi) / n
    assert m.training_metrics["logloss"] < -(freq * np.log(freq)).sum() - 0.1     # beats the class prior


def test_interactions():
    rng = np.random.default_rng(3)
    n = 4000
    a = rng.normal(size=n)
    b = rng.normal(size=n)
    g = rng.choice(["p", "q"], n)
    y = 1 + a + 2 * a * b + np.where(g == "q", 1.5, -0.5) * b + 0.01 * rng.normal(size=n)
    df = pd.DataFrame({"a": a, "b": b, "g": pd.Categorical(g), "y": y})
    fr = Frame.from_pandas(df)
    m = H2OGeneralizedLinearEstimator(lambda_=0.0, interaction_pairs=[("a", "b"), ("g", "b")]).train(
        x=["a", "b", "g"], y="y", training_frame=fr)
    c = m.coef()
    assert abs(c["a_b"] - 2.0) < 0.01
    assert abs(c["g.q_b"] - c["g.p_b"] - 2.0) < 0.02
    r2 = 1 - ((m.predict(fr).vec("predict").data.numpy() - y) ** 2).mean() / y.var()
    assert r2 > 0.999
    m2 = H2OGeneralizedLinearEstimator(lambda_=0.0, interactions=["a", "b"]).train(x=["a", "b"], y="y",
                                                                                   training_frame=fr)
    assert "a_b" in m2.coef()


@pytest.mark.gpu
def test_negative_binomial_gpu_matches_cpu(cuda_dev):
    df, theta = _nb_data(3000)
    kw = dict(family="negativebinomial", theta=theta, lambda_=0.0)
    a = H2OGeneralizedLinearEstimator(**kw).train(x=["a", "b"], y="y", training_frame=Frame.from_pandas(df))
    b = H2OGeneralizedLinearEstimator(**kw).train(x=["a", "b"], y="y",
                                                  training_frame=Frame.from_pandas(df, device=cuda_dev))
    for k, v in a.coef().items():
        assert abs(b.coef()[k] - v) < 1e-3, k
    assert abs(b.stats["residual_deviance"] - a.stats["residual_deviance"]) < 1e-3 * a.stats["residual_deviance"]
