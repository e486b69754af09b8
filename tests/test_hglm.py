"""HGLM (Gaussian LMM, random intercept + slopes) against a direct numerical
maximisation of the marginal likelihood (numpy, explicit V_g), prediction
with / without known groups, and multi-group parameter recovery."""
import numpy as np
import pandas as pd
import pytest
from scipy.optimize import minimize

from h2omx.frame import Frame
from h2omx.models import H2OHGLMEstimator


def _data(G=20, n=400, seed=0, slope=False):
    rng = np.random.default_rng(seed)
    g = rng.integers(0, G, n)
    u0 = rng.normal(scale=1.0, size=G)
    u1 = rng.normal(scale=0.5, size=G)
    x = rng.normal(size=n)
    y = 2 + 1.5 * x + u0[g] + (u1[g] * x if slope else 0) + rng.normal(scale=0.7, size=n)
    return pd.DataFrame({"x": x, "g": pd.Categorical([f"g{i:02d}" for i in g]), "y": y}), g


def test_random_intercept_matches_direct_mle():
    df, g = _data()
    m = H2OHGLMEstimator(group_column="g", em_epsilon=1e-10, max_iterations=500).train(
        x=["x"], y="y", training_frame=Frame.from_pandas(df))
    X = np.c_[np.ones(len(df)), df.x.values]
    y = df.y.values

    def nll(th):
        b, ls2, lt2 = th[:2], th[2], th[3]
        s2, t2 = np.exp(ls2), np.exp(lt2)
        out = 0.0
        for k in np.unique(g):
            idx = g == k
            nk = idx.sum()
            V = s2 * np.eye(nk) + t2 * np.ones((nk, nk))
            r = y[idx] - X[idx] @ b
            out += 0.5 * (np.linalg.slogdet(V)[1] + r @ np.linalg.solve(V, r) + nk * np.log(2 * np.pi))
        return out

    ref = minimize(nll, np.array([0.0, 0.0, 0.0, 0.0]), method="L-BFGS-B").x
    c = m.coef()
    np.testing.assert_allclose([c["Intercept"], c["x"]], ref[:2], atol=2e-3)
    np.testing.assert_allclose(m.sigma2, np.exp(ref[2]), rtol=2e-3)
    np.testing.assert_allclose(m.T[0, 0], np.exp(ref[3]), rtol=5e-3)
    np.testing.assert_allclose(m.stats["loglik"], -nll(ref), rtol=1e-5)


def test_random_slope_and_prediction():
    df, _ = _data(G=60, n=6000, seed=1, slope=True)
    fr = Frame.from_pandas(df)
    m = H2OHGLMEstimator(group_column="g", random_columns=["x"]).train(x=["x"], y="y", training_frame=fr)
    assert abs(m.coef()["x"] - 1.5) < 0.2
    assert abs(m.sigma2 - 0.49) < 0.05
    assert m.T.shape == (2, 2) and 0.1 < m.T[1, 1] < 0.5
    P = m.predict(fr).vec("predict").data.numpy()
    resid = df.y.values - P
    assert resid.var() < 0.6                 # random effects explain the group structure
    new = df.copy()
    new["g"] = pd.Categorical(["unseen"] * len(new))
    Pn = m.predict(Frame.from_pandas(new)).vec("predict").data.numpy()
    c = m.coef()
    np.testing.assert_allclose(Pn, c["Intercept"] + c["x"] * df.x.values, atol=1e-4)
    assert set(m.coefs_random()) == set(df.g.cat.categories)


def test_hglm_requires_group_column():
    df, _ = _data()
    with pytest.raises(ValueError):
        H2OHGLMEstimator().train(x=["x"], y="y", training_frame=Frame.from_pandas(df))
