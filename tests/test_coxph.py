"""CoxPH vs a naive O(n^2) partial likelihood maximised with scipy (Breslow and
Efron ties, counting-process start times, strata, weights)."""
import numpy as np
import pandas as pd
import pytest
from scipy.optimize import minimize

from h2omx.frame import Frame
from h2omx.models.coxph import H2OCoxProportionalHazardsEstimator


def _naive_nll(beta, X, t, d, w, start, strata, ties):
    eta = X @ beta
    ll = 0.0
    for s in np.unique(strata):
        idx = np.nonzero(strata == s)[0]
        for tau in np.unique(t[idx][d[idx] > 0]):
            D = idx[(t[idx] == tau) & (d[idx] > 0)]
            R = idx[(t[idx] >= tau) & ((start[idx] < tau) if start is not None else True)]
            S0 = np.sum(w[R] * np.exp(eta[R]))
            A0 = np.sum(w[D] * np.exp(eta[D]))
            ll += np.sum(w[D] * eta[D])
            m = len(D)
            wbar = w[D].mean()
            if ties == "breslow":
                ll -= w[D].sum() * np.log(S0)
            else:
                for k in range(m):
                    ll -= wbar * np.log(S0 - k / m * A0)
    return -ll


def _data(n=300, seed=0, ties=True, counting=False):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 2))
    beta = np.array([0.8, -0.5])
    T = rng.exponential(np.exp(-X @ beta))
    C = rng.exponential(1.5, n)
    t = np.minimum(T, C)
    if ties:
        t = np.ceil(t * 10) / 10
    d = (T <= C).astype(float)
    df = pd.DataFrame({"x1": X[:, 0], "x2": X[:, 1], "t": t, "ev": d, "w": rng.uniform(0.5, 1.5, n),
                       "g": rng.integers(0, 2, n).astype(float)})
    if counting:
        df["s"] = np.maximum(0.0, t - rng.uniform(0.2, 2.0, n))
    return df


@pytest.mark.parametrize("ties", ["efron", "breslow"])
@pytest.mark.parametrize("variant", ["plain", "weights_strata", "counting"])
def test_coxph_matches_naive_mle(ties, variant):
    df = _data(counting=variant == "counting", seed={"plain": 0, "weights_strata": 1, "counting": 2}[variant])
    kw = dict(stop_column="t", ties=ties)
    w = np.ones(len(df))
    strata = np.zeros(len(df))
    start = None
    if variant == "weights_strata":
        kw.update(weights_column="w", stratify_by=["g"])
        w = df.w.to_numpy()
        strata = df.g.to_numpy()
    if variant == "counting":
        kw["start_column"] = "s"
        start = df.s.to_numpy()
    fr = Frame.from_pandas(df)
    m = H2OCoxProportionalHazardsEstimator(**kw).train(x=["x1", "x2"], y="ev", training_frame=fr)
    X = df[["x1", "x2"]].to_numpy()
    X = X - (X * w[:, None]).sum(0) / w.sum()
    res = minimize(_naive_nll, np.zeros(2), args=(X, df.t.to_numpy(), df.ev.to_numpy(), w, start, strata, ties),
                   method="BFGS", options={"gtol": 1e-9})
    np.testing.assert_allclose(m.beta, res.x, rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(m.stats["loglik"], -res.fun, rtol=1e-8)
    assert 0.5 < m.stats["concordance"] <= 1.0
    lp = m.predict(fr).to_pandas()["lp"].to_numpy()
    np.testing.assert_allclose(lp, X @ m.beta, rtol=1e-4, atol=1e-5)
    tab = m.coefficients_table
    assert len(tab["se_coef"]) == 2 and all(s > 0 for s in tab["se_coef"])


def test_coxph_requires_stop_column():
    fr = Frame.from_pandas(_data(n=50))
    with pytest.raises(ValueError):
        H2OCoxProportionalHazardsEstimator().train(x=["x1"], y="ev", training_frame=fr)
