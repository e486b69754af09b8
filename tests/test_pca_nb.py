"""PCA and Naive Bayes vs independent references (NumPy / scikit-learn)."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models import H2ONaiveBayesEstimator, H2OPrincipalComponentAnalysisEstimator


def _corr_data(n=5000, seed=0):
    rng = np.random.default_rng(seed)
    Z = rng.normal(size=(n, 3))
    A = np.array([[2.0, 0.5, 0.0, 1.0, 0.0], [0.0, 1.0, 1.5, 0.0, 0.3], [0.2, 0.0, 0.0, 0.5, 2.0]])
    X = Z @ A + rng.normal(scale=0.1, size=(n, 5)) + np.array([1.0, -2.0, 0.5, 3.0, 0.0])
    return X


@pytest.mark.parametrize("transform", ["DEMEAN", "STANDARDIZE", "NONE"])
def test_pca_matches_numpy(transform):
    X = _corr_data()
    names = [f"x{i}" for i in range(5)]
    m = H2OPrincipalComponentAnalysisEstimator(k=3, transform=transform).train(
        training_frame=Frame.from_numpy(X.astype(np.float32), names=names))
    Xt = X.copy()
    if transform in ("DEMEAN", "STANDARDIZE"):
        Xt = Xt - X.mean(0)
    if transform == "STANDARDIZE":
        Xt = Xt / X.std(0, ddof=1)
    w, V = np.linalg.eigh(Xt.T @ Xt / (len(X) - 1))
    w, V = w[::-1], V[:, ::-1]
    np.testing.assert_allclose(m.eigenvalues, w[:3], rtol=1e-3)
    for j in range(3):
        assert abs(abs(np.dot(m.eigenvectors[:, j], V[:, j])) - 1) < 1e-3
    pv = m.importance["Proportion of Variance"]
    np.testing.assert_allclose(pv, w[:3] / w.sum(), rtol=1e-3)
    S = m.predict(Frame.from_numpy(X[:50].astype(np.float32), names=names)).to_pandas().values
    ref = Xt[:50] @ m.eigenvectors
    np.testing.assert_allclose(S, ref, atol=2e-3 * np.abs(ref).max())


def test_pca_vs_sklearn_and_categoricals():
    from sklearn.decomposition import PCA

    X = _corr_data(seed=1)
    names = [f"x{i}" for i in range(5)]
    m = H2OPrincipalComponentAnalysisEstimator(k=2, transform="DEMEAN").train(
        training_frame=Frame.from_numpy(X.astype(np.float32), names=names))
    sk = PCA(n_components=2).fit(X)
    np.testing.assert_allclose(m.std_deviation ** 2, sk.explained_variance_, rtol=1e-3)
    df = pd.DataFrame(X, columns=names)
    df["c"] = pd.Categorical(np.random.default_rng(2).choice(["a", "b", "c"], len(df)))
    m2 = H2OPrincipalComponentAnalysisEstimator(k=4, transform="STANDARDIZE", use_all_factor_levels=True).train(
        training_frame=Frame.from_pandas(df))
    assert m2.eigenvectors.shape == (8, 4)
    assert m2.to_json()["output"]["eigenvectors"]["names"][-3:] == ["c.a", "c.b", "c.c"]


def test_naive_bayes_gaussian_vs_sklearn():
    from sklearn.naive_bayes import GaussianNB

    rng = np.random.default_rng(3)
    n = 20000
    y = rng.integers(0, 3, n)
    X = rng.normal(size=(n, 4)) + y[:, None] * np.array([0.5, -0.3, 1.0, 0.0])
    df = pd.DataFrame(X, columns=list("abcd"))
    df["y"] = pd.Categorical([f"k{v}" for v in y])
    m = H2ONaiveBayesEstimator().train(y="y", training_frame=Frame.from_pandas(df))
    P = m.predict_raw(Frame.from_pandas(df)).numpy().T
    sk = GaussianNB().fit(X, y).predict_proba(X)
    assert np.abs(P - sk).max() < 2e-3
    assert m.training_metrics["logloss"] < 1.0


def test_naive_bayes_categorical_laplace_and_na():
    df = pd.DataFrame({"c": pd.Categorical(["u", "u", "v", "w", "u", "v"]),
                       "y": pd.Categorical(["p", "p", "q", "q", "q", "p"])})
    m = H2ONaiveBayesEstimator(laplace=1.0).train(y="y", training_frame=Frame.from_pandas(df))
    # P(c=u | p) = (2 + 1) / (3 + 3), P(c=w | p) = (0 + 1) / 6
    T = m.tables["c"]
    dom = list(df["c"].cat.categories)
    np.testing.assert_allclose(T[0, dom.index("u")], 3 / 6)
    np.testing.assert_allclose(T[0, dom.index("w")], 1 / 6)
    np.testing.assert_allclose(m.prior, [0.5, 0.5])
    test = pd.DataFrame({"c": pd.Categorical([None, "w"], categories=dom), "y": pd.Categorical(["p", "q"])})
    P = m.predict_raw(Frame.from_pandas(test)).numpy()
    np.testing.assert_allclose(P[:, 0], [0.5, 0.5])              # NA feature: prior only
    assert P[1, 1] > P[0, 1]
