"""CPU tests of the estimators (H2O-3 pyunit style: train on a small frame,
check metrics against an independent implementation).  The tree builders
run their NumPy reference path here; GPU parity of the HIP kernels against
that reference is in test_tree_gpu.py / test_dense_gpu.py."""
import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame import Frame
from h2omx.models import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                          H2OKMeansEstimator, H2ORandomForestEstimator, H2OXGBoostEstimator)

sk = pytest.importorskip("sklearn")
from sklearn.cluster import KMeans  # noqa: E402
from sklearn.linear_model import LinearRegression, LogisticRegression, PoissonRegressor  # noqa: E402
from sklearn.metrics import roc_auc_score  # noqa: E402


def _binary_frame(n=3000, p=6, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, p))
    logit = X[:, 0] - 0.7 * X[:, 1] + 0.5 * X[:, 2] * X[:, 3]
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(p)])
    df["y"] = pd.Categorical(np.where(y == 1, "yes", "no"))
    return df


@pytest.mark.parametrize("est", [H2OGradientBoostingEstimator(ntrees=20, max_depth=3, seed=1),
                                 H2OXGBoostEstimator(ntrees=20, max_depth=3, seed=1),
                                 H2ORandomForestEstimator(ntrees=10, max_depth=8, seed=1)])
def test_tree_estimators_binomial(est):
    df = _binary_frame()
    fr = Frame.from_pandas(df)
    m = est.train(y="y", training_frame=fr)
    # DRF's training metrics are out-of-bag (as in H2O): score the frame instead
    auc = m.model_performance(fr)["AUC"] if est.algo == "drf" else m.training_metrics["AUC"]
    p = m.predict(fr).to_pandas()
    assert list(p.columns) == ["predict", "no", "yes"]
    ref = roc_auc_score((df["y"] == "yes").astype(int), p["yes"])
    assert abs(auc - ref) < 2e-3
    assert auc > 0.75
    assert m.training_metrics["AUC"] > 0.7
    vi = m.varimp()
    assert vi[0][0] in ("x0", "x1")


def test_gbm_regression_and_cv():
    rng = np.random.default_rng(1)
    X = rng.normal(size=(2000, 4))
    y = 2 * X[:, 0] + np.sin(X[:, 1]) + 0.1 * rng.normal(size=2000)
    fr = Frame.from_numpy(np.column_stack([X, y]), names=["a", "b", "c", "d", "y"])
    m = H2OGradientBoostingEstimator(ntrees=30, max_depth=4, seed=2, nfolds=3).train(y="y", training_frame=fr)
    assert m.training_metrics["r2"] > 0.9
    assert m.cross_validation_metrics["r2"] > 0.8
    assert len(m.cv_models) == 3
    assert m.cross_validation_holdout.shape == (1, 2000)


def test_glm_binomial_matches_sklearn():
    df = _binary_frame(seed=3)
    fr = Frame.from_pandas(df)
    m = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0, standardize=True).train(y="y", training_frame=fr)
    lr = LogisticRegression(C=1e10, max_iter=2000).fit(df.iloc[:, :6].values, (df["y"] == "yes").astype(int))
    co = m.coef()
    assert abs(co["Intercept"] - lr.intercept_[0]) < 1e-3
    for j in range(6):
        assert abs(co[f"x{j}"] - lr.coef_[0][j]) < 1e-3


def test_glm_gaussian_and_poisson():
    rng = np.random.default_rng(4)
    X = rng.normal(size=(2000, 3))
    y = 1 + X @ np.array([0.5, -1.0, 2.0]) + 0.1 * rng.normal(size=2000)
    fr = Frame.from_numpy(np.column_stack([X, y]), names=["a", "b", "c", "y"])
    m = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0.0).train(y="y", training_frame=fr)
    lr = LinearRegression().fit(X, y)
    assert np.allclose([m.coef()[c] for c in "abc"], lr.coef_, atol=1e-6)
    lam = np.exp(0.3 + X @ np.array([0.2, -0.3, 0.1]))
    yc = rng.poisson(lam)
    fr2 = Frame.from_numpy(np.column_stack([X, yc]), names=["a", "b", "c", "y"])
    mp = H2OGeneralizedLinearEstimator(family="poisson", lambda_=0.0).train(y="y", training_frame=fr2)
    pr = PoissonRegressor(alpha=0.0, max_iter=1000, tol=1e-10).fit(X, yc)
    assert np.allclose([mp.coef()[c] for c in "abc"], pr.coef_, atol=1e-4)


def test_glm_lasso_sparsity():
    rng = np.random.default_rng(5)
    X = rng.normal(size=(1000, 10))
    y = X[:, 0] * 3 + rng.normal(size=1000)
    fr = Frame.from_numpy(np.column_stack([X, y]), names=[f"x{i}" for i in range(10)] + ["y"])
    m = H2OGeneralizedLinearEstimator(family="gaussian", alpha=1.0, lambda_=0.3).train(y="y", training_frame=fr)
    co = m.coef()
    assert abs(co["x0"]) > 2
    assert sum(abs(co[f"x{i}"]) > 0 for i in range(1, 10)) <= 2


def test_kmeans_matches_sklearn_inertia():
    rng = np.random.default_rng(0)
    cent = rng.normal(0, 5, (4, 6))
    X = np.concatenate([c + rng.normal(0, 1, (400, 6)) for c in cent])
    fr = Frame.from_numpy(X, names=[f"x{i}" for i in range(6)])
    m = H2OKMeansEstimator(k=4, seed=1, standardize=False, max_iterations=50).train(training_frame=fr)
    skm = KMeans(4, n_init=5, random_state=0).fit(X)
    assert abs(m.stats["tot_withinss"] - skm.inertia_) / skm.inertia_ < 1e-6
    assert sorted(int(s) for s in m.stats["size"]) == [400] * 4
    pred = m.predict(fr).to_pandas()["predict"].values
    assert len(np.unique(pred)) == 4
    for init in ("PlusPlus", "Random"):
        m2 = H2OKMeansEstimator(k=4, seed=2, init=init, max_iterations=50).train(training_frame=fr)
        assert m2.stats["betweenss"] > 0


def test_deeplearning_classification_regression_autoencoder():
    df = _binary_frame(n=2000, seed=6)
    fr = Frame.from_pandas(df)
    m = H2ODeepLearningEstimator(hidden=[32, 32], epochs=10, seed=3).train(y="y", training_frame=fr)
    assert m.training_metrics["AUC"] > 0.72  # Bayes AUC of this data is 0.76
    assert len(m.scoring_history) >= 1
    mo = H2ODeepLearningEstimator(hidden=[16], epochs=5, seed=3, activation="MaxoutWithDropout",
                                  adaptive_rate=False, rate=0.01, momentum_start=0.5, momentum_stable=0.9,
                                  l2=1e-5).train(y="y", training_frame=fr)
    assert mo.training_metrics["AUC"] > 0.65
    rng = np.random.default_rng(7)
    X = rng.normal(size=(2000, 3))
    y = X[:, 0] * 2 + X[:, 1] ** 2
    frr = Frame.from_numpy(np.column_stack([X, y]), names=["a", "b", "c", "y"])
    mr = H2ODeepLearningEstimator(hidden=[32, 32], epochs=20, seed=3, activation="Tanh").train(y="y", training_frame=frr)
    assert mr.training_metrics["r2"] > 0.8
    ae = H2ODeepLearningEstimator(hidden=[2], epochs=10, seed=3, autoencoder=True).train(training_frame=frr)
    an = ae.anomaly(frr).to_pandas()
    assert an.shape == (2000, 1) and np.isfinite(an.values).all()


def test_parse_csv_native(tmp_path):
    path = tmp_path / "d.csv"
    path.write_text("a,b,c\n1,x,2.5\n2,y,NA\n3,x,4\n")
    from h2omx.frame.parse import import_file, parse_setup

    st = parse_setup(str(path))
    assert st["column_names"] == ["a", "b", "c"]
    fr = import_file(str(path))
    pdf = fr.to_pandas()
    assert fr.shape == (3, 3)
    assert list(pdf["b"].astype(str)) == ["x", "y", "x"]
    assert np.isnan(pdf["c"].iloc[1])


def test_tree_early_stopping_checkpoint_and_scoring_history():
    df = _binary_frame(n=4000, seed=1)
    fr = Frame.from_pandas(df)
    tr, va = fr.split_frame((0.7,), seed=3)
    m = H2OGradientBoostingEstimator(ntrees=200, max_depth=6, learn_rate=0.3, stopping_rounds=3,
                                     stopping_tolerance=1e-3, seed=1).train(y="y", training_frame=tr,
                                                                            validation_frame=va)
    assert m.ens.ntrees < 200                       # overfitting stopped early
    assert "validation_logloss" in m.scoring_history[-1]
    a = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1).train(y="y", training_frame=tr)
    b = H2OGradientBoostingEstimator(ntrees=25, max_depth=3, seed=1, checkpoint=a.model_id).train(
        y="y", training_frame=tr)
    c = H2OGradientBoostingEstimator(ntrees=25, max_depth=3, seed=1).train(y="y", training_frame=tr)
    assert b.ens.ntrees == 25
    assert abs(b.training_metrics["AUC"] - c.training_metrics["AUC"]) < 1e-9   # continuation == one run
    d = H2ORandomForestEstimator(ntrees=20, seed=1, score_tree_interval=10).train(y="y", training_frame=tr,
                                                                                  validation_frame=va)
    assert [e["number_of_trees"] for e in d.scoring_history] == [10, 20]


def test_deeplearning_checkpoint_continues():
    df = _binary_frame(n=2000, seed=2)
    fr = Frame.from_pandas(df)
    a = H2ODeepLearningEstimator(hidden=[16], epochs=2, seed=1).train(y="y", training_frame=fr)
    b = H2ODeepLearningEstimator(hidden=[16], epochs=6, seed=1, checkpoint=a.model_id).train(y="y", training_frame=fr)
    assert abs(b.epochs_trained - 6) < 0.2
    assert b.scoring_history[0]["epochs"] > 2
    with pytest.raises(ValueError):
        H2ODeepLearningEstimator(hidden=[8], epochs=3, checkpoint=a.model_id).train(y="y", training_frame=fr)


def test_scoring_adapts_categorical_domains():
    """A scored frame whose categorical levels differ from training (subset,
    other order, unseen level) is mapped onto the training domains by name."""
    from h2omx.models import H2OGradientBoostingEstimator

    rng = np.random.default_rng(5)
    n = 3000
    c = rng.choice(["a", "b", "c"], n)
    yv = np.where(rng.random(n) < np.where(c == "a", 0.9, np.where(c == "b", 0.5, 0.1)), "yes", "no")
    df = pd.DataFrame({"c": pd.Categorical(c), "z": rng.normal(size=n), "y": pd.Categorical(yv)})
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=2, seed=1).train(y="y", training_frame=Frame.from_pandas(df))
    t = pd.DataFrame({"c": pd.Categorical(["c", "a", "zzz"], categories=["zzz", "c", "a"]), "z": [0.0, 0.0, 0.0],
                      "y": pd.Categorical(["no", "yes", "no"], categories=["yes", "no"])})
    P = m.predict_raw(Frame.from_pandas(t)).numpy()
    ref = m.predict_raw(Frame.from_pandas(df.iloc[[list(c).index("c"), list(c).index("a")]].assign(z=0.0))).numpy()
    np.testing.assert_allclose(P[:, :2], ref, rtol=1e-6)
    assert P[1, 1] > 0.7 and P[1, 0] < 0.3
    perf = m.model_performance(Frame.from_pandas(t))
    assert perf["AUC"] == 1.0
