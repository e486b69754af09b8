"""Isotonic regression, Aggregator, AdaBoost, DecisionTree (CPU paths; oracles:
sklearn isotonic / plain NumPy)."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models.adaboost import H2OAdaBoostEstimator, H2ODecisionTreeEstimator
from h2omx.models.aggregator import H2OAggregatorEstimator
from h2omx.models.isotonic import H2OIsotonicRegressionEstimator, pav


def test_isotonic_matches_sklearn():
    from sklearn.isotonic import IsotonicRegression

    rng = np.random.default_rng(0)
    x = rng.uniform(0, 10, 800).round(1)
    y = np.log1p(x) + rng.normal(scale=0.3, size=x.size)
    w = rng.uniform(0.5, 2.0, x.size)
    fr = Frame.from_pandas(pd.DataFrame({"x": x, "y": y, "w": w}))
    m = H2OIsotonicRegressionEstimator(weights_column="w").train(x=["x"], y="y", training_frame=fr)
    ref = IsotonicRegression(out_of_bounds="nan").fit(x, y, sample_weight=w)
    q = np.linspace(-1, 11, 97)
    got = m.predict(Frame.from_pandas(pd.DataFrame({"x": q}))).to_pandas()["predict"].to_numpy()
    np.testing.assert_allclose(got, ref.predict(q), rtol=1e-4, atol=1e-4)
    clip = H2OIsotonicRegressionEstimator(out_of_bounds="clip").train(x=["x"], y="y", training_frame=fr)
    g2 = clip.predict(Frame.from_pandas(pd.DataFrame({"x": [-5.0, 50.0]}))).to_pandas()["predict"].to_numpy()
    assert np.isfinite(g2).all() and g2[0] <= g2[1]
    t, v = pav(np.array([1.0, 2, 3]), np.array([3.0, 1, 2]), np.ones(3))
    assert np.all(np.diff(v) >= 0)


def test_aggregator_reduces_and_conserves_counts():
    rng = np.random.default_rng(1)
    centers = rng.normal(size=(20, 4)) * 5
    X = np.concatenate([c + 0.05 * rng.normal(size=(300, 4)) for c in centers])
    df = pd.DataFrame(X, columns=list("abcd"))
    df["k"] = pd.Categorical(np.where(X[:, 0] > 0, "pos", "neg"))
    fr = Frame.from_pandas(df)
    m = H2OAggregatorEstimator(target_num_exemplars=40, rel_tol_num_exemplars=0.5,
                               save_mapping_frame=True).train(training_frame=fr)
    agg = m.aggregated_frame.to_pandas()
    assert 20 <= len(agg) <= 60
    assert agg["counts"].sum() == len(df)
    assert set(agg["k"].astype(str)) <= {"pos", "neg"}
    small = H2OAggregatorEstimator(target_num_exemplars=10000).train(training_frame=fr)
    assert len(small.aggregated_frame.to_pandas()) == len(df)


def _binary(n=3000, seed=0, xor=True):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    y = ((X[:, 0] > 0) ^ (X[:, 1] > 0.5)).astype(int) if xor else (X[:, 0] + X[:, 1] - 0.7 * X[:, 2] > 0).astype(int)
    df = pd.DataFrame(X, columns=list("abcd"))
    df["y"] = pd.Categorical(np.where(y == 1, "t", "f"))
    return df


def test_adaboost_stumps_beat_single_stump():
    df = _binary(xor=False)
    fr = Frame.from_pandas(df)
    one = H2OAdaBoostEstimator(nlearners=1, seed=1).train(y="y", training_frame=fr)
    many = H2OAdaBoostEstimator(nlearners=30, seed=1).train(y="y", training_frame=fr)
    assert many.training_metrics["AUC"] > one.training_metrics["AUC"] + 0.05
    assert len(many.alphas) >= 2 and all(a > 0 for a in many.alphas)
    g = H2OAdaBoostEstimator(nlearners=5, weak_learner="GLM", seed=1).train(y="y", training_frame=fr)
    assert np.isfinite(g.training_metrics["AUC"])
    with pytest.raises(ValueError):
        H2OAdaBoostEstimator(nlearners=2).train(y="a", training_frame=fr)


def test_decision_tree_fits_xor():
    df = _binary(seed=2)
    fr = Frame.from_pandas(df)
    m = H2ODecisionTreeEstimator(max_depth=4, seed=1).train(y="y", training_frame=fr)
    assert m.training_metrics["AUC"] > 0.95


@pytest.mark.parametrize("ext", [0, 2])
def test_extended_isolation_forest_ranks_outliers(ext):
    from sklearn.metrics import roc_auc_score

    from h2omx.models.extended_isolation_forest import H2OExtendedIsolationForestEstimator

    rng = np.random.default_rng(4)
    inl = rng.normal(size=(3000, 3))
    out = rng.uniform(-6, 6, size=(60, 3))
    out = out[np.linalg.norm(out, axis=1) > 4]
    X = np.concatenate([inl, out])
    lab = np.r_[np.zeros(len(inl)), np.ones(len(out))]
    fr = Frame.from_pandas(pd.DataFrame(X, columns=list("abc")))
    m = H2OExtendedIsolationForestEstimator(ntrees=50, sample_size=256, extension_level=ext, seed=3).train(
        training_frame=fr)
    pr = m.predict(fr).to_pandas()
    assert roc_auc_score(lab, pr["anomaly_score"]) > 0.95
    assert ((pr["anomaly_score"] > 0) & (pr["anomaly_score"] < 1)).all()
    assert pr["mean_length"].max() <= 8 + 10
