"""Isolation Forest: outlier detection, agreement with scikit-learn's
IsolationForest score distribution, contamination labels, MOJO round trip,
REST build (CPU)."""
import numpy as np
import pytest

from h2omx.frame import Frame
from h2omx.models import H2OIsolationForestEstimator
from h2omx.models.isolation_forest import avg_path


@pytest.fixture(scope="module")
def data():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(20000, 5)).astype(np.float32)
    X[:60] += rng.choice([-6.0, 6.0], size=(60, 5)).astype(np.float32)
    X[100:110, 2] = np.nan
    lab = np.zeros(len(X))
    lab[:60] = 1
    return X, lab


def test_avg_path():
    # c(n) for n = 256 (the default sample size) ~ 10.24
    assert abs(avg_path([256])[0] - 10.2448) < 1e-3
    assert avg_path([1])[0] == 0.0 and avg_path([2])[0] == 1.0


def test_isolation_forest_detects_outliers(data):
    from sklearn.ensemble import IsolationForest
    from sklearn.metrics import roc_auc_score

    X, lab = data
    fr = Frame.from_numpy(X, names=list("abcde"))
    m = H2OIsolationForestEstimator(ntrees=100, seed=3).train(training_frame=fr)
    P = m.predict(fr).to_pandas()
    assert list(P.columns) == ["predict", "mean_length"]
    assert roc_auc_score(lab, P["predict"]) > 0.99
    assert 0.0 <= P["predict"].min() and P["predict"].max() <= 1.0 + 1e-6
    assert m.summary()["max_depth"] <= 8
    ok = ~np.isnan(X).any(1)
    sk = IsolationForest(n_estimators=100, random_state=0).fit(X[ok])
    ours = m.anomaly_score(Frame.from_numpy(X[ok], names=list("abcde"))).numpy()
    ref = -sk.score_samples(X[ok])
    assert abs(ours.mean() - ref.mean()) < 0.01
    assert np.corrcoef(ours, ref)[0, 1] > 0.9


def test_contamination_and_mojo(data, tmp_path):
    from h2omx.mojo import import_mojo

    X, lab = data
    fr = Frame.from_numpy(X, names=list("abcde"))
    m = H2OIsolationForestEstimator(ntrees=40, seed=5, contamination=0.01).train(training_frame=fr)
    P = m.predict(fr).to_pandas()
    assert list(P.columns) == ["predict", "score", "mean_length"]
    frac = P["predict"].mean()
    assert 0.005 <= frac <= 0.02
    assert P["predict"][:60].mean() > 0.9
    path = m.download_mojo(str(tmp_path))
    g = import_mojo(path)
    np.testing.assert_allclose(g.predict_raw(fr).numpy(), m.predict_raw(fr).numpy(), rtol=1e-5, atol=1e-5)


def test_sample_rate_and_column_sampling(data):
    X, _ = data
    fr = Frame.from_numpy(X, names=list("abcde"))
    m = H2OIsolationForestEstimator(ntrees=5, sample_rate=0.2, max_depth=12, col_sample_rate_per_tree=0.6,
                                    seed=1).train(training_frame=fr)
    used = {int(f) for t in m.ens.trees for f in t["feat"] if f >= 0}
    assert m.sample_size == 4000 and len(used) <= 5
    assert m.training_metrics["mean_score"] > 5
