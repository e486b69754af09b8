"""offset_column for GBM / XGBoost (H2O: margin = init_f + offset + trees).

Gaussian: the model trained with an offset grows the same trees as the model
trained on ``y - offset`` (identical residuals), so its predictions differ by
exactly the offset.  Bernoulli / Poisson: the initial margin is the fit with
the offset held fixed (mean of sigmoid(c + o) equals the mean response;
c = log(sum y / sum exp(o)))."""
import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame import Frame
from h2omx.models import H2OGradientBoostingEstimator


def _frame(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({"x1": rng.normal(size=n), "x2": rng.normal(size=n), "o": 0.5 * rng.normal(size=n)})
    df["y"] = 1.5 + df.o + np.sin(df.x1) + 0.1 * rng.normal(size=n)
    df["yo"] = df.y - df.o
    eta = -0.3 + df.o + df.x1
    df["yb"] = pd.Categorical(np.where(rng.random(n) < 1 / (1 + np.exp(-eta)), "1", "0"))
    df["cnt"] = rng.poisson(np.exp(0.2 + df.o + 0.3 * df.x2)).astype(float)
    return df


def test_gaussian_offset_equals_shifted_response():
    df = _frame()
    fr = Frame.from_pandas(df)
    kw = dict(ntrees=20, max_depth=3, seed=1, learn_rate=0.2)
    m = H2OGradientBoostingEstimator(offset_column="o", **kw).train(x=["x1", "x2"], y="y", training_frame=fr)
    m0 = H2OGradientBoostingEstimator(**kw).train(x=["x1", "x2"], y="yo", training_frame=fr)
    assert "o" not in m.x
    np.testing.assert_allclose(float(m.ens.init_f[0]), float(df.yo.mean()), rtol=1e-6)
    p = m.predict(fr).to_pandas()["predict"].to_numpy()
    p0 = m0.predict(fr).to_pandas()["predict"].to_numpy()
    np.testing.assert_allclose(p - df.o.to_numpy(), p0, atol=2e-5)


def test_bernoulli_and_poisson_offset_init():
    df = _frame(seed=1)
    fr = Frame.from_pandas(df)
    mb = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1, offset_column="o").train(
        x=["x1", "x2"], y="yb", training_frame=fr)
    c = float(mb.ens.init_f[0])
    yb = (df.yb == "1").to_numpy(float)
    np.testing.assert_allclose(np.mean(1 / (1 + np.exp(-(c + df.o.to_numpy())))), yb.mean(), rtol=1e-8)
    auc_off = mb.training_metrics["AUC"]
    assert auc_off > 0.7
    mp = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1, distribution="poisson",
                                      offset_column="o").train(x=["x1", "x2"], y="cnt", training_frame=fr)
    np.testing.assert_allclose(float(mp.ens.init_f[0]), np.log(df.cnt.sum() / np.exp(df.o).sum()), rtol=1e-6)
    pred = mp.predict(fr).to_pandas()["predict"].to_numpy()
    assert np.all(pred > 0) and abs(pred.mean() - df.cnt.mean()) < 0.05 * df.cnt.mean()


def test_offset_rejected_for_drf():
    from h2omx.models import H2ORandomForestEstimator

    fr = Frame.from_pandas(_frame(500))
    with pytest.raises(ValueError, match="offset_column"):
        H2ORandomForestEstimator(ntrees=2, offset_column="o").train(x=["x1", "x2"], y="y", training_frame=fr)


@pytest.mark.gpu
def test_gaussian_and_bernoulli_offset_gpu(cuda_dev):
    """Device-resident frame through the HIP tree engine: the gaussian offset
    model equals the shifted-response model; bernoulli init solves the offset fit."""
    df = _frame(20000, seed=2)
    fr = Frame.from_pandas(df, device=cuda_dev)
    kw = dict(ntrees=10, max_depth=4, seed=1, learn_rate=0.2)
    m = H2OGradientBoostingEstimator(offset_column="o", **kw).train(x=["x1", "x2"], y="y", training_frame=fr)
    m0 = H2OGradientBoostingEstimator(**kw).train(x=["x1", "x2"], y="yo", training_frame=fr)
    p = m.predict(fr).to_pandas()["predict"].to_numpy()
    p0 = m0.predict(fr).to_pandas()["predict"].to_numpy()
    np.testing.assert_allclose(p - df.o.to_numpy(), p0, atol=1e-4)
    mb = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1, offset_column="o").train(
        x=["x1", "x2"], y="yb", training_frame=fr)
    c = float(mb.ens.init_f[0])
    yb = (df.yb == "1").to_numpy(float)
    np.testing.assert_allclose(np.mean(1 / (1 + np.exp(-(c + df.o.to_numpy())))), yb.mean(), rtol=1e-6)
    assert mb.training_metrics["AUC"] > 0.7
