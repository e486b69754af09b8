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


@pytest.mark.parametrize("dist,y", [("gaussian", "y"), ("bernoulli", "yb"), ("poisson", "cnt")])
def test_offset_model_mojo_round_trip(dist, y):
    """The MOJO of an offset model records the offset column and its Generic
    scorer adds it to the margin before the link: predictions match the native
    model's."""
    from h2omx.mojo import GenericModel, mojo_bytes

    df = _frame(seed=3)
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=8, max_depth=3, seed=1, distribution=dist, offset_column="o").train(
        x=["x1", "x2"], y=y, training_frame=fr)
    g = GenericModel(mojo_bytes(m))
    assert g.info["offset_column"] == "o"
    a, b = m.predict(fr).to_pandas(), g.predict(fr).to_pandas()
    for c in a.columns:
        if c == "predict" and dist == "bernoulli":
            assert (a[c].astype(str) == b[c].astype(str)).all()
        else:
            np.testing.assert_allclose(a[c].to_numpy(float), b[c].to_numpy(float), rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError, match="offset_column"):
        g.predict(Frame.from_pandas(df.drop(columns=["o"])))


def test_tweedie_offset_init():
    """H2O Tweedie initF with an offset: log(sum w y e^{o(1-p)} / sum w e^{o(2-p)})."""
    df = _frame(seed=4)
    fr = Frame.from_pandas(df)
    p = 1.3
    m = H2OGradientBoostingEstimator(ntrees=2, max_depth=2, seed=1, distribution="tweedie", tweedie_power=p,
                                     offset_column="o").train(x=["x1", "x2"], y="cnt", training_frame=fr)
    o, yv = df.o.to_numpy(), df.cnt.to_numpy()
    want = np.log((yv * np.exp(o * (1 - p))).sum() / np.exp(o * (2 - p)).sum())
    np.testing.assert_allclose(float(m.ens.init_f[0]), want, rtol=1e-6)


def test_laplace_quantile_init_weighted_quantile():
    """laplace / quantile initial margins are weighted (alpha-)quantiles of
    y - offset at any row count (no torch.quantile 2^24 limit)."""
    from h2omx.models.tree.boost import weighted_quantile

    rng = np.random.default_rng(5)
    r = torch.from_numpy(rng.normal(size=20001))
    w = torch.from_numpy(rng.random(20001))
    for q in (0.1, 0.5, 0.9):
        v = weighted_quantile(r, w, q)
        order = np.argsort(r.numpy())
        cw = np.cumsum(w.numpy()[order])
        want = r.numpy()[order][np.searchsorted(cw, q * cw[-1])]
        assert v == want, (q, v, want)
    assert weighted_quantile(r, None, 0.5) == float(np.sort(r.numpy())[10000])


def test_weighted_quantile_extreme_ranges_exact():
    """Bisection on the ordered int64 key of the value: exact for values
    spanning hundreds of decades, ties and tiny non-zero targets."""
    import torch

    from h2omx.models.tree.boost import weighted_quantile

    rng = np.random.default_rng(0)
    for trial in range(200):
        n = int(rng.integers(1, 40))
        r = rng.standard_normal(n) * 10.0 ** int(rng.integers(-300, 300))
        if trial % 3 == 0:
            r = np.round(r)
        if trial % 7 == 0:
            r[0] = 5e-324                       # smallest subnormal
        w = rng.random(n)
        q = float(rng.random())
        v = weighted_quantile(torch.from_numpy(r), torch.from_numpy(w), q)
        want = min(x for x in np.unique(r) if w[r <= x].sum() >= q * w.sum())
        assert v == want, (trial, v, want)
