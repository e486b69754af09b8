"""Target encoding vs pandas group-by oracles."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models.target_encoder import H2OTargetEncoderEstimator


def _df(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.choice(list("abcdefg"), n, p=[.3, .2, .15, .15, .1, .06, .04])
    b = rng.choice(["u", "v", "w"], n)
    eff = {"a": -1, "b": 0, "c": 1, "d": .5, "e": 2, "f": -2, "g": 0}
    logit = np.array([eff[x] for x in a]) + 0.3 * rng.normal(size=n)
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame({"a": pd.Categorical(a), "b": pd.Categorical(b), "x": rng.normal(size=n),
                       "fold": rng.integers(0, 3, n).astype(float),
                       "y": pd.Categorical(np.where(y == 1, "yes", "no")),
                       "r": logit + rng.normal(size=n)})
    return df


def test_te_plain_and_blending_match_groupby():
    df = _df()
    fr = Frame.from_pandas(df)
    te = H2OTargetEncoderEstimator(columns_to_encode=["a", "b"], noise=0.0).train(
        x=["a", "b"], y="y", training_frame=fr)
    out = te.transform(fr).to_pandas()
    yy = (df.y == "yes").astype(float)
    g = yy.groupby(df.a, observed=True).mean()
    np.testing.assert_allclose(out["a_te"].to_numpy(), df.a.map(g).astype(float).to_numpy(), rtol=1e-6)
    # blending
    te2 = H2OTargetEncoderEstimator(blending=True, inflection_point=5, smoothing=10, noise=0.0).train(
        x=["a"], y="y", training_frame=fr)
    out2 = te2.transform(fr).to_pandas()
    prior = yy.mean()
    n = yy.groupby(df.a, observed=True).count()
    lam = 1 / (1 + np.exp((5 - n) / 10))
    exp = lam * g + (1 - lam) * prior
    np.testing.assert_allclose(out2["a_te"].to_numpy(), df.a.map(exp).astype(float).to_numpy(), rtol=1e-6)
    assert "a" in out2.columns      # originals kept by default


def test_te_leave_one_out_kfold_noise_and_unseen():
    df = _df(seed=1)
    fr = Frame.from_pandas(df)
    te = H2OTargetEncoderEstimator(data_leakage_handling="LeaveOneOut", noise=0.0).train(
        x=["a"], y="r", training_frame=fr)
    out = te.transform(fr, as_training=True).to_pandas()
    s = df.r.groupby(df.a, observed=True).transform("sum")
    c = df.r.groupby(df.a, observed=True).transform("count")
    np.testing.assert_allclose(out["a_te"].to_numpy(), ((s - df.r) / (c - 1)).to_numpy(), rtol=1e-5)
    # k-fold: statistics of the other folds
    tk = H2OTargetEncoderEstimator(data_leakage_handling="KFold", fold_column="fold", noise=0.0).train(
        x=["a"], y="r", training_frame=fr)
    ok = tk.transform(fr, as_training=True).to_pandas()
    exp = np.empty(len(df))
    for f in range(3):
        other = df[df.fold != f]
        m = other.r.groupby(other.a, observed=True).mean()
        sel = (df.fold == f).to_numpy()
        exp[sel] = df.a[sel].map(m).astype(float).to_numpy()
    np.testing.assert_allclose(ok["a_te"].to_numpy(), exp, rtol=1e-5)
    # noise is bounded and seeded; scoring (as_training=False) is noise-free
    tn = H2OTargetEncoderEstimator(noise=0.05, seed=3).train(x=["a"], y="r", training_frame=fr)
    d = tn.transform(fr, as_training=True).to_pandas()["a_te"] - tn.transform(fr).to_pandas()["a_te"]
    assert 0 < d.abs().max() <= 0.05 + 1e-6
    # unseen level -> prior
    new = Frame.from_pandas(pd.DataFrame({"a": pd.Categorical(["zzz", "a"]), "r": [0.0, 0.0]}))
    enc = te.transform(new).to_pandas()["a_te"].to_numpy()
    np.testing.assert_allclose(enc[0], df.r.mean(), rtol=1e-5)


def test_te_multinomial_columns():
    df = _df(seed=2)
    df["m"] = pd.Categorical(np.array(["p", "q", "s"])[np.arange(len(df)) % 3])
    fr = Frame.from_pandas(df)
    te = H2OTargetEncoderEstimator(noise=0.0, keep_original_categorical_columns=False).train(
        x=["a"], y="m", training_frame=fr)
    out = te.transform(fr).to_pandas()
    assert {"a_q_te", "a_s_te"} <= set(out.columns) and "a" not in out.columns
    g = (df.m == "s").astype(float).groupby(df.a, observed=True).mean()
    np.testing.assert_allclose(out["a_s_te"].to_numpy(), df.a.map(g).astype(float).to_numpy(), rtol=1e-6)


def test_te_bad_kfold_config():
    fr = Frame.from_pandas(_df(n=100))
    with pytest.raises(ValueError):
        H2OTargetEncoderEstimator(data_leakage_handling="KFold").train(x=["a"], y="y", training_frame=fr)
