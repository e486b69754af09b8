"""H2O ``categorical_encoding`` (h2omx/frame/encoding.py): every scheme is
either handled natively by the algorithm or applied as a fitted frame
transform that scoring frames and MOJOs reuse; unknown or unsupported values
raise instead of being ignored."""
from __future__ import annotations

import numpy as np
import pandas as pd
import pytest

from h2omx.frame.encoding import CategoricalEncoder, normalize_scheme
from h2omx.frame.frame import ENUM, Frame
from h2omx.models.deeplearning import H2ODeepLearningEstimator
from h2omx.models.tree_models import H2OGradientBoostingEstimator, H2OXGBoostEstimator


def _df(n=2000, seed=0):
    rng = np.random.default_rng(seed)
    levels = [f"L{i}" for i in range(15)]
    eff = rng.normal(size=15) * 2
    c = rng.integers(0, 15, n)
    x = rng.normal(size=n)
    y = eff[c] + 0.5 * x + 0.3 * rng.normal(size=n) > 0
    cc = np.array([levels[i] for i in c], object)
    cc[rng.uniform(size=n) < 0.05] = None
    return pd.DataFrame({"c": pd.Categorical(cc, categories=levels), "x": x,
                         "y": pd.Categorical(np.where(y, "b", "a"))})


def _fit_enc(scheme, df):
    fr = Frame.from_pandas(df)
    ce = CategoricalEncoder(normalize_scheme(scheme), ["c", "x"], {"c": ENUM, "x": "real"},
                            {"c": list(df["c"].cat.categories), "x": None}, max_levels=4, y="y")
    ce.fit(fr)
    return ce, ce.transform(fr).to_pandas()


def test_one_hot_explicit_and_binary_columns():
    df = _df()
    ce, out = _fit_enc("OneHotExplicit", df)
    assert ce.x_out[:2] == ["c.L0", "c.L1"] and "c.missing(NA)" in ce.x_out and ce.x_out[-1] == "x"
    oh = out[[c for c in ce.x_out if c.startswith("c.")]].to_numpy()
    assert (oh.sum(1) == 1).all()
    na = df["c"].isna().to_numpy()
    assert (out["c.missing(NA)"].to_numpy()[na] == 1).all()
    ce, out = _fit_enc("Binary", df)
    bits = [c for c in ce.x_out if c.startswith("c:")]
    assert len(bits) == 4                     # ceil(log2(15 + 1))
    val = sum(out[b].to_numpy() * (1 << k) for k, b in enumerate(bits))
    codes = df["c"].cat.codes.to_numpy()
    np.testing.assert_array_equal(val, np.where(codes >= 0, codes + 1, 0))


def test_enum_limited_eigen_label_sortbyresponse():
    df = _df()
    ce, out = _fit_enc("EnumLimited", df)
    dom = ce.out_domains["c"]
    assert len(dom) == 5 and dom[-1] == "other"          # 4 most frequent + other
    ce, out = _fit_enc("Eigen", df)
    assert ce.x_out == ["c.Eigen", "x"] and np.isfinite(out["c.Eigen"].to_numpy()[~df["c"].isna().to_numpy()]).all()
    ce, out = _fit_enc("LabelEncoder", df)
    codes = df["c"].cat.codes.to_numpy()
    np.testing.assert_array_equal(np.nan_to_num(out["c"].to_numpy(), nan=-1), codes)
    ce, out = _fit_enc("SortByResponse", df)
    yb = (df["y"] == "b").to_numpy()
    means = [yb[df["c"] == lv].mean() for lv in ce.out_domains["c"]]
    assert all(a <= b + 1e-12 for a, b in zip(means, means[1:]))


@pytest.mark.parametrize("scheme", ["OneHotExplicit", "Binary", "Eigen", "LabelEncoder", "EnumLimited",
                                    "SortByResponse", "AUTO", "Enum"])
def test_gbm_schemes_score_and_mojo_round_trip(tmp_path, scheme):
    from h2omx.mojo import import_mojo

    fr = Frame.from_pandas(_df())
    m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1, categorical_encoding=scheme).train(
        y="y", training_frame=fr)
    assert m.training_metrics["AUC"] > 0.8
    g = import_mojo(m.download_mojo(str(tmp_path)))
    np.testing.assert_allclose(g.predict(fr).to_pandas().iloc[:, -1].to_numpy(),
                               m.predict(fr).to_pandas().iloc[:, -1].to_numpy(), atol=1e-6)
    # a scoring frame with unseen / reordered levels goes through the same encoding
    test = pd.DataFrame({"c": pd.Categorical(["L3", "NEW", None]), "x": [0.1, 0.2, 0.3]})
    p = m.predict(Frame.from_pandas(test)).to_pandas().iloc[:, -1].to_numpy()
    assert np.isfinite(p).all()


def test_xgboost_auto_is_one_hot_and_dl_binary():
    fr = Frame.from_pandas(_df())
    xg = H2OXGBoostEstimator(ntrees=5, max_depth=3, seed=1).train(y="y", training_frame=fr)
    assert "c.L0" in xg.x and "c.missing(NA)" in xg.x
    dl = H2ODeepLearningEstimator(hidden=[8], epochs=1, seed=1, categorical_encoding="Binary").train(
        y="y", training_frame=fr)
    assert dl.x[:4] == ["c:0", "c:1", "c:2", "c:3"]


def test_unknown_and_unsupported_encodings_raise():
    fr = Frame.from_pandas(_df(n=300))
    with pytest.raises(ValueError, match="unknown categorical_encoding"):
        H2OGradientBoostingEstimator(ntrees=2, categorical_encoding="Hash").train(y="y", training_frame=fr)
    with pytest.raises(ValueError, match="OneHotInternal is not supported by tree"):
        H2OGradientBoostingEstimator(ntrees=2, categorical_encoding="OneHotInternal").train(y="y", training_frame=fr)
