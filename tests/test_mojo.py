"""MOJO round trips: export every algorithm, re-import it as a Generic model
and check the scores match the original model.  (Binary parity with H2O's
h2o-genmodel jar is unpinned: no JVM / jar in this environment.)"""
import io
import zipfile

import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame import Frame
from h2omx.models import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                          H2OKMeansEstimator, H2ORandomForestEstimator, H2OStackedEnsembleEstimator,
                          H2OXGBoostEstimator)
from h2omx.mojo import GenericModel, decode_tree, encode_tree, mojo_bytes, read_mojo


def _df(n=1500, seed=0, classes=2):
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n),
                       "c": rng.choice(["u", "v", "w"], n), "d": rng.normal(size=n)})
    df.loc[rng.random(n) < 0.05, "a"] = np.nan
    df.loc[rng.random(n) < 0.05, "c"] = None
    s = df.a.fillna(0) - df.b + (df.c == "u") * 1.5
    if classes == 2:
        df["y"] = np.where(rng.random(n) < 1 / (1 + np.exp(-s)), "pos", "neg")
    elif classes > 2:
        df["y"] = np.array(["k0", "k1", "k2"])[np.digitize(s + rng.normal(size=n) * 0.5, [-0.5, 0.8])]
    else:
        df["y"] = s + rng.normal(size=n) * 0.1
    return df


def _roundtrip(model, fr, atol):
    data = mojo_bytes(model)
    names = zipfile.ZipFile(io.BytesIO(data)).namelist()
    assert "model.ini" in names
    g = GenericModel(data)
    a = model.predict_raw(fr).cpu().double()
    b = g.predict_raw(fr).cpu().double()
    assert a.shape == b.shape
    assert torch.allclose(a, b, atol=atol, rtol=0), (a - b).abs().max()
    return g, names


@pytest.mark.parametrize("cls,kw", [(H2OGradientBoostingEstimator, dict(ntrees=8, max_depth=4)),
                                    (H2OXGBoostEstimator, dict(ntrees=8, max_depth=4)),
                                    (H2ORandomForestEstimator, dict(ntrees=5, max_depth=12))])
@pytest.mark.parametrize("classes", [2, 3, 0])
def test_tree_mojo(cls, kw, classes):
    fr = Frame.from_pandas(_df(classes=classes))
    m = cls(seed=1, **kw).train(y="y", training_frame=fr)
    g, names = _roundtrip(m, fr, 1e-6)
    assert any(n.startswith("trees/t00_") for n in names)
    info = read_mojo(mojo_bytes(m))["info"]
    assert info["n_trees"] == kw["ntrees"] and info["algo"] == m.algo


def test_tree_codec_single_leaf_and_deep():
    from h2omx.models.tree.structs import TREE_NODE_DTYPE

    t = np.zeros(1, TREE_NODE_DTYPE)
    t["feat"] = -1
    t["value"] = 3.5
    d = decode_tree(encode_tree(t))
    assert d["feat"][0] == -1 and d["value"][0] == np.float32(3.5)


@pytest.mark.parametrize("family,classes", [("binomial", 2), ("multinomial", 3), ("gaussian", 0)])
def test_glm_mojo(family, classes):
    fr = Frame.from_pandas(_df(classes=classes))
    m = H2OGeneralizedLinearEstimator(family=family, lambda_=0.0).train(y="y", training_frame=fr)
    _roundtrip(m, fr, 1e-5)


def test_kmeans_dl_mojo():
    df = _df(classes=2)
    fr = Frame.from_pandas(df)
    km = H2OKMeansEstimator(k=4, seed=3).train(x=["a", "b", "c", "d"], training_frame=fr)
    _roundtrip(km, fr, 0)
    for act in ("Rectifier", "Tanh", "Maxout"):
        dl = H2ODeepLearningEstimator(hidden=[8, 8], epochs=2, seed=2, activation=act).train(y="y", training_frame=fr)
        _roundtrip(dl, fr, 1e-5)
    dlr = H2ODeepLearningEstimator(hidden=[8], epochs=2, seed=2).train(y="y", training_frame=Frame.from_pandas(
        _df(classes=0)))
    _roundtrip(dlr, Frame.from_pandas(_df(classes=0)), 1e-4)


def test_stacked_ensemble_mojo():
    fr = Frame.from_pandas(_df(classes=2))
    cv = dict(nfolds=3, fold_assignment="Modulo", keep_cross_validation_predictions=True, seed=1)
    a = H2OGradientBoostingEstimator(ntrees=5, **cv).train(y="y", training_frame=fr)
    b = H2OGeneralizedLinearEstimator(lambda_=0.0, **cv).train(y="y", training_frame=fr)
    se = H2OStackedEnsembleEstimator(base_models=[a.model_id, b.model_id]).train(y="y", training_frame=fr)
    assert se.training_metrics["AUC"] >= min(a.training_metrics["AUC"], b.training_metrics["AUC"]) - 0.02
    _roundtrip(se, fr, 1e-5)
