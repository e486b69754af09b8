"""Newer estimators on device-resident frames (HIP GEMMs / tree engine) match
their CPU runs."""
import numpy as np
import pandas as pd
import pytest
import torch

from h2omx import _native
from h2omx.frame import Frame
from h2omx.models import (H2OAdaBoostEstimator, H2OAggregatorEstimator, H2OCoxProportionalHazardsEstimator,
                          H2OExtendedIsolationForestEstimator, H2OGeneralizedAdditiveEstimator,
                          H2OGeneralizedLowRankEstimator, H2OIsotonicRegressionEstimator, H2OModelSelectionEstimator,
                          H2ORuleFitEstimator, H2OSingularValueDecompositionEstimator, H2OTargetEncoderEstimator,
                          H2OWord2vecEstimator)

pytestmark = pytest.mark.gpu


def _df(n=6000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 5)).astype(np.float32)
    df = pd.DataFrame(X, columns=list("abcde"))
    df["g"] = pd.Categorical(rng.choice(list("pqrst"), n))
    f = np.sin(2 * X[:, 0]) + X[:, 1] - 0.5 * X[:, 2]
    df["y"] = f + 0.2 * rng.normal(size=n)
    df["yb"] = pd.Categorical(np.where(rng.random(n) < 1 / (1 + np.exp(-2 * f)), "1", "0"))
    df["t"] = np.ceil(rng.exponential(np.exp(-0.5 * X[:, 0])) * 10) / 10
    df["ev"] = (rng.random(n) < 0.7).astype(float)
    return df


@pytest.fixture(scope="module")
def frames():
    df = _df()
    return df, Frame.from_pandas(df), Frame.from_pandas(df, device="cuda")


def test_dimred_and_te_gpu(cuda_dev, frames):
    df, fc, fg = frames
    sc = H2OSingularValueDecompositionEstimator(nv=3).train(x=list("abcde"), training_frame=fc)
    sg = H2OSingularValueDecompositionEstimator(nv=3).train(x=list("abcde"), training_frame=fg)
    np.testing.assert_allclose(sg.d, sc.d, rtol=1e-4)
    gc = H2OGeneralizedLowRankEstimator(k=3, init="SVD", max_iterations=40).train(x=list("abcde"), training_frame=fc)
    gg = H2OGeneralizedLowRankEstimator(k=3, init="SVD", max_iterations=40).train(x=list("abcde"), training_frame=fg)
    np.testing.assert_allclose(gg.objective, gc.objective, rtol=1e-3)
    assert gg.representation.vecs[0].data.is_cuda
    tc = H2OTargetEncoderEstimator(noise=0.0).train(x=["g"], y="y", training_frame=fc)
    tg = H2OTargetEncoderEstimator(noise=0.0).train(x=["g"], y="y", training_frame=fg)
    np.testing.assert_allclose(tg.transform(fg).to_pandas()["g_te"], tc.transform(fc).to_pandas()["g_te"], rtol=1e-5)
    ag = H2OAggregatorEstimator(target_num_exemplars=200).train(x=list("abc"), training_frame=fg)
    assert ag.aggregated_frame.to_pandas()["counts"].sum() == len(df)
    assert any("dense" in p for p in _native.loaded_libraries())


def test_glm_family_gpu(cuda_dev, frames):
    df, fc, fg = frames
    kw = dict(family="gaussian", gam_columns=["a"], num_knots=[8], lambda_=0.0)
    mc = H2OGeneralizedAdditiveEstimator(**kw).train(x=list("abc"), y="y", training_frame=fc)
    mg = H2OGeneralizedAdditiveEstimator(**kw).train(x=list("abc"), y="y", training_frame=fg)
    for k, v in mc.coef().items():
        assert abs(mg.coef()[k] - v) < 2e-3 * max(1.0, abs(v)), k
    sc = H2OModelSelectionEstimator(mode="maxr", max_predictor_number=3).train(x=list("abcde"), y="y",
                                                                              training_frame=fc)
    sg = H2OModelSelectionEstimator(mode="maxr", max_predictor_number=3).train(x=list("abcde"), y="y",
                                                                              training_frame=fg)
    assert [r["predictors"] for r in sg.result()] == [r["predictors"] for r in sc.result()]
    cc = H2OCoxProportionalHazardsEstimator(stop_column="t").train(x=["a", "b"], y="ev", training_frame=fc)
    cg = H2OCoxProportionalHazardsEstimator(stop_column="t").train(x=["a", "b"], y="ev", training_frame=fg)
    np.testing.assert_allclose(cg.beta, cc.beta, rtol=1e-5)
    ic = H2OIsotonicRegressionEstimator().train(x=["a"], y="y", training_frame=fc)
    ig = H2OIsotonicRegressionEstimator().train(x=["a"], y="y", training_frame=fg)
    np.testing.assert_allclose(ig.thresholds_y, ic.thresholds_y, rtol=1e-5, atol=1e-6)


def test_tree_based_gpu(cuda_dev, frames):
    df, fc, fg = frames
    rf = H2ORuleFitEstimator(min_rule_length=2, max_rule_length=2, rule_generation_ntrees=10, seed=1).train(
        x=list("abcde"), y="y", training_frame=fg)
    assert rf.training_metrics["MSE"] < 0.3
    ab = H2OAdaBoostEstimator(nlearners=10, seed=1).train(x=list("abcde"), y="yb", training_frame=fg)
    assert ab.training_metrics["AUC"] > 0.75
    ei = H2OExtendedIsolationForestEstimator(ntrees=30, extension_level=2, seed=1).train(x=list("abcde"),
                                                                                      training_frame=fg)
    sc = ei.predict(fg).to_pandas()["anomaly_score"]
    assert sc.between(0, 1).all()
    ecpu = H2OExtendedIsolationForestEstimator(ntrees=30, extension_level=2, seed=1).train(x=list("abcde"),
                                                                                        training_frame=fc)
    np.testing.assert_allclose(sc.to_numpy(), ecpu.predict(fc).to_pandas()["anomaly_score"].to_numpy(), rtol=1e-4)
    assert any("tree" in p for p in _native.loaded_libraries())


def test_word2vec_gpu(cuda_dev):
    rng = np.random.default_rng(0)
    topics = [[f"a{i}" for i in range(6)], [f"b{i}" for i in range(6)]]
    toks = []
    for _ in range(2000):
        toks += list(rng.choice(topics[rng.integers(0, 2)], size=6)) + [None]
    fr = Frame.from_pandas(pd.DataFrame({"w": toks}), device="cuda")
    m = H2OWord2vecEstimator(vec_size=16, window_size=3, epochs=5, min_word_freq=3, seed=1, init_learning_rate=0.05,
                             sent_sample_rate=0.0).train(training_frame=fr)
    assert m.vectors.is_cuda
    syn = m.find_synonyms("a0", 4)
    assert sum(w.startswith("a") for w in syn) >= 3, syn
