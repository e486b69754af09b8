"""Estimator-level GPU tests: every algorithm trains on a device-resident
frame through its HIP kernels and matches the CPU path / an independent
reference (sklearn) within tolerance."""
import numpy as np
import pandas as pd
import pytest
import torch

from h2omx import _native
from h2omx.frame import Frame
from h2omx.models import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                          H2OKMeansEstimator, H2ORandomForestEstimator, H2OXGBoostEstimator)

pytestmark = pytest.mark.gpu


def _binary_df(n=20000, p=8, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, p)).astype(np.float32)
    logit = X[:, 0] - 0.7 * X[:, 1] + 0.5 * X[:, 2] * X[:, 3]
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(int)
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(p)])
    df["y"] = pd.Categorical(np.where(y == 1, "yes", "no"))
    return df


def test_glm_binomial_gpu_matches_cpu(cuda_dev):
    df = _binary_df()
    cpu = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0).train(y="y", training_frame=Frame.from_pandas(df))
    gpu = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0).train(
        y="y", training_frame=Frame.from_pandas(df, device=cuda_dev))
    for k, v in cpu.coef().items():
        assert abs(gpu.coef()[k] - v) < 2e-3, k
    assert abs(gpu.training_metrics["AUC"] - cpu.training_metrics["AUC"]) < 1e-3
    assert "dense" in " ".join(_native.loaded_libraries())


def test_glm_wide_categorical_gpu_matches_cpu(cuda_dev):
    """A 400-level categorical (one-hot > 254 columns) no longer fails on the
    GPU: the wide IRLS path matches the CPU reference coefficients."""
    rng = np.random.default_rng(7)
    n = 30000
    lev = rng.integers(0, 400, n)
    eff = rng.normal(scale=0.5, size=400)
    x = rng.normal(size=n)
    eta = eff[lev] + 0.7 * x
    y = np.where(rng.random(n) < 1 / (1 + np.exp(-eta)), "1", "0")
    df = pd.DataFrame({"cat": pd.Categorical([f"L{v}" for v in lev]), "x": x, "y": pd.Categorical(y)})
    kw = dict(family="binomial", lambda_=1e-4, alpha=0.0, max_iterations=10)
    g = H2OGeneralizedLinearEstimator(**kw).train(y="y", training_frame=Frame.from_pandas(df, device=cuda_dev))
    c = H2OGeneralizedLinearEstimator(**kw).train(y="y", training_frame=Frame.from_pandas(df))
    cg, cc = g.coef(), c.coef()
    assert len(cg) > 300
    err = max(abs(cg[k] - cc[k]) for k in cc)
    assert err < 2e-3, err
    assert abs(g.training_metrics["AUC"] - c.training_metrics["AUC"]) < 1e-4


def test_glm_multinomial_and_poisson_gpu(cuda_dev):
    rng = np.random.default_rng(1)
    X = rng.normal(size=(30000, 5)).astype(np.float32)
    logits = X @ rng.normal(size=(5, 3))
    y = np.array([rng.choice(3, p=np.exp(l) / np.exp(l).sum()) for l in logits])
    df = pd.DataFrame(X, columns=list("abcde"))
    df["y"] = pd.Categorical([f"c{v}" for v in y])
    m = H2OGeneralizedLinearEstimator(family="multinomial", lambda_=0.0).train(
        y="y", training_frame=Frame.from_pandas(df, device=cuda_dev))
    mc = H2OGeneralizedLinearEstimator(family="multinomial", lambda_=0.0).train(y="y", training_frame=Frame.from_pandas(df))
    assert abs(m.training_metrics["logloss"] - mc.training_metrics["logloss"]) < 1e-3
    yc = rng.poisson(np.exp(0.2 + X[:, 0] * 0.3))
    dfp = pd.DataFrame(X, columns=list("abcde"))
    dfp["y"] = yc.astype(np.float32)
    mp = H2OGeneralizedLinearEstimator(family="poisson", lambda_=0.0).train(
        y="y", training_frame=Frame.from_pandas(dfp, device=cuda_dev))
    assert abs(mp.coef()["a"] - 0.3) < 0.03


def test_kmeans_gpu_matches_cpu(cuda_dev):
    rng = np.random.default_rng(2)
    cent = rng.normal(0, 6, (6, 10))
    X = np.concatenate([c + rng.normal(0, 1, (3000, 10)) for c in cent]).astype(np.float32)
    names = [f"x{i}" for i in range(10)]
    mc = H2OKMeansEstimator(k=6, seed=3, max_iterations=30).train(training_frame=Frame.from_numpy(X, names=names))
    mg = H2OKMeansEstimator(k=6, seed=3, max_iterations=30).train(
        training_frame=Frame.from_numpy(X, names=names, device=cuda_dev))
    assert abs(mg.stats["tot_withinss"] - mc.stats["tot_withinss"]) / mc.stats["tot_withinss"] < 1e-4
    assert sorted(mg.stats["size"]) == sorted(mc.stats["size"])


@pytest.mark.parametrize("d,k", [(300, 5), (40, 200), (520, 150)])
def test_kmeans_gpu_wide_hip_path_matches_reference(cuda_dev, d, k):
    """Shapes beyond the fused kernel (d > 256 or k > 128) run on the HIP
    staging / MFMA GEMM / argmin / one-hot kernels; one Lloyd pass agrees with
    the fp64 reference."""
    import torch

    from h2omx.ops import dense as Dev
    from h2omx.reference import dense as Ref

    rng = np.random.default_rng(d + k)
    n = 20000
    X = rng.normal(size=(d, n)).astype(np.float32)
    X[0, ::97] = np.nan
    C = X[:, rng.choice(n, k, replace=False)].T.copy()
    C[np.isnan(C)] = 0
    Xt = torch.from_numpy(X)
    a_g, s_g, c_g, e_g = Dev.kmeans_step(Xt.to(cuda_dev), torch.from_numpy(C).to(cuda_dev))
    a_r, s_r, c_r, e_r = Ref.kmeans_step(torch.nan_to_num(Xt), torch.from_numpy(C))
    agree = (a_g.cpu().numpy() == a_r.numpy()).mean()
    assert agree > 0.999, agree
    if agree == 1.0:
        np.testing.assert_allclose(s_g, s_r, rtol=1e-4, atol=1e-2)
        np.testing.assert_array_equal(c_g, c_r)
        np.testing.assert_allclose(e_g, e_r, rtol=1e-4, atol=1e-3)   # singleton clusters: SSE ~ 0
    assert c_g.sum() == n
    m = H2OKMeansEstimator(k=5, seed=1, max_iterations=5).train(
        training_frame=Frame.from_numpy(X.T[:4000, :300].copy() if d >= 300 else X.T[:4000].copy(),
                                        names=[f"c{i}" for i in range(min(d, 300))], device=cuda_dev))
    assert sum(m.stats["size"]) == 4000


def test_deeplearning_gpu(cuda_dev):
    df = _binary_df(n=50000)
    fr = Frame.from_pandas(df, device=cuda_dev)
    m = H2ODeepLearningEstimator(hidden=[64, 64], epochs=3, seed=1).train(y="y", training_frame=fr)
    assert m.training_metrics["AUC"] > 0.74
    assert next(iter(m.net.flat.device.type for _ in [0])) == "cuda"
    r = H2ODeepLearningEstimator(hidden=[32], epochs=3, seed=1, activation="Tanh", adaptive_rate=False,
                                 rate=0.001).train(y="x0", training_frame=fr)
    assert np.isfinite(r.training_metrics["MSE"])


@pytest.mark.parametrize("act,precision", [("Rectifier", "fp32"), ("Maxout", "fp32"), ("Tanh", "bf16")])
def test_deeplearning_graph_replay_matches_eager(cuda_dev, monkeypatch, act, precision):
    """The HIP-graph replay of the update step (models/deeplearning.py _DLTrainer)
    runs the same kernels in the same order as the eager step: identical weights."""
    df = _binary_df(n=30000)
    fr = Frame.from_pandas(df, device=cuda_dev)
    kw = dict(hidden=[64, 32], epochs=2, seed=4, activation=act, precision=precision)
    out = {}
    from h2omx.models.deeplearning import _DLTrainer

    for g in ("0", "1"):
        monkeypatch.setattr(_DLTrainer, "GRAPH", g == "1")
        out[g] = H2ODeepLearningEstimator(**kw).train(y="y", training_frame=fr)
    assert torch.equal(out["0"].net.flat, out["1"].net.flat)
    assert out["1"].training_metrics["AUC"] == out["0"].training_metrics["AUC"]


def test_deeplearning_folds_in_adadelta_match_separate_reduces(cuda_dev, monkeypatch):
    """Bias-gradient slices and the output layer's split partials folded inside
    the ADADELTA kernel (_DLTrainer.FOLD) train the same model as the separate
    reduce launches: the bias folds are the same fp64 sums, the output layer's
    fold only changes the fp32 summation order."""
    from h2omx.models import deeplearning as DLM

    df = _binary_df(n=30000)
    fr = Frame.from_pandas(df, device=cuda_dev)
    kw = dict(hidden=[64, 64, 32], epochs=1, seed=6)
    out = {}
    for fold in (False, True):
        monkeypatch.setattr(DLM._DLTrainer, "FOLD", fold)
        out[fold] = H2ODeepLearningEstimator(**kw).train(y="y", training_frame=fr)
    a, b = out[False].net.flat, out[True].net.flat
    assert float((a - b).abs().max()) < 1e-3 * float(a.abs().max())
    assert abs(out[False].training_metrics["AUC"] - out[True].training_metrics["AUC"]) < 0.005


@pytest.mark.parametrize("cls", [H2OGradientBoostingEstimator, H2OXGBoostEstimator, H2ORandomForestEstimator])
def test_tree_estimators_gpu(cuda_dev, cls):
    df = _binary_df()
    kw = dict(ntrees=20, max_depth=5, seed=1)
    m = cls(**kw).train(y="y", training_frame=Frame.from_pandas(df, device=cuda_dev))
    mc = cls(**kw).train(y="y", training_frame=Frame.from_pandas(df))
    assert abs(m.training_metrics["AUC"] - mc.training_metrics["AUC"]) < 0.01
    # DRF reports out-of-bag training metrics (H2O semantics): lower than in-sample
    assert m.training_metrics["AUC"] > (0.72 if cls is H2ORandomForestEstimator else 0.75)
    assert "tree" in " ".join(_native.loaded_libraries())


def test_gbm_gpu_early_stopping_and_checkpoint(cuda_dev):
    df = _binary_df(n=30000, seed=4)
    fr = Frame.from_pandas(df, device=cuda_dev)
    tr, va = fr.split_frame((0.7,), seed=3)
    m = H2OGradientBoostingEstimator(ntrees=300, max_depth=8, learn_rate=0.5, stopping_rounds=3, seed=1,
                                     score_tree_interval=5).train(y="y", training_frame=tr, validation_frame=va)
    assert m.ens.ntrees < 300 and "validation_auc" in m.scoring_history[-1]
    a = H2OGradientBoostingEstimator(ntrees=6, max_depth=4, seed=1).train(y="y", training_frame=tr)
    b = H2OGradientBoostingEstimator(ntrees=15, max_depth=4, seed=1, checkpoint=a.model_id).train(
        y="y", training_frame=tr)
    c = H2OGradientBoostingEstimator(ntrees=15, max_depth=4, seed=1).train(y="y", training_frame=tr)
    assert abs(b.training_metrics["AUC"] - c.training_metrics["AUC"]) < 1e-6


def test_pca_and_naive_bayes_gpu(cuda_dev):
    from h2omx.models import H2ONaiveBayesEstimator, H2OPrincipalComponentAnalysisEstimator

    rng = np.random.default_rng(9)
    X = (rng.normal(size=(40000, 3)) @ rng.normal(size=(3, 12))).astype(np.float32)
    names = [f"x{i}" for i in range(12)]
    g = H2OPrincipalComponentAnalysisEstimator(k=3, transform="STANDARDIZE").train(
        training_frame=Frame.from_numpy(X, names=names, device=cuda_dev))
    c = H2OPrincipalComponentAnalysisEstimator(k=3, transform="STANDARDIZE").train(
        training_frame=Frame.from_numpy(X, names=names))
    np.testing.assert_allclose(g.eigenvalues, c.eigenvalues, rtol=1e-3)
    assert sum(g.importance["Proportion of Variance"]) > 0.999
    df = _binary_df(n=20000)
    nb_g = H2ONaiveBayesEstimator().train(y="y", training_frame=Frame.from_pandas(df, device=cuda_dev))
    nb_c = H2ONaiveBayesEstimator().train(y="y", training_frame=Frame.from_pandas(df))
    assert abs(nb_g.training_metrics["AUC"] - nb_c.training_metrics["AUC"]) < 1e-4


def test_isolation_forest_gpu(cuda_dev):
    from h2omx.models import H2OIsolationForestEstimator

    rng = np.random.default_rng(4)
    X = rng.normal(size=(200000, 6)).astype(np.float32)
    X[:100] += 7
    names = [f"x{i}" for i in range(6)]
    fr = Frame.from_numpy(X, names=names, device=cuda_dev)
    m = H2OIsolationForestEstimator(ntrees=50, seed=2).train(training_frame=fr)
    S = m.predict_raw(fr)
    assert S.is_cuda
    s = S[0].cpu().numpy()
    assert s[:100].mean() > 0.8 > s[100:].mean() + 0.4
    c = H2OIsolationForestEstimator(ntrees=50, seed=2).train(training_frame=Frame.from_numpy(X, names=names))
    assert abs(c.training_metrics["mean_score"] - m.training_metrics["mean_score"]) < 0.2
    assert "tree" in " ".join(_native.loaded_libraries())


def test_deeplearning_bf16_precision_gpu(cuda_dev):
    """precision="bf16" (bf16 matrix-core GEMMs, fp32 master weights) reaches the
    fp32 model's quality; regression and Tanh included."""
    df = _binary_df(n=50000)
    fr = Frame.from_pandas(df, device=cuda_dev)
    kw = dict(hidden=[64, 64], epochs=3, seed=1)
    a32 = H2ODeepLearningEstimator(**kw).train(y="y", training_frame=fr).training_metrics["AUC"]
    m = H2ODeepLearningEstimator(precision="bf16", **kw).train(y="y", training_frame=fr)
    assert m.training_metrics["AUC"] > a32 - 0.01 and m.training_metrics["AUC"] > 0.74
    r = H2ODeepLearningEstimator(hidden=[32], epochs=3, seed=1, activation="Tanh", precision="bf16").train(
        y="x0", training_frame=fr)
    assert np.isfinite(r.training_metrics["MSE"]) and r.training_metrics["MSE"] < 1.0


def test_gpu_fits_never_touch_the_cpu_reference(cuda_dev):
    """The backend router sends every op with a device tensor to the HIP layer:
    GBM / XGBoost / DRF / GLM / DL / K-Means fits on a GPU frame import no
    module of h2omx.reference (fresh interpreter)."""
    import json
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, os.path.join(here, "_gpu_no_reference_worker.py")], capture_output=True,
                       text=True, timeout=300, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["reference_loaded"] == [], out
