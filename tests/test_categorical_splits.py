"""Categorical group splits (H2O GBM / DRF default for enum predictors under
categorical_encoding AUTO / Enum): a split of an enum column sends a SET of
levels left (levels ordered by G / S inside the node, best prefix), stored as
a 256-bit left-set bitset per node (TreeEnsemble.catbits, TreeNode.na_left
bit 1).  CPU tests run the NumPy oracle (h2omx/reference/tree.py); GPU tests
compare the HIP scan (feat_best_cat_wave), routing (part_right) and scoring
(predict_raw / predict_binned / TreeSHAP) against it."""
from __future__ import annotations

import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame.frame import Frame
from h2omx.models.tree.structs import bitset_has
from h2omx.models.tree_models import (H2OGradientBoostingEstimator, H2ORandomForestEstimator,
                                      H2OXGBoostEstimator)


def _data(n=4000, nlev=20, seed=0, na_frac=0.0, binary=False):
    rng = np.random.default_rng(seed)
    levels = [f"L{i:02d}" for i in range(nlev)]
    hi = {lv for i, lv in enumerate(levels) if (i * 7) % 3 == 0}        # scattered "high" levels
    g = rng.choice(levels, n).astype(object)
    x = rng.normal(size=n)
    f = np.array([2.5 if v in hi else -0.5 for v in g]) + 0.4 * x
    if na_frac:
        g[rng.uniform(size=n) < na_frac] = None
        f = np.where(pd.isna(g), 4.0, f)
    df = pd.DataFrame({"g": pd.Categorical(g, categories=levels), "x": x})
    if binary:
        df["y"] = pd.Categorical(np.where(rng.uniform(size=n) < 1 / (1 + np.exp(-f)), "b", "a"))
    else:
        df["y"] = f + 0.1 * rng.normal(size=n)
    return df, levels, hi


def test_group_split_stump_separates_level_set():
    df, levels, hi = _data()
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=1, max_depth=1, learn_rate=1.0, min_rows=1, seed=1).train(
        x=["g", "x"], y="y", training_frame=fr)
    root = m.ens.trees[0][0]
    assert root["feat"] == 0 and (int(root["na_left"]) & 2)
    left = bitset_has(m.ens.catbits[0][0], np.arange(len(levels)))
    got = {levels[i] for i in range(len(levels)) if left[i]}
    assert got in (hi, set(levels) - hi)
    pred = m.predict(fr).to_pandas()["predict"].to_numpy()
    assert np.mean((pred - df["y"].to_numpy()) ** 2) < 0.3


def test_na_level_follows_na_direction_and_unseen_levels():
    df, levels, hi = _data(na_frac=0.1, seed=3)
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=20, max_depth=3, learn_rate=0.5, seed=1).train(
        x=["g", "x"], y="y", training_frame=fr)
    na = df["g"].isna().to_numpy()
    pred = m.predict(fr).to_pandas()["predict"].to_numpy()
    assert abs(pred[na].mean() - df["y"].to_numpy()[na].mean()) < 0.3
    # a level unseen in training scores like NA (adapt_frame) without errors
    test = pd.DataFrame({"g": pd.Categorical(["L00", "ZZZ", None]), "x": [0.0, 0.0, 0.0]})
    p = m.predict(Frame.from_pandas(test)).to_pandas()["predict"].to_numpy()
    assert np.isfinite(p).all() and abs(p[1] - p[2]) < 1e-6


def test_auto_beats_label_encoder_and_drf_uses_group_splits():
    df, _, _ = _data(binary=True, seed=5)
    fr = Frame.from_pandas(df)
    kw = dict(ntrees=5, max_depth=2, seed=1)
    a = H2OGradientBoostingEstimator(**kw).train(x=["g", "x"], y="y", training_frame=fr)
    b = H2OGradientBoostingEstimator(categorical_encoding="LabelEncoder", **kw).train(
        x=["g", "x"], y="y", training_frame=fr)
    assert a.training_metrics["AUC"] > b.training_metrics["AUC"] + 0.02
    assert b.ens.catbits is None
    d = H2ORandomForestEstimator(ntrees=5, max_depth=6, seed=1).train(x=["g", "x"], y="y", training_frame=fr)
    assert d.ens.catbits is not None
    assert any((int(tr[0]["na_left"]) & 2) for tr in d.ens.trees)
    # XGBoost keeps H2O's non-group behaviour (no bitset splits)
    xg = H2OXGBoostEstimator(ntrees=3, max_depth=3, seed=1).train(x=["g", "x"], y="y", training_frame=fr)
    assert xg.ens.catbits is None


def test_mojo_round_trip_with_bitset_splits(tmp_path):
    from h2omx.mojo import import_mojo

    df, _, _ = _data(na_frac=0.05, binary=True, seed=7, nlev=40)
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=8, max_depth=4, seed=1).train(x=["g", "x"], y="y", training_frame=fr)
    g = import_mojo(m.download_mojo(str(tmp_path)))
    assert g.ens.catbits is not None
    np.testing.assert_allclose(g.predict(fr).to_pandas().iloc[:, -1].to_numpy(),
                               m.predict(fr).to_pandas().iloc[:, -1].to_numpy(), atol=1e-6)


def test_shap_and_leaf_assignment_with_categorical_splits():
    from h2omx.explain import predict_contributions
    from h2omx.explain_more import predict_leaf_node_assignment

    df, _, _ = _data(na_frac=0.05, seed=9)
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=6, max_depth=3, seed=1).train(x=["g", "x"], y="y", training_frame=fr)
    C = predict_contributions(m, fr).to_pandas().to_numpy()
    margin = m.ens.raw_margin(fr.feature_matrix(m.x))[0].numpy()
    np.testing.assert_allclose(C.sum(1), margin, atol=1e-4)
    la = predict_leaf_node_assignment(m, fr)
    assert la.nrows == fr.nrows


def test_many_levels_fall_back_to_ordinal_bins():
    rng = np.random.default_rng(1)
    n = 3000
    levels = [f"v{i:03d}" for i in range(300)]
    g = rng.choice(levels, n)
    y = rng.normal(size=n) + np.array([int(v[1:]) % 2 for v in g])
    fr = Frame.from_pandas(pd.DataFrame({"g": pd.Categorical(g, categories=levels), "y": y}))
    m = H2OGradientBoostingEstimator(ntrees=3, max_depth=3, seed=1).train(y="y", training_frame=fr)
    assert m.ens.catbits is None     # > 255 levels: ordinal quantile bins of the codes


@pytest.mark.gpu
@pytest.mark.parametrize("binary", [False, True])
def test_categorical_gpu_matches_reference(cuda_dev, binary):
    from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble
    from h2omx.models.tree.binning import categorical_bins

    df, levels, _ = _data(n=30000, nlev=37, na_frac=0.03, binary=binary, seed=11)
    codes = df["g"].cat.codes.to_numpy().astype(np.float32)
    codes[codes < 0] = np.nan
    X = torch.tensor(np.stack([codes, df["x"].to_numpy(np.float32)]))
    y = (df["y"].cat.codes.to_numpy() if binary else df["y"].to_numpy()).astype(np.float32)
    e, nv, nbt = compute_edges(X, 64)
    e, nv, nbt, cat = categorical_bins(e, nv, nbt, {0: len(levels)})
    tp = TreeParams(max_depth=4, min_rows=10.0, learn_rate=0.2, seed=3)
    dist = "bernoulli" if binary else "gaussian"
    ec = train_ensemble(bin_matrix(X, e, nv, nbt, cat=cat), y, dist=dist, ntrees=6, tparams=tp)
    eg = train_ensemble(bin_matrix(X.to(cuda_dev), e, nv, nbt, cat=cat), y, dist=dist, ntrees=6, tparams=tp)
    assert eg.catbits is not None

    def reach(tr):
        keep, stack = [], [0]
        while stack:
            i = stack.pop()
            keep.append(i)
            if tr[i]["feat"] >= 0:
                stack += [int(tr[i]["left"]), int(tr[i]["left"]) + 1]
        return sorted(keep)

    # reachable structure (GPU heaps keep garbage in unreachable slots; CPU trees are compact)
    same = np.mean([reach(a) == reach(b) and (a[reach(a)]["feat"] == b[reach(b)]["feat"]).all()
                    for a, b in zip(ec.trees, eg.trees)])
    assert same >= 0.6
    # first tree: identical root split incl. the level set
    assert ec.trees[0][0]["feat"] == eg.trees[0][0]["feat"] == 0
    np.testing.assert_array_equal(ec.catbits[0][0], eg.catbits[0][0])
    mc = ec.raw_margin(X)[0].numpy()
    mg = eg.raw_margin(X.to(cuda_dev))[0].cpu().numpy()
    assert (np.abs(mc - mg) < 1e-3 * max(1.0, np.abs(mc).max())).mean() > 0.95
    # the binned-code scorer agrees with the raw-value scorer on the device
    from h2omx import ops

    bg = bin_matrix(X.to(cuda_dev), e, nv, nbt, cat=cat)
    T = eg.trees.shape[0]
    nodes = torch.from_numpy(eg.trees.reshape(-1).view(np.uint8).copy()).to(cuda_dev)
    cbits = torch.from_numpy(eg.catbits.reshape(-1).view(np.int32).copy()).to(cuda_dev)
    roots = torch.arange(T, dtype=torch.int32, device=cuda_dev) * eg.trees.shape[1]
    out = torch.zeros((1, bg.n), dtype=torch.float32, device=cuda_dev)
    lib = ops.tree_lib()
    ops.check(lib.h2omx_predict_binned(ops.P(bg.codes), bg.npad, bg.n, ops.P(nodes), ops.P(roots), T, 1, nbt,
                                       ops.P(out), out.stride(0), ops.P(cbits), ops.stream(cuda_dev)),
              "predict_binned")
    np.testing.assert_allclose(out[0].cpu().numpy() + float(eg.init_f[0]), mg, atol=1e-4)


@pytest.mark.gpu
def test_categorical_shap_gpu_matches_cpu(cuda_dev):
    from h2omx.explain import predict_contributions

    df, _, _ = _data(n=5000, na_frac=0.05, seed=13)
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1).train(x=["g", "x"], y="y", training_frame=fr)
    c_cpu = predict_contributions(m, fr).to_pandas().to_numpy()
    c_gpu = predict_contributions(m, fr.to(cuda_dev)).to_pandas().to_numpy()
    np.testing.assert_allclose(c_gpu, c_cpu, atol=1e-4)
