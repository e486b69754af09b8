"""interaction_constraints for GBM / XGBoost (H2O GBMParameters
._interaction_constraints, XGBoost interaction_constraints): the features on
any root-to-node path all belong to one interaction set; a predictor outside
every set only combines with itself.

CPU tests run the NumPy reference builder (interaction_allowed /
interaction_child); the GPU test checks the HIP kernels (inter_ok in the split
scans and the direct deep-level engine, SplitParams::istate written by the
level finalisation) against the same rule and against the reference."""
from __future__ import annotations

import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame.frame import Frame
from h2omx.models.tree_models import H2OGradientBoostingEstimator, H2OXGBoostEstimator

COLS = ["x0", "x1", "x2", "x3", "x4"]


def _frame(n=5000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 5))
    f = X[:, 0] * X[:, 1] + X[:, 2] * X[:, 3] + 1.5 * X[:, 0] * X[:, 2] + 0.7 * X[:, 4]
    df = pd.DataFrame(X, columns=COLS)
    df["y"] = f + 0.2 * rng.normal(size=n)
    return df


def _path_sets(trees):
    """feature sets of every root-to-node path of every tree"""
    out = []
    for tr in trees:
        stack = [(0, frozenset())]
        while stack:
            i, fs = stack.pop()
            if i < 0 or i >= len(tr) or tr[i]["feat"] < 0:
                continue
            fs2 = fs | {int(tr[i]["feat"])}
            out.append(fs2)
            left = int(tr[i]["left"])
            stack += [(left, fs2), (left + 1, fs2)]
    return out


def _valid(fs, sets):
    return any(fs <= set(s) for s in sets) or (len(fs) == 1 and not any(fs <= set(s) for s in sets))


SETS = [[0, 1], [2, 3]]   # x4 unlisted


@pytest.mark.parametrize("est_cls", [H2OGradientBoostingEstimator, H2OXGBoostEstimator])
def test_interaction_constraints_paths(est_cls):
    fr = Frame.from_pandas(_frame())
    free = est_cls(ntrees=15, max_depth=5, seed=3).train(y="y", training_frame=fr)
    assert not all(_valid(fs, SETS) for fs in _path_sets(free.ens.trees)), "free trees should mix the sets"
    m = est_cls(ntrees=15, max_depth=5, seed=3,
                interaction_constraints=[["x0", "x1"], ["x2", "x3"]]).train(y="y", training_frame=fr)
    paths = _path_sets(m.ens.trees)
    assert paths and all(_valid(fs, SETS) for fs in paths)
    assert m.model_performance(fr)["r2"] > 0.05   # x0 * x2 is out of reach by construction


def test_interaction_constraints_unlisted_solo_and_validation():
    df = _frame(n=2000)
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=8, max_depth=4, seed=1,
                                     interaction_constraints=[["x0", "x1"]]).train(y="y", training_frame=fr)
    for fs in _path_sets(m.ens.trees):
        assert fs <= {0, 1} or len(fs) == 1, fs
    with pytest.raises(ValueError, match="not a predictor"):
        H2OGradientBoostingEstimator(ntrees=2, interaction_constraints=[["x0", "zz"]]).train(
            y="y", training_frame=fr)
    # one set holding every predictor is the unconstrained model
    a = H2OGradientBoostingEstimator(ntrees=4, max_depth=3, seed=2).train(y="y", training_frame=fr)
    b = H2OGradientBoostingEstimator(ntrees=4, max_depth=3, seed=2, interaction_constraints=[COLS]).train(
        y="y", training_frame=fr)
    np.testing.assert_array_equal(a.predict(fr).to_pandas()["predict"], b.predict(fr).to_pandas()["predict"])


@pytest.mark.gpu
@pytest.mark.parametrize("mode,depth", [(0, 5), (1, 6), (0, 12)])
def test_interaction_gpu_matches_reference(cuda_dev, mode, depth):
    """scan engine (depth 5/6) and the segmented engine with direct deep levels (depth 12)"""
    from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble

    df = _frame(n=30000, seed=4)
    X = torch.tensor(df[COLS].to_numpy().T.copy(), dtype=torch.float32)
    y = df["y"].to_numpy().astype(np.float32)
    tp = TreeParams(max_depth=depth, min_rows=5.0 if mode == 0 else 0.0, min_child_weight=1.0, learn_rate=0.2,
                    mode=mode, reg_lambda=1.0 if mode else 0.0, seed=5, interactions=((0, 1), (2, 3)))
    e, nv, nbt = compute_edges(X, 64)
    bg = bin_matrix(X.cuda(), e, nv, nbt)
    eg = train_ensemble(bg, y, dist="gaussian", ntrees=6, tparams=tp)
    paths = _path_sets(eg.trees)
    assert paths and all(_valid(fs, SETS) for fs in paths)
    if depth <= 6:
        bc = bin_matrix(X, e, nv, nbt)
        ec = train_ensemble(bc, y, dist="gaussian", ntrees=6, tparams=tp)
        # the first tree splits identically (later trees fit residuals that a
        # fixed-point near-tie may already have steered apart)
        reach = ec.compact()[0]
        assert reach == eg.compact()[0]
        np.testing.assert_array_equal(ec.trees[0][reach]["feat"], eg.trees[0][reach]["feat"])
        r2 = lambda m: 1 - np.mean((m - y) ** 2) / np.var(y)   # noqa: E731
        assert abs(r2(ec.raw_margin(X)[0].numpy()) - r2(eg.raw_margin(X.cuda())[0].cpu().numpy())) < 0.02
