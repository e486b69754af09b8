"""monotone_constraints for GBM / XGBoost (H2O GBMModel.GBMParameters
._monotone_constraints; hex/tree/DTree.java constrained splits and
hex/tree/Constraints.java bounds): every tree's leaves respect the sign of
each constrained predictor, so the whole model's margin is monotone in it.

CPU tests exercise the NumPy reference builder; the GPU test checks the HIP
kernels (mono_ok in the split scans, SplitParams::gbound intervals written by
the level finalisation and clamped in leaf_finalize) against it."""
from __future__ import annotations

import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame.frame import Frame
from h2omx.models.tree_models import H2OGradientBoostingEstimator, H2OXGBoostEstimator


def _frame(n=4000, seed=0, binary=False):
    rng = np.random.default_rng(seed)
    x0 = rng.uniform(-3, 3, n)
    x1 = rng.normal(size=n)
    x2 = rng.uniform(0, 1, n)
    # response rises with x0 overall but wiggles (non-monotone without constraints)
    f = x0 + 1.5 * np.sin(3 * x0) + 0.5 * x1 - 2.0 * x2
    df = pd.DataFrame({"x0": x0, "x1": x1, "x2": x2})
    if binary:
        p = 1 / (1 + np.exp(-f))
        df["y"] = pd.Categorical(np.where(rng.uniform(size=n) < p, "b", "a"))
    else:
        df["y"] = f + 0.3 * rng.normal(size=n)
    return df


def _sweep(model, col, base_rows=6, grid=61):
    """predictions along a grid of ``col`` for a few fixed rows of the others"""
    rng = np.random.default_rng(7)
    xs = np.linspace(-3.5, 3.5, grid) if col == "x0" else np.linspace(-0.2, 1.2, grid)
    out = []
    for _ in range(base_rows):
        r = {"x0": rng.uniform(-3, 3), "x1": rng.normal(), "x2": rng.uniform(0, 1)}
        df = pd.DataFrame({k: np.full(grid, v) for k, v in r.items()})
        df[col] = xs
        fr = Frame.from_pandas(df)
        p = model.predict(fr).to_pandas()
        out.append(p.iloc[:, -1].to_numpy() if p.shape[1] > 1 else p["predict"].to_numpy())
    return np.stack(out)


@pytest.mark.parametrize("est_cls", [H2OGradientBoostingEstimator, H2OXGBoostEstimator])
def test_monotone_increasing_and_decreasing(est_cls):
    df = _frame()
    fr = Frame.from_pandas(df)
    free = est_cls(ntrees=30, max_depth=4, seed=3).train(y="y", training_frame=fr)
    d = np.diff(_sweep(free, "x0"), axis=1)
    assert (d < -1e-6).any(), "unconstrained fit should follow the sin wiggle"
    m = est_cls(ntrees=30, max_depth=4, seed=3,
                monotone_constraints={"x0": 1, "x2": -1}).train(y="y", training_frame=fr)
    assert (np.diff(_sweep(m, "x0"), axis=1) >= -1e-6).all()
    assert (np.diff(_sweep(m, "x2"), axis=1) <= 1e-6).all()
    # the constrained model still fits the trend
    perf = m.model_performance(fr)
    assert perf["r2"] > 0.6


def test_monotone_bernoulli_rest_form():
    df = _frame(binary=True)
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=25, max_depth=3, seed=1,
                                     monotone_constraints=[{"key": "x0", "value": 1}]).train(
        y="y", training_frame=fr)
    s = _sweep(m, "x0")
    assert (np.diff(s, axis=1) >= -1e-6).all()
    assert m.training_metrics["AUC"] > 0.75


def test_monotone_validation():
    df = _frame(n=500)
    df["c"] = pd.Categorical(np.where(df["x1"] > 0, "p", "q"))
    fr = Frame.from_pandas(df)
    with pytest.raises(ValueError, match="not a predictor"):
        H2OGradientBoostingEstimator(ntrees=2, monotone_constraints={"zz": 1}).train(y="y", training_frame=fr)
    with pytest.raises(ValueError, match="categorical"):
        H2OGradientBoostingEstimator(ntrees=2, monotone_constraints={"c": 1}).train(y="y", training_frame=fr)
    with pytest.raises(ValueError, match="must be -1, 0 or 1"):
        H2OGradientBoostingEstimator(ntrees=2, monotone_constraints={"x0": 2}).train(y="y", training_frame=fr)
    # all-zero constraints are a no-op: identical to the unconstrained model
    a = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=2).train(y="y", training_frame=fr, x=["x0", "x1"])
    b = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=2, monotone_constraints={"x0": 0}).train(
        y="y", training_frame=fr, x=["x0", "x1"])
    np.testing.assert_array_equal(a.predict(fr).to_pandas()["predict"], b.predict(fr).to_pandas()["predict"])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_monotone_gpu_matches_reference(cuda_dev, mode):
    from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble

    df = _frame(n=20000)
    X = torch.tensor(df[["x0", "x1", "x2"]].to_numpy().T.copy(), dtype=torch.float32)
    y = df["y"].to_numpy().astype(np.float32)
    tp = TreeParams(max_depth=4, min_rows=10.0 if mode == 0 else 0.0, min_child_weight=1.0, learn_rate=0.2,
                    mode=mode, reg_lambda=1.0 if mode else 0.0, seed=5, monotone=(1, 0, -1))
    e, nv, nbt = compute_edges(X, 64)
    bc = bin_matrix(X, e, nv, nbt)
    bg = bin_matrix(X.cuda(), e, nv, nbt)
    ec = train_ensemble(bc, y, dist="gaussian", ntrees=8, tparams=tp)
    eg = train_ensemble(bg, y, dist="gaussian", ntrees=8, tparams=tp)
    from treecmp import frac_same

    same = frac_same(ec.trees, eg.trees)
    assert same >= 0.75
    mc = ec.raw_margin(X)[0].numpy()
    mg = eg.raw_margin(X.cuda())[0].cpu().numpy()
    assert (np.abs(mc - mg) < 1e-3 * max(1.0, np.abs(mc).max())).mean() > 0.9
    # monotone along x0 (+1) and x2 (-1) on the GPU ensemble
    for col, sign, lo, hi in ((0, 1, -3.5, 3.5), (2, -1, -0.2, 1.2)):
        Xs = X[:, :8].repeat_interleave(101, dim=1).clone()
        Xs[col] = torch.linspace(lo, hi, 101).repeat(8)
        s = eg.raw_margin(Xs.cuda())[0].cpu().numpy().reshape(8, 101)
        assert (sign * np.diff(s, axis=1) >= -1e-6).all()
    # ... and the unconstrained GPU ensemble is not (the data wiggles in x0)
    tp.monotone = None
    ef = train_ensemble(bg, y, dist="gaussian", ntrees=8, tparams=tp)
    Xs = X[:, :8].repeat_interleave(101, dim=1).clone()
    Xs[0] = torch.linspace(-3.5, 3.5, 101).repeat(8)
    s = ef.raw_margin(Xs.cuda())[0].cpu().numpy().reshape(8, 101)
    assert (np.diff(s, axis=1) < -1e-6).any()


def _mono_signal(n=6000, seed=4):
    rng = np.random.default_rng(seed)
    X = np.stack([rng.uniform(-2, 2, n), rng.normal(size=n)]).astype(np.float32)
    p = 1 / (1 + np.exp(-(1.5 * X[0] + 0.7 * X[1])))
    y = (rng.uniform(size=n) < p).astype(np.float32)
    return X, y


def _fit_bernoulli(X, y, monotone, dev=None):
    from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble

    Xt = torch.tensor(X)
    if dev is not None:
        Xt = Xt.to(dev)
    tp = TreeParams(max_depth=3, min_rows=10.0, learn_rate=0.3, mode=0, seed=1, monotone=monotone)
    e, nv, nbt = compute_edges(Xt, 64)
    ens = train_ensemble(bin_matrix(Xt, e, nv, nbt), y, dist="bernoulli", ntrees=10, tparams=tp)
    return ens, ens.raw_margin(Xt)[0].cpu().numpy()


def test_monotone_bernoulli_newton_scale_bounds():
    """Bernoulli GBM (squared-error splits on (G, W), Newton leaves -G/H with
    H <= W / 4): on an already monotone signal the constraint should barely
    bind.  Bounds cut at -G/W midpoints would clamp the 4x larger Newton
    values of deeper leaves and shrink the constrained model's margins."""
    X, y = _mono_signal()
    _, free = _fit_bernoulli(X, y, None)
    ens, con = _fit_bernoulli(X, y, (1, 0))
    spread = np.ptp(free)
    assert np.abs(con - free).mean() < 0.02 * spread, (np.abs(con - free).mean(), spread)
    assert np.ptp(con) > 0.9 * spread
    # monotone in x0 for fixed x1
    xs = np.linspace(-2.5, 2.5, 81, dtype=np.float32)
    for x1 in (-1.0, 0.0, 1.3):
        Xs = np.stack([xs, np.full_like(xs, x1)])
        s = ens.raw_margin(torch.tensor(Xs))[0].numpy()
        assert (np.diff(s) >= -1e-9).all()


@pytest.mark.gpu
def test_monotone_bernoulli_gpu_matches_reference(cuda_dev):
    X, y = _mono_signal(n=20000, seed=9)
    ec, mc = _fit_bernoulli(X, y, (1, -1))
    eg, mg = _fit_bernoulli(X, y, (1, -1), dev=cuda_dev)
    from treecmp import frac_same

    same = frac_same(ec.trees, eg.trees)
    assert same >= 0.75
    assert (np.abs(mc - mg) < 1e-3 * max(1.0, np.abs(mc).max())).mean() > 0.9
    _, free = _fit_bernoulli(X, y, None, dev=cuda_dev)
    assert np.ptp(mg) > 0.5 * np.ptp(free)
