"""Per-node histogram semantics (H2O ``histogram_type`` UniformAdaptive - the
GBM / DRF default AUTO - Random and RoundRobin; hex/tree/DHistogram).

Every node re-bins its own [min, max] into nb = max(nbins_top_level >> depth,
nbins) equal-width bins (Random: nb - 1 uniform random cuts); h2omx keeps the
fine histogram and lets a node split only at the fine edges nearest those cuts
(``reference/tree.adaptive_mask`` on the CPU, ``adaptive_candidates`` in
csrc/tree_kernels.hip).  The oracle below re-derives the allowed edges by brute
force (argmin distance of every cut to the node's interior fine edges, from the
node's own rows) - a different mechanism from the kernels' cut counting.
GPU parts are marked ``gpu``."""
import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble
from h2omx.models.tree.binning import adaptive_ranges, node_bins, resolve_histogram_type
from h2omx.models.tree.hashing import hash4, u01
from h2omx.reference.tree import adaptive_mask


def oracle_allowed(S, e, fr, m, nbt, nb, mode, seed=0, tree_index=0, depth=0, node=0, f=0):
    """Brute-force allowed threshold set of one (node, feature)."""
    T = min(m, nbt - 1)
    ne = np.nonzero(S[:T] > 0)[0]
    if ne.size == 0 or ne[-1] - ne[0] < 1:
        return set(range(T))
    lo, hi = int(ne[0]), int(ne[-1])
    fmin, fmax, exact, isint = (float(v) for v in fr)
    if exact:
        lo_v = float(e[lo]) if lo < m - 1 else fmax
        hi_v = float(e[hi]) if hi < m - 1 else fmax
    else:
        lo_v = fmin if lo == 0 else float(e[lo - 1])
        hi_v = fmax if hi == m - 1 else float(e[hi])
    span = hi_v - lo_v
    if not span > 0 or (isint and span + 1 <= nb):
        return set(range(T))
    if mode == 1:
        cuts = [lo_v + (span * k) / nb for k in range(1, nb)]
    else:
        key = ((tree_index * 131 + depth) & 0xFFFFFFFF) ^ ((f * 0x9E3779B1) & 0xFFFFFFFF)
        cuts = list(lo_v + span * u01(hash4((seed & 0xFFFFFFFF) ^ 0x52414E44, key, node, np.arange(1, nb))))
    interior = np.arange(lo, hi)
    x = e[interior].astype(np.float64)
    keep = set(range(T)) - set(interior.tolist())
    for c in cuts:
        keep.add(int(interior[int(np.argmin(np.abs(x - c)))]))
    return keep


@pytest.mark.parametrize("mode", [1, 2])
def test_adaptive_mask_matches_brute_force_oracle(mode):
    rng = np.random.default_rng(mode)
    nbt = 256
    for trial in range(300):
        m = int(rng.integers(3, 255))
        e = np.sort(rng.normal(size=m - 1).astype(np.float32) * rng.choice([1.0, 100.0]))
        e = np.unique(e)
        m = e.size + 1
        edges = np.full(nbt, np.inf, np.float32)
        edges[: m - 1] = e
        S = rng.random(nbt) * (rng.random(nbt) < rng.uniform(0.05, 1.0))
        exact = bool(rng.random() < 0.3)
        isint = bool(rng.random() < 0.2)
        fr = np.array([e[0] - abs(rng.normal()), e[-1] + abs(rng.normal()), float(exact), float(isint)], np.float32)
        depth = int(rng.integers(0, 12))
        tp = TreeParams(hist_mode=mode, hist_top=1024, hist_nbins=int(rng.choice([8, 20, 40])), seed=trial)
        nb = node_bins(tp.hist_top, tp.hist_nbins, depth)
        node, f, ti = int(rng.integers(0, 50)), int(rng.integers(0, 30)), int(rng.integers(0, 9))
        keep = adaptive_mask(tp, edges, fr, S, m, nbt, node, f, depth, ti)
        want = oracle_allowed(S, edges, fr, m, nbt, nb, mode, trial, ti, depth, node, f)
        got = set(range(min(m, nbt - 1))) if keep is None else set(np.nonzero(keep)[0].tolist())
        assert got == want, (trial, sorted(got ^ want)[:10])


def test_node_bins_follow_h2o_halving():
    assert [node_bins(1024, 20, d) for d in range(8)] == [1024, 512, 256, 128, 64, 32, 20, 20]
    assert node_bins(64, 20, 0) == 64 and node_bins(16, 20, 0) == 20
    assert resolve_histogram_type("AUTO", auto="uniformadaptive") == "uniformadaptive"
    assert resolve_histogram_type("AUTO") == "quantilesglobal"
    assert resolve_histogram_type("RoundRobin") == "roundrobin"
    with pytest.raises(ValueError):
        resolve_histogram_type("bogus")


def _data(n=5000, F=6, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(F, n)).astype(np.float32)
    X[1] = np.exp(X[1] * 1.5)                       # heavy right tail: uniform != quantile cuts
    X[2, rng.random(n) < 0.1] = np.nan
    X[4] = rng.integers(0, 6, n)                    # integer, exact bins
    X[5] = np.round(X[5] * 40)                      # integer, span > nb at depth
    logit = 1.2 * X[0] - 0.5 * np.log(X[1]) + np.nan_to_num(X[2]) * X[3] + 0.4 * X[4] + 0.02 * X[5]
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    return X, y


def _bm(X, dev=None):
    Xt = torch.from_numpy(X)
    e, nv, nbt = compute_edges(Xt, 255)
    bm = bin_matrix(Xt if dev is None else Xt.to(dev), e, nv, nbt)
    bm.frange = adaptive_ranges(Xt if dev is None else Xt.to(dev), bm)
    return bm


def _check_tree_oracle(tree, bm, tp, tree_index, rows=None):
    """Every split of ``tree`` sits on an edge the oracle allows for the node's rows."""
    codes = bm.codes.cpu().numpy()[:, : bm.n]
    edges = bm.edges.cpu().numpy()
    nvb = bm.nvb.cpu().numpy()
    fr = bm.frange.cpu().numpy()
    nbt = bm.nbt
    rows = np.arange(bm.n) if rows is None else rows
    level = [(0, rows)]
    depth, checked = 0, 0
    while level:
        nxt = []
        for i, (gid, r) in enumerate(level):
            rec = tree[gid]
            if rec["feat"] < 0:
                continue
            f, t = int(rec["feat"]), int(rec["bin"])
            S = np.bincount(codes[f, r], minlength=nbt).astype(np.float64)
            mode = tp.hist_mode if tp.hist_mode != 3 else (1, 1, 2, 0)[tree_index & 3]
            if mode:
                nb = node_bins(tp.hist_top, tp.hist_nbins, depth)
                ok = oracle_allowed(S, edges[f], fr[f], int(nvb[f]), nbt, nb, mode, tp.seed, tree_index, depth, i, f)
                assert t in ok, (gid, depth, f, t)
                checked += 1
            c = codes[f, r]
            nal = (int(rec["na_left"]) & 1) == 1
            left = np.where(c == nbt - 1, nal, c <= t)
            nxt.append((int(rec["left"]), r[left]))
            nxt.append((int(rec["left"]) + 1, r[~left]))
        # the builder numbers a level's nodes in split order
        level = sorted(nxt, key=lambda z: z[0])
        depth += 1
    return checked


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_cpu_reference_trees_split_on_oracle_edges(mode):
    X, y = _data()
    bm = _bm(X)
    tp = TreeParams(max_depth=6, min_rows=5, learn_rate=0.3, min_split_improvement=0, hist_mode=mode,
                    hist_top=64, hist_nbins=6, seed=3)
    ens = train_ensemble(bm, y, dist="bernoulli", ntrees=4, tparams=tp)
    checked = sum(_check_tree_oracle(ens.trees[t], bm, tp, t) for t in range(4))
    assert checked > 20
    # the rule changes the model (QuantilesGlobal scans every fine edge)
    tq = TreeParams(max_depth=6, min_rows=5, learn_rate=0.3, min_split_improvement=0, seed=3)
    eq = train_ensemble(bm, y, dist="bernoulli", ntrees=4, tparams=tq)
    assert not np.array_equal(eq.trees[0]["bin"], ens.trees[0]["bin"])


def test_zero_weight_rows_do_not_widen_the_node_range():
    """A node's [min, max] (the span UniformAdaptive re-bins) comes from its rows
    of POSITIVE weight: a fine bin counts as occupied when its weight plane is
    > 0 (adaptive_candidates in csrc/tree_kernels.hip, reference adaptive_mask),
    as H2O's histograms skip zero-weight rows.  So zero-weight rows - here
    placed at the extremes of a feature, where they would widen every node's
    range - give the same trees as leaving those rows out (same grid)."""
    X, y = _data(4000, seed=11)
    rng = np.random.default_rng(5)
    zero = rng.random(X.shape[1]) < 0.2
    X[0, zero] = np.where(rng.random(int(zero.sum())) < 0.5, -40.0, 40.0)   # out-of-range rows
    w = np.where(zero, 0.0, 1.0).astype(np.float32)
    Xt = torch.from_numpy(X)
    e, nv, nbt = compute_edges(Xt, 255)
    fr = None
    tp = TreeParams(max_depth=5, min_rows=5, learn_rate=0.3, min_split_improvement=0, seed=3, hist_mode=1,
                    hist_top=1024, hist_nbins=20)
    keep = ~zero
    bm_all = bin_matrix(Xt, e, nv, nbt)
    bm_all.frange = fr = adaptive_ranges(Xt, bm_all)
    bm_kept = bin_matrix(torch.from_numpy(np.ascontiguousarray(X[:, keep])), e, nv, nbt)
    bm_kept.frange = fr
    ea = train_ensemble(bm_all, torch.from_numpy(y), torch.from_numpy(w), dist="bernoulli", ntrees=3, tparams=tp)
    ek = train_ensemble(bm_kept, torch.from_numpy(y[keep]), dist="bernoulli", ntrees=3, tparams=tp)
    for t in range(3):
        for k in ("feat", "bin", "left"):
            np.testing.assert_array_equal(ea.trees[t][k], ek.trees[t][k])
        np.testing.assert_allclose(ea.trees[t]["value"], ek.trees[t]["value"], rtol=1e-5, atol=1e-7)


def _frame(n=3000, seed=0):
    from h2omx.frame import Frame

    X, y = _data(n, seed=seed)
    df = pd.DataFrame(X.T, columns=[f"x{i}" for i in range(X.shape[0])])
    df["y"] = pd.Categorical(np.where(y > 0, "1", "0"), categories=["0", "1"])
    return Frame.from_pandas(df), df


def test_estimator_auto_is_per_node_uniform_adaptive(tmp_path):
    from h2omx.models import H2OGradientBoostingEstimator, H2ORandomForestEstimator, H2OXGBoostEstimator
    from h2omx.mojo import import_mojo

    fr, df = _frame()
    gbm = H2OGradientBoostingEstimator(ntrees=5, seed=1)
    assert gbm.params["nbins"] == 20 and gbm.params["histogram_type"] == "AUTO"
    m = gbm.train(y="y", training_frame=fr)
    assert any("nbins_top_level=1024" in w for w in m.warnings)
    assert m.to_json()["output"]["warnings"] == list(m.warnings)
    with pytest.warns(UserWarning, match="snap to 255 fine quantile bins"):
        H2OGradientBoostingEstimator(ntrees=2, nbins_top_level=4096).train(y="y", training_frame=fr)
    # AUTO == explicit UniformAdaptive; QuantilesGlobal is a different model
    m2 = H2OGradientBoostingEstimator(ntrees=5, seed=1, histogram_type="UniformAdaptive").train(y="y", training_frame=fr)
    mq = H2OGradientBoostingEstimator(ntrees=5, seed=1, histogram_type="QuantilesGlobal", nbins=255).train(
        y="y", training_frame=fr)
    p, p2, pq = (x.predict(fr).to_pandas()["1"].to_numpy() for x in (m, m2, mq))
    np.testing.assert_array_equal(p, p2)
    assert not np.allclose(p, pq)
    assert not mq.warnings
    # MOJO round trip scores identically (thresholds are raw fine edges)
    g = import_mojo(m.download_mojo(str(tmp_path)))
    np.testing.assert_allclose(g.predict(fr).to_pandas()["1"].to_numpy(), p, rtol=1e-6, atol=1e-7)
    # DRF: Random per node runs; RoundRobin is accepted
    for ht in ("Random", "RoundRobin"):
        d = H2ORandomForestEstimator(ntrees=4, max_depth=8, seed=2, histogram_type=ht, nbins_top_level=128)
        dm = d.train(y="y", training_frame=fr)
        assert dm.training_metrics["AUC"] > 0.7
    # builders without the per-node scan say so
    with pytest.warns(UserWarning, match="one global grid"):
        rm = H2OGradientBoostingEstimator(ntrees=2, histogram_type="UniformRobust").train(y="y", training_frame=fr)
    assert rm.warnings
    # XGBoost 'hist' has no histogram_type: global bins, no warning
    assert not H2OXGBoostEstimator(ntrees=2).train(y="y", training_frame=fr).warnings


# ---------------------------------------------------------------------------
# GPU: the HIP split scan applies the same rule
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_gpu_trees_match_cpu_and_oracle(cuda_dev, mode):
    X, y = _data()
    bc, bg = _bm(X), _bm(X, cuda_dev)
    np.testing.assert_array_equal(bc.frange.numpy(), bg.frange.cpu().numpy())
    tp = TreeParams(max_depth=6, min_rows=5, learn_rate=0.3, min_split_improvement=0, hist_mode=mode,
                    hist_top=64, hist_nbins=6, seed=3)
    ec = train_ensemble(bc, y, dist="bernoulli", ntrees=4, tparams=tp)
    eg = train_ensemble(bg, torch.from_numpy(y).to(cuda_dev), dist="bernoulli", ntrees=4, tparams=tp)
    checked = 0
    for t in range(4):
        checked += _check_tree_oracle(np.asarray(eg.trees[t]), bg, tp, t)
        tc, tg = ec.trees[t], eg.trees[t]
        for i in [j for j in ec.compact()[t] if j < 7]:     # top levels identical (deep ties aside)
            assert tc[i]["feat"] == tg[i]["feat"], (t, i)
            if tc[i]["feat"] >= 0:
                assert tc[i]["bin"] == tg[i]["bin"] and tc[i]["na_left"] == tg[i]["na_left"], (t, i)
    assert checked > 20


@pytest.mark.gpu
def test_gpu_segmented_engine_identical_under_uniform_adaptive(cuda_dev, monkeypatch):
    """Deep DRF trees: the row-partitioned engine builds bit-identical trees to
    the scan engine with the per-node rule on (both run adaptive_candidates)."""
    from h2omx.models.tree import engine as E

    X, y = _data(n=20000)
    bg = _bm(X, cuda_dev)
    tp = TreeParams(max_depth=12, min_rows=1, learn_rate=1.0, leaf_mode=1, mtries=3, min_split_improvement=0,
                    seed=7, hist_mode=1, hist_top=1024, hist_nbins=20)
    yt = torch.from_numpy(y).to(cuda_dev)
    out = {}
    # the direct deep-level kernels (from level 1 on: per-wave cut tables wherever
    # the level has <= 64 cuts, the division form above) in their node-workgroup,
    # wave-per-node and row-chunk forms, with and without column-major code planes
    cfgs = (("scan", 16, {}), ("seg", 0, {}), ("seg", 0, {"DIRECT_MIN_NODES": 2}),
            ("seg", 0, {"DIRECT_MIN_NODES": 2, "DIRECT_WAVE_ROWS": 1 << 30}),
            ("seg", 0, {"DIRECT_MIN_NODES": 2, "DIRECT_CHUNKED": False, "COLMAJOR_EVERY": 0}),
            ("seg", 0, {"DIRECT_MIN_NODES": 2, "DIRECT_WAVE_ROWS": 0, "COLMAJOR_EVERY": 1}),
            ("seg", 0, {"DIRECT_MIN_NODES": 2, "DIRECT_WAVE_ROWS": 0, "COLMAJOR_EVERY": 3}))
    names = ("DIRECT_MIN_NODES", "DIRECT_WAVE_ROWS", "DIRECT_CHUNKED", "COLMAJOR_EVERY")
    defaults = {name: getattr(E.HipTreeBuilder, name) for name in names}
    for k, (eng, scan_slots, attrs) in enumerate(cfgs):
        monkeypatch.setenv("H2OMX_TREE_ENGINE", eng)
        monkeypatch.setattr(E.HipTreeBuilder, "SCAN_SLOTS", scan_slots)
        for name in names:
            monkeypatch.setattr(E.HipTreeBuilder, name, attrs.get(name, defaults[name]))
        out[k] = train_ensemble(bg, yt, dist="drf", ntrees=3, tparams=tp, sample_rate=0.632, nclass=2, seed=11)
    a = out[0]
    for k in range(1, len(cfgs)):
        b = out[k]
        for t in range(a.trees.shape[0]):
            for i in a.compact()[t]:
                assert a.trees[t][i]["feat"] == b.trees[t][i]["feat"], (cfgs[k], t, i)
                assert a.trees[t][i]["bin"] == b.trees[t][i]["bin"], (cfgs[k], t, i)
