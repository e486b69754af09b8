"""HIP tree kernels vs the NumPy reference implementation of the same algorithm."""
import os

import numpy as np
import pytest
import torch

from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble
from h2omx.models.tree.binning import BinnedMatrix

pytestmark = pytest.mark.gpu


def _data(n=6000, F=7, seed=0, task="bin"):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(F, n)).astype(np.float32)
    X[2, rng.random(n) < 0.1] = np.nan
    X[5] = rng.integers(0, 4, n)  # low-cardinality column
    logit = 1.5 * X[0] - X[1] * X[3] + np.nan_to_num(X[2]) + 0.7 * X[5]
    if task == "bin":
        y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    elif task == "reg":
        y = (logit + rng.normal(size=n)).astype(np.float32)
    else:
        y = np.digitize(logit, [-1, 0.5, 2]).astype(np.float32)
    return X, y


def _both(X, y, nbins=255, **kw):
    Xt = torch.from_numpy(X)
    e, nv, nbt = compute_edges(Xt, nbins)
    bm_cpu = bin_matrix(Xt, e, nv, nbt)
    dev = torch.device("cuda", 0)
    bm_gpu = bin_matrix(Xt.to(dev), e, nv, nbt)
    return bm_cpu, bm_gpu


def test_binning_matches_cpu(cuda_dev):
    X, y = _data()
    for nbins in (255, 63, 20):
        bc, bg = _both(X, y, nbins)
        np.testing.assert_array_equal(bc.codes.numpy(), bg.codes.cpu().numpy())


@pytest.mark.parametrize("nbins", [255, 63, 31])
def test_gbm_bernoulli_matches_reference(cuda_dev, nbins):
    X, y = _data()
    bc, bg = _both(X, y, nbins)
    tp = TreeParams(max_depth=5, min_rows=10, learn_rate=0.2)
    ec = train_ensemble(bc, y, dist="bernoulli", ntrees=6, tparams=tp)
    eg = train_ensemble(bg, torch.from_numpy(y).cuda(), dist="bernoulli", ntrees=6, tparams=tp)
    # first tree: identical structure on the top levels (deep small nodes can
    # hold exact gain ties between features that produce the same partition;
    # fp32-vs-fp64 summation order then legitimately breaks them differently)
    t0c, t0g = ec.trees[0], eg.trees[0]
    for i in [j for j in ec.compact()[0] if j < 7]:
        assert t0c[i]["feat"] == t0g[i]["feat"], i
        if t0c[i]["feat"] >= 0:
            assert t0c[i]["bin"] == t0g[i]["bin"]
            assert t0c[i]["na_left"] == t0g[i]["na_left"]
        np.testing.assert_allclose(t0c[i]["weight"], t0g[i]["weight"], rtol=1e-5)
        if t0c[i]["feat"] < 0:  # leaf values (internal node values are informational)
            np.testing.assert_allclose(t0c[i]["value"], t0g[i]["value"], rtol=1e-4, atol=1e-6)
    Xt = torch.from_numpy(X)
    mc = ec.raw_margin(Xt)[0].numpy()
    mg = eg.raw_margin(Xt.cuda())[0].cpu().numpy()
    assert (np.abs(mc - mg) < 1e-3).mean() > 0.9
    from sklearn.metrics import roc_auc_score
    assert abs(roc_auc_score(y, mc) - roc_auc_score(y, mg)) < 3e-3
    # training margins from the fused update agree with re-scoring
    np.testing.assert_allclose(eg._state.Fm[0, : bg.n].cpu().numpy(), mg, atol=1e-4)


@pytest.mark.parametrize("dist", ["gaussian", "poisson", "laplace"])
def test_gbm_regression_matches_reference(cuda_dev, dist):
    X, y = _data(task="reg")
    if dist == "poisson":
        y = np.floor(np.exp(np.clip(y, -3, 3) * 0.5)).astype(np.float32)
    bc, bg = _both(X, y)
    tp = TreeParams(max_depth=4, min_rows=5, learn_rate=0.3)
    ec = train_ensemble(bc, y, dist=dist, ntrees=4, tparams=tp)
    eg = train_ensemble(bg, y, dist=dist, ntrees=4, tparams=tp)
    Xt = torch.from_numpy(X)
    mc = ec.raw_margin(Xt)[0].numpy()
    mg = eg.raw_margin(Xt.cuda())[0].cpu().numpy()
    assert (np.abs(mc - mg) < 1e-3 * max(1.0, np.abs(mc).max())).mean() > 0.9


def test_multinomial_and_drf(cuda_dev):
    X, y = _data(task="multi")
    bc, bg = _both(X, y)
    tp = TreeParams(max_depth=4, min_rows=5, learn_rate=0.2)
    ec = train_ensemble(bc, y, dist="multinomial", nclass=4, ntrees=3, tparams=tp)
    eg = train_ensemble(bg, y, dist="multinomial", nclass=4, ntrees=3, tparams=tp)
    Xt = torch.from_numpy(X)
    d = np.abs(ec.raw_margin(Xt).numpy() - eg.raw_margin(Xt.cuda()).cpu().numpy())
    assert (d < 1e-3).mean() > 0.9
    # DRF with row bagging + mtries (hash-identical sampling on both sides)
    tpd = TreeParams(max_depth=6, min_rows=1, learn_rate=1.0, leaf_mode=1, mtries=3, min_split_improvement=0, seed=7)
    yb = (y > 1).astype(np.float32)
    ec = train_ensemble(bc, yb, dist="drf", ntrees=4, tparams=tpd, sample_rate=0.632, seed=11)
    eg = train_ensemble(bg, yb, dist="drf", ntrees=4, tparams=tpd, sample_rate=0.632, seed=11)
    t0c, t0g = ec.trees[0], eg.trees[0]
    for i in [j for j in ec.compact()[0] if j < 3]:
        assert t0c[i]["feat"] == t0g[i]["feat"]
    # depth-6 / min_rows=1 DRF trees hold many exact gain ties in small nodes:
    # compare model quality, not leaf membership
    from sklearn.metrics import roc_auc_score
    mc, mg = ec.raw_margin(Xt).numpy()[0], eg.raw_margin(Xt.cuda()).cpu().numpy()[0]
    assert np.abs(mc - mg).mean() < 0.02
    assert abs(roc_auc_score(yb, mc) - roc_auc_score(yb, mg)) < 0.01


def test_deep_tree_multipass(cuda_dev):
    """Depth 9 forces several LDS slot passes per level at 256 bins."""
    X, y = _data(n=20000)
    bc, bg = _both(X, y)
    tp = TreeParams(max_depth=9, min_rows=2, learn_rate=0.5, min_split_improvement=0)
    ec = train_ensemble(bc, y, dist="bernoulli", ntrees=2, tparams=tp)
    eg = train_ensemble(bg, y, dist="bernoulli", ntrees=2, tparams=tp)
    Xt = torch.from_numpy(X)
    mc = ec.raw_margin(Xt)[0].numpy()
    mg = eg.raw_margin(Xt.cuda())[0].cpu().numpy()
    # deep trees can diverge on near-ties; compare quality, not bits
    from sklearn.metrics import roc_auc_score
    assert abs(roc_auc_score(y, mc) - roc_auc_score(y, mg)) < 5e-3
    assert (np.abs(mc - mg) < 1e-3).mean() > 0.7


@pytest.mark.parametrize("dist,depth,sample_rate,nbins", [("bernoulli", 5, 1.0, 255), ("bernoulli", 8, 0.7, 63),
                                                          ("gaussian", 6, 1.0, 20), ("multinomial", 4, 1.0, 255),
                                                          ("drf", 12, 0.632, 20)])
def test_segmented_engine_matches_scan_engine(cuda_dev, monkeypatch, dist, depth, sample_rate, nbins):
    """The row-partitioned engine builds bit-identical trees to the scan engine:
    both quantise every row with the same dither and sum integers."""
    import h2omx.models.tree.engine as E

    task = {"bernoulli": "bin", "gaussian": "reg", "multinomial": "multi", "drf": "bin"}[dist]
    X, y = _data(n=40000, F=9, seed=3, task=task)
    _, bg = _both(X, y, nbins)
    tp = TreeParams(max_depth=depth, min_rows=3, learn_rate=0.2,
                    leaf_mode=1 if dist == "drf" else 0, mtries=3 if dist == "drf" else 0)
    yt = torch.from_numpy(y).cuda()
    nclass = 3 if dist == "multinomial" else (2 if dist == "drf" else 1)
    out = {}
    for eng, scan_slots, close_sb in (("scan", 16, 2048), ("seg", 0, 2048), ("seg2", 2, 2048), ("seg3", 0, 0)):
        monkeypatch.setenv("H2OMX_TREE_ENGINE", eng[:3] if eng != "scan" else "scan")
        # seg: chunked histograms at every level; seg2: scan histograms while <= 2 built
        # nodes; seg3: multi-block level close at every level
        monkeypatch.setattr(E.HipTreeBuilder, "SCAN_SLOTS", scan_slots)
        monkeypatch.setattr(E.HipTreeBuilder, "CLOSE_SINGLE_BLOCK", close_sb)
        out[eng] = train_ensemble(bg, yt, dist=dist, ntrees=4, tparams=tp, sample_rate=sample_rate, nclass=nclass,
                                  seed=11)
    a = out["scan"]
    for b in (out["seg"], out["seg2"], out["seg3"]):
        for t in range(a.trees.shape[0]):
            for i in a.compact()[t]:
                assert a.trees[t][i]["feat"] == b.trees[t][i]["feat"], (t, i)
                assert a.trees[t][i]["bin"] == b.trees[t][i]["bin"], (t, i)
                np.testing.assert_allclose(a.trees[t][i]["value"], b.trees[t][i]["value"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("dist,depth,sample_rate,nbins,mtries,col_rate,mode", [
    ("drf", 12, 0.632, 20, 3, 1.0, 0), ("bernoulli", 13, 0.8, 255, 0, 0.7, 1), ("gaussian", 14, 1.0, 63, 0, 1.0, 0),
    ("multinomial", 11, 1.0, 255, 0, 1.0, 0), ("drf", 16, 1.0, 127, 4, 1.0, 0)])
def test_direct_deep_levels_match_subtraction(cuda_dev, monkeypatch, dist, depth, sample_rate, nbins, mtries,
                                              col_rate, mode):
    """Deep levels in direct mode - one workgroup per node (seg_direct_kernel)
    or one wave per node (seg_direct_wave_kernel), packed or two-plane LDS
    histograms built and scanned in LDS - grow the same trees as the
    parent-minus-sibling histogram path; so does the multi-block level
    finalisation against the single-workgroup one."""
    import h2omx.models.tree.engine as E

    task = {"bernoulli": "bin", "gaussian": "reg", "multinomial": "multi", "drf": "bin"}[dist]
    X, y = _data(n=50000, F=13, seed=6, task=task)
    _, bg = _both(X, y, nbins)
    tp = TreeParams(max_depth=depth, min_rows=2, learn_rate=0.2, leaf_mode=1 if dist == "drf" else 0,
                    mtries=mtries, col_sample_rate=col_rate, mode=mode, reg_lambda=1.0 if mode else 0.0,
                    min_child_weight=1.0 if mode else 0.0)
    yt = torch.from_numpy(y).cuda()
    monkeypatch.setenv("H2OMX_TREE_ENGINE", "seg")
    nclass = 3 if dist == "multinomial" else (2 if dist == "drf" else 1)
    out = {}
    # engine switches: direct from this many nodes, wave-per-node below this many rows per node,
    # multi-block finalise, wave-chunk partition from this many nodes, chunked direct workgroups,
    # (g, s2) moved into segment order, eligible-feature codes stored for the partition,
    # column-major code planes every k direct levels
    keys = ("DIRECT_MIN_NODES", "DIRECT_WAVE_ROWS", "LF_MULTI_BLOCK", "PART_WAVE_NODES", "DIRECT_CHUNKED",
            "PERMUTE_GS", "ECODES", "COLMAJOR_EVERY")
    for cfg in ((0, 0, False, 1 << 30, True, False, False, 0), (0, 0, True, 1, True, True, True, 0),
                (2, 0, True, 1 << 30, True, True, True, 0), (64, 0, True, 1 << 30, False, False, True, 0),
                (64, 1 << 30, True, 1, True, True, False, 0), (64, 1 << 30, False, 2048, True, False, True, 0),
                (64, 0, True, 1 << 30, True, True, True, 0), (2, 0, True, 1 << 30, True, True, True, 1),
                (2, 0, True, 1, True, True, False, 3), (64, 0, True, 1 << 30, True, False, True, 2)):
        for k, v in zip(keys, cfg):
            monkeypatch.setattr(E.HipTreeBuilder, k, v)
        out[cfg] = train_ensemble(bg, yt, dist=dist, ntrees=3, tparams=tp, sample_rate=sample_rate,
                                  nclass=nclass, seed=13)
    a = out[(0, 0, False, 1 << 30, True, False, False, 0)]
    for cfg, b in out.items():
        for t in range(a.trees.shape[0]):
            reach = a.compact()[t]
            assert reach == b.compact()[t], (cfg, t)
            for f in ("feat", "bin", "value", "weight"):
                np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f], err_msg=f"{cfg} tree {t} {f}")


@pytest.mark.parametrize("dist,depth,sample_rate", [("bernoulli", 5, 1.0), ("gaussian", 7, 0.7)])
def test_pk32_rows_match_pk64(cuda_dev, monkeypatch, dist, depth, sample_rate):
    """32-bit packed rows (large row chunks: per-row values fit 16 bits) build
    bit-identical trees to the 64-bit rows."""
    import h2omx.models.tree.engine as E

    X, y = _data(n=600_000, F=9, seed=8, task="bin" if dist == "bernoulli" else "reg")
    _, bg = _both(X, y, 255)
    tp = TreeParams(max_depth=depth, min_rows=3, learn_rate=0.2)
    yt = torch.from_numpy(y).cuda()
    monkeypatch.setattr(E.HipTreeBuilder, "TARGET_WGS", 8)   # few, large row chunks
    made = []
    init = E.HipTreeBuilder.__init__

    def spy(self, *a, **k):
        init(self, *a, **k)
        made.append(self)

    monkeypatch.setattr(E.HipTreeBuilder, "__init__", spy)
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setattr(E.HipTreeBuilder, "PK32", flag == "1")
        out[flag] = train_ensemble(bg, yt, dist=dist, ntrees=3, tparams=tp, sample_rate=sample_rate, seed=5)
    assert [m.pk32 for m in made] == [False, True]
    a, b = out["0"], out["1"]
    for t in range(a.trees.shape[0]):
        reach = a.compact()[t]
        assert reach == b.compact()[t]
        for f in ("feat", "bin", "value"):
            np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f])


@pytest.mark.parametrize("dist,depth,min_rows", [("bernoulli", 5, 3), ("gaussian", 7, 400), ("multinomial", 4, 3)])
def test_level_finalisation_in_reduce_launch(cuda_dev, monkeypatch, dist, depth, min_rows):
    """The level finalisation folded into the last workgroup of the reduce +
    split scan (write-through split records, ticket, agent-scope loads:
    FUSE_FIN_LOCAL) builds bit-identical trees to its separate launch."""
    import h2omx.models.tree.engine as E

    X, y = _data(n=300_000, F=10, seed=31, task={"bernoulli": "bin", "gaussian": "reg"}.get(dist, "multi"))
    _, bg = _both(X, y, 255)
    tp = TreeParams(max_depth=depth, min_rows=min_rows, learn_rate=0.2)
    yt = torch.from_numpy(y).cuda()
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(E.HipTreeBuilder, "FUSE_FIN_LOCAL", flag)
        out[flag] = train_ensemble(bg, yt, dist=dist, ntrees=4, tparams=tp, seed=3,
                                   nclass=int(y.max()) + 1 if dist == "multinomial" else 1)
    a, b = out[False], out[True]
    assert a.trees.shape == b.trees.shape
    for t in range(a.trees.shape[0]):
        reach = a.compact()[t]
        assert reach == b.compact()[t]
        for f in ("feat", "bin", "value"):
            np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f])


@pytest.mark.parametrize("dist,depth,sample_rate,min_rows,lds_kb", [
    ("bernoulli", 5, 1.0, 3, 0), ("bernoulli", 6, 0.6, 400, 0), ("gaussian", 8, 0.8, 50, 0),
    ("multinomial", 4, 1.0, 3, 0), ("bernoulli", 1, 1.0, 3, 0), ("gaussian", 6, 1.0, 3, 16)])
def test_fused_routing_matches_partition(cuda_dev, monkeypatch, dist, depth, sample_rate, min_rows, lds_kb):
    """Partition fused into the next level's histogram kernel (double-buffered
    node ids, whole-tree leaf sums at the last level) builds bit-identical
    trees and margins: early leaves (large min_rows), bagging, several slot
    passes per level (small LDS budget) and depth 1 included."""
    import h2omx.models.tree.engine as E

    task = {"bernoulli": "bin", "gaussian": "reg", "multinomial": "multi"}[dist]
    X, y = _data(n=30000, F=9, seed=9, task=task)
    _, bg = _both(X, y, 255)
    tp = TreeParams(max_depth=depth, min_rows=min_rows, learn_rate=0.2)
    yt = torch.from_numpy(y).cuda()
    if lds_kb:
        monkeypatch.setattr(E.HipTreeBuilder, "LDS_BUDGET", lds_kb * 1024)
        monkeypatch.setattr(E.HipTreeBuilder, "DEEP_LDS_BUDGET", lds_kb * 1024)
    out = {}
    # unfused; fused while the previous level has <= 4 nodes (routing pass after);
    # fused at every level
    for key, flag, max_prev in (("off", "0", 4), ("mixed", "1", 4), ("all", "1", 1 << 20)):
        monkeypatch.setattr(E.HipTreeBuilder, "FUSE_ROUTE", flag == "1")
        monkeypatch.setattr(E.HipTreeBuilder, "FUSE_MAX_PREV", max_prev)
        out[key] = train_ensemble(bg, yt, dist=dist, ntrees=3, tparams=tp, sample_rate=sample_rate,
                                  nclass=3 if dist == "multinomial" else 1, seed=4)
    Xd = torch.from_numpy(X).cuda()

    def margin(e):
        m = e.raw_margin(Xd)
        return m.cpu().numpy() if torch.is_tensor(m) else np.asarray(m)

    a = out["off"]
    for b in (out["mixed"], out["all"]):
        for t in range(a.trees.shape[0]):
            reach = a.compact()[t]
            assert reach == b.compact()[t]
            for f in ("feat", "bin", "value", "weight"):
                np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f])
        np.testing.assert_array_equal(margin(a), margin(b))


@pytest.mark.parametrize("nbins", [20, 255])
def test_device_edges_match_host_edges(cuda_dev, nbins):
    """compute_edges on the device == the NumPy sketch on the same sample."""
    rng = np.random.default_rng(5)
    n = 300_000
    X = np.stack([rng.normal(size=n), rng.integers(0, 7, n).astype(float), rng.exponential(size=n),
                  np.round(rng.normal(size=n), 1), np.full(n, 3.0)]).astype(np.float32)
    X[0, rng.random(n) < 0.2] = np.nan
    X[2, :] = np.nan
    Xt = torch.from_numpy(X)
    eh, nh, bh = compute_edges(Xt, nbins, sample_rows=100_000, seed=3)
    ed, nd, bd = compute_edges(Xt.to(cuda_dev), nbins, sample_rows=100_000, seed=3)
    assert bh == bd
    np.testing.assert_array_equal(nh, nd)
    np.testing.assert_array_equal(eh, ed)


@pytest.mark.parametrize("n,mode,depth", [(40000, 0, 5), (40000, 1, 4), (600000, 0, 5), (600000, 1, 6)])
def test_fused_gradient_level_matches_boost_update(cuda_dev, monkeypatch, n, mode, depth):
    """Level 0 with the gradient pass fused in (hist_build PKM 5: F += previous
    tree, (g, h) from (F, y), bound-based quantisation scales) grows the same
    trees and margins as the separate boost_update pass; 600k rows run the
    32-bit packed rows, 40k rows the 64-bit ones."""
    from h2omx.models.tree.boost import GpuBooster, TreeEnsemble, _GpuView
    from h2omx.models.tree.engine import HipTreeBuilder

    X, y = _data(n=n, F=9, seed=12, task="bin")
    _, bg = _both(X, y, 255)
    tp = TreeParams(max_depth=depth, min_rows=3, learn_rate=0.2, mode=mode, reg_lambda=1.0 if mode else 0.0)
    yt = torch.from_numpy(y).cuda()
    monkeypatch.setenv("H2OMX_TREE_ENGINE", "scan")
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setattr(HipTreeBuilder, "FUSE_GRAD", flag == "1")   # (default: see HipTreeBuilder.can_fuse_grad)
        ens = TreeEnsemble(trees=np.zeros((0, 1)), K=1, dist="bernoulli", init_f=np.array([0.1]), nbt=bg.nbt,
                           feature_names=bg.names)
        gb = GpuBooster(bg, yt, None, ens, tp, 1.0, 3, None, {})
        assert gb.fused == (flag == "1")
        margins = []
        for t in range(4):
            gb.step()
            if t == 1:   # a mid-training read flushes; the next step must not re-apply
                margins.append(_GpuView(gb).margin[0].clone())
        out[flag] = (gb.finish(), margins, gb.st.Fm[0, :n].clone())
    (a, ma, fa), (b, mb, fb) = out["0"], out["1"]
    for t in range(a.trees.shape[0]):
        reach = a.compact()[t]
        assert reach == b.compact()[t]
        for f in ("feat", "bin", "value", "weight"):
            np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f])
    torch.testing.assert_close(ma[0], mb[0], rtol=0, atol=0)
    torch.testing.assert_close(fa, fb, rtol=0, atol=0)


@pytest.mark.parametrize("dist,depth,min_rows,n,ntrees", [("bernoulli", 5, 10, 400_000, 6),
                                                          ("gaussian", 7, 3, 150_000, 6),
                                                          ("bernoulli", 1, 3, 50_000, 6),
                                                          ("bernoulli", 4, 3, 60_000, 70)])
def test_graph_replay_matches_eager(cuda_dev, monkeypatch, dist, depth, min_rows, n, ntrees):
    """Each boosting step replayed as one HIP graph (tree index / dither salt
    taken from the device counter) builds bit-identical trees and margins to
    the eager launch sequence.  Bernoulli (fixed gradient bounds) replays the
    chained step (next tree's begin inside the leaf finalisation, the tree
    archive inside boost_update); even depth puts the final control block in
    the level-0 slot the chained begin rewrites; 70 trees wrap the 64-slot
    archive ring."""
    from h2omx.models.tree import boost as B

    X, y = _data(n=n, F=11, seed=21, task="bin" if dist == "bernoulli" else "reg")
    _, bg = _both(X, y, 255)
    tp = TreeParams(max_depth=depth, min_rows=min_rows, learn_rate=0.2)
    yt = torch.from_numpy(y).cuda()
    made = []
    init = B.GpuBooster.__init__

    def spy(self, *a, **k):
        init(self, *a, **k)
        made.append(self)

    monkeypatch.setattr(B.GpuBooster, "__init__", spy)
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("H2OMX_TREE_GRAPH", flag)
        out[flag] = train_ensemble(bg, yt, dist=dist, ntrees=ntrees, tparams=tp, seed=5)
    assert not made[0].graph_used and made[1].graph_used, made[1].graph_error
    from h2omx.models.tree.engine import HipTreeBuilder as _HTB

    if dist == "bernoulli" and _HTB.CHAIN_BEGIN:
        assert made[1].graph_chain
    a, b = out["0"], out["1"]
    assert a.trees.shape == b.trees.shape
    for t in range(a.trees.shape[0]):
        reach = a.compact()[t]
        assert reach == b.compact()[t], t
        for f in ("feat", "bin", "value", "weight"):
            np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f], err_msg=f"tree {t} {f}")
    torch.testing.assert_close(a._state.Fm, b._state.Fm, rtol=0, atol=0)



@pytest.mark.parametrize("dist,mode", [("bernoulli", 0), ("bernoulli", 1), ("gaussian", 0)])
def test_level0_copies_match_plain_slices(cuda_dev, monkeypatch, dist, mode):
    """Level 0 with 8 / 4 interleaved lane copies - low-cardinality columns laid
    out as up to 64 slices inside the copies' space, high-cardinality ones
    interleaved - builds bit-identical trees to the plain one-slice kernel."""
    import h2omx.models.tree.engine as E

    rng = np.random.default_rng(23)
    X, y = _data(n=400_000, F=9, seed=23, task="bin" if dist == "bernoulli" else "reg")
    X[6] = rng.integers(0, 7, X.shape[1])       # weekday-like
    X[7] = rng.integers(1, 13, X.shape[1])      # month-like
    X[8] = rng.integers(0, 30, X.shape[1]).astype(np.float32)
    X[8, rng.random(X.shape[1]) < 0.05] = np.nan
    y = y + (dist != "bernoulli") * 0.3 * X[7]
    _, bg = _both(X, y, 255)
    tp = TreeParams(max_depth=5, min_rows=3, learn_rate=0.2, mode=mode, reg_lambda=1.0 if mode else 0.0)
    yt = torch.from_numpy(y.astype(np.float32)).cuda()
    out = {}
    for cop in (1, 4, 8):
        monkeypatch.setattr(E.HipTreeBuilder, "L0_COPIES", cop)
        out[cop] = train_ensemble(bg, yt, dist=dist, ntrees=3, tparams=tp, seed=5)
    a = out[1]
    for cop in (4, 8):
        b = out[cop]
        for t in range(a.trees.shape[0]):
            reach = a.compact()[t]
            assert reach == b.compact()[t], (cop, t)
            for f in ("feat", "bin", "value"):
                np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f], err_msg=f"{cop} {t} {f}")


@pytest.mark.parametrize("F,fp", [(13, 16), (100, 128), (200, 256), (37, 40), (6, 8), (300, 384)])
def test_seg_colmajor_transpose(cuda_dev, F, fp):
    """h2omx_seg_colmajor: plane f, position j holds code f of row idx[j]
    (16-byte row chunks when fp % 16 == 0, dwords otherwise); positions whose
    row id is out of range read as zeros."""
    from h2omx import ops

    lib = ops.tree_lib()
    g = torch.Generator().manual_seed(F)
    nrows, n = 5000, 3001
    codes = torch.randint(0, 256, (nrows, fp), generator=g, dtype=torch.uint8)
    idx = torch.randint(0, nrows, (n + 64,), generator=g, dtype=torch.int32)
    idx[::97] = nrows + 5   # stale ids of retired segments
    plane = -(-n // 256) * 256
    ccol = torch.full((F * plane,), 7, dtype=torch.uint8, device=cuda_dev)
    cd, idd = codes.to(cuda_dev), idx.to(cuda_dev)
    ops.check(lib.h2omx_seg_colmajor(ops.P(cd), fp, F, ops.P(idd), n, nrows, ops.P(ccol), plane,
                                     ops.stream(cuda_dev)), "seg_colmajor")
    got = ccol.view(F, plane)[:, :n].cpu()
    ok = idx[:n].long() < nrows
    want = torch.zeros((F, n), dtype=torch.uint8)
    want[:, ok] = codes[idx[:n].long()[ok], :F].T
    assert torch.equal(got, want)


def test_mean_leaves_without_h_match(cuda_dev, monkeypatch):
    """DRF (mean leaves) on the segmented engine: partitions given no h (their
    H sums are unused) grow the same trees, values and weights."""
    import h2omx.models.tree.engine as E

    X, y = _data(n=40000, F=11, seed=9, task="bin")
    _, bg = _both(X, y, 64)
    tp = TreeParams(max_depth=14, min_rows=2, learn_rate=1.0, leaf_mode=1, mtries=4)
    yt = torch.from_numpy(y).cuda()
    monkeypatch.setenv("H2OMX_TREE_ENGINE", "seg")
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(E.HipTreeBuilder, "MEAN_LEAVES_NO_H", flag)
        out[flag] = train_ensemble(bg, yt, dist="drf", ntrees=3, tparams=tp, sample_rate=0.632, nclass=2, seed=3)
    a, b = out[False], out[True]
    for t in range(a.trees.shape[0]):
        reach = a.compact()[t]
        assert reach == b.compact()[t]
        for f in ("feat", "bin", "value", "weight"):
            np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f], err_msg=f"tree {t} {f}")


@pytest.mark.parametrize("F,n", [(100, 70000), (13, 5000), (6, 300), (37, 1000), (300, 2000)])
def test_codes_rowmajor_matches_torch(cuda_dev, F, n):
    """BinnedMatrix.codes_rm (h2omx_codes_rowmajor): row j holds the F codes of
    row j, the pad bytes up to fp are zero - as the strided torch copy."""
    X = torch.from_numpy(np.random.default_rng(F).normal(size=(F, n)).astype(np.float32))
    e, nv, nbt = compute_edges(X, 63)
    bm = bin_matrix(X.to(cuda_dev), e, nv, nbt)
    got = bm.codes_rm.cpu()
    want = torch.zeros((bm.n, bm.fp), dtype=torch.uint8)
    want[:, :F] = bm.codes[:, : bm.n].t().cpu()
    assert bm.fp >= F and torch.equal(got, want)


def test_async_forest_download_matches(cuda_dev, monkeypatch):
    """Deep trees are downloaded per tree by a helper thread while the next
    one builds: the host forest equals the one copied at the end of the fit."""
    from h2omx.models.tree.boost import GpuBooster

    X, y = _data(n=30000, F=9, seed=4, task="bin")
    _, bg = _both(X, y, 64)
    tp = TreeParams(max_depth=16, min_rows=1, learn_rate=1.0, leaf_mode=1, mtries=3)
    yt = torch.from_numpy(y).cuda()
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(GpuBooster, "ASYNC_DOWNLOAD", flag)
        out[flag] = train_ensemble(bg, yt, dist="drf", ntrees=4, tparams=tp, sample_rate=0.632, nclass=2, seed=2)
    a, b = out[False], out[True]
    assert a.trees.shape == b.trees.shape and not b.trees.flags["C_CONTIGUOUS"]
    assert a.trees.tobytes() == b.trees.tobytes()
    Xd = torch.from_numpy(X).cuda()
    np.testing.assert_array_equal(a.raw_margin(Xd).cpu().numpy(), b.raw_margin(Xd).cpu().numpy())


@pytest.mark.parametrize("dist,mode,nclass", [("drf", 0, 2), ("drf", 0, 3), ("gaussian", 0, 1), ("bernoulli", 1, 1),
                                             ("multinomial", 0, 3)])
def test_bag_compact_matches(cuda_dev, monkeypatch, dist, mode, nclass):
    """Bagged deep trees whose root segment holds only in-bag rows (the
    others walk the finished tree for their leaf) grow the same trees and
    leave the same margins and out-of-bag sums as trees that carry every row."""
    import h2omx.models.tree.engine as E

    X, y = _data(n=30000, F=9, seed=7, task="reg" if dist == "gaussian" else ("multi" if nclass == 3 else "bin"))
    _, bg = _both(X, y, 64)
    tp = TreeParams(max_depth=13, min_rows=2, learn_rate=1.0 if dist == "drf" else 0.2,
                    leaf_mode=1 if dist == "drf" else 0, mtries=4 if dist == "drf" else -1, mode=mode,
                    reg_lambda=1.0 if mode else 0.0, min_child_weight=1.0 if mode else 0.0)
    yt = torch.from_numpy(y).cuda()
    monkeypatch.setenv("H2OMX_TREE_ENGINE", "seg")
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(E.HipTreeBuilder, "BAG_COMPACT", flag)
        out[flag] = train_ensemble(bg, yt, dist=dist, ntrees=3, tparams=tp, sample_rate=0.6,
                                   nclass=nclass if nclass > 1 else 1, seed=11)
    a, b = out[False], out[True]
    assert a.trees.tobytes() == b.trees.tobytes()
    sa, sb = getattr(a, "_state", None), getattr(b, "_state", None)
    if sa is not None:
        np.testing.assert_array_equal(sa.Fm.cpu().numpy(), sb.Fm.cpu().numpy())
    oa, ob = getattr(a, "_oob", None), getattr(b, "_oob", None)
    if oa is not None:
        for u, v in zip(oa, ob):
            np.testing.assert_array_equal(u.cpu().numpy(), v.cpu().numpy())


def test_bag_compact_early_finish(cuda_dev, monkeypatch):
    """A bagged deep tree that runs out of splittable nodes before max_depth
    still routes its out-of-bag rows (the walk then runs after the loop)."""
    import h2omx.models.tree.engine as E

    X, y = _data(n=3000, F=7, seed=3, task="bin")
    _, bg = _both(X, y, 16)
    tp = TreeParams(max_depth=18, min_rows=40, learn_rate=1.0, leaf_mode=1, mtries=2)
    yt = torch.from_numpy(y).cuda()
    monkeypatch.setenv("H2OMX_TREE_ENGINE", "seg")
    monkeypatch.setattr(E.HipTreeBuilder, "SYNC_NODE_CAP", 4)   # read node counts back early: the loop may stop
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(E.HipTreeBuilder, "BAG_COMPACT", flag)
        out[flag] = train_ensemble(bg, yt, dist="drf", ntrees=3, tparams=tp, sample_rate=0.6, nclass=2, seed=5)
    a, b = out[False], out[True]
    assert a.trees.tobytes() == b.trees.tobytes()
    for u, v in zip(a._oob, b._oob):
        np.testing.assert_array_equal(u.cpu().numpy(), v.cpu().numpy())


def test_seg_feature_groups_match(cuda_dev, monkeypatch):
    """The segmented histograms split into several feature groups (small LDS
    budget) build the same trees as one group of every feature."""
    import h2omx.models.tree.engine as E

    X, y = _data(n=30000, F=13, seed=12, task="bin")
    _, bg = _both(X, y, 63)   # 64-wide histograms
    tp = TreeParams(max_depth=12, min_rows=2, learn_rate=1.0, leaf_mode=1, mtries=4)
    yt = torch.from_numpy(y).cuda()
    monkeypatch.setenv("H2OMX_TREE_ENGINE", "seg")
    out = {}
    for budget in (64 * 1024, 2048):
        monkeypatch.setattr(E.HipTreeBuilder, "SEG_LDS_BUDGET", budget)
        monkeypatch.setattr(E.HipTreeBuilder, "SEG_LDS_BUDGET_WIDE", budget)
        out[budget] = train_ensemble(bg, yt, dist="drf", ntrees=3, tparams=tp, sample_rate=0.632, nclass=2, seed=4)
    a, b = out[64 * 1024], out[2048]
    for t in range(a.trees.shape[0]):
        reach = a.compact()[t]
        assert reach == b.compact()[t], t
        for f in ("feat", "bin", "value", "weight"):
            np.testing.assert_array_equal(a.trees[t][reach][f], b.trees[t][reach][f], err_msg=f"tree {t} {f}")
