"""Boosting / bagging driver shared by GBM, XGBoost and DRF.

One call to :func:`train_ensemble` grows ``ntrees`` iterations (``K`` trees
per iteration for multinomial / multi-class DRF).  On the GPU every
iteration is a fixed sequence of enqueued kernels (no host sync): the fused
``boost_update`` kernel applies the finished tree to the margins and
produces the next gradients, bagging weights and node ids in one pass.
"""
from __future__ import annotations

import ctypes
import gc
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ... import ops
from .binning import BinnedMatrix
from .engine import (GRAD_BOUNDS, HipTreeBuilder, TreeParams, grad_bounds_tensor, make_grad_params, tree_capacity,
                     trees_from_bytes)
from .structs import TREE_NODE_DTYPE


def concat_trees(*parts: np.ndarray) -> np.ndarray:
    """Stack tree heaps of different widths (compact deep-tree snapshots):
    narrower heaps are padded with unreachable zero nodes."""
    parts = [p for p in parts if p.size]
    if not parts:
        return np.zeros((0, 1), TREE_NODE_DTYPE)
    width = max(p.shape[1] for p in parts)
    out = np.zeros((sum(p.shape[0] for p in parts), width), TREE_NODE_DTYPE)
    r = 0
    for p in parts:
        out[r: r + p.shape[0], : p.shape[1]] = p
        r += p.shape[0]
    return out


def concat_catbits(first, second) -> np.ndarray:
    """Categorical bitsets of two ensembles stacked like concat_trees (trees
    without categorical splits get zero bitsets)."""
    parts = []
    for e in (first, second):
        n, w = e.trees.shape[0], e.trees.shape[1] if e.trees.ndim == 2 else 1
        c = e.catbits if e.catbits is not None else np.zeros((n, w, 8), np.uint32)
        parts.append(c)
    width = max(p.shape[1] for p in parts)
    out = np.zeros((sum(p.shape[0] for p in parts), width, 8), np.uint32)
    r = 0
    for p in parts:
        out[r: r + p.shape[0], : p.shape[1]] = p
        r += p.shape[0]
    return out


@dataclass
class TreeEnsemble:
    trees: np.ndarray            # [n_trees_total][capacity] TREE_NODE_DTYPE
    K: int                       # trees per iteration (classes for multinomial)
    dist: str
    init_f: np.ndarray           # [K] initial margin
    average: bool = False        # DRF: prediction = sum / ntrees
    nbt: int = 256
    feature_names: list = field(default_factory=list)
    edges: list = field(default_factory=list)   # per-feature numpy cut points
    timings: dict = field(default_factory=dict)
    # categorical group splits: [n_trees_total][capacity][8] uint32 left-set
    # bitsets by node (TreeNode.na_left bit 1 marks such a split); None = none
    catbits: np.ndarray | None = None

    @property
    def ntrees(self) -> int:
        return self.trees.shape[0] // max(self.K, 1)

    def compact(self):
        """Per tree, the list of reachable node records (for export)."""
        out = []
        for t in range(self.trees.shape[0]):
            tr = self.trees[t]
            keep, stack = [], [0]
            while stack:
                i = stack.pop()
                keep.append(i)
                if tr[i]["feat"] >= 0:
                    stack += [int(tr[i]["left"]) + 1, int(tr[i]["left"])]
            out.append(sorted(keep))
        return out

    # -- scoring ---------------------------------------------------------------
    def raw_margin(self, X: torch.Tensor, ntrees: int | None = None) -> torch.Tensor:
        """Margins [K][n] for feature-major raw data X [F][n]."""
        nt = self.ntrees if ntrees is None else ntrees
        T = nt * self.K
        n = X.shape[1]
        if X.is_cuda:
            dev = X.device
            Xc = X.float().contiguous()
            key = (T, str(dev), self.trees.shape, id(self.trees), id(self.catbits))
            cache = getattr(self, "_dev_nodes", None)
            if cache is not None and cache[0] == key:
                nodes, cbits = cache[1], cache[2]
            else:
                nodes = torch.from_numpy(self.trees[:T].reshape(-1).view(np.uint8).copy()).to(dev)
                cbits = None
                if self.catbits is not None:
                    cb = np.ascontiguousarray(self.catbits[:T], np.uint32).reshape(-1)
                    cbits = torch.from_numpy(cb.view(np.int32).copy()).to(dev)
                self._dev_nodes = (key, nodes, cbits)
            cap = self.trees.shape[1]
            roots = torch.arange(T, dtype=torch.int32, device=dev) * cap
            out = torch.empty((self.K, n), dtype=torch.float32, device=dev)
            if self.average:
                out.zero_()
            else:
                out.copy_(torch.from_numpy(self.init_f.astype(np.float32)).to(dev)[:, None].expand(self.K, n))
            if T:
                lib = ops.tree_lib()
                ops.check(lib.h2omx_predict_raw(ops.P(Xc), Xc.stride(0), n, ops.P(nodes), ops.P(roots), T, self.K,
                                                ops.P(out), out.stride(0), ops.P(cbits), ops.stream(dev)),
                          "predict_raw")
            if self.average and nt > 0:
                out /= nt
            return out
        from ...reference.tree import raw_margin_cpu

        return raw_margin_cpu(self, X, nt)



def init_margin(dist: str, y, w, K: int) -> np.ndarray:
    """Initial margin (H2O's init_f).  ``y`` / ``w`` may be device tensors: the
    weighted sums then run on the device and only scalars reach the host."""
    if torch.is_tensor(y):
        if dist in ("multinomial", "drf"):
            return np.zeros(K)
        if dist in ("laplace", "quantile"):
            return init_margin(dist, y.detach().float().cpu().numpy(), None, K)
        yd = y.detach().double()
        sw = float(yd.numel()) if w is None else float(w.detach().double().sum())
        swy = float(yd.sum()) if w is None else float((w.detach().double() * yd).sum())
        m = swy / sw
        if dist == "bernoulli":
            p = float(np.clip(m, 1e-6, 1 - 1e-6))
            return np.array([np.log(p / (1 - p))])
        if dist in ("poisson", "gamma", "tweedie"):
            return np.array([np.log(max(m, 1e-12))])
        return np.array([m])
    ww = np.ones_like(y, dtype=np.float64) if w is None else w.astype(np.float64)
    sw = ww.sum()
    if dist == "bernoulli":
        p = float(np.clip((ww * y).sum() / sw, 1e-6, 1 - 1e-6))
        return np.array([np.log(p / (1 - p))])
    if dist == "multinomial":
        return np.zeros(K)
    if dist in ("poisson", "gamma", "tweedie"):
        return np.array([np.log(max((ww * y).sum() / sw, 1e-12))])
    if dist in ("laplace", "quantile"):
        return np.array([float(np.median(y))])
    if dist == "drf":
        return np.zeros(K)
    return np.array([(ww * y).sum() / sw])


def _order_keys(r: torch.Tensor) -> torch.Tensor:
    """int64 keys ordered like the float64 values (IEEE bits, negative values
    with the magnitude bits flipped)."""
    b = r.contiguous().view(torch.int64)
    return torch.where(b < 0, b ^ 0x7FFFFFFFFFFFFFFF, b)


def _key_value(k: int) -> float:
    b = k ^ 0x7FFFFFFFFFFFFFFF if k < 0 else k
    return float(np.array([b], np.int64).view(np.float64)[0])


def weighted_quantile(r, w, q: float, comm=None) -> float:
    """Weighted 'lower' q-quantile of ``r`` over every rank: the smallest value
    v of the data with sum(w[r <= v]) >= q * sum(w).  Bisection on the
    order-preserving int64 key of the float64 value (at most 64 steps, exact:
    the bracket ends on adjacent keys, and the upper one is a data value),
    one all-reduced weight sum per step (no gather of the rows, any row
    count; torch.quantile is limited to 2^24 elements)."""
    multi = comm is not None and comm.world_size > 1
    r = r.detach().double() if torch.is_tensor(r) else torch.from_numpy(np.asarray(r, np.float64))
    wt = torch.ones_like(r) if w is None else (w.detach().double() if torch.is_tensor(w)
                                               else torch.from_numpy(np.asarray(w, np.float64))).to(r.device)
    keep = wt > 0
    r, wt = r[keep], wt[keep]
    keys = _order_keys(r)

    def red(v, op="sum"):
        a = np.array(v, np.float64)
        return comm.all_reduce_numpy(a, op) if multi else a

    W = float(red([float(wt.sum())])[0])
    if W <= 0:
        return 0.0
    # key range over every rank: reduce the min / max values, then key them
    lo_v = -float(red([-(float(r.min()) if r.numel() else 1e300)], "max")[0])
    hi_v = float(red([float(r.max()) if r.numel() else -1e300], "max")[0])
    lo = int(_order_keys(torch.tensor([lo_v], dtype=torch.float64))[0])
    hi = int(_order_keys(torch.tensor([hi_v], dtype=torch.float64))[0])
    target = q * W
    if float(red([float(wt[keys <= lo].sum())])[0]) >= target:
        return lo_v
    while hi - lo > 1:              # invariant: cum(lo) < target <= cum(hi)
        mid = lo + (hi - lo) // 2
        if float(red([float(wt[keys <= mid].sum())])[0]) >= target:
            hi = mid
        else:
            lo = mid
    return _key_value(hi)


def train_ensemble(bm: BinnedMatrix, y, w=None, *, dist: str = "bernoulli", ntrees: int = 50,
                   tparams: TreeParams | None = None, sample_rate: float = 1.0, nclass: int = 1,
                   seed: int = 0, comm=None, init_f: np.ndarray | None = None, callback=None,
                   dist_kw: dict | None = None, base_margin=None, tree_offset: int = 0) -> TreeEnsemble:
    """Grow an ensemble on binned data.

    ``y``: float targets (class index for multinomial / multi-class DRF).
    ``dist``: gaussian|bernoulli|multinomial|poisson|gamma|tweedie|laplace|quantile|huber|drf.
    ``base_margin``: [K][n] starting margins (checkpoint continuation) instead of ``init_f``.
    ``tree_offset``: iterations already in the model being continued: iteration t
    is global iteration tree_offset + t (learn-rate annealing, bagging / column
    sampling hashes, dither), so a continued model equals one long run.
    ``callback(t, view)``: called after every iteration; returning True stops training.
    """
    tparams = tparams or TreeParams()
    dist_kw = dist_kw or {}
    n = bm.n
    multi = dist == "multinomial" or (dist == "drf" and nclass > 2)
    K = nclass if multi else 1
    if bm.codes.is_cuda:
        # device-resident labels / weights stay on the device (no 11M-row host round trip)
        def _dev(v):
            return v.detach().float().to(bm.device) if torch.is_tensor(v) else \
                torch.from_numpy(np.asarray(v, np.float32)).to(bm.device)
        y_np = _dev(y)
        w_np = None if w is None else _dev(w)
    else:
        y_np = y.detach().float().cpu().numpy() if torch.is_tensor(y) else np.asarray(y, np.float32)
        w_np = None if w is None else (w.detach().float().cpu().numpy() if torch.is_tensor(w)
                                       else np.asarray(w, np.float32))
    if init_f is None:
        if dist in ("laplace", "quantile"):
            # H2O: weighted median / alpha-quantile of the response, over all ranks
            q = 0.5 if dist == "laplace" else float(dist_kw.get("quantile_alpha", 0.5))
            init_f = np.array([weighted_quantile(y_np, w_np, q, comm)])
        elif comm is not None and comm.world_size > 1:
            init_f = _global_init(dist, y_np, w_np, K, comm)
        else:
            init_f = init_margin(dist, y_np, w_np, K)
    ens = TreeEnsemble(trees=np.zeros((0, tree_capacity(tparams.max_depth)), TREE_NODE_DTYPE), K=K, dist=dist,
                       init_f=np.asarray(init_f, np.float64), average=(dist == "drf"), nbt=bm.nbt,
                       feature_names=list(bm.names), edges=bm.edges_numpy())
    ens._base_margin = base_margin
    if bm.codes.is_cuda:
        _train_gpu(bm, y_np, w_np, ens, ntrees, tparams, sample_rate, seed, comm, callback, dist_kw, tree_offset)
    else:
        # host-resident bins: the fp64 reference builder (test oracle, CPU-only clouds)
        from ...reference.tree import train_cpu

        train_cpu(bm, y_np, w_np, ens, ntrees, tparams, sample_rate, seed, comm, callback, dist_kw, tree_offset)
    return ens


def _global_init(dist, y, w, K, comm):
    if torch.is_tensor(y):
        yd = y.double()
        wd = None if w is None else w.double()
        loc = [float(yd.sum() if wd is None else (wd * yd).sum()), float(yd.numel() if wd is None else wd.sum())]
        s = comm.all_reduce_numpy(np.array(loc, np.float64))
    else:
        ww = np.ones_like(y, dtype=np.float64) if w is None else w.astype(np.float64)
        s = comm.all_reduce_numpy(np.array([(ww * y).sum(), ww.sum()], np.float64))
    m = s[0] / max(s[1], 1e-300)
    if dist == "bernoulli":
        p = float(np.clip(m, 1e-6, 1 - 1e-6))
        return np.array([np.log(p / (1 - p))])
    if dist in ("multinomial", "drf"):
        return np.zeros(K)
    if dist in ("poisson", "gamma", "tweedie"):
        return np.array([np.log(max(m, 1e-12))])
    return np.array([m])


class _GpuState:
    def __init__(self, bm, y_np, w_np, K, dist, init_f, base_margin=None):
        dev = bm.device
        npad, n = bm.npad, bm.n
        self.Fm = torch.zeros((K, npad), dtype=torch.float32, device=dev)
        if base_margin is not None:
            self.Fm[:, :n] = base_margin.to(dev).float()
        else:
            for k in range(K):
                self.Fm[k, :n] = float(init_f[k])
        if torch.is_tensor(y_np):
            self.y = torch.zeros(npad, dtype=torch.float32, device=dev)
            self.y[:n] = y_np.to(dev)
        else:
            yp = np.zeros(npad, np.float32)
            yp[:n] = y_np
            self.y = torch.from_numpy(yp).to(dev)
        self.yk = self.y.to(torch.int32) if K > 1 else None
        if dist == "drf" and K > 1:
            self.ycls = torch.stack([(self.y == k).float() for k in range(K)])
        self.w = None
        if w_np is not None and torch.is_tensor(w_np):
            self.w = torch.zeros(npad, dtype=torch.float32, device=dev)
            self.w[:n] = w_np.to(dev)
        elif w_np is not None:
            wp = np.zeros(npad, np.float32)
            wp[:n] = w_np
            self.w = torch.from_numpy(wp).to(dev)
        self.g = torch.empty((K, npad), dtype=torch.float32, device=dev)
        self.h = torch.empty((K, npad), dtype=torch.float32, device=dev)


class GpuBooster:
    """Step-wise GPU boosting loop (one ``step()`` = one iteration = K trees)."""

    def __init__(self, bm, y_np, w_np, ens, tp, sample_rate, seed, comm, dist_kw, ntrees_hint=64, tree_offset=0):
        self.lib = ops.tree_lib()
        self.bm, self.ens, self.tp = bm, ens, tp
        self.sample_rate, self.seed = sample_rate, seed
        self.dev = bm.device
        self.K, self.dist = ens.K, ens.dist
        self.st = _GpuState(bm, y_np, w_np, self.K, self.dist, ens.init_f, getattr(ens, "_base_margin", None))
        self.builder = HipTreeBuilder(bm, tp, comm)
        self.builder.bag_compact = sample_rate < 1.0
        self.cap = self.builder.capacity
        self.trees_dev = []
        self.cats_dev = []         # categorical left-set bitsets, parallel to trees_dev
        self.graph_used = False   # a step graph was captured (finish() releases the graph itself)
        self.graph_chain = False  # ... with tree_begin / archive folded into neighbours (TreeGraph.chain)
        need_w = sample_rate < 1.0 or self.st.w is not None
        self.wout = torch.empty((bm.npad,), dtype=torch.float32, device=self.dev) if need_w else None
        self.kw = dict(tweedie_power=dist_kw.get("tweedie_power", 1.5),
                       quantile_alpha=dist_kw.get("quantile_alpha", 0.5),
                       huber_delta=dist_kw.get("huber_delta", 1.0))
        self.t = tree_offset       # global iteration index (checkpoint continuation)
        self.t_start = tree_offset
        # K == 1 with bounded gradients: each tree's level 0 applies the previous
        # tree and computes the gradients itself (no boost_update pass); the
        # margins then lag one tree until flush()
        self.fused = (self.K == 1 and self.builder.can_fuse_grad(self.dist, self.st.w is not None, sample_rate))
        # HIP-graph replay of the step (TreeGraph): H2OMX_TREE_GRAPH=0 off, 1 / auto on
        # when graph_eligible(); captured at the second step (the first allocates buffers)
        self.use_graph = os.environ.get("H2OMX_TREE_GRAPH", "auto") != "0" and self.graph_eligible()
        self.graph = None
        self.graph_error = None
        # DRF out-of-bag predictions (H2O reports DRF training metrics on them):
        # per row the sum of the leaf values of the trees whose bag left it out
        self.oob = None
        if self.dist == "drf" and sample_rate < 1.0:
            self.oob = (torch.zeros((self.K, bm.npad), dtype=torch.float32, device=self.dev),
                        torch.zeros((bm.npad,), dtype=torch.float32, device=self.dev))
            self.use_graph = False
        self.pending = False
        # 0 / 1 labels as bytes for the gradient passes (bernoulli; exact as floats)
        self.y8 = None
        if self.K == 1 and self.dist == "bernoulli":
            yv = self.st.y
            if bool(((yv == 0) | (yv == 1)).all()):
                self.y8 = yv.to(torch.uint8)
        self.deferred: list = []  # graph mode: steps held back for a multi-tree replay
        self._archive = None     # TreeGraph capture: (ring, slots, counter offset)
        # bounded gradients (unweighted rows; bagging only zeroes rows) quantise with
        # the bound scales on every path, fused or not
        self._bounds = None
        if self.K == 1 and self.st.w is None and self.dist in GRAD_BOUNDS:
            self._bounds = grad_bounds_tensor(self.dist, self.dev)
        self._stall = self._stall_plan()
        if self.fused:
            pass
        elif self.K == 1:
            self._update(apply=False, next_tree=self.t, k=0)

    def _health(self):
        """Raise PeerLost when a peer is gone (watchdog) or a P2P exchange of an
        earlier step timed out on the device (pinned host word: no sync).  In
        graph mode no collective is host-issued, so this is the check that
        stops a multi-rank fit from returning a model built on timed-out sums."""
        c = self.builder.comm
        if c is not None and c.world_size > 1 and hasattr(c, "check_health"):
            c.check_health()

    # Test-only fault injection, resolved once per booster:
    # (tree, seconds) for this rank, or None.  tests/_p2p_fault_worker.py sets it
    # through FAULT_STALL_SPEC ("rank:tree:seconds"); the production step only
    # compares a cached None.
    FAULT_STALL_SPEC: str | None = None

    def _stall_plan(self):
        spec = type(self).FAULT_STALL_SPEC
        c = self.builder.comm
        if not spec or c is None:
            return None
        r, t, sec = spec.split(":")
        return (int(t), float(sec)) if int(r) == c.rank else None

    def _fault_stall(self):
        if self._stall is not None and self._stall[0] == self.t:
            time.sleep(self._stall[1])

    def flush(self):
        """Bring the margins up to date (fused mode applies each tree inside the
        next tree's first level; graph mode may hold steps back to replay them
        as one multi-tree graph)."""
        self._health()
        if self.graph is not None and self.deferred:
            for t in self.deferred:
                self.graph.replay(t)
            self.deferred = []
        if self.pending:
            b = self.builder
            ops.check(self.lib.h2omx_apply_tree(ops.P(self.st.Fm[0]), self.bm.n, ops.P(b.nid), ops.P(b.tree_buf),
                                                ops.stream(self.dev)), "apply_tree")
            self.pending = False

    def _update(self, apply: bool, next_tree: int, k: int, dist=None, pack: bool = False):
        P, st, b = ops.P, self.st, self.builder
        gp = make_grad_params(dist or self.dist, apply, self.sample_rate, self.seed, next_tree,
                              row_base=self.builder.row_base, **self.kw)
        gp.skip_nid = 1 if getattr(self.builder, "implicit_root", False) else 0
        y = st.ycls[k] if (self.dist == "drf" and self.K > 1) else st.y
        # bounded gradients: the next build() takes the bounds (stat=), so no
        # per-block maxima, no maxima reduction and no bounds copy per tree
        fixed = self._bounds is not None and k == 0 and self.K == 1
        with b.timer.phase("grad"):
            arch = self._archive    # (ring, slots, counter offset): graph replay's tree archive
            pk = b.pk if (pack or (arch is not None and b.pk_in_boost)) else None
            ops.check(self.lib.h2omx_boost_update(P(st.Fm[k]), P(y), P(st.w), self.bm.n, self.bm.npad, P(b.nid),
                                                  P(b.tree_buf), ctypes.addressof(gp), P(st.g[k]), P(st.h[k]),
                                                  P(self.wout), P(None if fixed else b.stat_slab),
                                                  b.tree_buf.numel(), P(arch[0] if arch else None),
                                                  arch[1] if arch else 0, P(b.tree_ctr if arch else None),
                                                  arch[2] if arch else 0, P(pk), P(b.qscale if pk is not None else None),
                                                  1 if b.p.mode == 1 else 0,
                                                  0 if (arch is not None and b.regrad is not None) else 1,
                                                  P(self.y8 if y is st.y else None),
                                                  P(b.leaf16_buf if (arch is not None and apply) else None),
                                                  ops.stream(self.dev)),
                      "boost_update")
            if not fixed:
                b.reduce_stats()

    def graph_eligible(self) -> bool:
        """A step is a fixed launch sequence whose only per-tree host input is
        the tree index (dither salt, read on the device from builder.tree_ctr):
        one tree per iteration, no bagging / column sampling / learn-rate
        annealing (those bake per-tree host values into the launches), the scan
        engine (the segmented one reads node counts on the host) and no phase
        timers (events are host objects)."""
        tp, b = self.tp, self.builder
        return (self.K == 1 and not self.fused and self.sample_rate >= 1.0 and tp.col_sample_rate >= 1.0
                and tp.col_sample_rate_per_tree >= 1.0 and tp.mtries == 0 and tp.learn_rate_annealing == 1.0
                and not b.segmented and not b.timer.enabled and self.cap <= self.COMPACT_CAP
                and self.dev.type == "cuda" and b.catf is None
                and tp.hist_mode in (0, 1))   # Random / RoundRobin draw per tree index

    def _body_k1(self, t: int, fresh: bool, chain: bool = False):
        b = self.builder
        if fresh:
            # grow the tree straight into its own buffer (no copy afterwards);
            # the next boost_update applies it from there
            b.tree_buf = torch.empty_like(b.tree_buf)
        b.build(self.st.g[0], self.st.h[0], self.wout, t, None, stat=self._bounds, chain=chain)

    def step(self):
        P, st, b, bm, t = ops.P, self.st, self.builder, self.bm, self.t
        self._health()
        self._fault_stall()
        if self.graph is None and self.use_graph and t >= self.t_start + 1:
            self._try_capture()
        if self.graph is not None:
            if self.graph.group > 1:
                # consecutive steps replay as one G-tree graph (no inter-graph gap
                # between them); readers of the margins / trees flush() first
                self.deferred.append(t)
                if len(self.deferred) == self.graph.group:
                    self.graph.replay_group(self.deferred[0])
                    self.deferred = []
            else:
                self.graph.replay(t)
            self.t += 1
            return
        fmask = _tree_fmask(self.tp, bm.F, t, self.dev)
        if self.K == 1 and self.fused:
            gp = make_grad_params(self.dist, False, 1.0, self.seed, t, row_base=b.row_base, **self.kw)
            gf = dict(F=st.Fm[0], y=st.y, apply=self.pending, gp=gp, bounds=self._bounds)
            b.build(st.g[0], st.h[0], None, t, fmask, grad_fuse=gf)
            self.pending = True
            self.trees_dev.append(self._snapshot())
            self._snap_cat()
        elif self.K == 1:
            fresh = self.cap <= self.COMPACT_CAP
            if fresh:
                # grow the tree straight into its own buffer (no copy afterwards);
                # the next boost_update applies it from there
                b.tree_buf = torch.empty_like(b.tree_buf)
            b.build(st.g[0], st.h[0], self.wout, t, fmask, stat=self._bounds)
            self.trees_dev.append(b.tree_buf if fresh else self._snapshot())
            self._snap_cat()
            self._oob(t, 0)
            self._update(apply=True, next_tree=t + 1, k=0)
        else:
            s = ops.stream(self.dev)
            gp = make_grad_params("bernoulli", False, self.sample_rate, self.seed, t,
                                  row_base=self.builder.row_base, **self.kw)
            # all classes' gradients from the margins at the start of the iteration;
            # per-class maxima are kept for the per-class quantisation scales
            maxes = []
            for k in range(self.K):
                if self.dist == "drf":
                    self._update(apply=False, next_tree=t, k=k)
                else:
                    ops.check(self.lib.h2omx_softmax_grad(P(st.Fm), self.K, st.Fm.stride(0), P(st.yk), P(st.w),
                                                          bm.n, bm.npad, k, ctypes.addressof(gp), P(b.nid),
                                                          P(st.g[k]), P(st.h[k]), P(self.wout), P(b.stat_slab), s),
                                  "softmax_grad")
                    b.reduce_stats()
                maxes.append(b.stat_max.clone())
            for k in range(self.K):
                b.nid[: bm.n].zero_()
                b.stat_max.copy_(maxes[k])
                b.build(st.g[k], st.h[k], self.wout, t * self.K + k, fmask)
                self.trees_dev.append(self._snapshot())
                self._snap_cat()
                self._oob(t, k)
                ops.check(self.lib.h2omx_apply_tree(P(st.Fm[k]), bm.n, P(b.nid), P(b.tree_buf), s), "apply_tree")
        self.t += 1

    COMPACT_CAP = 8191   # deeper trees: copy only the nodes actually created

    def _oob(self, t: int, k: int):
        """Add tree (t, k) to the out-of-bag sums of the rows its bag left out
        (bag hash of iteration t, as boost_update / softmax_grad draw it)."""
        if self.oob is None:
            return
        b = self.builder
        ops.check(self.lib.h2omx_oob_accumulate(ops.P(self.oob[0][k]), ops.P(self.oob[1]), self.bm.n, ops.P(b.nid),
                                                ops.P(b.tree_buf), ops.P(self.st.w), self.seed & 0xFFFFFFFF, t,
                                                self.sample_rate, b.row_base, 1 if k == 0 else 0,
                                                ops.stream(self.dev)), "oob_accumulate")

    def _try_capture(self):
        b = self.builder
        try:
            g = TreeGraph(self)
            g.capture()
        except Exception as e:   # capture unsupported here: keep stepping eagerly
            b.tree_ctr = None
            self.use_graph = False
            self.graph_error = f"{type(e).__name__}: {e}"
            import warnings

            warnings.warn(f"h2omx: tree step graph capture failed, running eagerly ({self.graph_error})")
            return
        self.graph = g
        self.graph_used = True
        self.graph_chain = g.chain

    def _snap_cat(self) -> None:
        """Copy of the finished tree's categorical bitsets (nodes of the tree only)."""
        b = self.builder
        if b.treecat is None:
            return
        if self.cap <= self.COMPACT_CAP:
            self.cats_dev.append(b.treecat.clone())
        else:
            total = max(1, int(b.tree_size()))
            self.cats_dev.append(b.treecat[: total * 8].clone())

    def _snapshot(self) -> torch.Tensor:
        """Copy of the finished tree.  Shallow trees copy the whole capacity-sized
        heap without a host sync; deep trees (DRF depth 20: 2^21 slots, 64 MB)
        read the node count and copy only the used prefix."""
        b = self.builder
        if self.cap <= self.COMPACT_CAP:
            return b.tree_buf.clone()
        total = max(1, int(b.tree_size()))
        snap = b.tree_buf[: total * TREE_NODE_DTYPE.itemsize].clone()
        self._download(len(self.trees_dev), snap)
        return snap

    # deep trees: each snapshot is downloaded by a helper thread on its own stream
    # while the next tree builds (a 10-tree DRF depth-20 forest is ~190 MB: the
    # staged copy at finish() cost ~17 ms a fit), straight into the row of a
    # zero-initialised host array (calloc'd: untouched pages stay unmapped)
    ntrees_hint = None
    ASYNC_DOWNLOAD = True

    def _download(self, i: int, snap: torch.Tensor) -> None:
        dl = getattr(self, "_dl", None)
        if dl is None:
            if not (self.ASYNC_DOWNLOAD and self.ntrees_hint and self.dev.type == "cuda"):
                self._dl = False
                return
            import queue
            import threading

            host = np.zeros((int(self.ntrees_hint) * self.K, self.cap * TREE_NODE_DTYPE.itemsize), np.uint8)
            q: queue.Queue = queue.Queue()
            state = {"host": host, "q": q, "err": None, "n": 0}

            def run():
                side = torch.cuda.Stream(self.dev)
                while True:
                    item = q.get()
                    if item is None:
                        return
                    j, src, ev = item
                    try:
                        with torch.cuda.stream(side):
                            side.wait_event(ev)
                            torch.from_numpy(host[j, : src.numel()]).copy_(src)
                    except Exception as e:   # reported (and the forest downloaded again) by finish()
                        state["err"] = e

            state["thread"] = threading.Thread(target=run, name="h2omx-tree-download", daemon=True)
            state["thread"].start()
            self._dl = dl = state
        if dl is False:
            return
        if i >= dl["host"].shape[0]:
            dl["err"] = IndexError("more trees than ntrees_hint")
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        dl["q"].put((i, snap, ev))
        dl["n"] += 1

    def _downloaded(self, width: int):
        """The host forest [ntrees][width] bytes from the helper thread (None:
        not used or failed - finish() copies the device forest)."""
        dl = getattr(self, "_dl", None)
        if not dl:
            return None
        dl["q"].put(None)
        dl["thread"].join()
        self._dl = None
        if dl["err"] is not None or dl["n"] != len(self.trees_dev):
            return None
        return dl["host"][: len(self.trees_dev), :width]

    def finish(self) -> TreeEnsemble:
        self.flush()
        if self.graph is not None:
            # trees out of the ring, then drop the graph: booster <-> TreeGraph is
            # a reference cycle, and a graph freed later by the cyclic collector
            # could land inside another capture
            self.graph.freeze()
            self.graph.gb = None
            self.graph = None
        torch.cuda.synchronize(self.dev)
        self._health()     # every exchange of the fit has completed: a timeout raises here
        if self.builder.timer.enabled:
            self.ens.timings.update({f"gpu_ms_{k}": v for k, v in self.builder.timer.totals().items()})
        if self.trees_dev:
            width = max(t.numel() for t in self.trees_dev)
            if all(t.numel() == width for t in self.trees_dev):
                raw = torch.stack(self.trees_dev)
            else:   # compact snapshots: pad to the largest tree with unreachable zero nodes
                raw = torch.zeros((len(self.trees_dev), width), dtype=torch.uint8, device=self.dev)
                for i, t in enumerate(self.trees_dev):
                    raw[i, : t.numel()] = t
            host = self._downloaded(width)
            if host is None:
                host = raw.cpu().numpy()
            self.ens.trees = trees_from_bytes(host, width // TREE_NODE_DTYPE.itemsize)
            if self.cats_dev:
                self.ens.catbits = _stack_cats(self.cats_dev, width // TREE_NODE_DTYPE.itemsize)
            else:
                # the device node array raw_margin would rebuild from ens.trees (a copy
                # and an upload of the whole forest: ~0.1 s for a 50-tree depth-20 DRF,
                # paid by every cross-validation holdout prediction) is this one
                e = self.ens
                key = (e.ntrees * e.K, str(self.dev), e.trees.shape, id(e.trees), id(e.catbits))
                e._dev_nodes = (key, raw.reshape(-1), None)
        self.ens._state = self.st
        if self.oob is not None:
            self.ens._oob = (self.oob[0][:, : self.bm.n], self.oob[1][: self.bm.n])
        return self.ens


def _train_gpu(bm, y_np, w_np, ens, ntrees, tp, sample_rate, seed, comm, callback, dist_kw, tree_offset=0):
    t0 = time.perf_counter()
    gb = GpuBooster(bm, y_np, w_np, ens, tp, sample_rate, seed, comm, dist_kw, tree_offset=tree_offset)
    gb.ntrees_hint = ntrees
    lr0, ann = tp.learn_rate, tp.learn_rate_annealing
    for t in range(ntrees):
        if ann != 1.0:
            gb.builder.p.learn_rate = lr0 * ann ** (tree_offset + t)
        gb.step()
        if callback is not None and callback(t, _GpuView(gb)) is True:
            break
    gb.finish()
    gb.builder.p.learn_rate = lr0
    ens.timings["train_s"] = time.perf_counter() - t0


def _stack_cats(cats: list, width_nodes: int) -> np.ndarray:
    """[n_trees][width_nodes][8] uint32 from per-tree device bitset snapshots."""
    out = np.zeros((len(cats), width_nodes, 8), np.uint32)
    for i, c in enumerate(cats):
        a = c.cpu().numpy().view(np.uint32).reshape(-1, 8)
        out[i, : a.shape[0]] = a[:width_nodes]
    return out


class _GpuView:
    """What a training callback sees (scoring / early stopping / cancel)."""

    def __init__(self, gb):
        self.gb = gb
        self.init_f = gb.ens.init_f

    @property
    def margin(self) -> torch.Tensor:
        self.gb.flush()
        return self.gb.st.Fm[:, : self.gb.bm.n]

    def trees(self, lo: int, hi: int) -> np.ndarray:
        """Tree records of iterations [lo, hi) (K trees each)."""
        self.gb.flush()
        K = self.gb.K
        if self.gb.graph is not None:
            self.gb.graph.freeze()
        bufs = self.gb.trees_dev[lo * K: hi * K]
        if not bufs:
            return np.zeros((0, self.gb.cap), TREE_NODE_DTYPE)
        width = max(t.numel() for t in bufs)
        raw = torch.zeros((len(bufs), width), dtype=torch.uint8, device=bufs[0].device)
        for i, t in enumerate(bufs):
            raw[i, : t.numel()] = t
        return trees_from_bytes(raw.cpu().numpy(), width // TREE_NODE_DTYPE.itemsize)

    def catbits(self, lo: int, hi: int) -> np.ndarray | None:
        """Categorical bitsets of iterations [lo, hi) aligned with trees(lo, hi)."""
        K = self.gb.K
        cats = self.gb.cats_dev[lo * K: hi * K]
        if not cats:
            return None
        width = max(t.numel() for t in self.gb.trees_dev[lo * K: hi * K]) // TREE_NODE_DTYPE.itemsize
        return _stack_cats(cats, width)



def _tree_fmask(tp: TreeParams, F: int, t: int, dev):
    if tp.col_sample_rate_per_tree >= 1.0:
        return None
    from .hashing import hash4, u01

    hs = hash4(tp.seed & 0xFFFFFFFF, 0xC0FFEE, t, np.arange(F))
    m = (u01(hs) < tp.col_sample_rate_per_tree).astype(np.uint8)
    if m.sum() == 0:
        m[int(np.argmin(hs))] = 1
    return torch.from_numpy(m).to(dev) if dev is not None else m


class TreeGraph:
    """HIP-graph replay of one boosting step (K == 1): tree_begin -> per level
    {hist_build, hist_reduce, [all-reduce], split_find, level_finalize,
    partition} -> leaf_finalize -> boost_update, i.e. ~30 launches that the
    host otherwise enqueues one ctypes call at a time.

    The only per-tree host input of the sequence is the tree index (dither
    salt); replays take it from ``builder.tree_ctr``, which tree_begin reads
    and advances on the device, so replayed trees are bit-identical to eager
    ones.  Buffers are the builder's fixed ones (allocated by the first, eager
    step) and the tree is grown in place in ``builder.tree_buf``; the caller
    snapshots it after every replay.

    Multi-rank: with the one-shot P2P all-reduce (``parallel/p2p.py``, on by
    default when peer memory maps) the collectives are kernels of the step, so
    the whole N-rank step is ONE graph replay with no host-issued collective.
    Otherwise the step is captured in SEGMENTS split at the collectives, which
    are issued eagerly between segment replays (works with any backend; a Comm
    whose ``graph_collectives`` is set has them captured inside one graph).
    """

    # finished trees go to a device ring of RING slots inside the graph
    # (tree_archive kernel); trees_dev holds views of the live ring until
    # freeze() swaps them for views of one ring snapshot (every RING trees, and
    # whenever the trees are read)
    RING = 64
    GROUP = 4      # trees per replay of the multi-tree graph

    def __init__(self, booster):
        self.gb = booster
        self.comm = booster.builder.comm
        self.graphs: list = []
        self.colls: list = []
        self.pool = None
        self.ring = None
        self.live: list = []      # (trees_dev index, ring slot) still pointing into the ring
        self.expect = None        # tree index the device counter holds
        self.chain = False        # tree_begin folded into the previous step (see capture)
        # chained single-graph steps: GROUP consecutive trees per replay
        self.group = 1
        self.graph_g = None

    def capture(self):
        gb, b = self.gb, self.gb.builder
        dev = gb.dev
        b.tree_ctr = torch.zeros((1,), dtype=torch.int32, device=dev)
        # the graph's own tree buffer: eager steps hand their tree_buf to trees_dev
        # (fresh buffers), which replays must not overwrite
        b.tree_buf = torch.zeros_like(b.tree_buf)
        self.ring = torch.zeros((self.RING, b.tree_buf.numel()), dtype=torch.uint8, device=dev)
        multi = self.comm is not None and self.comm.world_size > 1
        # P2P collectives are ordinary kernels: the whole step is one graph.  RCCL
        # calls become segment boundaries
        segmented = multi and not getattr(self.comm, "graph_collectives", False)
        self.pool = torch.cuda.graph_pool_handle()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.synchronize(dev)
        # no garbage collection while capturing: a collected graph / event / pool
        # of an earlier model would be destroyed inside the capture (illegal while
        # a stream captures).  (No gc.collect() up front: in a large process it
        # costs tens of ms per fit; reference-counted frees of tensors from the
        # regular pool are safe during capture.)
        gc_was = gc.isenabled()
        gc.disable()
        # tree_begin of the next tree runs inside this tree's leaf finalisation
        # (fixed gradient bounds), the tree archive inside boost_update: the
        # replayed step is levels -> leaf_finalize(+begin) -> boost_update(+archive)
        self.chain = b.can_chain(gb._bounds is not None)
        b.pk_in_boost = self.chain and b.can_pack_in_boost()
        b.regrad = None
        if b.pk_in_boost and gb.wout is None and gb.K == 1:
            # the final partition re-derives (g, h) from the margins: boost_update
            # stores only the packed rows (8 bytes per row less each way)
            gpr = make_grad_params(gb.dist, False, 1.0, gb.seed, 0, row_base=b.row_base, **gb.kw)
            b.regrad = (gb.st.Fm[0], gb.st.y, gpr, gb.y8)
        try:
            with torch.cuda.stream(side):
                g = torch.cuda.CUDAGraph()
                g.capture_begin(pool=self.pool)
                self._open = g
                if segmented:
                    b.comm = _SegmentComm(self, self.comm)
                # archive slot: tree_ctr - 1 after this tree's begin, - 2 once the
                # leaf finalisation has begun the next tree
                gb._archive = (self.ring, self.RING, 2 if self.chain else 1)
                try:
                    gb._body_k1(gb.t, fresh=False, chain=self.chain)
                    gb._update(apply=True, next_tree=gb.t + 1, k=0)
                finally:
                    gb._archive = None
                    b.comm = self.comm
                    self._open.capture_end()
                    self.graphs.append(self._open)
                    self._open = None
                group = self.GROUP
                if self.chain and not segmented and group > 1:
                    # the same step G times in one graph: the chained step's only
                    # state hand-off is on the device (tree counter, scales, leaf sums)
                    g = torch.cuda.CUDAGraph()
                    g.capture_begin(pool=self.pool)
                    gb._archive = (self.ring, self.RING, 2)
                    try:
                        for _ in range(group):
                            gb._body_k1(gb.t, fresh=False, chain=True)
                            gb._update(apply=True, next_tree=gb.t + 1, k=0)
                    finally:
                        gb._archive = None
                        g.capture_end()
                    self.graph_g, self.group = g, group
        finally:
            if gc_was:
                gc.enable()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)

    def _cut(self, t, op):
        """segment boundary at a collective: close the open graph, remember the
        collective, open the next graph"""
        self._open.capture_end()
        self.graphs.append(self._open)
        self.colls.append((t, op))
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self.pool)
        self._open = g

    def replay(self, t: int):
        """Grow tree ``t`` (and update margins / gradients for tree t + 1)."""
        if self.expect != t:   # tree_begin advances the counter: set only when out of step
            b = self.gb.builder
            b.tree_ctr.fill_(t & 0x7FFFFFFF)
            if self.chain:     # the graph starts at level 0: begin this tree here
                self._begin_eager(t)
        self.expect = t + 1
        if len(self.live) >= self.RING:
            self.freeze()
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.colls):
                buf, op = self.colls[i]
                self.comm.all_reduce_(buf, op)
        slot = (t & 0x7FFFFFFF) % self.RING
        self.live.append((len(self.gb.trees_dev), slot))
        self.gb.trees_dev.append(self.ring[slot])

    def _begin_eager(self, t: int):
        """Out of step (first replay, or after eager steps): begin tree t here and,
        when level 0 reads boost_update's packed rows, re-derive them from the
        current margins (same gradients, this tree's scales and dither salt)."""
        gb, b = self.gb, self.gb.builder
        b.begin(gb._bounds, t)
        if b.pk_in_boost:
            gb._update(apply=False, next_tree=t, k=0, pack=True)

    def replay_group(self, t: int):
        """Grow trees t .. t + group - 1 with one replay of the multi-tree graph."""
        if self.expect != t:
            self.gb.builder.tree_ctr.fill_(t & 0x7FFFFFFF)
            self._begin_eager(t)
        self.expect = t + self.group
        if len(self.live) + self.group > self.RING:
            self.freeze()
        self.graph_g.replay()
        for u in range(t, t + self.group):
            slot = (u & 0x7FFFFFFF) % self.RING
            self.live.append((len(self.gb.trees_dev), slot))
            self.gb.trees_dev.append(self.ring[slot])

    def freeze(self):
        """Point the trees still living in the ring at one copy of their slots
        (only the live ones: scoring reads the trees every few replays)."""
        if self.live:
            slots = torch.tensor([slot for _, slot in self.live], dtype=torch.int64, device=self.ring.device)
            snap = self.ring.index_select(0, slots)
            for j, (i, _) in enumerate(self.live):
                self.gb.trees_dev[i] = snap[j]
            self.live = []


class _SegmentComm:
    """Stand-in for the builder's Comm while a segmented TreeGraph is captured:
    every collective becomes a segment boundary instead of a captured call."""

    def __init__(self, graph: TreeGraph, comm):
        self._graph, self._comm = graph, comm
        self.world_size, self.rank, self.device = comm.world_size, comm.rank, comm.device

    def all_reduce_(self, t, op: str = "sum"):
        self._graph._cut(t, op)
        return t

