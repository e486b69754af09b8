"""Isolation Forest (H2O IsolationForest equivalent).

Each tree isolates a random subsample of ``sample_size`` rows (or
``sample_rate`` × rows) with random axis-aligned splits: at every node a
feature is drawn uniformly among the node's non-constant features and the
split point uniformly between the node's min and max of that feature.  A
leaf at depth e holding m sample rows has path length e + c(m), where
c(m) = 2 H(m-1) - 2 (m-1)/m is the average unsuccessful-search length of a
BST (Liu et al., 2008).

Distributed, device-resident construction: every rank samples its own
rows (its share of the global sample), trees grow level by level, and a
level needs only the per-node feature minima / maxima / counts of the
sampled rows (scatter reductions on the device, one all-reduce per level
across ranks).  Split choices come from a host RNG seeded by (seed, tree),
so every rank builds the same trees without exchanging rows.  Trees use
the shared tree-node heap, so scoring runs the GPU ensemble kernel
(csrc/tree_kernels.hip predict_raw_kernel) and MOJO export reuses the tree
codec.

Outputs per row (H2O): ``predict`` = normalised score
(max_len - len) / (max_len - min_len) with the min / max mean path length
seen on the training data (higher = more anomalous), ``mean_length`` =
mean path length over the trees.  With ``contamination`` in (0, 0.5],
``predict`` is the 0/1 label at that training quantile and ``score`` holds
the normalised score.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import Frame, Vec
from .base import Model, ModelBuilder, ModelCategory
from .tree.boost import TreeEnsemble
from .tree.structs import TREE_NODE_DTYPE

EULER = 0.5772156649015329


def avg_path(m) -> np.ndarray:
    """c(m): average path length of an unsuccessful BST search over m points."""
    m = np.asarray(m, np.float64)
    out = np.zeros_like(m)
    big = m > 2
    out[m == 2] = 1.0
    mb = m[big]
    out[big] = 2.0 * (np.log(mb - 1.0) + EULER) - 2.0 * (mb - 1.0) / mb
    return out


class IsolationForestModel(Model):
    algo = "isolationforest"
    algo_full_name = "Isolation Forest"

    def __init__(self, builder, model_id, ens, sample_size):
        super().__init__(builder, model_id)
        self.ens = ens
        self.sample_size = sample_size
        self.min_path_length = 0.0
        self.max_path_length = 1.0
        self.threshold = None

    def mean_length(self, frame: Frame) -> torch.Tensor:
        X = frame.feature_matrix(self.x)
        return self.ens.raw_margin(X)[0].to(X.device)

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        L = self.mean_length(frame)
        span = max(self.max_path_length - self.min_path_length, 1e-12)
        score = (self.max_path_length - L) / span
        return torch.stack([score, L])

    def predict(self, frame: Frame) -> Frame:
        S = self.predict_raw(frame)
        if self.threshold is not None:
            lab = (S[0] >= self.threshold).to(torch.int32)
            return Frame([Vec("predict", lab, "int"), Vec("score", S[0].float(), "real"),
                          Vec("mean_length", S[1].float(), "real")])
        return Frame([Vec("predict", S[0].float(), "real"), Vec("mean_length", S[1].float(), "real")])

    def anomaly_score(self, frame: Frame) -> torch.Tensor:
        """Liu et al. score 2^(-E[h] / c(psi)) in (0, 1]."""
        c = float(avg_path([self.sample_size])[0]) or 1.0
        return torch.pow(2.0, -self.mean_length(frame) / c)

    def model_performance(self, frame: Frame | None = None):
        if frame is None:
            return self.training_metrics
        S = self.predict_raw(frame)
        return {"mean_score": float(S[1].double().mean()), "mean_normalized_score": float(S[0].double().mean())}

    def summary(self):
        d = [int(_depth(t)) for t in self.ens.trees]
        return {"model_id": self.model_id, "number_of_trees": int(self.ens.trees.shape[0]),
                "min_depth": min(d) if d else 0, "max_depth": max(d) if d else 0,
                "mean_depth": float(np.mean(d)) if d else 0.0}

    def to_json(self):
        j = super().to_json()
        j["output"]["min_path_length"] = self.min_path_length
        j["output"]["max_path_length"] = self.max_path_length
        return j


def _depth(tree) -> int:
    best, stack = 0, [(0, 0)]
    while stack:
        i, d = stack.pop()
        if tree[i]["feat"] >= 0:
            stack += [(int(tree[i]["left"]), d + 1), (int(tree[i]["left"]) + 1, d + 1)]
        else:
            best = max(best, d)
    return best


class H2OIsolationForestEstimator(ModelBuilder):
    algo = "isolationforest"
    UNSUPERVISED_CATEGORY = ModelCategory.ANOMALY
    DEFAULTS = dict(ntrees=50, max_depth=8, sample_size=256, sample_rate=-1.0, mtries=-1, min_rows=1.0,
                    col_sample_rate_per_tree=1.0, contamination=-1.0, categorical_encoding="AUTO",
                    score_each_iteration=False, score_tree_interval=0, stopping_rounds=0, stopping_metric="AUTO",
                    stopping_tolerance=0.01, validation_response_column=None)

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        return super().train(x=x, y=None, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        comm = self.comm if (self.comm is not None and self.comm.world_size > 1) else None
        X = train.feature_matrix(self.x)                 # [F][n] float32, NaN = missing
        F, n = X.shape
        dev = X.device
        rank = comm.rank if comm else 0
        counts = torch.tensor([float(n)], dtype=torch.float64, device=dev)
        if comm:
            all_n = comm.all_gather_cat(counts).cpu().numpy()
        else:
            all_n = counts.cpu().numpy()
        N = float(all_n.sum())
        sr = float(p_["sample_rate"])
        psi = int(round(sr * N)) if sr > 0 else min(int(p_["sample_size"]), int(N))
        psi = max(psi, 2)
        D = int(p_["max_depth"]) if int(p_["max_depth"]) > 0 else int(math.ceil(math.log2(psi)))
        D = min(D, 30)
        cap = (1 << (D + 1)) - 1
        ntrees = int(p_["ntrees"])
        seed = self._seed()
        # this rank's share of every tree's global sample (largest remainder)
        share = psi * all_n / max(N, 1.0)
        base = np.floor(share).astype(np.int64)
        extra = int(psi - base.sum())
        order = np.argsort(-(share - base), kind="stable")
        base[order[:extra]] += 1
        m_local = int(base[rank])
        min_rows = float(p_["min_rows"])
        mtries = int(p_["mtries"])
        colrate = float(p_["col_sample_rate_per_tree"])
        trees = np.zeros((ntrees, cap), TREE_NODE_DTYPE)
        trees["feat"] = -1
        gen = torch.Generator(device="cpu")
        for t in range(ntrees):
            rng = np.random.default_rng([seed & 0x7FFFFFFF, t])
            gen.manual_seed((seed * 1_000_003 + 7919 * t + 104729 * rank) & 0x7FFFFFFFFFFF)
            idx = torch.randperm(n, generator=gen)[:m_local].to(dev) if m_local > 0 else \
                torch.zeros(0, dtype=torch.long, device=dev)
            feats = np.arange(F)
            if colrate < 1.0:
                feats = np.sort(rng.choice(F, max(1, int(round(colrate * F))), replace=False))
            trees[t] = self._grow(X[:, idx], feats, rng, D, cap, min_rows, mtries, comm)
        ens = TreeEnsemble(trees=trees, K=1, dist="isolation", init_f=np.zeros(1), average=True,
                           feature_names=list(self.x))
        model = IsolationForestModel(self, model_id, ens, psi)
        L = model.mean_length(train)
        stats = torch.stack([L.double().min(), -L.double().max(), L.double().sum()])
        if comm:
            mm = torch.stack([stats[0], stats[1]])
            comm.all_reduce_(mm, "min")
            s = stats[2:].clone()
            comm.all_reduce_(s)
            stats = torch.cat([mm, s])
        model.min_path_length = float(stats[0])
        model.max_path_length = float(-stats[1])
        cont = float(p_["contamination"])
        S = model.predict_raw(train)
        if 0.0 < cont <= 0.5:
            sc = S[0].double()
            if comm:
                sc = comm.all_gather_cat(sc)
            model.threshold = float(torch.quantile(sc.float().cpu(), 1.0 - cont))
        tot = torch.stack([S[1].double().sum(), S[0].double().sum()])
        if comm:
            comm.all_reduce_(tot)
        model.training_metrics = {"mean_score": float(tot[0]) / N, "mean_normalized_score": float(tot[1]) / N,
                                  "nobs": N}
        return model

    @staticmethod
    def _grow(Xs, feats, rng, D, cap, min_rows, mtries, comm):
        """One tree on this rank's sample Xs [F][m] (possibly empty)."""
        F, m = Xs.shape
        dev = Xs.device
        tree = np.zeros(cap, TREE_NODE_DTYPE)
        tree["feat"] = -1
        node = torch.zeros(m, dtype=torch.long, device=dev)     # index into the current level's node list
        level = [0]                                              # heap ids of this level's nodes
        nxt_free = 1
        Xf = torch.nan_to_num(Xs, nan=0.0)
        ok = ~torch.isnan(Xs)
        for d in range(D + 1):
            k = len(level)
            live = node >= 0
            nd = torch.where(live, node, torch.zeros_like(node))
            cnt = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(0, nd, live.double())
            big = torch.tensor(float("inf"), dtype=torch.float32, device=dev)
            valid = ok & live[None, :]
            lo = torch.full((F, k), float("inf"), dtype=torch.float32, device=dev)
            hi = torch.full((F, k), float("-inf"), dtype=torch.float32, device=dev)
            if m:
                idx = nd[None, :].expand(F, m)
                lo.scatter_reduce_(1, idx, torch.where(valid, Xf, big), "amin")
                hi.scatter_reduce_(1, idx, torch.where(valid, Xf, -big), "amax")
            if comm is not None:
                comm.all_reduce_(lo, "min")
                comm.all_reduce_(hi, "max")
                comm.all_reduce_(cnt)
            lo_h, hi_h, cnt_h = lo.cpu().numpy(), hi.cpu().numpy(), cnt.cpu().numpy()
            split_feat = np.full(k, -1, np.int64)
            split_thr = np.zeros(k, np.float32)
            child = np.full(k, -1, np.int64)
            new_level = []
            for j, hid in enumerate(level):
                c = cnt_h[j]
                tree["weight"][hid] = c
                cand = [f for f in feats if hi_h[f, j] > lo_h[f, j]]
                if mtries > 0 and len(cand) > mtries:
                    cand = list(rng.choice(cand, mtries, replace=False))
                if d == D or c <= min_rows or not cand or nxt_free + 2 > cap:
                    tree["value"][hid] = d + float(avg_path([c])[0])
                    continue
                f = int(cand[int(rng.integers(len(cand)))])
                a, b = float(lo_h[f, j]), float(hi_h[f, j])
                thr = np.float32(a + (b - a) * rng.random())
                if thr >= b:            # keep both sides non-empty in float32
                    thr = np.nextafter(np.float32(b), np.float32(a))
                tree["feat"][hid] = f
                tree["thr"][hid] = thr
                tree["left"][hid] = nxt_free
                tree["na_left"][hid] = 1
                split_feat[j], split_thr[j] = f, thr
                child[j] = len(new_level)
                new_level += [nxt_free, nxt_free + 1]
                nxt_free += 2
            if not new_level:
                break
            if m:
                sf = torch.from_numpy(split_feat).to(dev)
                st = torch.from_numpy(split_thr).to(dev)
                ch = torch.from_numpy(child).to(dev)
                f_r = sf[nd]
                inner = live & (f_r >= 0)
                v = Xs[f_r.clamp_min(0), torch.arange(m, device=dev)]
                left = torch.isnan(v) | (v <= st[nd])
                node = torch.where(inner, ch[nd] + (~left).long(), torch.full_like(node, -1))
            level = new_level
        return tree
