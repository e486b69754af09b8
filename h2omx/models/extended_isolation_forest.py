"""Extended Isolation Forest (H2O ``H2OExtendedIsolationForestEstimator``;
Hariri, Kind & Brunner 2018).

Each tree isolates ``sample_size`` rows with random hyperplanes: at a node
the normal vector n ~ N(0, I) keeps ``extension_level + 1`` random non-zero
coordinates (0 = axis-parallel, the classic forest) and the intercept point
is uniform in the node's bounding box; rows with (x − q)·n ≤ 0 go left.
Trees grow to depth ceil(log2(sample_size)).

Training samples are drawn per rank (its share of the global sample, seeded
by (seed, tree, rank)) and all-gathered once, so every rank builds the same
small trees on the host.  Scoring is GEMM-shaped: the hyperplane offsets of
every node of a block of trees are ONE fp32 matrix-core product X·Nᵀ
(ops.dense.gemm) per row block, after which rows walk their trees with
gathers.  Path length = depth + c(leaf size); outputs ``anomaly_score`` =
2^(−E[h(x)] / c(sample_size)) and ``mean_length`` = E[h(x)].
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import Frame, Vec
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo
from .isolation_forest import avg_path


def _build_tree(S: np.ndarray, limit: int, ext: int, rng: np.random.Generator, cap: int):
    """Heap-indexed tree over sample S [m][p]: normals [cap][p], offsets [cap], leaf size [cap] (-1 inner)."""
    m, p = S.shape
    normals = np.zeros((cap, p), np.float32)
    offs = np.zeros(cap, np.float32)
    size = np.full(cap, -1.0, np.float32)
    stack = [(0, np.arange(m), 0)]
    while stack:
        node, idx, depth = stack.pop()
        if depth >= limit or idx.size <= 1:
            size[node] = idx.size
            continue
        pts = S[idx]
        lo, hi = pts.min(0), pts.max(0)
        live = np.nonzero(hi > lo)[0]
        if live.size == 0:
            size[node] = idx.size
            continue
        n = np.zeros(p, np.float64)
        k = min(ext + 1, live.size)
        dims = rng.choice(live, size=k, replace=False)
        n[dims] = rng.normal(size=k)
        q = lo + rng.random(p) * (hi - lo)
        b = float(n @ q)
        proj = pts @ n
        left = idx[proj <= b]
        right = idx[proj > b]
        normals[node] = n
        offs[node] = b
        stack.append((2 * node + 1, left, depth + 1))
        stack.append((2 * node + 2, right, depth + 1))
    return normals, offs, size


class ExtendedIsolationForestModel(Model):
    algo = "extendedisolationforest"
    algo_full_name = "Extended Isolation Forest"

    def __init__(self, builder, model_id, design, normals, offs, sizes, limit, sample_size):
        super().__init__(builder, model_id)
        self.design = design
        self.normals = normals      # [T][cap][p]
        self.offs = offs            # [T][cap]
        self.sizes = sizes          # [T][cap] leaf sizes, -1 inner
        self.limit = limit
        self.sample_size = sample_size

    def mean_length(self, frame: Frame, block: int = 8192, tree_block: int = 32) -> torch.Tensor:
        Xraw = self.design.raw_matrix(frame)
        dev = Xraw.device
        m = torch.from_numpy(self.design.means.astype(np.float32)).to(dev)[:, None]
        X = torch.where(torch.isnan(Xraw), m.expand_as(Xraw), Xraw).T.contiguous()    # [n][p]
        T, cap, p = self.normals.shape
        n = X.shape[0]
        cpath = torch.from_numpy(np.where(self.sizes >= 0, avg_path(np.maximum(self.sizes, 0)), 0.0)
                                 .astype(np.float32)).to(dev)                         # [T][cap]
        depth_of = torch.floor(torch.log2(torch.arange(cap, device=dev, dtype=torch.float32) + 1))
        is_leaf = torch.from_numpy(self.sizes >= 0).to(dev)
        offs = torch.from_numpy(self.offs).to(dev)
        total = torch.zeros(n, dtype=torch.float32, device=dev)
        for t0 in range(0, T, tree_block):
            t1 = min(T, t0 + tree_block)
            Nb = torch.from_numpy(self.normals[t0:t1].reshape(-1, p)).to(dev)          # [(t1-t0)*cap][p]
            for r0 in range(0, n, block):
                r1 = min(n, r0 + block)
                P = D.gemm(X[r0:r1], Nb, tb=True).view(r1 - r0, t1 - t0, cap)        # x . n per node
                node = torch.zeros((r1 - r0, t1 - t0), dtype=torch.long, device=dev)
                tid = torch.arange(t0, t1, device=dev)[None, :].expand_as(node)
                for _ in range(self.limit):
                    leaf = is_leaf[tid, node]
                    proj = P.gather(2, node[..., None]).squeeze(-1)
                    go = (proj > offs[tid, node]).long()
                    node = torch.where(leaf, node, 2 * node + 1 + go)
                h = depth_of[node] + cpath[tid, node]
                total[r0:r1] += h.sum(1)
        return total / T

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        ml = self.mean_length(frame)
        c = float(avg_path(np.array([self.sample_size]))[0]) or 1.0
        score = torch.pow(2.0, -ml / c)
        return torch.stack([score, ml])

    def predict(self, frame: Frame) -> Frame:
        P = self.predict_raw(frame)
        return Frame([Vec("anomaly_score", P[0].float(), "real"), Vec("mean_length", P[1].float(), "real")])

    def model_performance(self, frame=None):
        return self.training_metrics

    def summary(self):
        return {"model_id": self.model_id, "ntrees": int(self.normals.shape[0]), "sample_size": self.sample_size,
                "extension_level": int(self.params["extension_level"])}


class H2OExtendedIsolationForestEstimator(ModelBuilder):
    algo = "extendedisolationforest"
    UNSUPERVISED_CATEGORY = ModelCategory.ANOMALY
    DEFAULTS = dict(ntrees=100, sample_size=256, extension_level=0, disable_training_metrics=True,
                    categorical_encoding="AUTO")

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        return super().train(x=x, y=None, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        comm = self.comm
        world = comm.world_size if comm is not None else 1
        rank = comm.rank if comm is not None else 0
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, use_all_levels=True)
        Xraw = design.raw_matrix(train)
        design.fit_standardization(Xraw, False, comm)
        m = torch.from_numpy(design.means.astype(np.float32)).to(Xraw.device)[:, None]
        X = torch.where(torch.isnan(Xraw), m.expand_as(Xraw), Xraw).T.contiguous()    # [n][p]
        n, p = X.shape
        ext = int(p_["extension_level"])
        if not 0 <= ext <= max(p - 1, 0):
            raise ValueError(f"extendedisolationforest: extension_level must be in [0, {p - 1}]")
        T = int(p_["ntrees"])
        counts = np.array([float(n)]) if world == 1 else comm.all_gather_cat(
            torch.tensor([float(n)], dtype=torch.float64, device=X.device)).cpu().numpy()
        N = float(counts.sum())
        psi = int(min(int(p_["sample_size"]), N))
        if psi < 2:
            raise ValueError("extendedisolationforest: needs at least 2 rows")
        seed = self._seed()
        # this rank's share of every tree's sample (deterministic in (seed, tree, rank))
        share = int(round(psi * n / N)) if world > 1 else psi
        g = torch.Generator().manual_seed(seed * 1000003 + rank)
        idx = torch.stack([torch.randperm(n, generator=g)[:share] for _ in range(T)]) if share > 0 else \
            torch.zeros((T, 0), dtype=torch.long)
        samp = X[idx.flatten().to(X.device)].view(T, -1, p)
        if world > 1:
            samp = comm.all_gather_cat(samp.transpose(0, 1).contiguous()).transpose(0, 1)
        samp = samp.double().cpu().numpy()
        limit = int(math.ceil(math.log2(max(psi, 2))))
        cap = (1 << (limit + 1)) - 1
        rng = np.random.default_rng(seed)
        normals = np.zeros((T, cap, p), np.float32)
        offs = np.zeros((T, cap), np.float32)
        sizes = np.zeros((T, cap), np.float32)
        for t in range(T):
            normals[t], offs[t], sizes[t] = _build_tree(samp[t], limit, ext, rng, cap)
        model = ExtendedIsolationForestModel(self, model_id, design, normals, offs, sizes, limit, psi)
        if not p_["disable_training_metrics"]:
            ml = model.mean_length(train)
            model.training_metrics = {"mean_length": float(ml.mean()), "nobs": N}
        else:
            model.training_metrics = {"nobs": N}
        return model
