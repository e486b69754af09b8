"""Aggregator (H2O ``H2OAggregatorEstimator``): radius-based exemplar
reduction of a large frame (Wilkinson's leader algorithm).

Rows are normalised (``transform``, default NORMALIZE: demean / range), then
streamed in blocks: every row joins the nearest existing exemplar within
radius δ, otherwise it starts a new exemplar (greedy inside the block).  The
block-to-exemplar distances are one fp32 matrix-core GEMM per block
(||x||² − 2 x·e + ||e||², ops.dense.gemm).  δ is adjusted geometrically
until the exemplar count is within ``rel_tol_num_exemplars`` of
``target_num_exemplars`` (or the iteration cap).  Multi-rank: every rank
aggregates its shard with the same δ, the leaders are all-gathered and
re-aggregated once more, counts summed.

The result (``aggregated_frame``) holds the exemplar rows in the original
units plus a ``counts`` column; ``save_mapping_frame`` adds the row →
exemplar mapping (local rows, ``exemplar_assignment``).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import DKV, ENUM, Frame, Vec
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo
from .pca import TRANSFORMS
from .svd import transform_params, transformed


def _leaders(Z: torch.Tensor, delta: float, block: int = 4096):
    """Greedy leader clustering of rows of Z [n][p] -> (leader row ids, assignment [n])."""
    n = Z.shape[0]
    dev = Z.device
    assign = torch.full((n,), -1, dtype=torch.long, device=dev)
    leaders = torch.zeros((0,), dtype=torch.long, device=dev)
    d2 = delta * delta
    for s0 in range(0, n, block):
        s1 = min(n, s0 + block)
        B = Z[s0:s1]
        if leaders.numel():
            E = Z[leaders]
            dist = ((B * B).sum(1, keepdim=True) - 2 * D.gemm(B.contiguous(), E.contiguous(), tb=True)
                    + (E * E).sum(1)[None, :]).clamp_min(0)
            md, arg = dist.min(1)
            hit = md <= d2
            assign[s0:s1] = torch.where(hit, arg, torch.full_like(arg, -1))
        rest = torch.nonzero(assign[s0:s1] < 0).flatten()
        while rest.numel():
            lead = rest[0]
            dd = ((B[rest] - B[lead]) ** 2).sum(1)
            mine = rest[dd <= d2]
            li = leaders.numel()
            leaders = torch.cat([leaders, (s0 + lead).reshape(1)])
            assign[s0 + mine] = li
            rest = rest[dd > d2]
    return leaders, assign


class AggregatorModel(Model):
    algo = "aggregator"
    algo_full_name = "Aggregator"

    def __init__(self, builder, model_id, frame_key, mapping_key, delta):
        super().__init__(builder, model_id)
        self.aggregated_frame_key = frame_key
        self.mapping_frame_key = mapping_key
        self.radius = delta

    @property
    def aggregated_frame(self) -> Frame:
        return DKV.get(self.aggregated_frame_key)

    def predict_raw(self, frame):
        raise ValueError("aggregator models do not score frames; use aggregated_frame")

    def model_performance(self, frame=None):
        return self.training_metrics

    def to_json(self):
        j = super().to_json()
        j["output"]["output_frame"] = {"name": self.aggregated_frame_key}
        j["output"]["mapping_frame"] = {"name": self.mapping_frame_key} if self.mapping_frame_key else None
        return j


class H2OAggregatorEstimator(ModelBuilder):
    algo = "aggregator"
    UNSUPERVISED_CATEGORY = ModelCategory.DIMREDUCTION
    DEFAULTS = dict(target_num_exemplars=5000, rel_tol_num_exemplars=0.5, transform="NORMALIZE",
                    categorical_encoding="AUTO", save_mapping_frame=False, num_iteration_without_new_exemplar=500)

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        return super().train(x=x, y=None, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        tr = str(p_["transform"]).upper()
        if tr not in TRANSFORMS:
            raise ValueError(f"aggregator: unknown transform {p_['transform']!r}")
        comm = self.comm
        world = comm.world_size if comm is not None else 1
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, use_all_levels=True)
        Xraw = design.raw_matrix(train)
        design.fit_standardization(Xraw, True, comm)
        center, scale = transform_params(design, Xraw, tr, comm)
        del Xraw
        Z = transformed(design, center, scale, train).T.contiguous()      # [n][p]
        n, p = Z.shape
        target = int(p_["target_num_exemplars"])
        tol = float(p_["rel_tol_num_exemplars"])
        lo_t, hi_t = target * (1 - tol), target * (1 + tol)
        ntot = float(n) if world == 1 else float(comm.all_reduce_numpy(np.array([float(n)]))[0])
        if ntot <= hi_t:
            leaders = torch.arange(n, device=Z.device)
            assign = torch.arange(n, device=Z.device)
            delta = 0.0
        else:
            # initial radius: a target-sized grid over the unit cube of the normalised space
            delta = max(1e-6, 0.5 * math.sqrt(p) / max(target, 1) ** (1.0 / max(min(p, 8), 1)))
            for _ in range(30):
                leaders, assign = _leaders(Z, delta)
                cnt = float(leaders.numel())
                if world > 1:
                    cnt = float(comm.all_reduce_numpy(np.array([cnt]))[0])
                if lo_t <= cnt <= hi_t:
                    break
                delta *= (cnt / target) ** (1.0 / max(min(p, 8), 1)) if cnt > 0 else 0.5
        counts = torch.bincount(assign, minlength=leaders.numel()).double()
        E = Z[leaders]
        if world > 1:
            E = comm.all_gather_cat(E)
            counts = comm.all_gather_cat(counts)
            l2, a2 = _leaders(E, delta) if delta > 0 else (torch.arange(E.shape[0], device=E.device),
                                                          torch.arange(E.shape[0], device=E.device))
            c2 = torch.zeros(l2.numel(), dtype=torch.float64, device=E.device).index_add_(0, a2, counts)
            E, counts = E[l2], c2
        # back to original units (categoricals: the one-hot argmax level)
        Ez = E.T.double().cpu().numpy() * np.asarray(scale)[:, None] + np.asarray(center)[:, None]
        vecs = []
        col = 0
        for c in self.x:
            if self.feature_types[c] == ENUM:
                dom = self.feature_domains[c] or []
                blk = Ez[col:col + len(dom)]
                vecs.append(Vec(c, torch.from_numpy(blk.argmax(0).astype(np.int32)), ENUM, list(dom)))
                col += len(dom)
            else:
                vecs.append(Vec(c, torch.from_numpy(Ez[col].astype(np.float32)), "real"))
                col += 1
        vecs.append(Vec("counts", torch.from_numpy(counts.cpu().numpy().astype(np.float32)), "real"))
        out = Frame([Vec(v.name, v.data.to(train.device), v.vtype, v.domain) for v in vecs])
        DKV.put(out.key, out)
        mkey = None
        if p_["save_mapping_frame"]:
            mp = Frame([Vec("exemplar_assignment", assign.to(torch.float32), "real")])
            DKV.put(mp.key, mp)
            mkey = mp.key
        model = AggregatorModel(self, model_id, out.key, mkey, delta)
        model.training_metrics = {"num_exemplars": int(E.shape[0]), "radius": delta, "nobs": ntot}
        return model
