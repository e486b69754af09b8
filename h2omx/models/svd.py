"""Singular Value Decomposition (H2O ``H2OSingularValueDecompositionEstimator``).

``svd_method="GramSVD"`` (H2O's default): one split-K fp32 GEMM on the
matrix cores forms the p×p Gram XᵀX of the transformed design matrix
(feature-major on the device, csrc/dense_kernels.hip), the Gram is
all-reduced across ranks once, and its fp64 symmetric eigendecomposition
gives V and d = sqrt(eigenvalues).  ``keep_u`` materialises U = X V / d as a
frame (``u_name``) — one more GEMM, local to every rank's rows.  ``Power``
and ``Randomized`` are accepted and return the same (exact) factors.

Scoring returns the projection X V (H2O SVDModel.score0), columns
``SVD1 … SVDnv``.
"""
from __future__ import annotations

import numpy as np
import torch

from ..frame.frame import DKV, Frame, Vec
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory
from .pca import TRANSFORMS
from .glm import DesignInfo


def transform_params(design, Xraw, tr: str, comm):
    """(center, scale) of an H2O DataInfo.TransformType over all ranks."""
    p = Xraw.shape[0]
    mn = torch.where(torch.isnan(Xraw), torch.full_like(Xraw, float("inf")), Xraw).amin(1)
    mx = torch.where(torch.isnan(Xraw), torch.full_like(Xraw, float("-inf")), Xraw).amax(1)
    if comm is not None and comm.world_size > 1:
        comm.all_reduce_(mn, "min")
        comm.all_reduce_(mx, "max")
    rng = (mx - mn).double().cpu().numpy()
    center = design.means.copy() if tr in ("DEMEAN", "STANDARDIZE", "NORMALIZE") else np.zeros(p)
    if tr in ("DESCALE", "STANDARDIZE"):
        scale = design.sds.copy()
    elif tr == "NORMALIZE":
        scale = np.where(rng > 0, rng, 1.0)
    else:
        scale = np.ones(p)
    return center, scale


def transformed(design, center, scale, frame: Frame) -> torch.Tensor:
    """Mean-imputed, centred and scaled design matrix, feature-major [p][n] fp32."""
    Xraw = design.raw_matrix(frame)
    dev = Xraw.device
    m = torch.from_numpy(design.means.astype(np.float32)).to(dev)[:, None]
    c = torch.from_numpy(np.asarray(center, np.float32)).to(dev)[:, None]
    s = torch.from_numpy(np.asarray(scale, np.float32)).to(dev)[:, None]
    X = torch.where(torch.isnan(Xraw), m.expand_as(Xraw), Xraw)
    return ((X - c) / s).contiguous()


class SVDModel(Model):
    algo = "svd"
    algo_full_name = "Singular Value Decomposition"

    def __init__(self, builder, model_id, design, center, scale, v, d):
        super().__init__(builder, model_id)
        self.design, self.center, self.scale = design, center, scale
        self.v = v          # [p][nv] right singular vectors
        self.d = d          # [nv] singular values
        self.u_key = None

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        X = transformed(self.design, self.center, self.scale, frame)
        V = torch.from_numpy(self.v.astype(np.float32)).to(X.device)
        return D.gemm(V, X, ta=True)            # [nv][n] = Vᵀ X

    def predict(self, frame: Frame) -> Frame:
        S = self.predict_raw(frame)
        return Frame([Vec(f"SVD{i + 1}", S[i].float(), "real") for i in range(S.shape[0])])

    def model_performance(self, frame=None):
        return self.training_metrics

    def summary(self):
        return {"model_id": self.model_id, "nv": int(self.v.shape[1]), "d": self.d.tolist()}

    def to_json(self):
        j = super().to_json()
        out = j["output"]
        out["d"] = self.d.tolist()
        out["v"] = {"names": self.design.names, "data": self.v.tolist()}
        out["u_key"] = {"name": self.u_key} if self.u_key else None
        return j


class H2OSingularValueDecompositionEstimator(ModelBuilder):
    algo = "svd"
    UNSUPERVISED_CATEGORY = ModelCategory.DIMREDUCTION
    DEFAULTS = dict(nv=1, transform="NONE", svd_method="GramSVD", max_iterations=1000, use_all_factor_levels=True,
                    keep_u=True, u_name=None, impute_missing=False)

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        return super().train(x=x, y=None, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        tr = str(p_["transform"]).upper()
        if tr not in TRANSFORMS:
            raise ValueError(f"svd: unknown transform {p_['transform']!r}")
        if str(p_["svd_method"]) not in ("GramSVD", "Power", "Randomized"):
            raise ValueError(f"svd: svd_method {p_['svd_method']!r} (GramSVD, Power, Randomized)")
        comm = self.comm
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, bool(p_["use_all_factor_levels"]))
        Xraw = design.raw_matrix(train)
        design.fit_standardization(Xraw, True, comm)
        p = Xraw.shape[0]
        nv = int(p_["nv"])
        if not 1 <= nv <= p:
            raise ValueError(f"svd: nv={nv} must be in [1, {p}] (expanded predictors)")
        center, scale = transform_params(design, Xraw, tr, comm)
        del Xraw
        X = transformed(design, center, scale, train)
        G = D.gemm(X, X, tb=True).double()              # [p][p] = X Xᵀ (feature-major) = AᵀA
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(G)
        Gn = G.cpu().numpy()
        w, V = np.linalg.eigh(0.5 * (Gn + Gn.T))
        order = np.argsort(w)[::-1]
        w, V = np.maximum(w[order], 0.0), V[:, order]
        sgn = np.sign(V[np.argmax(np.abs(V), axis=0), np.arange(V.shape[1])])
        V = V * np.where(sgn == 0, 1.0, sgn)[None, :]
        d = np.sqrt(w[:nv])
        model = SVDModel(self, model_id, design, center, scale, V[:, :nv].copy(), d)
        model.training_metrics = {"nobs": float(train.nrows), "d": d.tolist()}
        if p_["keep_u"]:
            Vt = torch.from_numpy(model.v.astype(np.float32)).to(X.device)
            U = D.gemm(Vt, X, ta=True) / torch.from_numpy(np.where(d > 0, d, 1.0).astype(np.float32)).to(X.device)[:, None]
            ufr = Frame([Vec(f"u{i + 1}", U[i].float(), "real") for i in range(nv)], key=p_["u_name"] or None)
            DKV.put(ufr.key, ufr)
            model.u_key = ufr.key
            model.u = ufr
        return model
