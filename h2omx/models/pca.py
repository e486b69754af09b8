"""Principal Component Analysis (H2O PCA equivalent).

``pca_method="GramSVD"`` (H2O's default): the transformed design matrix X
(feature-major [p][n] on the device) is reduced to its Gram matrix
X Xᵀ / (n - 1) with one split-K fp32 GEMM on the matrix cores
(csrc/dense_kernels.hip gemm_kernel, deterministic split-K reduce), the
p×p Gram is all-reduced across ranks (one collective per model, SURVEY.md
§2.5 C4-style), and its symmetric eigendecomposition runs on the host in
fp64.  ``Power`` and ``Randomized`` are accepted and give the same
eigenpairs (the Gram is exact and small); ``GLRM`` is not provided.

``transform``: NONE | DEMEAN | DESCALE | STANDARDIZE | NORMALIZE (demean,
divide by the range), like H2O's DataInfo.TransformType.  Categorical
columns are one-hot expanded (first level dropped unless
``use_all_factor_levels``).  Scoring projects rows onto the first k
eigenvectors: columns ``PC1 … PCk``.
"""
from __future__ import annotations

import numpy as np
import torch

from ..frame.frame import Frame, Vec
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo

TRANSFORMS = ("NONE", "DEMEAN", "DESCALE", "STANDARDIZE", "NORMALIZE")


class PCAModel(Model):
    algo = "pca"
    algo_full_name = "Principal Components Analysis"

    def __init__(self, builder, model_id, design, center, scale, eigvec, eigval, total_var):
        super().__init__(builder, model_id)
        self.design = design
        self.center = center            # [p] subtracted before projection
        self.scale = scale              # [p] divided after centering
        self.eigenvectors = eigvec      # [p][k]
        self.eigenvalues = eigval       # [k]
        self.std_deviation = np.sqrt(np.maximum(eigval, 0.0))
        self.total_variance = total_var
        pv = eigval / total_var if total_var > 0 else np.zeros_like(eigval)
        self.importance = {"Standard deviation": self.std_deviation.tolist(),
                           "Proportion of Variance": pv.tolist(), "Cumulative Proportion": np.cumsum(pv).tolist()}

    def _X(self, frame: Frame) -> torch.Tensor:
        Xraw = self.design.raw_matrix(frame)
        dev = Xraw.device
        m = torch.from_numpy(self.design.means.astype(np.float32)).to(dev)[:, None]
        c = torch.from_numpy(self.center.astype(np.float32)).to(dev)[:, None]
        s = torch.from_numpy(self.scale.astype(np.float32)).to(dev)[:, None]
        X = torch.where(torch.isnan(Xraw), m.expand_as(Xraw), Xraw)
        return ((X - c) / s).contiguous()

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        X = self._X(frame)                                              # [p][n]
        V = torch.from_numpy(self.eigenvectors.astype(np.float32)).to(X.device)   # [p][k]
        return D.gemm(V, X, ta=True)                                    # [k][n]

    def predict(self, frame: Frame) -> Frame:
        S = self.predict_raw(frame)
        return Frame([Vec(f"PC{i + 1}", S[i].float(), "real") for i in range(S.shape[0])])

    def model_performance(self, frame: Frame | None = None):
        return self.training_metrics

    def summary(self):
        return {"model_id": self.model_id, "k": int(self.eigenvectors.shape[1]), **self.importance}

    def to_json(self):
        j = super().to_json()
        out = j["output"]
        k = self.eigenvectors.shape[1]
        out["eigenvectors"] = {"names": self.design.names, "columns": [f"PC{i + 1}" for i in range(k)],
                               "data": self.eigenvectors.tolist()}
        out["importance"] = self.importance
        out["std_deviation"] = self.std_deviation.tolist()
        out["total_variance"] = self.total_variance
        return j


class H2OPrincipalComponentAnalysisEstimator(ModelBuilder):
    algo = "pca"
    UNSUPERVISED_CATEGORY = ModelCategory.DIMREDUCTION
    DEFAULTS = dict(k=1, transform="NONE", pca_method="GramSVD", pca_impl="MTJ_EVD_SYMMMATRIX", max_iterations=1000,
                    use_all_factor_levels=False, compute_metrics=True, impute_missing=False)

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        return super().train(x=x, y=None, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        tr = str(p_["transform"]).upper()
        if tr not in TRANSFORMS:
            raise ValueError(f"pca: unknown transform {p_['transform']!r}")
        method = str(p_["pca_method"])
        if method not in ("GramSVD", "Power", "Randomized"):
            raise ValueError(f"pca: pca_method {method!r} is not supported (GramSVD, Power, Randomized)")
        comm = self.comm
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, bool(p_["use_all_factor_levels"]))
        Xraw = design.raw_matrix(train)
        design.fit_standardization(Xraw, True, comm)      # means / sds over all ranks (NA-aware)
        p = Xraw.shape[0]
        k = int(p_["k"])
        if not 1 <= k <= p:
            raise ValueError(f"pca: k={k} must be in [1, {p}] (expanded predictors)")
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
        model = PCAModel(self, model_id, design, center, scale, np.zeros((p, k)), np.zeros(k), 0.0)
        X = model._X(train)
        del Xraw
        G = D.gemm(X, X, tb=True).double()                # [p][p] = X Xᵀ
        n = torch.tensor([float(X.shape[1])], dtype=torch.float64, device=X.device)
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(G)
            comm.all_reduce_(n)
        N = float(n.item())
        Gn = G.cpu().numpy() / max(N - 1.0, 1.0)
        Gn = 0.5 * (Gn + Gn.T)
        w, V = np.linalg.eigh(Gn)
        order = np.argsort(w)[::-1]
        w, V = w[order], V[:, order]
        # deterministic sign: the largest-magnitude loading of each component is positive
        sgn = np.sign(V[np.argmax(np.abs(V), axis=0), np.arange(V.shape[1])])
        V = V * np.where(sgn == 0, 1.0, sgn)[None, :]
        total = float(np.maximum(w, 0).sum())
        model = PCAModel(self, model_id, design, center, scale, V[:, :k].copy(), w[:k].copy(), total)
        model.training_metrics = {"nobs": N, "total_variance": total, **model.importance}
        model.gram = Gn
        return model
