"""Generalized Low Rank Model (H2O ``H2OGeneralizedLowRankEstimator``).

Factorises the (transformed, one-hot expanded) n×p data A ≈ X Y with X n×k
(rows, kept on the rank that owns them) and Y k×p (archetypes, replicated),
minimising the quadratic loss over the OBSERVED entries plus
``gamma_x r_x(X) + gamma_y r_y(Y)``.

Alternating minimisation, every product on the fp32 matrix cores
(ops.dense.gemm, feature-major A [p][n]):

* X-step (local to each rank): X = (Y Yᵀ + γx I)⁻¹ Y A;
* Y-step: Y = (X Xᵀ + γy I)⁻¹ X Aᵀ, with X Xᵀ (k×k) and X Aᵀ (k×p) summed over
  ranks in ONE all-reduce per iteration (the only communication);
* with missing entries each row (X-step) / column (Y-step) has its own
  normal equations over its observed entries: batched k×k solves of
  Y diag(m_i) Yᵀ and X diag(m_j) Xᵀ (exact masked ALS), the column systems
  all-reduced as one p×k×(k+1) tensor;
* ``NonNegative`` projects onto X, Y ≥ 0 after each half-step and ``L1``
  soft-thresholds (proximal step); ``Quadratic`` / ``L2`` are the ridge
  terms above; ``None`` uses γ = 0.

Stops after ``max_iterations`` or when the relative objective change drops
below ``min_step_size``.  ``loss`` other than ``Quadratic`` is rejected.
``init``: ``SVD`` (top-k right singular vectors of the Gram, scaled),
``PlusPlus`` (k-means++ row seeding), ``Random``.  Scoring a frame solves its
X with Y fixed and returns the reconstruction ``reconstr_<col>`` (H2O
``predict``); ``transform_frame`` returns X (``Arch1 … Archk``).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import DKV, Frame, Vec
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo
from .pca import TRANSFORMS
from .svd import transform_params


class GLRMModel(Model):
    algo = "glrm"
    algo_full_name = "Generalized Low Rank Modeling"

    def __init__(self, builder, model_id, design, center, scale, Y, objective, iterations):
        super().__init__(builder, model_id)
        self.design, self.center, self.scale = design, center, scale
        self.Y = Y                  # [k][p] archetypes (transformed scale)
        self.objective = objective
        self.iterations = iterations
        self.representation_key = None

    def _A(self, frame: Frame):
        Xraw = self.design.raw_matrix(frame)
        dev = Xraw.device
        c = torch.from_numpy(np.asarray(self.center, np.float32)).to(dev)[:, None]
        s = torch.from_numpy(np.asarray(self.scale, np.float32)).to(dev)[:, None]
        A = (Xraw - c) / s
        mask = ~torch.isnan(A)
        return torch.where(mask, A, torch.zeros_like(A)).contiguous(), mask

    def transform_frame(self, frame: Frame) -> Frame:
        """X (n×k) of a frame with the archetypes fixed (H2O ``transform_frame``)."""
        A, mask = self._A(frame)
        Xk = _solve_x(A, mask, torch.from_numpy(self.Y.astype(np.float32)).to(A.device), self.params)
        return Frame([Vec(f"Arch{i + 1}", Xk[i].float(), "real") for i in range(Xk.shape[0])])

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        A, mask = self._A(frame)
        Yt = torch.from_numpy(self.Y.astype(np.float32)).to(A.device)
        Xk = _solve_x(A, mask, Yt, self.params)
        R = D.gemm(Yt, Xk, ta=True)                                       # [p][n]
        s = torch.from_numpy(np.asarray(self.scale, np.float32)).to(R.device)[:, None]
        c = torch.from_numpy(np.asarray(self.center, np.float32)).to(R.device)[:, None]
        return R * s + c

    def predict(self, frame: Frame) -> Frame:
        R = self.predict_raw(frame)
        return Frame([Vec(f"reconstr_{n}", R[j].float(), "real") for j, n in enumerate(self.design.names)])

    def model_performance(self, frame=None):
        return self.training_metrics

    def archetypes(self):
        return self.Y.copy()

    def summary(self):
        return {"model_id": self.model_id, "k": int(self.Y.shape[0]), "objective": self.objective,
                "iterations": self.iterations}

    def to_json(self):
        j = super().to_json()
        out = j["output"]
        out["archetypes"] = {"names": self.design.names, "data": self.Y.tolist()}
        out["objective"] = self.objective
        out["iterations"] = self.iterations
        out["representation_name"] = self.representation_key
        return j


def _prox(M: torch.Tensor, reg: str, gamma: float):
    reg = reg.lower()
    if reg == "nonnegative":
        return M.clamp_min(0.0)
    if reg == "l1" and gamma > 0:
        return torch.sign(M) * (M.abs() - gamma).clamp_min(0.0)
    return M


def _ridge(reg: str, gamma: float) -> float:
    return gamma if reg.lower() in ("quadratic", "l2") else 0.0


def _solve_x(A: torch.Tensor, mask: torch.Tensor, Y: torch.Tensor, p_) -> torch.Tensor:
    """X [k][n] minimising the masked quadratic loss (+ x regulariser) with Y fixed."""
    k = Y.shape[0]
    rx, gx = str(p_["regularization_x"]), float(p_["gamma_x"])
    lam = _ridge(rx, gx) + 1e-8
    if bool(mask.all()):
        Gy = D.gemm(Y, Y, tb=True).double() + lam * torch.eye(k, dtype=torch.float64, device=Y.device)
        return _prox(torch.linalg.inv(Gy.cpu()).to(Y.device, torch.float32) @ D.gemm(Y, A), rx, gx)
    # per-row normal equations over the observed columns: G_i = Y diag(m_i) Y^T
    m = mask.float()
    out = torch.empty((k, A.shape[1]), dtype=torch.float32, device=A.device)
    eye = lam * torch.eye(k, dtype=torch.float64, device=A.device)
    for s0 in range(0, A.shape[1], 1 << 16):
        s1 = min(A.shape[1], s0 + (1 << 16))
        mb = m[:, s0:s1]
        G = torch.einsum("jn,aj,bj->nab", mb, Y, Y).double() + eye
        r = (Y @ (A[:, s0:s1] * mb)).T.double()                           # [n][k]
        out[:, s0:s1] = torch.linalg.solve(G, r.unsqueeze(-1)).squeeze(-1).T.float()
    return _prox(out, rx, gx)


def _solve_y(A: torch.Tensor, mask: torch.Tensor, X: torch.Tensor, p_, comm, full: bool) -> torch.Tensor:
    """Y [k][p] with X fixed; one all-reduce of the (summed) normal equations.
    ``full`` (no missing entry on ANY rank) must agree across ranks."""
    k = X.shape[0]
    ry, gy = str(p_["regularization_y"]), float(p_["gamma_y"])
    lam = _ridge(ry, gy) + 1e-8
    world = comm.world_size if comm is not None else 1
    dev = A.device
    if full:
        S = torch.cat([D.gemm(X, X, tb=True), D.gemm(X, A, tb=True)], 1).double()
        if world > 1:
            comm.all_reduce_(S)
        Gx = S[:, :k] + lam * torch.eye(k, dtype=torch.float64, device=dev)
        return _prox(torch.linalg.solve(Gx.cpu(), S[:, k:].cpu()).to(dev, torch.float32), ry, gy)
    m = mask.float()
    G = torch.einsum("jn,an,bn->jab", m, X, X).double()                    # [p][k][k]
    r = (X @ (A * m).T).T.double()                                         # [p][k]
    S = torch.cat([G, r.unsqueeze(-1)], -1)
    if world > 1:
        comm.all_reduce_(S)
    G = S[..., :k] + lam * torch.eye(k, dtype=torch.float64, device=dev)
    Y = torch.linalg.solve(G, S[..., k:]).squeeze(-1).T                    # [k][p]
    return _prox(Y.float().contiguous(), ry, gy)


class H2OGeneralizedLowRankEstimator(ModelBuilder):
    algo = "glrm"
    UNSUPERVISED_CATEGORY = ModelCategory.DIMREDUCTION
    DEFAULTS = dict(k=1, transform="NONE", loss="Quadratic", multi_loss="Categorical", regularization_x="None",
                    regularization_y="None", gamma_x=0.0, gamma_y=0.0, max_iterations=1000, max_updates=2000,
                    init_step_size=1.0, min_step_size=1e-4, init="PlusPlus", svd_method="Randomized",
                    user_y=None, user_x=None, expand_user_y=True, impute_original=False, recover_svd=False,
                    representation_name=None, period=1, max_runtime_secs=0.0)

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        return super().train(x=x, y=None, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        if str(p_["loss"]).lower() != "quadratic":
            raise ValueError(f"glrm: loss {p_['loss']!r} is not supported (Quadratic)")
        tr = str(p_["transform"]).upper()
        if tr not in TRANSFORMS:
            raise ValueError(f"glrm: unknown transform {p_['transform']!r}")
        for r in ("regularization_x", "regularization_y"):
            if str(p_[r]).lower() not in ("none", "quadratic", "l2", "l1", "nonnegative"):
                raise ValueError(f"glrm: {r}={p_[r]!r} (None, Quadratic, L2, L1, NonNegative)")
        comm = self.comm
        world = comm.world_size if comm is not None else 1
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, use_all_levels=True)
        Xraw = design.raw_matrix(train)
        design.fit_standardization(Xraw, True, comm)
        center, scale = transform_params(design, Xraw, tr, comm)
        del Xraw
        model = GLRMModel(self, model_id, design, center, scale, np.zeros((1, 1)), float("nan"), 0)
        A, mask = model._A(train)
        p, n = A.shape
        k = int(p_["k"])
        if not 1 <= k <= p:
            raise ValueError(f"glrm: k={k} must be in [1, {p}]")
        dev = A.device
        seed = self._seed()
        g = torch.Generator().manual_seed(seed)
        # missing entries start at the column means (0 on the transformed scale when demeaned)
        colmean = (A.double().sum(1) / mask.double().sum(1).clamp_min(1))
        cm = torch.stack([A.double().sum(1), mask.double().sum(1)])
        if world > 1:
            comm.all_reduce_(cm)
        colmean = (cm[0] / cm[1].clamp_min(1)).float()
        Af = torch.where(mask, A, colmean[:, None].expand_as(A)).contiguous()
        Y = self._init_y(Af, k, str(p_["init"]), g, comm).to(dev)
        rx, ry = str(p_["regularization_x"]), str(p_["regularization_y"])
        gx, gy = float(p_["gamma_x"]), float(p_["gamma_y"])
        nobs = mask.double().sum()
        anymiss = torch.tensor([0.0 if bool(mask.all()) else 1.0], dtype=torch.float64, device=dev)
        if world > 1:
            comm.all_reduce_(anymiss, "max")
        full = float(anymiss) == 0.0
        if world > 1:
            comm.all_reduce_(nobs)
        prev = math.inf
        obj = math.inf
        it = 0
        X = None
        hist = []
        for it in range(1, int(p_["max_iterations"]) + 1):
            X = _solve_x(A, mask, Y, p_)                                   # rows are local
            Y = _solve_y(A, mask, X, p_, comm, full)
            R = D.gemm(Y, X, ta=True)                                     # reconstruction [p][n]
            err = torch.where(mask, A - R, torch.zeros_like(R)).double().pow(2).sum()
            regx = (X.double().pow(2).sum() * _ridge(rx, gx) + (X.double().abs().sum() * gx if rx.lower() == "l1"
                                                                 else 0.0))
            parts = torch.stack([err, torch.as_tensor(regx, dtype=torch.float64, device=dev)])
            if world > 1:
                comm.all_reduce_(parts)
            regy = float(Y.double().pow(2).sum()) * _ridge(ry, gy) + (float(Y.double().abs().sum()) * gy
                                                                      if ry.lower() == "l1" else 0.0)
            obj = float(parts[0] + parts[1]) + regy
            hist.append({"iterations": it, "objective": obj})
            if abs(prev - obj) <= float(p_["min_step_size"]) * max(abs(prev), 1e-12):
                break
            prev = obj
        model = GLRMModel(self, model_id, design, center, scale, Y.double().cpu().numpy(), obj, it)
        model.scoring_history = hist
        model.training_metrics = {"objective": obj, "iterations": it, "numerr": float(parts[0]),
                                  "nobs": float(nobs), "caterr": 0.0}
        rep = Frame([Vec(f"Arch{i + 1}", X[i].float(), "real") for i in range(k)],
                    key=p_["representation_name"] or None)
        DKV.put(rep.key, rep)
        model.representation_key = rep.key
        model.representation = rep
        return model

    def _init_y(self, Af: torch.Tensor, k: int, init: str, g, comm) -> torch.Tensor:
        p, n = Af.shape
        world = comm.world_size if comm is not None else 1
        init = init.lower()
        if init == "svd":
            G = D.gemm(Af, Af, tb=True).double()
            if world > 1:
                comm.all_reduce_(G)
            w, V = np.linalg.eigh(G.cpu().numpy())
            order = np.argsort(w)[::-1][:k]
            nrows = float(n) * world
            Y = (V[:, order] * np.sqrt(np.maximum(w[order], 0) / max(nrows, 1.0))).T
            return torch.from_numpy(np.ascontiguousarray(Y, dtype=np.float32))
        if init == "random":
            return torch.randn((k, p), generator=g)
        if init in ("plusplus", "user"):
            # k-means++ seeding over a sample of the rank's rows, gathered to every rank
            m = min(n, 20000)
            idx = torch.randperm(n, generator=g)[:m].to(Af.device)
            S = Af[:, idx].T.contiguous().float()                        # [m][p]
            if world > 1:
                S = comm.all_gather_cat(S)
            S = S.cpu()
            rows = [int(torch.randint(0, S.shape[0], (1,), generator=g))]
            d2 = ((S - S[rows[0]]) ** 2).sum(1)
            for _ in range(1, k):
                pr = d2 / d2.sum().clamp_min(1e-30)
                j = int(torch.multinomial(pr, 1, generator=g)) if float(d2.sum()) > 0 else int(
                    torch.randint(0, S.shape[0], (1,), generator=g))
                rows.append(j)
                d2 = torch.minimum(d2, ((S - S[j]) ** 2).sum(1))
            return S[rows].contiguous()
        raise ValueError(f"glrm: init {init!r} (SVD, PlusPlus, Random)")
