"""Generalized Additive Model (H2O ``H2OGeneralizedAdditiveEstimator``).

Each ``gam_columns`` predictor x is replaced by a penalised cubic regression
spline (H2O ``bs=0``; Wood 2006, §4.1.2): ``num_knots`` knots at quantiles
of x (over all ranks), basis functions parameterised by the function values
at the knots with natural end conditions, and the wiggliness penalty
∫ f''(x)² dx = βᵀ S β with S = Dᵀ B⁻¹ D.  The basis is made identifiable by
the sum-to-zero constraint (null space of the column sums, QR), so each gam
column contributes ``num_knots − 1`` centred columns ``<col>_cr_<i>``.

The model is then a GLM (same families / links / IRLS kernels — the Gram is
the fp32 MFMA kernel of ops.dense.glm_irls_pass) whose normal equations get
the block-diagonal penalty Σ scale_j S_j (estimator hook
``_penalty_matrix``).  Scoring rebuilds the basis from the stored knots.
"""
from __future__ import annotations

import numpy as np
import torch

from ..frame.frame import Frame, Vec
from .glm import GLMModel, H2OGeneralizedLinearEstimator


def cr_basis_matrices(knots: np.ndarray):
    """(F, S) for cubic regression splines on sorted knots: second derivatives
    at the knots = F β, penalty = S."""
    k = knots.size
    h = np.diff(knots)
    Dm = np.zeros((k - 2, k))
    Bm = np.zeros((k - 2, k - 2))
    for i in range(k - 2):
        Dm[i, i] = 1.0 / h[i]
        Dm[i, i + 1] = -1.0 / h[i] - 1.0 / h[i + 1]
        Dm[i, i + 2] = 1.0 / h[i + 1]
        Bm[i, i] = (h[i] + h[i + 1]) / 3.0
        if i + 1 < k - 2:
            Bm[i, i + 1] = Bm[i + 1, i] = h[i + 1] / 6.0
    BinvD = np.linalg.solve(Bm, Dm)
    F = np.zeros((k, k))
    F[1:-1] = BinvD
    S = Dm.T @ BinvD
    return F, 0.5 * (S + S.T)


def cr_basis(x: torch.Tensor, knots: np.ndarray, F: np.ndarray) -> torch.Tensor:
    """[n][k] cubic-regression-spline basis (linear extrapolation outside the knots)."""
    dev = x.device
    kn = torch.from_numpy(knots).to(dev, torch.float64)
    Ft = torch.from_numpy(F).to(dev, torch.float64)
    k = kn.numel()
    xd = x.double()
    xc = xd.clamp(kn[0], kn[-1])
    j = (torch.searchsorted(kn, xc, right=True) - 1).clamp(0, k - 2)
    x0, x1 = kn[j], kn[j + 1]
    h = x1 - x0
    am = (x1 - xc) / h
    ap = (xc - x0) / h
    cm = ((x1 - xc) ** 3 / h - h * (x1 - xc)) / 6.0
    cp = ((xc - x0) ** 3 / h - h * (xc - x0)) / 6.0
    n = x.numel()
    X = cm[:, None] * Ft[j] + cp[:, None] * Ft[j + 1]
    rows = torch.arange(n, device=dev)
    X[rows, j] += am
    X[rows, j + 1] += ap
    # natural (linear) extrapolation: f(x) = f(edge) + f'(edge) (x - edge)
    lo, hi = xd < kn[0], xd > kn[-1]
    if bool(lo.any()) or bool(hi.any()):
        h0, hl = kn[1] - kn[0], kn[-1] - kn[-2]
        d0 = torch.zeros(k, dtype=torch.float64, device=dev)      # f'(x_0) as a linear map of beta
        d0[0], d0[1] = -1.0 / h0, 1.0 / h0
        d0 = d0 - h0 / 3.0 * Ft[0] - h0 / 6.0 * Ft[1]
        dl = torch.zeros(k, dtype=torch.float64, device=dev)
        dl[-2], dl[-1] = -1.0 / hl, 1.0 / hl
        dl = dl + hl / 6.0 * Ft[-2] + hl / 3.0 * Ft[-1]
        X = torch.where(lo[:, None], X + (xd - kn[0])[:, None] * d0[None, :], X)
        X = torch.where(hi[:, None], X + (xd - kn[-1])[:, None] * dl[None, :], X)
    return X


class GAMModel(GLMModel):
    algo = "gam"
    algo_full_name = "Generalized Additive Model"

    def augment(self, frame: Frame) -> Frame:
        return _augment(frame, self.gam_spec)

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        return super().predict_raw(self.augment(frame))

    def to_json(self):
        j = super().to_json()
        j["output"]["gam_knots"] = {c: sp["knots"].tolist() for c, sp in self.gam_spec.items()}
        return j


def _augment(frame: Frame, spec: dict) -> Frame:
    names = set(frame.names)
    vecs = list(frame.vecs)
    for c, sp in spec.items():
        cols = [f"{c}_cr_{i}" for i in range(sp["Z"].shape[1])]
        if all(n in names for n in cols):
            continue
        x = frame.vec(c).as_float()
        x = torch.where(torch.isnan(x), torch.full_like(x, float(sp["mean"])), x)
        B = cr_basis(x, sp["knots"], sp["F"]) @ torch.from_numpy(sp["Z"]).to(x.device, torch.float64)
        vecs += [Vec(n, B[:, i].float(), "real") for i, n in enumerate(cols)]
    return Frame(vecs, key=frame.key)


class H2OGeneralizedAdditiveEstimator(H2OGeneralizedLinearEstimator):
    algo = "gam"
    DEFAULTS = {**H2OGeneralizedLinearEstimator.DEFAULTS, "gam_columns": None, "num_knots": None, "bs": None,
                "scale": None, "knot_ids": None, "keep_gam_cols": False}

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        if training_frame is None:
            raise ValueError("training_frame is required")
        self.params.update(kw)
        p_ = self.params
        gcols = [c if isinstance(c, str) else c[0] for c in (p_.get("gam_columns") or [])]
        if not gcols:
            raise ValueError("gam: gam_columns is required")
        nk = p_.get("num_knots") or [10] * len(gcols)
        sc = p_.get("scale") or [0.001] * len(gcols)
        bs = p_.get("bs") or [0] * len(gcols)
        if any(int(b) != 0 for b in bs):
            raise ValueError("gam: only bs=0 (cubic regression splines) is supported")
        spec = {}
        for c, k, s in zip(gcols, nk, sc):
            v = training_frame.vec(c).as_float()
            v = v[~torch.isnan(v)]
            samp = v[torch.randperm(v.numel(), device=v.device)[:200_000]] if v.numel() > 200_000 else v
            if comm is not None and comm.world_size > 1:
                samp = comm.all_gather_cat(samp)
            k = int(k)
            qs = torch.quantile(samp.double().cpu(), torch.linspace(0, 1, k, dtype=torch.float64)).numpy()
            knots = np.unique(qs)
            if knots.size < 3:
                raise ValueError(f"gam: column {c} has too few distinct values for {k} knots")
            F, S = cr_basis_matrices(knots)
            xf = training_frame.vec(c).as_float()
            mean = float(samp.double().mean())
            xf = torch.where(torch.isnan(xf), torch.full_like(xf, mean), xf)
            Bfull = cr_basis(xf, knots, F)
            csum = Bfull.sum(0)
            if comm is not None and comm.world_size > 1:
                comm.all_reduce_(csum)
            Q, _ = np.linalg.qr(csum.cpu().numpy()[:, None], mode="complete")
            Z = Q[:, 1:]                                                  # sum-to-zero null space
            spec[c] = {"knots": knots, "F": F, "S": Z.T @ S @ Z, "Z": Z, "scale": float(s), "mean": mean}
        self.gam_spec = spec
        aug = _augment(training_frame, spec)
        vaug = _augment(validation_frame, spec) if validation_frame is not None else None
        base_x = x if x is not None else [n for n in training_frame.names if n != y]
        keep = [c for c in base_x if c not in spec and c not in self._special(y)]
        new_x = keep + [f"{c}_cr_{i}" for c in spec for i in range(spec[c]["Z"].shape[1])]
        model = super().train(x=new_x, y=y, training_frame=aug, validation_frame=vaug, comm=comm)
        model.__class__ = GAMModel
        model.gam_spec = spec
        return model

    def _special(self, y):
        p_ = self.params
        return {y, p_.get("weights_column"), p_.get("fold_column"), p_.get("offset_column")}

    def _penalty_matrix(self, design):
        spec = getattr(self, "gam_spec", None)
        if not spec:
            return None
        p = len(design.names)
        P = np.zeros((p, p))
        pos = {n: i for i, n in enumerate(design.names)}
        for c, sp in spec.items():
            idx = [pos[f"{c}_cr_{i}"] for i in range(sp["Z"].shape[1]) if f"{c}_cr_{i}" in pos]
            if len(idx) == sp["S"].shape[0]:
                P[np.ix_(idx, idx)] += sp["scale"] * sp["S"]
        return P
