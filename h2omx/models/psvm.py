"""Parallel SVM (H2O ``H2OSupportVectorMachineEstimator``, PSVM).

This is a binary kernel SVM trained with the PSVM scheme (Chang et al.,
"PSVM: Parallelizing Support Vector Machines on Distributed Computers", 2007).

1. Pivoted incomplete Cholesky factorisation (ICF) of the kernel matrix,
   K ~ H H^T with H of shape [n][p].  The rank is
   p = rank_ratio * n (default sqrt(n)).  The Gaussian kernel is
   K(a, b) = exp(-gamma ||a - b||^2), with gamma = 1 / #features by default.
   Rows stay sharded over ranks.  Each pivot step is:
     * a global arg-max of the residual diagonal (one all-gather);
     * a broadcast of the pivot row and its H row from the owner rank;
     * a kernel column computed locally on every rank.
2. A primal-dual interior-point method on the dual
       min 1/2 a^T Q a - 1^T a,  y^T a = 0,  0 <= a_i <= C_i,
   with Q = diag(y) H H^T diag(y) and C_i = hyper_param times the class weight.
   The Newton system (D + Hy Hy^T) is solved with Sherman-Morrison-Woodbury:
   each iteration needs one p x p Gram Hy^T D^-1 Hy, which is all-reduced, and
   p x p Cholesky solves.  Everything else is row-local vector work plus
   scalar / p-vector all-reduces.  The barrier weight mu shrinks by
   ``mu_factor`` per iteration.  The loop stops when both the surrogate
   duality gap and the primal / dual residuals are below their thresholds.
3. Support vectors are rows with a_i > sv_threshold.  The bias b is averaged
   over the free support vectors, 0 < a_i < C_i.
Scoring: f(x) = sum_sv a_i y_i K(x_i, x) + b.  The cross term x . sv is the
fp32 MFMA GEMM of ops.dense.gemm, with the squared norms and exp fused after it.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import Frame, Vec
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory


def _allsum(t: torch.Tensor, comm) -> torch.Tensor:
    if comm is not None and comm.world_size > 1:
        comm.all_reduce_(t)
    return t


def _kernel_col(X: torch.Tensor, xsq: torch.Tensor, xp: torch.Tensor, gamma: float) -> torch.Tensor:
    """exp(-gamma ||X_i - xp||^2) for every local row, fp64."""
    d2 = (xsq - 2.0 * (X @ xp) + (xp * xp).sum()).clamp_min(0.0)
    return torch.exp(-gamma * d2)


def icf(X: torch.Tensor, gamma: float, p: int, thresh: float, comm=None) -> torch.Tensor:
    """Pivoted incomplete Cholesky of the Gaussian kernel over the (sharded)
    rows of X [n][d] fp64 -> H [n][rank] with K ~ H H^T."""
    n, d = X.shape
    dev = X.device
    world = comm.world_size if comm is not None else 1
    rank = comm.rank if comm is not None else 0
    H = torch.zeros((n, p), dtype=torch.float64, device=dev)
    diag = torch.ones(n, dtype=torch.float64, device=dev)      # K(x, x) = 1 for the Gaussian kernel
    xsq = (X * X).sum(1)
    k_used = 0
    for k in range(p):
        if n > 0:
            v, i = diag.max(0)
            v, i = float(v), int(i)
        else:
            v, i = -1.0, -1
        if world > 1:
            cand = comm.all_gather_cat(torch.tensor([[v, float(rank), float(i)]], dtype=torch.float64, device=dev))
            j = int(torch.argmax(cand[:, 0]))
            v, owner, i = float(cand[j, 0]), int(cand[j, 1]), int(cand[j, 2])
        else:
            owner = 0
        if v < thresh:
            break
        buf = torch.zeros(d + k, dtype=torch.float64, device=dev)
        if rank == owner:
            buf[:d] = X[i]
            buf[d:] = H[i, :k]
        if world > 1:
            comm.broadcast_(buf, owner)
        xp, hp = buf[:d], buf[d:]
        piv = math.sqrt(v)
        col = _kernel_col(X, xsq, xp, gamma)
        if k:
            col = col - H[:, :k] @ hp
        H[:, k] = col / piv
        if rank == owner:
            H[i, k] = piv
        diag = (diag - H[:, k] ** 2).clamp_min(0.0)
        if rank == owner:
            diag[i] = 0.0
        k_used = k + 1
    return H[:, :k_used].contiguous()


class PSVMModel(Model):
    algo = "psvm"
    algo_full_name = "Support Vector Machine (PSVM)"

    def __init__(self, builder, model_id, sv, coef, b, gamma, means, scales):
        super().__init__(builder, model_id)
        self.sv = sv            # [nsv][d] float32 (standardised inputs)
        self.coef = coef        # [nsv] a_i y_i
        self.b = float(b)
        self.gamma = float(gamma)
        self.means = means
        self.scales = scales

    def decision_function(self, frame: Frame) -> torch.Tensor:
        X = _design(frame, self.x, self.means, self.scales).float()
        dev = X.device
        if self.sv.shape[0] == 0:
            return torch.full((X.shape[0],), self.b, device=dev)
        S = self.sv.to(dev)
        out = torch.zeros(X.shape[0], dtype=torch.float64, device=dev)
        ssq = (S.double() * S.double()).sum(1)
        coef = self.coef.to(dev)
        step = 1 << 16
        for r0 in range(0, X.shape[0], step):
            xb = X[r0:r0 + step].contiguous()
            G = D.gemm(xb, S, tb=True)                                   # [rows][nsv] x . sv
            d2 = ((xb.double() * xb.double()).sum(1)[:, None] - 2.0 * G.double() + ssq[None, :]).clamp_min(0.0)
            out[r0:r0 + step] = torch.exp(-self.gamma * d2) @ coef
        return (out + self.b).float()

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        f = self.decision_function(frame)
        p1 = (f > 0).float()
        return torch.stack([1 - p1, p1])

    def predict(self, frame: Frame) -> Frame:
        f = self.decision_function(frame)
        lab = (f > 0).to(torch.int32)
        return Frame([Vec("predict", lab, "enum", list(self.response_domain)),
                      Vec("decision_function", f.float(), "real")])

    def summary(self):
        return {"model_id": self.model_id, "number_of_support_vectors": int(self.sv.shape[0]),
                "number_of_bounded_support_vectors": int(self.timings.get("bounded_sv", 0)),
                "rho": -self.b, "gamma": self.gamma}


def _design(frame: Frame, cols, means, scales) -> torch.Tensor:
    X = frame.feature_matrix(cols).t().double()
    m = torch.from_numpy(means).to(X.device)
    s = torch.from_numpy(scales).to(X.device)
    X = torch.where(torch.isnan(X), m[None, :], X)
    return (X - m[None, :]) / s[None, :]


class H2OSupportVectorMachineEstimator(ModelBuilder):
    algo = "psvm"
    DEFAULTS = dict(hyper_param=1.0, kernel_type="gaussian", gamma=-1.0, rank_ratio=-1.0, positive_weight=1.0,
                    negative_weight=1.0, disable_training_metrics=True, sv_threshold=1e-4, fact_threshold=1e-5,
                    feasible_threshold=1e-3, surrogate_gap_threshold=1e-3, mu_factor=10.0, max_iterations=200,
                    standardize=True)

    def _fit(self, train: Frame, valid, model_id):
        if self.category != ModelCategory.BINOMIAL:
            raise ValueError("psvm: binary classification only")
        if str(self.params["kernel_type"]).lower() != "gaussian":
            raise ValueError("psvm: only kernel_type='gaussian' is supported (as in H2O)")
        p_ = self.params
        comm = self.comm
        yc = train.vec(self.y).data
        ok = yc >= 0
        Xall = train.feature_matrix(self.x).t().double()
        X, ycodes = Xall[ok], yc[ok]
        # standardisation statistics over all ranks (NA -> mean)
        Xz = torch.nan_to_num(X, nan=0.0)
        cnt = (~torch.isnan(X)).double()
        st = _allsum(torch.stack([Xz.sum(0), (Xz * Xz).sum(0), cnt.sum(0)]), comm)
        means = (st[0] / st[2].clamp_min(1)).cpu().numpy()
        var = (st[1] / st[2].clamp_min(1)).cpu().numpy() - means ** 2
        scales = np.sqrt(np.maximum(var, 1e-24)) if p_.get("standardize", True) else np.ones_like(means)
        m_t = torch.from_numpy(means).to(X.device)[None, :]
        X = (torch.where(torch.isnan(X), m_t, X) - m_t) / torch.from_numpy(scales).to(X.device)[None, :]
        n = X.shape[0]
        N = int(_allsum(torch.tensor([float(n)], dtype=torch.float64, device=X.device), comm)[0])
        d = X.shape[1]
        gamma = float(p_["gamma"]) if float(p_["gamma"]) > 0 else 1.0 / max(d, 1)
        rr = float(p_["rank_ratio"])
        p = int(math.ceil(math.sqrt(N))) if rr <= 0 else max(1, int(math.ceil(rr * N)))
        p = min(p, N)
        H = icf(X, gamma, p, float(p_["fact_threshold"]), comm)
        y = torch.where(ycodes == 1, 1.0, -1.0).double().to(X.device)
        C = float(p_["hyper_param"]) * torch.where(y > 0, float(p_["positive_weight"]),
                                                   float(p_["negative_weight"])).double()
        alpha, b, iters = self._ipm(H, y, C, comm)
        thr = float(p_["sv_threshold"])
        sv = alpha > thr
        free = sv & (alpha < C - thr)
        # b from the free support vectors (exact kernel values through the low-rank factor)
        Hy = H * y[:, None]
        Qa_over_y = H @ (_allsum(Hy.t() @ alpha, comm))            # sum_j a_j y_j K_ij
        bs = _allsum(torch.stack([(y - Qa_over_y)[free].sum(), free.double().sum()]), comm)
        if float(bs[1]) > 0:
            b = float(bs[0] / bs[1])
        sv_x = X[sv].float()
        coef = (alpha * y)[sv]
        if comm is not None and comm.world_size > 1:
            sv_x = comm.all_gather_cat(sv_x)
            coef = comm.all_gather_cat(coef)
        model = PSVMModel(self, model_id, sv_x.cpu(), coef.cpu(), b, gamma, means, scales)
        model.timings = {"ipm_iterations": iters, "icf_rank": int(H.shape[1]),
                         "bounded_sv": int(_allsum(torch.tensor([float((alpha >= C - thr).sum())],
                                                               dtype=torch.float64, device=X.device), comm)[0])}
        return model

    def _ipm(self, H, y, C, comm):
        p_ = self.params
        n, k = H.shape
        dev = H.device
        Hy = H * y[:, None]
        mu_f = float(p_["mu_factor"])
        alpha = C / 10.0
        lam = torch.ones(n, dtype=torch.float64, device=dev)     # multipliers of a >= 0
        xi = torch.ones(n, dtype=torch.float64, device=dev)      # multipliers of a <= C
        nu = 0.0
        N = float(_allsum(torch.tensor([float(n)], dtype=torch.float64, device=dev), comm)[0])
        it = 0
        for it in range(1, int(p_["max_iterations"]) + 1):
            Qa = Hy @ _allsum(Hy.t() @ alpha, comm)
            gap_v = _allsum(torch.stack([(lam * alpha).sum() + (xi * (C - alpha)).sum(), (y * alpha).sum()]), comm)
            gap, ya = float(gap_v[0]), float(gap_v[1])
            rd = Qa - 1.0 + nu * y - lam + xi
            rd_n = float(_allsum(torch.stack([(rd * rd).sum()]), comm)[0])
            if gap < float(p_["surrogate_gap_threshold"]) and math.sqrt(rd_n / N) < float(p_["feasible_threshold"]) \
                    and abs(ya) / N < float(p_["feasible_threshold"]):
                break
            mu = gap / N / mu_f
            z = -Qa + 1.0 - nu * y + mu / alpha - mu / (C - alpha)
            Dg = lam / alpha + xi / (C - alpha)
            # (Dg + Hy Hy^T)^-1 via Sherman-Morrison-Woodbury; M = I + Hy^T Dg^-1 Hy
            Hd = Hy / Dg[:, None]
            M = _allsum(Hy.t() @ Hd, comm)
            M += torch.eye(k, dtype=torch.float64, device=dev)
            L = torch.linalg.cholesky(M)

            def solve(v):
                t = _allsum(Hd.t() @ v, comm)
                return v / Dg - Hd @ torch.cholesky_solve(t[:, None], L)[:, 0]

            Sz, Sy = solve(z), solve(y)
            s = _allsum(torch.stack([(y * Sz).sum(), (y * Sy).sum()]), comm)
            dnu = (float(s[0]) + ya) / float(s[1])
            da = Sz - dnu * Sy
            dl = (mu - lam * alpha - lam * da) / alpha
            dx = (mu - xi * (C - alpha) + xi * da) / (C - alpha)
            # fraction-to-the-boundary step keeping 0 < a < C and lam, xi > 0
            steps = [torch.where(da < 0, -alpha / da, torch.full_like(da, math.inf)),
                     torch.where(da > 0, (C - alpha) / da, torch.full_like(da, math.inf)),
                     torch.where(dl < 0, -lam / dl, torch.full_like(dl, math.inf)),
                     torch.where(dx < 0, -xi / dx, torch.full_like(dx, math.inf))]
            smax = torch.stack([t.min() if t.numel() else torch.tensor(math.inf, device=dev) for t in steps]).min()
            if comm is not None and comm.world_size > 1:
                smax = torch.tensor([float(smax)], dtype=torch.float64, device=dev)
                comm.all_reduce_(smax, "min")
                smax = smax[0]
            step = min(1.0, 0.99 * float(smax))
            alpha = alpha + step * da
            lam = lam + step * dl
            xi = xi + step * dx
            nu = nu + step * dnu
        return alpha, nu, it           # free SVs: b = y_i - sum_j a_j y_j K_ij = nu
