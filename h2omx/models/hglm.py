"""Hierarchical GLM (H2O ``H2OHGLMEstimator``): a Gaussian linear mixed
model with a random intercept and optional random slopes per level of
``group_column``:

    y = X beta + Z_g u_g + e,   u_g ~ N(0, T),   e ~ N(0, sigma^2 I)

It is fitted by maximum likelihood with EM for the variance components
(H2O's HGLM method), plus an exact generalised-least-squares beta step
(ECME), which converges much faster than plain EM on the fixed effects.
One iteration:
  beta    = (X^T V^-1 X)^-1 X^T V^-1 y, with V_g^-1 applied through
            Woodbury using the per-group X_g^T Z_g and Z_g^T y_g
  E-step, per group g:
      C_g = (Z_g^T Z_g / sigma^2 + T^-1)^-1
      u_g = C_g Z_g^T (y_g - X_g beta) / sigma^2
  M-step:
      sigma^2 = [sum ||y_g - X_g beta - Z_g u_g||^2 + tr(Z_g C_g Z_g^T)] / N
      T       = mean_g (u_g u_g^T + C_g)
Group statistics (Z^T Z, Z^T r, counts) are built by index_add on the device
and all-reduced across ranks, so a group may span shards.  The q x q solves
(q = 1 + #random slopes) are batched over groups; all of it is fp64 on the
device.  Prediction is X beta plus Z u_g
for groups seen in training, and X beta (population level) otherwise.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo


def _allsum(t, comm):
    if comm is not None and comm.world_size > 1:
        comm.all_reduce_(t)
    return t


class HGLMModel(Model):
    algo = "hglm"
    algo_full_name = "Hierarchical Generalized Linear Model"

    def __init__(self, builder, model_id, design, beta, ranef, T, sigma2, levels, rcols, rint, stats):
        super().__init__(builder, model_id)
        self.design = design
        self.beta = beta                # [p + 1] raw scale (intercept last)
        self.ranef = ranef              # [G][q]
        self.T = T
        self.sigma2 = sigma2
        self.levels = levels
        self.random_columns = rcols
        self.random_intercept = rint
        self.stats = stats

    def _Z(self, frame: Frame) -> torch.Tensor:
        cols = [frame.vec(c).as_float().double() for c in self.random_columns]
        if self.random_intercept:
            cols = [torch.ones(frame.nrows, dtype=torch.float64, device=frame.device)] + cols
        return torch.stack(cols, 1)

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        X = self.design.raw_matrix(frame).double()
        m = torch.from_numpy(np.asarray(self.design.means, np.float64)).to(X.device)[:, None]
        X = torch.where(torch.isnan(X), m.expand_as(X), X)
        b = torch.from_numpy(self.beta).to(X.device)
        fixed = b[:-1] @ X + b[-1]
        g = frame.vec(self.params["group_column"])
        dom = list(g.domain or [])
        pos = {s: i for i, s in enumerate(self.levels)}
        lut = torch.tensor([pos.get(s, -1) for s in dom] + [-1], dtype=torch.long, device=X.device)
        c = g.data.long()
        gi = lut[torch.where(c >= 0, c, torch.full_like(c, len(dom)))]
        U = torch.from_numpy(self.ranef).to(X.device)
        Z = torch.nan_to_num(self._Z(frame))
        rand = torch.where(gi >= 0, (Z * U[gi.clamp_min(0)]).sum(1), torch.zeros_like(fixed))
        return (fixed + rand)[None, :].float()

    def coef(self) -> dict:
        out = {"Intercept": float(self.beta[-1])}
        out.update({n: float(v) for n, v in zip(self.design.names, self.beta[:-1])})
        return out

    def coefs_random(self) -> dict:
        names = (["Intercept"] if self.random_intercept else []) + list(self.random_columns)
        return {lvl: dict(zip(names, map(float, self.ranef[i]))) for i, lvl in enumerate(self.levels)}

    def summary(self):
        return {"model_id": self.model_id, "sigma2": self.sigma2, "T": self.T.tolist(), **self.stats}

    def to_json(self):
        j = super().to_json()
        j["output"].update(coefficients=self.coef(), tau_e_var=self.sigma2, tau_u_var=self.T.tolist(),
                           ubeta=self.ranef.tolist(), group_levels=self.levels, log_likelihood=self.stats["loglik"])
        return j


class H2OHGLMEstimator(ModelBuilder):
    algo = "hglm"
    DEFAULTS = dict(family="gaussian", rand_family="gaussian", group_column=None, random_columns=None,
                    random_intercept=True, max_iterations=200, em_epsilon=1e-6, tau_e_var_init=0.0,
                    tau_u_var_init=0.0, initial_t_matrix=None, method="EM", standardize=False,
                    use_all_factor_levels=False, missing_values_handling="MeanImputation")

    def _resolve_columns(self, frame, x, y):
        x, y = super()._resolve_columns(frame, x, y)
        gc = self.params.get("group_column")
        return [c for c in x if c != gc], y

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        if str(p_["family"]).lower() != "gaussian":
            raise ValueError("hglm: family='gaussian' (H2O HGLM supports the gaussian family)")
        if self.category != ModelCategory.REGRESSION:
            raise ValueError("hglm: numeric response required")
        gc = p_["group_column"]
        if not gc or train.vec(gc).vtype != ENUM:
            raise ValueError("hglm: group_column must name a categorical column")
        comm = self.comm
        rcols = list(p_.get("random_columns") or [])
        rint = bool(p_["random_intercept"])
        if not rcols and not rint:
            raise ValueError("hglm: need random_columns and/or random_intercept")
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, bool(p_["use_all_factor_levels"]))
        Xraw = design.raw_matrix(train)
        y = train.vec(self.y).as_float().double()
        gv = train.vec(gc)
        levels = list(gv.domain or [])
        gidx = gv.data.long()
        ok = ~torch.isnan(y) & (gidx >= 0)
        design.fit_standardization(Xraw[:, ok], False, comm)
        m = torch.from_numpy(np.asarray(design.means, np.float64)).to(Xraw.device)[:, None]
        X = torch.where(torch.isnan(Xraw.double()), m.expand_as(Xraw).double(), Xraw.double())[:, ok]
        y, gidx = y[ok], gidx[ok]
        n = y.numel()
        dev = y.device
        Xa = torch.cat([X, torch.ones((1, n), dtype=torch.float64, device=dev)])      # [p+1][n]
        zc = [train.vec(c).as_float().double()[ok] for c in rcols]
        Z = torch.stack(([torch.ones(n, dtype=torch.float64, device=dev)] if rint else []) +
                        [torch.nan_to_num(c) for c in zc], 1)                          # [n][q]
        q = Z.shape[1]
        G = len(levels)
        # fixed-effect Gram (all ranks)
        XtX = _allsum(Xa @ Xa.T, comm)
        N = float(_allsum(torch.tensor([float(n)], dtype=torch.float64, device=dev), comm)[0])
        # per-group Z^T Z and counts
        ZZ = torch.zeros((G, q, q), dtype=torch.float64, device=dev)
        ZZ.index_add_(0, gidx, Z[:, :, None] * Z[:, None, :])
        _allsum(ZZ, comm)
        cnt = _allsum(torch.bincount(gidx, minlength=G).double(), comm)
        seen = cnt > 0
        beta = torch.linalg.solve(XtX, _allsum(Xa @ y, comm))
        r0 = y - beta @ Xa
        s2 = float(_allsum(torch.stack([(r0 * r0).sum()]), comm)[0]) / N
        sigma2 = float(p_["tau_e_var_init"]) if float(p_["tau_e_var_init"]) > 0 else 0.5 * s2
        if p_.get("initial_t_matrix") is not None:
            T = torch.tensor(np.asarray(p_["initial_t_matrix"], np.float64), device=dev)
        else:
            tu = float(p_["tau_u_var_init"]) if float(p_["tau_u_var_init"]) > 0 else 0.5 * s2
            T = torch.eye(q, dtype=torch.float64, device=dev) * tu
        eps = float(p_["em_epsilon"])
        # per-group cross products (constant over the iterations)
        XZ = torch.zeros((G, Xa.shape[0], q), dtype=torch.float64, device=dev)
        XZ.index_add_(0, gidx, Xa.T[:, :, None] * Z[:, None, :])
        _allsum(XZ, comm)
        Zy = _allsum(torch.zeros((G, q), dtype=torch.float64, device=dev).index_add_(0, gidx, Z * y[:, None]), comm)
        Xty = _allsum(Xa @ y, comm)
        it = 0
        ll = -math.inf
        U = torch.zeros((G, q), dtype=torch.float64, device=dev)
        for it in range(1, int(p_["max_iterations"]) + 1):
            Tinv = torch.linalg.inv(T)
            C = torch.linalg.inv(ZZ / sigma2 + Tinv[None])                               # [G][q][q] = M_g^-1
            # beta by generalised least squares given (T, sigma^2) (ECME): X^T V^-1 X and X^T V^-1 y
            # through Woodbury, V_g^-1 = (I - Z_g M_g^-1 Z_g^T / sigma^2) / sigma^2
            XZC = torch.einsum("gpi,gij->gpj", XZ, C)
            A = XtX / sigma2 - torch.einsum("gpj,gkj->pk", XZC, XZ) / sigma2 ** 2
            b = Xty / sigma2 - torch.einsum("gpj,gj->p", XZC, Zy) / sigma2 ** 2
            beta_new = torch.linalg.solve(A, b)
            # E-step for the random effects at the new beta
            r = y - beta_new @ Xa
            Zr = _allsum(torch.zeros((G, q), dtype=torch.float64, device=dev).index_add_(0, gidx, Z * r[:, None]),
                         comm)
            U = torch.einsum("gij,gj->gi", C, Zr) / sigma2
            U[~seen] = 0.0
            zu = (Z * U[gidx]).sum(1)
            res = r - zu
            trz = (ZZ * C).sum((1, 2))[seen].sum()
            sse = _allsum(torch.stack([(res * res).sum()]), comm)[0]
            sigma2_new = float((sse + trz) / N)
            Gs = float(seen.sum())
            T_new = (U[seen, :, None] * U[seen, None, :] + C[seen]).sum(0) / max(Gs, 1.0)
            ll_new = _loglik(y, Xa, Z, gidx, beta_new, T_new, sigma2_new, ZZ, cnt, G, comm)
            delta = max(float((beta_new - beta).abs().max()), abs(sigma2_new - sigma2), float((T_new - T).abs().max()))
            beta, sigma2, T = beta_new, sigma2_new, T_new
            done = abs(ll_new - ll) < eps * max(1.0, abs(ll_new)) and delta < math.sqrt(eps)
            ll = ll_new
            if done:
                break
        model = HGLMModel(self, model_id, design, beta.cpu().numpy(), U.cpu().numpy(), T.cpu().numpy(),
                          float(sigma2), levels, rcols, rint,
                          {"iterations": it, "loglik": ll, "icc": _icc(T, sigma2, rint)})
        return model


def _icc(T, sigma2, rint):
    if not rint:
        return None
    t00 = float(T[0, 0])
    return t00 / (t00 + sigma2)


def _loglik(y, Xa, Z, gidx, beta, T, sigma2, ZZ, cnt, G, comm):
    """Marginal Gaussian log-likelihood via the matrix determinant lemma and
    Woodbury identity per group (V_g = sigma^2 I + Z_g T Z_g^T)."""
    q = T.shape[0]
    r = y - beta @ Xa
    Zr = torch.zeros((G, q), dtype=torch.float64, device=y.device).index_add_(0, gidx, Z * r[:, None])
    rr = torch.zeros(G, dtype=torch.float64, device=y.device).index_add_(0, gidx, r * r)
    _allsum(Zr, comm)
    _allsum(rr, comm)
    seen = cnt > 0
    Tinv = torch.linalg.inv(T)
    M = Tinv[None] + ZZ / sigma2                                                        # [G][q][q]
    sol = torch.linalg.solve(M, Zr[:, :, None])[:, :, 0]
    quad = rr / sigma2 - (Zr * sol).sum(1) / sigma2 ** 2
    logdet = cnt * math.log(sigma2) + torch.logdet(M) + torch.logdet(T)
    N = float(cnt.sum())
    return float(-0.5 * (N * math.log(2 * math.pi) + (logdet + quad)[seen].sum()))
