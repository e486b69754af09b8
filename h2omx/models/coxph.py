"""Cox Proportional Hazards (H2O ``H2OCoxProportionalHazardsEstimator``).

Newton-Raphson on the partial log-likelihood with Efron (default) or
Breslow handling of tied event times, optional counting-process data
(``start_column``), observation weights and ``stratify_by`` strata.  The
response ``y`` is the event indicator (0/1 or a two-level categorical),
``stop_column`` the event / censoring time.

Risk-set sums are computed for all distinct event times at once: rows are
sorted by stop time (descending) inside each stratum and the weighted sums
S0 = Σ w e^η, S1 = Σ w e^η x and S2 = Σ w e^η x xᵀ over the risk set come
from cumulative sums (minus the rows that entered after the time for
counting-process data), fp64, on the device that holds the frame.  Cox risk
sets couple every row of a stratum, so a multi-rank cluster all-gathers the
(time, event, weight, x) columns once and every rank runs the same solve.

Outputs: coefficients, exp(coef), se, z, p-values, log-likelihood (null
and final), likelihood-ratio / Wald statistics, Harrell's concordance and
``predict`` = linear predictor ``lp`` = (x − x̄)·β.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame, Vec
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo


def _event_sums(t, start, d, w, eta, X, strata, efron: bool):
    """Partial log-likelihood, gradient and Hessian (fp64)."""
    n, p = X.shape
    ll = torch.zeros((), dtype=torch.float64, device=X.device)
    grad = torch.zeros(p, dtype=torch.float64, device=X.device)
    hess = torch.zeros((p, p), dtype=torch.float64, device=X.device)
    for s in torch.unique(strata):
        sel = torch.nonzero(strata == s).flatten()
        ts, ds, ws, es, Xs = t[sel], d[sel], w[sel], eta[sel], X[sel]
        ss = start[sel] if start is not None else None
        r = ws * torch.exp(es)
        xr = Xs * r[:, None]
        xxr = Xs[:, :, None] * xr[:, None, :]
        # sort by stop time descending: cumulative sums = rows with stop >= time
        order = torch.argsort(ts, descending=True, stable=True)
        to = ts[order]
        c0 = torch.cumsum(r[order], 0)
        c1 = torch.cumsum(xr[order], 0)
        c2 = torch.cumsum(xxr[order], 0)
        ev = ds > 0
        if not bool(ev.any()):
            continue
        utimes = torch.unique(ts[ev])                          # ascending
        # last position (in descending order) with stop >= time
        pos = (to.numel() - torch.searchsorted(to.flip(0), utimes, right=False)) - 1
        S0, S1, S2 = c0[pos], c1[pos], c2[pos]
        if ss is not None:
            # remove rows that start at or after the event time (not yet at risk)
            o2 = torch.argsort(ss, descending=True, stable=True)
            so = ss[o2]
            e0 = torch.cumsum(r[o2], 0)
            e1 = torch.cumsum(xr[o2], 0)
            e2 = torch.cumsum(xxr[o2], 0)
            q = (so.numel() - torch.searchsorted(so.flip(0), utimes, right=False)) - 1
            has = q >= 0
            qq = q.clamp_min(0)
            S0 = S0 - torch.where(has, e0[qq], torch.zeros_like(S0))
            S1 = S1 - torch.where(has[:, None], e1[qq], torch.zeros_like(S1))
            S2 = S2 - torch.where(has[:, None, None], e2[qq], torch.zeros_like(S2))
        # tied events per distinct time
        ti = torch.searchsorted(utimes, ts[ev])
        U = utimes.numel()
        m = torch.zeros(U, dtype=torch.float64, device=X.device).index_add_(0, ti, torch.ones_like(ts[ev]))
        dw = torch.zeros(U, dtype=torch.float64, device=X.device).index_add_(0, ti, ws[ev])
        A0 = torch.zeros(U, dtype=torch.float64, device=X.device).index_add_(0, ti, r[ev])
        A1 = torch.zeros((U, p), dtype=torch.float64, device=X.device).index_add_(0, ti, xr[ev])
        A2 = torch.zeros((U, p, p), dtype=torch.float64, device=X.device).index_add_(0, ti, xxr[ev])
        ll = ll + (ws[ev] * es[ev]).sum()
        grad = grad + (ws[ev][:, None] * Xs[ev]).sum(0)
        mmax = int(m.max()) if efron else 1
        wbar = dw / m
        for k in range(mmax):
            if efron:
                act = m > k
                f = torch.where(act, k / m, torch.zeros_like(m))
                scale = torch.where(act, wbar, torch.zeros_like(m))
            else:
                f = torch.zeros_like(m)
                scale = dw
            phi0 = S0 - f * A0
            phi1 = S1 - f[:, None] * A1
            phi2 = S2 - f[:, None, None] * A2
            ok = scale > 0
            phi0s = torch.where(ok, phi0, torch.ones_like(phi0))
            ll = ll - (scale * torch.log(phi0s) * ok).sum()
            mu = phi1 / phi0s[:, None]
            grad = grad - (scale[:, None] * mu * ok[:, None]).sum(0)
            hess = hess - ((scale * ok)[:, None, None] * (phi2 / phi0s[:, None, None]
                                                          - mu[:, :, None] * mu[:, None, :])).sum(0)
    return ll, grad, hess


def concordance(t, d, lp, chunk: int = 2048) -> float:
    """Harrell's C: over comparable pairs (i event, t_j > t_i), P(lp_i > lp_j); ties count 1/2."""
    ev = torch.nonzero(d > 0).flatten()
    conc = torch.zeros((), dtype=torch.float64, device=t.device)
    tot = torch.zeros((), dtype=torch.float64, device=t.device)
    for c0 in range(0, ev.numel(), chunk):
        e = ev[c0:c0 + chunk]
        comp = t[None, :] > t[e][:, None]
        gt = (lp[e][:, None] > lp[None, :]) & comp
        eq = (lp[e][:, None] == lp[None, :]) & comp
        conc = conc + gt.sum() + 0.5 * eq.sum()
        tot = tot + comp.sum()
    return float(conc / tot) if float(tot) > 0 else float("nan")


class CoxPHModel(Model):
    algo = "coxph"
    algo_full_name = "Cox Proportional Hazards"

    def __init__(self, builder, model_id, design, beta, cov, x_mean, stats):
        super().__init__(builder, model_id)
        self.design = design
        self.beta = beta
        self.cov = cov
        self.x_mean = x_mean
        self.stats = stats
        se = np.sqrt(np.maximum(np.diag(cov), 0.0))
        z = np.where(se > 0, beta / np.where(se > 0, se, 1.0), np.nan)
        from scipy.stats import norm

        self.coefficients_table = {
            "names": list(design.names), "coefficients": beta.tolist(), "exp_coef": np.exp(beta).tolist(),
            "exp_negative_coef": np.exp(-beta).tolist(), "se_coef": se.tolist(), "z_coef": z.tolist(),
            "p_value": (2 * norm.sf(np.abs(z))).tolist()}

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        X = self.design.raw_matrix(frame).double()
        dev = X.device
        mu = torch.from_numpy(self.x_mean).to(dev)[:, None]
        X = torch.where(torch.isnan(X), mu.expand_as(X), X)
        b = torch.from_numpy(self.beta).to(dev)
        return ((X - mu) * b[:, None]).sum(0).float()[None, :]

    def predict(self, frame: Frame) -> Frame:
        return Frame([Vec("lp", self.predict_raw(frame)[0], "real")])

    def model_performance(self, frame=None):
        return self.training_metrics

    def coef(self):
        return dict(zip(self.design.names, self.beta.tolist()))

    def summary(self):
        return {"model_id": self.model_id, **self.stats}

    def to_json(self):
        j = super().to_json()
        j["output"]["coefficients_table"] = self.coefficients_table
        j["output"].update({k: v for k, v in self.stats.items()})
        j["output"]["var_coef"] = self.cov.tolist()
        return j


class H2OCoxProportionalHazardsEstimator(ModelBuilder):
    algo = "coxph"
    DEFAULTS = dict(start_column=None, stop_column=None, stratify_by=None, ties="efron", init=0.0, lre_min=9.0,
                    max_iterations=20, use_all_factor_levels=False, interactions=None, single_node_mode=False)

    def _resolve_columns(self, frame, x, y):
        x, y = super()._resolve_columns(frame, x, y)
        skip = {self.params.get("start_column"), self.params.get("stop_column")}
        skip |= set(self.params.get("stratify_by") or [])
        return [c for c in x if c not in skip], y

    def _response_category(self, frame, y):
        return ModelCategory.REGRESSION, None

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        if not p_.get("stop_column"):
            raise ValueError("coxph: stop_column is required")
        ties = str(p_["ties"]).lower()
        if ties not in ("efron", "breslow"):
            raise ValueError("coxph: ties must be 'efron' or 'breslow'")
        comm = self.comm
        yv = train.vec(self.y)
        d = (yv.data == 1).double() if yv.vtype == ENUM else yv.as_float().double()
        t = train.vec(p_["stop_column"]).as_float().double()
        start = train.vec(p_["start_column"]).as_float().double() if p_.get("start_column") else None
        w = (train.vec(p_["weights_column"]).as_float().double() if p_.get("weights_column")
             else torch.ones_like(t))
        strata_cols = list(p_.get("stratify_by") or [])
        strata = torch.zeros_like(t, dtype=torch.long)
        for c in strata_cols:
            v = train.vec(c)
            code = v.data.long() if v.vtype == ENUM else torch.unique(v.as_float(), return_inverse=True)[1]
            strata = strata * 100003 + code
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, bool(p_["use_all_factor_levels"]))
        X = design.raw_matrix(train).double()
        ok = ~torch.isnan(t) & ~torch.isnan(d) & ~torch.isnan(X).any(0) & (w > 0)
        if start is not None:
            ok &= ~torch.isnan(start)
        cols = [t, d, w, strata.double()] + ([start] if start is not None else [])
        M = torch.cat([torch.stack(cols, 1), X.T], 1)[ok]
        if comm is not None and comm.world_size > 1:
            M = comm.all_gather_cat(M.contiguous())
        t, d, w, strata = M[:, 0], M[:, 1], M[:, 2], M[:, 3].long()
        off = 4
        if start is not None:
            start = M[:, 4]
            off = 5
        X = M[:, off:].contiguous()
        n, p = X.shape
        x_mean = ((X * w[:, None]).sum(0) / w.sum()).cpu().numpy()
        design.means = x_mean
        Xc = X - torch.from_numpy(x_mean).to(X.device)[None, :]
        beta = torch.full((p,), float(p_["init"]), dtype=torch.float64, device=X.device)
        efron = ties == "efron"
        ll0, _, _ = _event_sums(t, start, d, w, torch.zeros(n, dtype=torch.float64, device=X.device), Xc, strata,
                                efron)
        ll_prev = None
        it = 0
        for it in range(1, int(p_["max_iterations"]) + 1):
            ll, g, H = _event_sums(t, start, d, w, Xc @ beta, Xc, strata, efron)
            if ll_prev is not None and float(ll) < float(ll_prev) - 1e-10:
                # step halving on a decrease (R coxph)
                beta = 0.5 * (beta + beta_prev)
                continue
            step = torch.linalg.solve(-H + 1e-12 * torch.eye(p, dtype=torch.float64, device=X.device), g)
            beta_prev = beta
            beta = beta + step
            if ll_prev is not None:
                rel = abs(float(ll) - float(ll_prev)) / max(abs(float(ll)), 1e-12)
                if rel == 0 or -math.log10(rel + 1e-300) >= float(p_["lre_min"]):
                    beta = beta_prev
                    break
            ll_prev = ll
        ll, g, H = _event_sums(t, start, d, w, Xc @ beta, Xc, strata, efron)
        cov = torch.linalg.inv(-H).cpu().numpy()
        b = beta.cpu().numpy()
        lp = Xc @ beta
        stats = {"loglik": float(ll), "null_loglik": float(ll0), "iter": it, "n": int(n),
                 "total_event": int(float((d > 0).sum())), "likelihood_ratio_test": float(2 * (ll - ll0)),
                 "wald_test": float(b @ np.linalg.solve(cov, b)) if p else 0.0,
                 "concordance": concordance(t, d, lp), "ties": ties}
        model = CoxPHModel(self, model_id, design, b, cov, x_mean, stats)
        model.training_metrics = dict(stats)
        return model
