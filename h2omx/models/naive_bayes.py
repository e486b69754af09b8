"""Naive Bayes (H2O NaiveBayes equivalent).

Classification only.  Per class c: prior P(c) = n_c / n; categorical
predictors get conditional tables (count(x=j, c) + laplace) /
(n_c + laplace · levels); numeric predictors a Gaussian with the class
mean and standard deviation (``sd <= eps_sdev`` is replaced by
``min_sdev``).  Scoring multiplies the per-feature likelihoods in log
space, skipping NA features; probabilities ``<= eps_prob`` are replaced
by ``min_prob``.

All statistics are device-resident scatter sums (one all-reduce of the
packed class tables across ranks); scoring is one fused pass per class.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame
from .base import Model, ModelBuilder, ModelCategory


class NaiveBayesModel(Model):
    algo = "naivebayes"
    algo_full_name = "Naive Bayes"

    def __init__(self, builder, model_id, prior, tables, gauss):
        super().__init__(builder, model_id)
        self.prior = prior              # [K]
        self.tables = tables            # {col: [K][levels] conditional probabilities}
        self.gauss = gauss              # {col: ([K] mean, [K] sd)}

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        p = self.params
        min_prob, eps_prob = float(p["min_prob"]), float(p["eps_prob"])
        K = len(self.prior)
        n = frame.nrows
        dev = frame.device
        logp = torch.log(torch.from_numpy(np.maximum(self.prior, 1e-300)).to(dev))[:, None].expand(K, n).clone()
        for c in self.x:
            v = frame.vec(c)
            if c in self.tables:
                T = torch.from_numpy(self.tables[c]).to(dev)              # [K][L]
                T = torch.where(T <= eps_prob, torch.full_like(T, min_prob), T)
                codes = v.data.long()
                ok = (codes >= 0) & (codes < T.shape[1])
                lp = torch.log(T[:, codes.clamp(0, T.shape[1] - 1)])        # [K][n]
                logp += torch.where(ok[None, :], lp, torch.zeros_like(lp))
            else:
                mu, sd = (torch.from_numpy(a).to(dev)[:, None] for a in self.gauss[c])
                x = v.as_float().double()[None, :]
                ok = ~torch.isnan(x)
                z = (x - mu) / sd
                dens = torch.exp(-0.5 * z * z) / (math.sqrt(2 * math.pi) * sd)
                dens = torch.where(dens <= eps_prob, torch.full_like(dens, min_prob), dens)
                logp += torch.where(ok, torch.log(dens), torch.zeros_like(dens))
        return torch.softmax(logp, 0).float()

    def summary(self):
        return {"model_id": self.model_id, "number_of_response_levels": len(self.prior),
                "min_apriori_probability": float(np.min(self.prior)),
                "max_apriori_probability": float(np.max(self.prior))}

    def to_json(self):
        j = super().to_json()
        out = j["output"]
        out["apriori"] = {"names": list(self.response_domain), "data": self.prior.tolist()}
        out["pcond"] = [{"name": c, "data": (self.tables[c].tolist() if c in self.tables else
                                            {"mean": self.gauss[c][0].tolist(), "sd": self.gauss[c][1].tolist()})}
                        for c in self.x]
        return j


class H2ONaiveBayesEstimator(ModelBuilder):
    algo = "naivebayes"
    DEFAULTS = dict(laplace=0.0, min_sdev=0.001, eps_sdev=0.0, min_prob=0.001, eps_prob=0.0, compute_metrics=True,
                    balance_classes=False)

    def _fit(self, train: Frame, valid, model_id):
        if self.category not in (ModelCategory.BINOMIAL, ModelCategory.MULTINOMIAL):
            raise ValueError("naivebayes: the response must be categorical")
        p_ = self.params
        comm = self.comm
        K = len(self.response_domain)
        y = train.vec(self.y).data.long()
        oky = y >= 0
        yk = y.clamp_min(0)
        dev = y.device
        parts, layout = [], []
        cnt = torch.zeros(K, dtype=torch.float64, device=dev).index_add_(0, yk, oky.double())
        parts.append(cnt.ravel())
        layout.append(("__count__", (K,)))
        for c in self.x:
            v = train.vec(c)
            if v.vtype == ENUM:
                L = len(v.domain or [])
                codes = v.data.long()
                ok = oky & (codes >= 0)
                t = torch.zeros(K * max(L, 1), dtype=torch.float64, device=dev)
                t.index_add_(0, yk * max(L, 1) + codes.clamp_min(0), ok.double())
                parts.append(t)
                layout.append((c, (K, max(L, 1))))
            else:
                x = v.as_float().double()
                ok = oky & ~torch.isnan(x)
                xz = torch.where(ok, x, torch.zeros_like(x))
                s = torch.zeros((3, K), dtype=torch.float64, device=dev)
                s[0].index_add_(0, yk, ok.double())
                s[1].index_add_(0, yk, xz)
                s[2].index_add_(0, yk, xz * xz)
                parts.append(s.ravel())
                layout.append((c, (3, K)))
        flat = torch.cat(parts)
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(flat)
        flat = flat.cpu().numpy()
        off = 0
        stats = {}
        for name, shape in layout:
            sz = int(np.prod(shape))
            stats[name] = flat[off: off + sz].reshape(shape)
            off += sz
        nc = stats.pop("__count__")
        prior = nc / max(nc.sum(), 1e-300)
        lap = float(p_["laplace"])
        tables, gauss = {}, {}
        for c in self.x:
            st = stats[c]
            if self.feature_types[c] == ENUM:
                L = st.shape[1]
                tables[c] = (st + lap) / np.maximum(st.sum(1, keepdims=True) + lap * L, 1e-300)
            else:
                m = st[0]
                mean = st[1] / np.maximum(m, 1)
                var = (st[2] - m * mean * mean) / np.maximum(m - 1, 1)
                sd = np.sqrt(np.maximum(var, 0.0))
                sd = np.where(sd <= float(p_["eps_sdev"]), float(p_["min_sdev"]), sd)
                gauss[c] = (mean, sd)
        return NaiveBayesModel(self, model_id, prior, tables, gauss)
