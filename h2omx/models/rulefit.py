"""RuleFit (H2O ``H2ORuleFitEstimator``; Friedman & Popescu 2008).

1. Rule generation: for every depth in [min_rule_length, max_rule_length]
   an ensemble of ``rule_generation_ntrees`` trees (DRF by default, or GBM)
   is trained on the HIP tree engine; every non-root node of every tree is a
   rule = the conjunction of the split conditions on its path.
2. Rule features: rows walk each tree once (device gathers) and every node
   they pass sets its rule indicator.  Linear terms (``model_type`` with
   LINEAR) are the numeric predictors winsorised at the 2.5 / 97.5 %
   quantiles, scaled by 0.4 / sd like the paper.
3. Sparse fit: an L1-penalised GLM (gaussian, or binomial via IRLS) on the
   standardised [rules | linear] design, solved by coordinate descent on the
   weighted Gram, which is ONE matrix-core GEMM per IRLS step over all rows
   (ops.dense.gemm, all-reduced across ranks).  ``lambda_`` (default
   λmax / 100) or, with ``max_num_rules`` > 0, the smallest λ on a
   20-point path that keeps at most that many rules.
4. ``rule_importance()``: rule, coefficient (original scale), support and
   importance |β| sqrt(s (1 − s)) (linear terms: |β| sd).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory


def _rules_from_ensemble(ens, names, types, domains):
    """[(tree index, node, text)] for every non-root reachable node."""
    out = []
    for t in range(ens.trees.shape[0]):
        tr = ens.trees[t]
        stack = [(0, [])]
        while stack:
            i, conds = stack.pop()
            if i != 0:
                out.append((t, i, " & ".join(conds)))
            if tr[i]["feat"] >= 0:
                f = int(tr[i]["feat"])
                thr = float(tr[i]["thr"])
                nal = bool(int(tr[i]["na_left"]) & 1)
                c = names[f]
                cb = getattr(ens, "catbits", None)
                if (int(tr[i]["na_left"]) & 2) and cb is not None:
                    from .tree.structs import bitset_has

                    dom = domains.get(c) or []
                    inl = bitset_has(cb[t][i], np.arange(len(dom)))
                    left = [d for k, d in enumerate(dom) if inl[k]]
                    right = [d for k, d in enumerate(dom) if not inl[k]]
                    lt = f"({c} in {{{', '.join(left)}}}{' or NA' if nal else ''})"
                    rt = f"({c} in {{{', '.join(right)}}}{'' if nal else ' or NA'})"
                elif types.get(c) == ENUM:
                    dom = domains.get(c) or []
                    left = [d for k, d in enumerate(dom) if k <= thr]
                    right = [d for k, d in enumerate(dom) if k > thr]
                    lt = f"({c} in {{{', '.join(left)}}}{' or NA' if nal else ''})"
                    rt = f"({c} in {{{', '.join(right)}}}{'' if nal else ' or NA'})"
                else:
                    lt = f"({c} <= {thr:.6g}{' or NA' if nal else ''})"
                    rt = f"({c} > {thr:.6g}{'' if nal else ' or NA'})"
                L = int(tr[i]["left"])
                stack.append((L + 1, conds + [rt]))
                stack.append((L, conds + [lt]))
    return out


def _rule_matrix(ens, rules, X: torch.Tensor) -> torch.Tensor:
    """Indicator matrix [n][R] (float32) of the rules for feature-major X [F][n]."""
    n = X.shape[1]
    dev = X.device
    R = torch.zeros((n, len(rules)), dtype=torch.float32, device=dev)
    col_of = {(t, i): k for k, (t, i, _) in enumerate(rules)}
    for t in range(ens.trees.shape[0]):
        tr = ens.trees[t]
        cap = tr.shape[0]
        from .tree.structs import TreeWalker

        cbt = getattr(ens, "catbits", None)
        tw = TreeWalker(tr, None if cbt is None else cbt[t], dev)
        feat, left = tw.feat, tw.left
        cmap = torch.full((cap,), -1, dtype=torch.long, device=dev)
        for (tt, i), k in col_of.items():
            if tt == t:
                cmap[i] = k
        node = torch.zeros(n, dtype=torch.long, device=dev)
        rows = torch.arange(n, device=dev)
        for _ in range(64):
            f = feat[node]
            inner = f >= 0
            if not bool(inner.any()):
                break
            x = X[f.clamp_min(0), rows]
            go_left = tw.go_left(node, x)
            child = torch.where(go_left, left[node], left[node] + 1)
            node = torch.where(inner, child, node)
            k = cmap[node]
            hit = inner & (k >= 0)
            R[rows[hit], k[hit]] = 1.0
    return R


def _cd_lasso(G: np.ndarray, b: np.ndarray, lam: float, beta0: np.ndarray, iters: int = 500, tol: float = 1e-8):
    """argmin 1/2 βᵀGβ − bᵀβ + lam |β|_1 by cyclic coordinate descent (G = XᵀWX / N),
    in the native covariance-update solver (csrc/host/solvers.cpp)."""
    from .glm import _enet_cd

    beta = np.ascontiguousarray(beta0, np.float64).copy()
    _enet_cd(np.ascontiguousarray(G, np.float64), np.ascontiguousarray(b, np.float64), np.zeros(beta.size), lam, -1,
             False, beta, iters, tol)
    return beta


class RuleFitModel(Model):
    algo = "rulefit"
    algo_full_name = "RuleFit"

    def __init__(self, builder, model_id, ensembles, rules, lin_cols, lin_params, mu, sd, beta, intercept):
        super().__init__(builder, model_id)
        self.ensembles = ensembles      # [(TreeEnsemble, rule list)]
        self.rules = rules              # [text]
        self.lin_cols = lin_cols
        self.lin_params = lin_params    # [(lo, hi, scale)]
        self.mu, self.sd = mu, sd
        self.beta = beta                # on standardised columns
        self.intercept = intercept

    def design(self, frame: Frame) -> torch.Tensor:
        X = frame.feature_matrix(self.x)
        parts = [_rule_matrix(ens, rl, X) for ens, rl in self.ensembles if rl]
        for c, (lo, hi, sc) in zip(self.lin_cols, self.lin_params):
            v = frame.vec(c).as_float()
            v = torch.where(torch.isnan(v), torch.full_like(v, 0.5 * (lo + hi)), v)
            parts.append((v.clamp(lo, hi) * sc)[:, None])
        return torch.cat(parts, 1) if parts else torch.zeros((frame.nrows, 0), device=frame.device)

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        Z = self.design(frame).double()
        mu = torch.from_numpy(self.mu).to(Z.device)
        sd = torch.from_numpy(self.sd).to(Z.device)
        eta = ((Z - mu) / sd) @ torch.from_numpy(self.beta).to(Z.device) + self.intercept
        if self.category == ModelCategory.BINOMIAL:
            p1 = torch.sigmoid(eta).float()
            return torch.stack([1 - p1, p1])
        return eta.float()[None, :]

    def rule_importance(self):
        names = self.rules + [f"linear.{c}" for c in self.lin_cols]
        coef = self.beta / self.sd
        out = []
        for j in np.nonzero(self.beta)[0]:
            if j < len(self.rules):
                s = float(self.mu[j])
                imp = abs(coef[j]) * math.sqrt(max(s * (1 - s), 0.0))
            else:
                s = float("nan")
                imp = abs(coef[j]) * float(self.sd[j])
            out.append({"variable": names[j], "coefficient": float(coef[j]), "support": s, "importance": imp})
        return sorted(out, key=lambda r: -r["importance"])

    def varimp(self):
        imp = np.zeros(len(self.x))
        for r in self.rule_importance():
            for i, c in enumerate(self.x):
                if f"({c} " in r["variable"] or r["variable"] == f"linear.{c}":
                    imp[i] += r["importance"]
        if imp.max() <= 0:
            return [(c, 0.0, 0.0, 0.0) for c in self.x]
        order = np.argsort(-imp)
        return [(self.x[i], float(imp[i]), float(imp[i] / imp.max()), float(imp[i] / imp.sum())) for i in order]

    def summary(self):
        return {"model_id": self.model_id, "rules": len(self.rules), "nonzero": int(np.count_nonzero(self.beta))}

    def to_json(self):
        j = super().to_json()
        j["output"]["rule_importance"] = self.rule_importance()
        return j


class H2ORuleFitEstimator(ModelBuilder):
    algo = "rulefit"
    DEFAULTS = dict(algorithm="AUTO", min_rule_length=3, max_rule_length=3, max_num_rules=-1,
                    model_type="RULES_AND_LINEAR", rule_generation_ntrees=50, remove_duplicates=True,
                    lambda_=None, max_categorical_levels=10)

    def _fit(self, train: Frame, valid, model_id):
        from .tree_models import H2OGradientBoostingEstimator, H2ORandomForestEstimator

        p_ = self.params
        if self.category == ModelCategory.MULTINOMIAL:
            raise ValueError("rulefit supports binomial and regression responses")
        comm = self.comm
        mt = str(p_["model_type"]).upper()
        if mt not in ("RULES_AND_LINEAR", "RULES", "LINEAR"):
            raise ValueError(f"rulefit: model_type {p_['model_type']!r}")
        algo = str(p_["algorithm"]).upper()
        seed = self._seed()
        ensembles, rule_text = [], []
        if mt != "LINEAR":
            lo, hi = int(p_["min_rule_length"]), int(p_["max_rule_length"])
            if not 1 <= lo <= hi:
                raise ValueError("rulefit: need 1 <= min_rule_length <= max_rule_length")
            seen = set()
            for depth in range(lo, hi + 1):
                kw = dict(ntrees=int(p_["rule_generation_ntrees"]), max_depth=depth, seed=seed + depth)
                est = (H2OGradientBoostingEstimator(learn_rate=0.1, **kw) if algo == "GBM"
                       else H2ORandomForestEstimator(**kw))
                m = est.train(x=self.x, y=self.y, training_frame=train, comm=comm)
                rl = _rules_from_ensemble(m.ens, self.x, self.feature_types, self.feature_domains)
                if p_["remove_duplicates"]:
                    rl = [r for r in rl if not (r[2] in seen or seen.add(r[2]))]
                ensembles.append((m.ens, [(t, i, txt) for t, i, txt in rl]))
                rule_text += [txt for _, _, txt in rl]
        lin_cols, lin_params = [], []
        if mt != "RULES":
            for c in self.x:
                if self.feature_types[c] == ENUM:
                    continue
                v = train.vec(c).as_float()
                v = v[~torch.isnan(v)]
                if v.numel() == 0:
                    continue
                lo_q, hi_q = (float(q) for q in torch.quantile(v.double()[: 1 << 24], torch.tensor(
                    [0.025, 0.975], dtype=torch.float64, device=v.device)))
                sd = float(v.clamp(lo_q, hi_q).double().std()) or 1.0
                lin_cols.append(c)
                lin_params.append((lo_q, hi_q, 0.4 / sd))
        model = RuleFitModel(self, model_id, ensembles, rule_text, lin_cols, lin_params, None, None, None, 0.0)
        Z = model.design(train).double()                                 # [n][q]
        y = train.vec(self.y)
        yv = (y.data == 1).double() if self.category == ModelCategory.BINOMIAL else y.as_float().double()
        ok = ~torch.isnan(yv)
        Z, yv = Z[ok], yv[ok]
        q = Z.shape[1]
        st = torch.cat([Z.sum(0), (Z * Z).sum(0), torch.tensor([float(Z.shape[0])], dtype=torch.float64,
                                                                device=Z.device)])
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(st)
        N = float(st[-1])
        mu = (st[:q] / N).cpu().numpy()
        sd = np.sqrt(np.maximum((st[q:2 * q] / N).cpu().numpy() - mu ** 2, 0.0))
        sd = np.where(sd > 1e-12, sd, 1.0)
        Zs = ((Z - torch.from_numpy(mu).to(Z.device)) / torch.from_numpy(sd).to(Z.device)).float().contiguous()
        beta, b0 = self._lasso(Zs, yv, N, comm)
        model.mu, model.sd, model.beta, model.intercept = mu, sd, beta, b0
        # keep only the ensembles' rules that survived (scoring cost)
        return model

    def _lasso(self, Zs: torch.Tensor, y: torch.Tensor, N: float, comm):
        p_ = self.params
        q = Zs.shape[1]
        binom = self.category == ModelCategory.BINOMIAL

        def allr(t):
            if comm is not None and comm.world_size > 1:
                comm.all_reduce_(t)
            return t

        def gram(w):
            # [X | 1]ᵀ W [X | 1 | z-part] through one fp32 GEMM (feature-major)
            A = torch.cat([Zs, torch.ones((Zs.shape[0], 1), device=Zs.device)], 1)
            Aw = (A * w[:, None].float()).T.contiguous()
            return allr(D.gemm(Aw, A).double())

        if not binom:
            ybar = float(allr(y.sum().reshape(1))[0]) / N
            r = (y - ybar).float()
            b = allr(D.gemm(Zs.T.contiguous(), r[:, None].contiguous()).double()[:, 0]) / N
            G = allr(D.gemm(Zs.T.contiguous(), Zs).double()) / N
            Gn, bn = G.cpu().numpy(), b.cpu().numpy()
            beta = self._path(Gn, bn, q)
            return beta, ybar
        # binomial: IRLS with an L1 penalty on the standardised rule/linear columns
        beta = np.zeros(q)
        b0 = 0.0
        ybar = float(allr(y.sum().reshape(1))[0]) / N
        b0 = math.log(max(ybar, 1e-6) / max(1 - ybar, 1e-6))
        for _ in range(25):
            eta = Zs.double() @ torch.from_numpy(beta).to(Zs.device) + b0
            pr = torch.sigmoid(eta)
            w = (pr * (1 - pr)).clamp_min(1e-6)
            z = eta + (y - pr) / w
            GA = gram(w) / N                                              # [(q+1)][(q+1)]
            rhs = allr(D.gemm(torch.cat([Zs, torch.ones((Zs.shape[0], 1), device=Zs.device)], 1).T.contiguous(),
                              (w * z).float()[:, None].contiguous()).double()[:, 0]) / N
            Gn, bn = GA.cpu().numpy(), rhs.cpu().numpy()
            # profile out the unpenalised intercept: centre with the weighted means
            sw = Gn[q, q]
            m = Gn[:q, q] / sw
            Gc = Gn[:q, :q] - np.outer(m, Gn[q, :q])
            bc = bn[:q] - m * bn[q]
            new = self._path(Gc, bc, q, warm=beta)
            nb0 = (bn[q] - Gn[q, :q] @ new) / sw
            done = np.max(np.abs(new - beta)) < 1e-6 and abs(nb0 - b0) < 1e-6
            beta, b0 = new, nb0
            if done:
                break
        return beta, float(b0)

    def _path(self, G, b, q, warm=None):
        p_ = self.params
        lam_max = float(np.max(np.abs(b))) if q else 0.0
        if p_.get("lambda_") is not None:
            lam = p_["lambda_"]
            lam = float(lam[0] if isinstance(lam, (list, tuple)) else lam)
            return _cd_lasso(G, b, lam, np.zeros(q) if warm is None else warm)
        cap = int(p_["max_num_rules"])
        if cap <= 0:
            return _cd_lasso(G, b, lam_max / 100.0, np.zeros(q) if warm is None else warm)
        beta = np.zeros(q)
        best = beta
        for lam in lam_max * np.logspace(0, -3, 20):
            beta = _cd_lasso(G, b, lam, beta)
            if np.count_nonzero(beta) > cap:
                break
            best = beta.copy()
        return best
