"""Model Selection (H2O ``H2OModelSelectionEstimator``) and ANOVA GLM
(H2O ``H2OANOVAGLMEstimator``).

ModelSelection, gaussian responses: the augmented Gram [x | 1 | y]ᵀ[x | 1 | y]
of ALL predictors is formed once (the fp32 MFMA IRLS-Gram kernel,
ops.dense.glm_irls_pass, all-reduced across ranks); every candidate subset
is then an exact least-squares solve on a sub-block of that Gram, so the
search never touches the rows again.  Modes: ``forward`` / ``backward``
(add / drop the predictor that changes R² most), ``maxr`` (forward steps
followed by pairwise replacements until R² stops improving — the H2O
"maximum R² improvement" sequential replacement) and ``allsubsets``
(exhaustive, up to ``max_predictor_number``).  For each subset size the best
subset gets a regular GLM (lambda 0) so coefficients, p-values and scoring
work as usual; ``result()`` lists size, R², predictors and model ids.

ANOVAGLM: type-III tests of every main effect and (numeric) interaction up
to ``highest_interaction_term``: the full GLM is refit without each term and
the deviance difference is reported with its degrees of freedom and a
chi-square (binomial / poisson) or F (gaussian and others) p-value.
"""
from __future__ import annotations

import itertools

import numpy as np
import torch

from ..frame.frame import DKV, ENUM, Frame, Vec
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo, H2OGeneralizedLinearEstimator


def _r2(G: np.ndarray, cols: list, p: int, tss: float) -> float:
    """R² of y ~ 1 + x[cols] from the augmented Gram (index p = intercept, p+1 = y)."""
    idx = list(cols) + [p]
    A = G[np.ix_(idx, idx)]
    b = G[idx, p + 1]
    try:
        beta = np.linalg.solve(A + 1e-10 * np.eye(len(idx)) * max(1.0, np.abs(A).max()), b)
    except np.linalg.LinAlgError:
        beta = np.linalg.lstsq(A, b, rcond=None)[0]
    rss = G[p + 1, p + 1] - 2 * beta @ b + beta @ A @ beta
    return 1.0 - rss / tss if tss > 0 else 0.0


class ModelSelectionModel(Model):
    algo = "modelselection"
    algo_full_name = "Model Selection"

    def __init__(self, builder, model_id, rows, models):
        super().__init__(builder, model_id)
        self.rows = rows        # [{size, r2, predictors, model_id}]
        self.models = models

    def result(self) -> list[dict]:
        return [dict(r) for r in self.rows]

    def get_best_model_predictors(self):
        return [r["predictors"] for r in self.rows]

    def get_best_r2_values(self):
        return [r["best_r2_value"] for r in self.rows]

    def coef(self, predictor_size: int | None = None):
        if predictor_size is None:
            return [m.coef() for m in self.models]
        return self.models[predictor_size - 1 - (self.rows[0]["size"] - 1)].coef()

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        return self.models[-1].predict_raw(frame)

    def summary(self):
        return {"model_id": self.model_id, "result": self.result()}

    def to_json(self):
        j = super().to_json()
        j["output"]["result"] = self.result()
        return j


class H2OModelSelectionEstimator(ModelBuilder):
    algo = "modelselection"
    DEFAULTS = dict(mode="maxr", max_predictor_number=1, min_predictor_number=1, family="gaussian",
                    standardize=True, intercept=True, lambda_=0.0, nparallelism=0, p_values_threshold=0.0)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        mode = str(p_["mode"]).lower()
        if mode not in ("maxr", "maxrsweep", "forward", "backward", "allsubsets"):
            raise ValueError(f"modelselection: mode {p_['mode']!r}")
        if self.category != ModelCategory.REGRESSION or str(p_["family"]).lower() not in ("gaussian", "auto"):
            raise ValueError("modelselection supports the gaussian family")
        comm = self.comm
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, False)
        if any(self.feature_types[c] == ENUM for c in self.x):
            raise ValueError("modelselection: numeric predictors only")
        Xraw = design.raw_matrix(train)
        y = train.vec(self.y).as_float()
        ok = ~torch.isnan(y) & ~torch.isnan(Xraw).any(0)
        Xraw, y = Xraw[:, ok], y[ok]
        design.fit_standardization(Xraw, True, comm)
        X = design.transform(Xraw)
        p = X.shape[0]
        beta = np.zeros((1, p + 1))
        G, _ = D.glm_irls_pass(X, y, None, None, beta, "gaussian", "identity", 0)
        if comm is not None and comm.world_size > 1:
            G = comm.all_reduce_numpy(np.ascontiguousarray(G))
        n = G[p, p]
        tss = G[p + 1, p + 1] - G[p + 1, p] ** 2 / n
        kmax = min(int(p_["max_predictor_number"]), p)
        kmin = max(1, int(p_["min_predictor_number"]))
        best = {}
        allv = list(range(p))
        if mode == "allsubsets":
            for k in range(1, kmax + 1):
                best[k] = max(itertools.combinations(allv, k), key=lambda s: _r2(G, list(s), p, tss))
        elif mode == "backward":
            cur = allv[:]
            best[len(cur)] = tuple(cur)
            while len(cur) > kmin:
                drop = max(cur, key=lambda j: _r2(G, [c for c in cur if c != j], p, tss))
                cur = [c for c in cur if c != drop]
                best[len(cur)] = tuple(cur)
            kmax = p
        else:
            cur = []
            for k in range(1, kmax + 1):
                add = max((j for j in allv if j not in cur), key=lambda j: _r2(G, cur + [j], p, tss))
                cur = cur + [add]
                if mode in ("maxr", "maxrsweep"):
                    improved = True
                    while improved:
                        improved = False
                        base = _r2(G, cur, p, tss)
                        for i in range(len(cur)):
                            for j in allv:
                                if j in cur:
                                    continue
                                trial = cur[:i] + [j] + cur[i + 1:]
                                r = _r2(G, trial, p, tss)
                                if r > base + 1e-12:
                                    cur, base, improved = trial, r, True
                best[k] = tuple(cur)
        rows, models = [], []
        for k in sorted(best):
            if k < kmin or k > kmax:
                continue
            cols = [self.x[j] for j in best[k]]
            mid = f"{model_id}_model_{k}"
            glm = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0.0, compute_p_values=True,
                                                model_id=mid, standardize=bool(p_["standardize"]))
            m = glm.train(x=cols, y=self.y, training_frame=train, comm=comm)
            models.append(m)
            rows.append({"size": k, "best_r2_value": float(_r2(G, list(best[k]), p, tss)), "predictors": cols,
                         "model_id": mid})
        return ModelSelectionModel(self, model_id, rows, models)


class ANOVAGLMModel(Model):
    algo = "anovaglm"
    algo_full_name = "ANOVA for GLM"

    def __init__(self, builder, model_id, table, full, interactions):
        super().__init__(builder, model_id)
        self.table = table
        self.full_model = full
        self.interactions = interactions

    def result(self):
        return [dict(r) for r in self.table]

    def predict_raw(self, frame):
        return self.full_model.predict_raw(_with_interactions(frame, self.interactions))

    def summary(self):
        return {"model_id": self.model_id, "anova_table": self.result()}

    def to_json(self):
        j = super().to_json()
        j["output"]["anova_table"] = self.result()
        return j


class H2OANOVAGLMEstimator(ModelBuilder):
    algo = "anovaglm"
    DEFAULTS = dict(family="AUTO", link="family_default", highest_interaction_term=2, type=3, lambda_=0.0,
                    standardize=True, compute_p_values=True, save_transformed_framekeys=False)

    def _fit(self, train: Frame, valid, model_id):
        from scipy import stats as sst

        p_ = self.params
        comm = self.comm
        hit = max(1, int(p_["highest_interaction_term"]))
        terms = [(c,) for c in self.x]
        num = [c for c in self.x if self.feature_types[c] != ENUM]
        for order in range(2, hit + 1):
            terms += list(itertools.combinations(num, order))
        # materialise the numeric interaction columns
        inter = [t for t in terms if len(t) > 1]
        fr = _with_interactions(train, inter)
        cols_of = {t: [":".join(t)] for t in terms}
        allcols = [c for t in terms for c in cols_of[t]]
        kw = dict(family=p_["family"], link=p_["link"], lambda_=0.0, standardize=bool(p_["standardize"]))
        full = H2OGeneralizedLinearEstimator(**kw).train(x=allcols, y=self.y, training_frame=fr, comm=comm)
        fam = full.family
        dev_full = full.stats["residual_deviance"]
        nobs = full.stats["nobs"]
        df_full = nobs - (len(full.design.names) + 1)
        table = []
        for t in terms:
            rest = [c for c in allcols if c not in cols_of[t]]
            red = H2OGeneralizedLinearEstimator(**kw).train(x=rest or None, y=self.y, training_frame=fr, comm=comm) \
                if rest else None
            dev_red = red.stats["residual_deviance"] if red is not None else full.stats["null_deviance"]
            dfs = len(full.design.names) - (len(red.design.names) if red is not None else 0)
            ss = max(dev_red - dev_full, 0.0)
            if fam in ("binomial", "poisson", "multinomial"):
                stat, pv = ss, float(sst.chi2.sf(ss, max(dfs, 1)))
                kind = "chi_square"
            else:
                stat = (ss / max(dfs, 1)) / max(dev_full / max(df_full, 1), 1e-300)
                pv = float(sst.f.sf(stat, max(dfs, 1), max(df_full, 1)))
                kind = "F"
            table.append({"term": ":".join(t), "family": fam, "df": dfs, "deviance_difference": ss,
                          "statistic": float(stat), "statistic_type": kind, "p_value": pv})
        return ANOVAGLMModel(self, model_id, table, full, inter)


def _with_interactions(frame: Frame, inter) -> Frame:
    vecs = list(frame.vecs)
    have = set(frame.names)
    for t in inter:
        name = ":".join(t)
        if name in have:
            continue
        v = torch.ones(frame.nrows, device=frame.device)
        for c in t:
            v = v * frame.vec(c).as_float()
        vecs.append(Vec(name, v, "real"))
    return Frame(vecs, key=frame.key)
