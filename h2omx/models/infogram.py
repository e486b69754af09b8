"""Infogram (H2O ``H2OInfogram``): admissible machine learning.

Each predictor gets two information measures.  A predictor is *admissible*
when both clear their thresholds (default 0.1).

Core infogram (no ``protected_columns``):
  * total information (relevance): the predictor's scaled variable importance
    in a model of y on all predictors;
  * net information: the conditional mutual information I(y; X_j | X_-j).
    It is estimated as the mean log-likelihood gain of the full model over a
    model trained without X_j,
        cmi_raw_j = mean_i [ log p_full(y_i | x_i) - log p_-j(y_i | x_i,-j) ]
    clipped at 0 and normalised by the largest value.
Fair infogram (``protected_columns`` A):
  * relevance index: the scaled variable importance in a model of y on the
    non-protected predictors;
  * safety index: I(y; X_j | A), estimated as the log-likelihood gain of
    y ~ A + X_j over y ~ A, normalised the same way.
Only the ``top_n_features`` most important predictors are scored.  Every
model is an h2omx estimator: GBM by default (the HIP tree engine), or any
``algorithm`` with its ``algorithm_params``, trained on the same (sharded)
frame and communicator.  Log-likelihoods are Bernoulli / multinomial for
classification and Gaussian (common variance) for regression.
``admissible_index`` = sqrt(a^2 + b^2) / sqrt(2) of the two normalised measures.

The estimates follow the published definitions, but not H2O's numbers
exactly ("parity unpinned": there is no H2O runtime here).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame, Vec
from .base import Model, ModelBuilder, ModelCategory


def _loglik(model, frame: Frame, y: str, category) -> torch.Tensor:
    P = model.predict_raw(frame)
    if category in (ModelCategory.BINOMIAL, ModelCategory.MULTINOMIAL):
        yc = frame.vec(y).data.long()
        ok = yc >= 0
        p = P[:, ok].double().gather(0, yc[ok][None, :].to(P.device)).clamp_min(1e-15)
        return torch.log(p).flatten()
    yv = frame.vec(y).as_float().double()
    ok = ~torch.isnan(yv)
    r = (yv[ok].to(P.device) - P[0][ok.to(P.device)].double())
    return -0.5 * r * r


def _mean(t: torch.Tensor, comm) -> float:
    s = torch.tensor([float(t.sum()), float(t.numel())], dtype=torch.float64)
    if comm is not None and comm.world_size > 1:
        s = torch.from_numpy(comm.all_reduce_numpy(s.numpy()))
    return float(s[0] / max(float(s[1]), 1.0))


class InfogramModel(Model):
    algo = "infogram"
    algo_full_name = "Information Diagram"

    def __init__(self, builder, model_id, table, fair, thresholds):
        super().__init__(builder, model_id)
        self.table = table
        self.fair = fair
        self.thresholds = thresholds

    def _cols(self):
        return ("relevance_index", "safety_index") if self.fair else ("total_information", "net_information")

    def get_admissible_features(self) -> list:
        return [r["column"] for r in self.table if r["admissible"]]

    def get_admissible_score_frame(self) -> Frame:
        a, b = self._cols()
        t = self.table
        vecs = [Vec("column", torch.arange(len(t), dtype=torch.int32), ENUM, [r["column"] for r in t])]
        vecs += [Vec("admissible", torch.tensor([float(r["admissible"]) for r in t]), "real")]
        for k in ("admissible_index", a, b, "cmi_raw"):
            vecs.append(Vec(k, torch.tensor([float(r[k]) for r in t]), "real"))
        return Frame(vecs)

    def get_admissible_cmi(self):
        return [r[self._cols()[1]] for r in self.table if r["admissible"]]

    def get_admissible_cmi_raw(self):
        return [r["cmi_raw"] for r in self.table if r["admissible"]]

    def get_admissible_relevance(self):
        return [r[self._cols()[0]] for r in self.table if r["admissible"]]

    def predict_raw(self, frame):
        raise ValueError("infogram: no predictions; use get_admissible_features() / get_admissible_score_frame()")

    def summary(self):
        return {"model_id": self.model_id, "admissible_features": self.get_admissible_features(), "fair": self.fair}

    def to_json(self):
        j = super().to_json()
        j["output"]["admissible_score"] = self.table
        j["output"]["admissible_features"] = self.get_admissible_features()
        return j


class H2OInfogram(ModelBuilder):
    algo = "infogram"
    DEFAULTS = dict(algorithm="AUTO", algorithm_params=None, protected_columns=None,
                    total_information_threshold=-1.0, net_information_threshold=-1.0,
                    relevance_index_threshold=-1.0, safety_index_threshold=-1.0, data_fraction=1.0,
                    top_n_features=50, nparallelism=0)

    def _learner(self, seed):
        from . import ESTIMATORS

        algo = str(self.params["algorithm"]).lower()
        algo = "gbm" if algo == "auto" else algo
        if algo not in ESTIMATORS or algo in ("infogram", "stackedensemble"):
            raise ValueError(f"infogram: algorithm {self.params['algorithm']!r}")
        kw = dict(self.params.get("algorithm_params") or {})
        kw.setdefault("seed", seed)
        return ESTIMATORS[algo], kw

    def _fit(self, train: Frame, valid, model_id):
        if self.y is None:
            raise ValueError("infogram needs a response column")
        p_ = self.params
        comm = self.comm
        seed = self._seed()
        frac = float(p_["data_fraction"])
        if frac < 1.0:
            g = torch.Generator().manual_seed(seed + (comm.rank if comm is not None else 0))
            keep = torch.rand(train.nrows, generator=g) < frac
            train = train.rows(torch.nonzero(keep).flatten().to(train.device))
        prot = [c for c in (p_.get("protected_columns") or [])]
        fair = bool(prot)
        cls, kw = self._learner(seed)
        cat = self.category
        y = self.y

        def fit(cols):
            return cls(**kw).train(x=list(cols), y=y, training_frame=train, comm=comm)

        preds = [c for c in self.x if c not in prot]
        full = fit(preds)
        vi = {v: s for v, _, s, _ in full.varimp()} if full.varimp() else {c: 1.0 for c in preds}
        ranked = sorted(preds, key=lambda c: -vi.get(c, 0.0))[: max(1, int(p_["top_n_features"]))]
        cmi = {}
        if fair:
            base = fit(prot)
            ll0 = _loglik(base, train, y, cat)
            for c in ranked:
                m = fit(prot + [c])
                cmi[c] = max(_mean(_loglik(m, train, y, cat) - ll0, comm), 0.0)
        else:
            llf = _loglik(full, train, y, cat)
            for c in ranked:
                rest = [d for d in preds if d != c]
                if not rest:
                    cmi[c] = max(_mean(llf - _null_loglik(train, y, cat, comm), comm), 0.0)
                    continue
                m = fit(rest)
                cmi[c] = max(_mean(llf - _loglik(m, train, y, cat), comm), 0.0)
        mx = max(cmi.values()) if cmi else 0.0
        t_a = float(p_["relevance_index_threshold" if fair else "total_information_threshold"])
        t_b = float(p_["safety_index_threshold" if fair else "net_information_threshold"])
        t_a = 0.1 if t_a < 0 else t_a
        t_b = 0.1 if t_b < 0 else t_b
        ka, kb = ("relevance_index", "safety_index") if fair else ("total_information", "net_information")
        table = []
        for c in ranked:
            a = float(vi.get(c, 0.0))
            b = cmi[c] / mx if mx > 0 else 0.0
            table.append({"column": c, ka: a, kb: b, "cmi_raw": cmi[c],
                          "admissible_index": math.sqrt(a * a + b * b) / math.sqrt(2.0),
                          "admissible": bool(a >= t_a and b >= t_b)})
        table.sort(key=lambda r: -r["admissible_index"])
        model = InfogramModel(self, model_id, table, fair, (t_a, t_b))
        model.training_metrics = {"admissible_features": model.get_admissible_features()}
        return model


def _null_loglik(frame, y, category, comm):
    """Log-likelihood of the intercept-only model (used when X_j is the only predictor)."""
    if category in (ModelCategory.BINOMIAL, ModelCategory.MULTINOMIAL):
        yc = frame.vec(y).data.long()
        yc = yc[yc >= 0]
        K = int(yc.max()) + 1 if yc.numel() else 1
        cnt = torch.bincount(yc, minlength=K).double()
        if comm is not None and comm.world_size > 1:
            cnt = torch.from_numpy(comm.all_reduce_numpy(cnt.cpu().numpy())).to(cnt.device)
        p = (cnt / cnt.sum()).clamp_min(1e-15)
        return torch.log(p[yc])
    yv = frame.vec(y).as_float().double()
    yv = yv[~torch.isnan(yv)]
    m = _mean(yv, comm)
    return -0.5 * (yv - m) ** 2
