"""AdaBoost and Decision Tree (H2O ``H2OAdaBoostEstimator`` /
``H2ODecisionTreeEstimator``).

AdaBoost (binary classification, SAMME): ``nlearners`` weak learners are
trained in sequence on re-weighted rows; learner t with weighted error e_t
gets weight a_t = learn_rate * log((1 - e_t) / e_t) and misclassified rows
are up-weighted by exp(a_t).  Weak learners are full h2omx estimators
trained through the ``weights_column`` (so a DRF / GBM weak learner runs on
the HIP tree engine and a GLM on the MFMA Gram kernel); the default is a
single depth-1 tree (a stump).  The committee score F = Σ a_t h_t(x) with
h_t ∈ {-1, +1} is reported as P(y = 1) = 1 / (1 + exp(-2 F)).

DecisionTree: one un-bagged tree on all features (DRF with ntrees=1,
sample_rate=1, mtries=all) with H2O DT's defaults (max_depth 20, min_rows 10).
"""
from __future__ import annotations

import math

import torch

from ..frame.frame import Frame, Vec
from .base import Model, ModelBuilder, ModelCategory
from .tree_models import H2ORandomForestEstimator


def _weak_learner(kind: str, params: dict, seed: int):
    from .deeplearning import H2ODeepLearningEstimator
    from .glm import H2OGeneralizedLinearEstimator
    from .tree_models import H2OGradientBoostingEstimator

    kind = kind.upper()
    if kind in ("AUTO", "DRF"):
        base = dict(ntrees=1, max_depth=1, min_rows=1.0, sample_rate=1.0, mtries=-2, seed=seed)
        return H2ORandomForestEstimator(**{**base, **params})
    if kind == "GBM":
        base = dict(ntrees=1, max_depth=1, min_rows=1.0, learn_rate=1.0, seed=seed)
        return H2OGradientBoostingEstimator(**{**base, **params})
    if kind == "GLM":
        return H2OGeneralizedLinearEstimator(**{**dict(family="binomial", lambda_=0.0, seed=seed), **params})
    if kind in ("DEEP_LEARNING", "DEEPLEARNING"):
        return H2ODeepLearningEstimator(**{**dict(hidden=[8], epochs=1, seed=seed), **params})
    raise ValueError(f"adaboost: weak_learner {kind!r} (AUTO, DRF, GBM, GLM, DEEP_LEARNING)")


class AdaBoostModel(Model):
    algo = "adaboost"
    algo_full_name = "AdaBoost"

    def __init__(self, builder, model_id, learners, alphas):
        super().__init__(builder, model_id)
        self.learners = learners
        self.alphas = alphas

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        F = None
        for m, a in zip(self.learners, self.alphas):
            h = m.predict_raw(frame)[-1].float() * 2 - 1             # P(y=1) -> [-1, 1]
            s = torch.sign(h)
            s = torch.where(s == 0, torch.ones_like(s), s)
            F = a * s if F is None else F + a * s
        p1 = torch.sigmoid(2.0 * F)
        return torch.stack([1 - p1, p1])

    def summary(self):
        return {"model_id": self.model_id, "nlearners": len(self.learners), "alphas": self.alphas}


class H2OAdaBoostEstimator(ModelBuilder):
    algo = "adaboost"
    DEFAULTS = dict(nlearners=50, weak_learner="AUTO", learn_rate=0.5, weak_learner_params=None)

    def _fit(self, train: Frame, valid, model_id):
        if self.category != ModelCategory.BINOMIAL:
            raise ValueError("adaboost supports binary classification only")
        p_ = self.params
        comm = self.comm
        y = train.vec(self.y).data
        ok = (y >= 0).double()
        sgn = (y == 1).double() * 2 - 1
        wname = "__adaboost_w__"
        base_w = (train.vec(p_["weights_column"]).as_float().double() if p_.get("weights_column")
                  else torch.ones(train.nrows, dtype=torch.float64, device=y.device)) * ok
        w = base_w.clone()
        tot = float(w.sum()) if comm is None or comm.world_size == 1 else float(
            comm.all_reduce_numpy(w.sum().reshape(1).cpu().numpy())[0])
        w = w / max(tot, 1e-300)
        learners, alphas = [], []
        seed = self._seed()
        lr = float(p_["learn_rate"])
        cols = [c for c in self.x]
        for t in range(int(p_["nlearners"])):
            fr = Frame([v for v in train.vecs if v.name != wname] + [Vec(wname, (w * train.nrows).float(), "real")])
            est = _weak_learner(str(p_["weak_learner"]), dict(p_.get("weak_learner_params") or {}), seed + t)
            est.params["weights_column"] = wname
            m = est.train(x=cols, y=self.y, training_frame=fr, comm=comm)
            h = m.predict_raw(train)[-1].double() * 2 - 1
            hs = torch.where(h >= 0, torch.ones_like(h), -torch.ones_like(h))
            miss = (hs != sgn).double() * ok
            parts = torch.stack([(w * miss).sum(), w.sum()])
            if comm is not None and comm.world_size > 1:
                comm.all_reduce_(parts)
            err = float(parts[0] / parts[1].clamp_min(1e-300))
            err = min(max(err, 1e-10), 1 - 1e-10)
            if err >= 0.5 and t > 0:
                break
            a = lr * math.log((1 - err) / err)
            learners.append(m)
            alphas.append(a)
            w = w * torch.exp(a * miss)
            s = w.sum()
            if comm is not None and comm.world_size > 1:
                s = torch.as_tensor(comm.all_reduce_numpy(s.reshape(1).cpu().numpy())[0], dtype=torch.float64)
            w = w / float(s)
        return AdaBoostModel(self, model_id, learners, alphas)


class H2ODecisionTreeEstimator(H2ORandomForestEstimator):
    """Single CART-style tree: DRF with one tree, no bagging, all features."""
    algo = "decision_tree"
    DEFAULTS = {**H2ORandomForestEstimator.DEFAULTS, "ntrees": 1, "max_depth": 20, "min_rows": 10.0,
                "sample_rate": 1.0, "mtries": -2}
