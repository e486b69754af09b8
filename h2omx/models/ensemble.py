"""Stacked Ensembles (H2O StackedEnsemble equivalent).

The level-one frame holds the base models' cross-validated holdout
predictions (``keep_cross_validation_predictions=True`` on the base models,
same folds) or their predictions on a ``blending_frame``; a metalearner —
by default a non-negative GLM, H2O's ``AUTO`` — is trained on it.  Scoring
runs every base model (each on its own GPU kernels) and feeds the stacked
predictions to the metalearner.  All level-one data stays on the device.
"""
from __future__ import annotations

import torch

from ..frame.frame import DKV, ENUM, Frame, Vec
from .base import Model, ModelBuilder, ModelCategory


def _level_one_columns(model, P, category):
    mid = model.model_id
    if category == ModelCategory.BINOMIAL:
        return [Vec(mid, P[-1].float(), "real")]
    if category == ModelCategory.MULTINOMIAL:
        dom = model.response_domain or [str(i) for i in range(P.shape[0])]
        return [Vec(f"{mid}/{d}", P[k].float(), "real") for k, d in enumerate(dom)]
    return [Vec(mid, P[0].float(), "real")]


def level_one_frame(base_models, frame: Frame, category, y_vec: Vec | None = None) -> Frame:
    vecs = []
    for m in base_models:
        vecs += _level_one_columns(m, m.predict_raw(frame).to(frame.device), category)
    if y_vec is not None:
        vecs.append(y_vec)
    return Frame(vecs)


class StackedEnsembleModel(Model):
    algo = "stackedensemble"
    algo_full_name = "Stacked Ensemble"

    def __init__(self, builder, model_id, base_models, metalearner):
        super().__init__(builder, model_id)
        self.base_models = base_models
        self.metalearner = metalearner

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        lvl1 = level_one_frame(self.base_models, frame, self.category)
        return self.metalearner.predict_raw(lvl1)

    def varimp(self):
        return self.metalearner.varimp() if hasattr(self.metalearner, "varimp") else []

    def summary(self):
        return {"model_id": self.model_id, "number_of_base_models": len(self.base_models),
                "metalearner": self.metalearner.algo,
                "base_models": ", ".join(m.model_id for m in self.base_models)}

    def to_json(self):
        j = super().to_json()
        j["output"]["base_models"] = [{"name": m.model_id} for m in self.base_models]
        j["output"]["metalearner"] = {"name": self.metalearner.model_id}
        return j


class H2OStackedEnsembleEstimator(ModelBuilder):
    algo = "stackedensemble"
    DEFAULTS = dict(base_models=[], metalearner_algorithm="AUTO", metalearner_nfolds=0,
                    metalearner_fold_assignment=None, metalearner_params=None, blending_frame=None,
                    keep_levelone_frame=False, score_training_samples=10000)

    def _resolve_base(self):
        out = []
        for b in self.params["base_models"]:
            m = DKV.get(b) if isinstance(b, str) else b
            if not isinstance(m, Model):
                raise ValueError(f"base model {b!r} not found")
            out.append(m)
        if not out:
            raise ValueError("base_models is empty")
        return out

    def _fit(self, train: Frame, valid, model_id):
        base = self._resolve_base()
        blend = self.params.get("blending_frame")
        if isinstance(blend, str):
            blend = DKV.get(blend)
        yv = train.vec(self.y) if blend is None else blend.vec(self.y)
        if blend is not None:
            lvl1 = level_one_frame(base, blend, self.category, yv)
        else:
            vecs = []
            n = train.nrows
            for m in base:
                H = m.cross_validation_holdout
                if H is None or H.shape[1] != n:
                    raise ValueError(f"base model {m.model_id} has no cross-validation holdout predictions "
                                     "(train base models with nfolds > 1 and keep_cross_validation_predictions)")
                vecs += _level_one_columns(m, H.to(train.device), self.category)
            vecs.append(Vec(self.y, yv.data if yv.vtype == ENUM else yv.as_float(), yv.vtype, yv.domain))
            lvl1 = Frame(vecs)
        meta = self._metalearner()
        meta.train(x=[v.name for v in lvl1.vecs if v.name != self.y], y=self.y, training_frame=lvl1, comm=self.comm)
        model = StackedEnsembleModel(self, model_id, base, meta.model)
        return model

    def _metalearner(self):
        from .glm import H2OGeneralizedLinearEstimator
        from .tree_models import H2OGradientBoostingEstimator, H2ORandomForestEstimator

        algo = str(self.params["metalearner_algorithm"]).lower()
        mp = dict(self.params.get("metalearner_params") or {})
        nf = int(self.params.get("metalearner_nfolds") or 0)
        if nf > 1:
            mp.setdefault("nfolds", nf)
        mp.setdefault("seed", self._seed())
        if algo in ("auto", "glm"):
            if algo == "auto":
                mp.setdefault("non_negative", True)
                mp.setdefault("lambda_", 0.0)
            return H2OGeneralizedLinearEstimator(**mp)
        if algo == "gbm":
            return H2OGradientBoostingEstimator(**mp)
        if algo == "drf":
            return H2ORandomForestEstimator(**mp)
        if algo == "deeplearning":
            from .deeplearning import H2ODeepLearningEstimator

            return H2ODeepLearningEstimator(**mp)
        raise ValueError(f"unsupported metalearner {algo}")
