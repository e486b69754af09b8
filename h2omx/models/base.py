"""Model-builder framework shared by every algorithm (H2O ModelBuilder /
Model / ModelOutput equivalents).

An estimator is configured with H2O parameter names, trained on a
:class:`~h2omx.frame.Frame` with ``train(x, y, training_frame, ...)`` and
produces a :class:`Model` that scores frames, reports H2O-style metrics and
can be exported as a MOJO.  Cross-validation (``nfolds``) and holdout
predictions (needed by StackedEnsemble) live here so every algorithm gets
them.
"""
from __future__ import annotations

import copy
import itertools
import time
import uuid

import numpy as np
import torch

from ..frame.frame import DKV, ENUM, Frame, Vec
from ..metrics import binomial_metrics, multinomial_metrics, regression_metrics

_model_counter = itertools.count(1)


def default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class ModelCategory:
    BINOMIAL = "Binomial"
    MULTINOMIAL = "Multinomial"
    REGRESSION = "Regression"
    CLUSTERING = "Clustering"
    DIMREDUCTION = "DimReduction"
    ANOMALY = "AnomalyDetection"


# categories whose models have no response column and no supervised metrics
UNSUPERVISED = (ModelCategory.CLUSTERING, ModelCategory.DIMREDUCTION, ModelCategory.ANOMALY)


class Model:
    """Trained model.  Subclasses implement ``predict_raw``; every such
    implementation is wrapped so categorical columns of the scored frame are
    first mapped onto the training domains by level name (H2O
    ``Model.adaptTestForTrain``: unseen levels become NA)."""

    algo = "model"
    # fitted transformers applied to a scored frame before predict_raw (H2O
    # AutoML preprocessing, e.g. a TargetEncoderModel); empty for plain models
    preprocessors: tuple = ()
    # deviations from H2O's semantics reported by the builder (output.warnings)
    warnings: tuple = ()

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        fn = cls.__dict__.get("predict_raw")
        if fn is not None and not getattr(fn, "_adapts_domains", False):
            def predict_raw(self, frame, *a, _fn=fn, **k):
                # preprocessing pipeline (AutoML target encoding) before the model
                for pp in self.preprocessors:
                    frame = pp.transform(frame)
                return _fn(self, self.adapt_frame(frame), *a, **k)

            predict_raw._adapts_domains = True
            predict_raw.__doc__ = fn.__doc__
            cls.predict_raw = predict_raw

    def adapt_frame(self, frame: Frame) -> Frame:
        enc = getattr(self, "cat_encoder", None)
        if enc is not None:
            frame = enc.transform(frame)
        cols = [c for c in self.x if self.feature_types.get(c) == ENUM]
        doms = {c: self.feature_domains.get(c) or [] for c in cols}
        if self.y is not None and self.response_domain is not None:
            cols.append(self.y)
            doms[self.y] = list(self.response_domain)
        repl = {}
        for c in cols:
            if c not in frame.names:
                continue
            v = frame.vec(c)
            if v.vtype != ENUM or list(v.domain or []) == list(doms[c]):
                continue
            idx = {d: i for i, d in enumerate(doms[c])}
            lut = torch.tensor([idx.get(d, -1) for d in (v.domain or [])] + [-1], dtype=torch.int32,
                               device=v.data.device)
            codes = v.data.long()
            codes = torch.where(codes >= 0, codes, torch.full_like(codes, lut.numel() - 1))
            repl[c] = Vec(c, lut[codes], ENUM, list(doms[c]))
        if not repl:
            return frame
        return Frame([repl.get(u.name, u) for u in frame.vecs], key=frame.key)

    def __init__(self, builder: "ModelBuilder", model_id: str):
        self.model_id = model_id
        self.params = dict(builder.params)
        self.x = list(builder.x or [])
        self.y = builder.y
        self.category = builder.category
        self.response_domain = builder.response_domain
        self.feature_types = dict(builder.feature_types)
        self.feature_domains = dict(builder.feature_domains)
        self.cat_encoder = getattr(builder, "cat_encoder", None)
        self.training_metrics: dict | None = None
        self.validation_metrics: dict | None = None
        self.cross_validation_metrics: dict | None = None
        self.cross_validation_holdout: torch.Tensor | None = None   # [K or 1][n] holdout predictions
        self.cv_models: list = []
        self.scoring_history: list = []
        self.run_time_ms = 0
        self.timings: dict = {}
        self.comm = builder.comm

    # -- scoring -------------------------------------------------------------------
    def predict_raw(self, frame: Frame) -> torch.Tensor:
        """Scores [K][n]: class probabilities (classification) or predictions."""
        raise NotImplementedError

    def predict(self, frame: Frame) -> Frame:
        P = self.predict_raw(frame)
        if self.category == ModelCategory.BINOMIAL:
            thr = (self.training_metrics or {}).get("max_f1_threshold", 0.5)
            p1 = P[-1]
            lab = (p1 >= thr).to(torch.int32)
            vecs = [Vec("predict", lab, ENUM, list(self.response_domain))]
            vecs += [Vec(d, P[i].float(), "real") for i, d in enumerate(self.response_domain)]
            return Frame(vecs)
        if self.category == ModelCategory.MULTINOMIAL:
            lab = P.argmax(0).to(torch.int32)
            vecs = [Vec("predict", lab, ENUM, list(self.response_domain))]
            vecs += [Vec(d, P[i].float(), "real") for i, d in enumerate(self.response_domain)]
            return Frame(vecs)
        if self.category == ModelCategory.CLUSTERING:
            return Frame([Vec("predict", P[0].to(torch.int32), "int")])
        if self.category == ModelCategory.ANOMALY:
            return Frame([Vec("predict", P[0].float(), "real"), Vec("mean_length", P[1].float(), "real")])
        if self.category == ModelCategory.DIMREDUCTION:
            return Frame([Vec(f"PC{i + 1}", P[i].float(), "real") for i in range(P.shape[0])])
        return Frame([Vec("predict", P[0].float(), "real")])

    def model_performance(self, frame: Frame | None = None) -> dict:
        if frame is None:
            return self.training_metrics
        return self._metrics(frame, self.predict_raw(frame))

    def _metrics(self, frame: Frame, P: torch.Tensor, comm=None) -> dict:
        frame = self.adapt_frame(frame)
        y = frame.vec(self.y)
        w = frame.vec(self.params["weights_column"]).as_float() if self.params.get("weights_column") else None
        return compute_metrics(self.category, P, y, w, comm, self.params.get("distribution"))

    def varimp(self) -> list[tuple]:
        return []

    def predict_contributions(self, frame: Frame) -> Frame:
        """SHAP contributions + BiasTerm (tree models; h2omx.explain)."""
        from ..explain import predict_contributions

        return predict_contributions(self, frame)

    # -- h2omx.explain_more (H2O model introspection APIs) ---------------------
    def predict_leaf_node_assignment(self, frame: Frame, type: str = "Path") -> Frame:  # noqa: A002
        from ..explain_more import predict_leaf_node_assignment

        return predict_leaf_node_assignment(self, frame, type)

    def staged_predict_proba(self, frame: Frame) -> Frame:
        from ..explain_more import staged_predict_proba

        return staged_predict_proba(self, frame)

    def feature_frequencies(self, frame: Frame) -> Frame:
        from ..explain_more import feature_frequencies

        return feature_frequencies(self, frame)

    def fairness_metrics(self, frame: Frame, protected_columns, reference=None, favorable_class=None) -> dict:
        from ..explain_more import fairness_metrics

        return fairness_metrics(self, frame, protected_columns, reference, favorable_class, self.comm)

    def permutation_importance(self, frame: Frame, metric="AUTO", n_repeats: int = 1, seed: int = -1,
                               features=None) -> list[dict]:
        from ..tools import permutation_importance

        return permutation_importance(self, frame, metric, n_repeats, seed, features)

    def ice(self, frame: Frame, column: str, nbins: int = 20, target=None) -> dict:
        from ..explain_more import ice

        return ice(self, frame, column, nbins, target)

    def explain(self, frame: Frame, **kw) -> dict:
        from ..explain_more import explain

        return explain([self], frame, **kw)

    def partial_dependence(self, frame: Frame, cols=None, nbins: int = 20, target=None) -> list[dict]:
        from ..explain import partial_dependence

        return [partial_dependence(self, frame, c, nbins=nbins, target=target, comm=self.comm)
                for c in (cols or self.x)]

    def summary(self) -> dict:
        return {"model_id": self.model_id, "algo": self.algo, "category": self.category}

    def to_json(self) -> dict:
        return {
            "model_id": {"name": self.model_id, "type": "Key<Model>"},
            "algo": self.algo,
            "algo_full_name": self.algo_full_name if hasattr(self, "algo_full_name") else self.algo,
            "response_column_name": self.y,
            "parameters": [{"name": k, "actual_value": _jsonable(v)} for k, v in self.params.items()],
            "output": {
                "model_category": self.category,
                "names": self.x + ([self.y] if self.y else []),
                "domains": [self.feature_domains.get(c) for c in self.x] + ([self.response_domain] if self.y else []),
                "training_metrics": _metrics_json(self.training_metrics),
                "validation_metrics": _metrics_json(self.validation_metrics),
                "cross_validation_metrics": _metrics_json(self.cross_validation_metrics),
                "variable_importances": [{"variable": v, "relative_importance": r, "scaled_importance": s,
                                          "percentage": p} for v, r, s, p in self.varimp()],
                "scoring_history": self.scoring_history,
                "run_time": self.run_time_ms,
                "h2omx_timings": {k: _jsonable(v) for k, v in (self.timings or {}).items()},
                "model_summary": self.summary(),
                "cross_validation_models": [{"name": m.model_id} for m in self.cv_models],
                "warnings": list(getattr(self, "warnings", None) or []) or None,
            },
        }

    def download_mojo(self, path: str) -> str:
        from ..mojo import export_mojo

        return export_mojo(self, path)


def _jsonable(v):
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {k: _jsonable(x) for k, x in v.items()}
    if isinstance(v, Frame):
        return v.key
    return v


def _metrics_json(m):
    if m is None:
        return None
    return {k: _jsonable(v) for k, v in m.items()}


def compute_metrics(category, P, yvec: Vec, w=None, comm=None, dist=None) -> dict:
    if category == ModelCategory.BINOMIAL:
        y = yvec.data.float() if yvec.vtype == ENUM else yvec.as_float()
        ok = y >= 0
        return binomial_metrics(P[-1][ok], y[ok], None if w is None else w[ok], comm)
    if category == ModelCategory.MULTINOMIAL:
        y = yvec.data
        ok = y >= 0
        return multinomial_metrics(P[:, ok], y[ok], None if w is None else w[ok], comm)
    y = yvec.as_float()
    ok = ~torch.isnan(y)
    return regression_metrics(P[0][ok], y[ok], None if w is None else w[ok], comm,
                              dist if dist in ("poisson", "gamma", "laplace") else "gaussian")


class ModelBuilder:
    """Base estimator.  Subclasses define ``algo``, ``DEFAULTS`` and ``_fit``."""

    algo = "base"
    DEFAULTS: dict = {}
    COMMON = dict(model_id=None, nfolds=0, fold_assignment="AUTO", fold_column=None, seed=-1,
                  keep_cross_validation_predictions=False, keep_cross_validation_models=True,
                  weights_column=None, ignored_columns=None, max_runtime_secs=0.0, distribution="AUTO",
                  # H2O ModelParameters shared by every builder; accepted so h2o-py
                  # call sites port unchanged (per-algorithm DEFAULTS override these)
                  keep_cross_validation_fold_assignment=False, score_each_iteration=False,
                  stopping_rounds=0, stopping_metric="AUTO", stopping_tolerance=1e-3,
                  categorical_encoding="AUTO", export_checkpoints_dir=None, custom_metric_func=None,
                  gainslift_bins=-1, auc_type="AUTO", ignore_const_cols=True, balance_classes=False,
                  class_sampling_factors=None, max_after_balance_size=5.0, max_confusion_matrix_size=20,
                  verbose=False, response_column=None, training_frame=None, validation_frame=None)

    def __init__(self, **params):
        unknown = set(params) - set(self.DEFAULTS) - set(self.COMMON)
        if unknown:
            raise ValueError(f"{self.algo}: unknown parameter(s) {sorted(unknown)}")
        self.params = {**self.COMMON, **self.DEFAULTS, **params}
        self._explicit_params = frozenset(params)   # what the user set (vs defaults)
        self.model: Model | None = None
        self.comm = None
        self.x = None
        self.y = None
        self.category = None
        self.response_domain = None
        self.feature_types = {}
        self.feature_domains = {}
        self.device = None

    # h2o-py style accessors
    def __getattr__(self, item):
        params = self.__dict__.get("params", {})
        if item in params:
            return params[item]
        raise AttributeError(item)

    def _seed(self) -> int:
        s = self.params.get("seed", -1)
        if s is None or s < 0:
            s = int(time.time() * 1000) & 0x7FFFFFFF
            self.params["seed"] = s
        return int(s)

    def _resolve_columns(self, frame: Frame, x, y):
        ignored = set(self.params.get("ignored_columns") or [])
        special = {y, self.params.get("weights_column"), self.params.get("fold_column"),
                   self.params.get("offset_column")}
        if x is None:
            x = [c for c in frame.names if c not in special and c not in ignored]
        x = [c for c in x if c not in special]
        return list(x), y

    UNSUPERVISED_CATEGORY = ModelCategory.CLUSTERING

    def _response_category(self, frame: Frame, y: str):
        if y is None:
            return self.UNSUPERVISED_CATEGORY, None
        v = frame.vec(y)
        dist = self.params.get("distribution", "AUTO")
        fam = self.params.get("family", "AUTO")
        if v.vtype == ENUM:
            dom = list(v.domain)
            return (ModelCategory.BINOMIAL if len(dom) == 2 else ModelCategory.MULTINOMIAL), dom
        if dist in ("bernoulli", "multinomial") or fam in ("binomial", "multinomial"):
            vals = torch.unique(v.as_float()[~torch.isnan(v.as_float())]).cpu().numpy()
            dom = [str(int(a)) if float(a).is_integer() else str(a) for a in vals]
            return (ModelCategory.BINOMIAL if len(dom) == 2 else ModelCategory.MULTINOMIAL), dom
        return ModelCategory.REGRESSION, None

    def train(self, x=None, y=None, training_frame: Frame | None = None, validation_frame: Frame | None = None,
              comm=None, **kw) -> Model:
        if training_frame is None:
            raise ValueError("training_frame is required")
        self.params.update(kw)
        t0 = time.time()
        self.comm = comm
        self.device = training_frame.device
        self.x, self.y = self._resolve_columns(training_frame, x, y)
        self.category, self.response_domain = self._response_category(training_frame, self.y)
        if self.y is not None and self.category != ModelCategory.REGRESSION and training_frame.vec(self.y).vtype != ENUM:
            training_frame = _as_enum_response(training_frame, self.y, self.response_domain)
            if validation_frame is not None:
                validation_frame = _as_enum_response(validation_frame, self.y, self.response_domain)
        for c in self.x:
            v = training_frame.vec(c)
            self.feature_types[c] = v.vtype
            self.feature_domains[c] = v.domain
        training_frame, validation_frame = self._encode_categoricals(training_frame, validation_frame)
        model_id = self.params.get("model_id") or f"{self.algo.upper()}_model_{next(_model_counter)}_{uuid.uuid4().hex[:6]}"
        nfolds = int(self.params.get("nfolds") or 0)
        cv_models, holdout = [], None
        if nfolds > 1:
            cv_models, holdout = self._cross_validate(training_frame, validation_frame, nfolds, model_id)
        model = self._fit(training_frame, validation_frame, model_id)
        model.comm = comm
        if model.training_metrics is None and self.category not in UNSUPERVISED:
            model.training_metrics = model._metrics(training_frame, model.predict_raw(training_frame), comm)
        if validation_frame is not None and self.category not in UNSUPERVISED:
            model.validation_metrics = model._metrics(validation_frame, model.predict_raw(validation_frame), comm)
        if nfolds > 1:
            model.cv_models = cv_models if self.params.get("keep_cross_validation_models", True) else []
            model.cross_validation_holdout = holdout
            if self.category not in UNSUPERVISED:
                model.cross_validation_metrics = model._metrics(training_frame, holdout, comm)
        model.run_time_ms = int((time.time() - t0) * 1000)
        DKV.put(model.model_id, model)
        self.model = model
        return model

    # categorical_encoding schemes the algorithm handles itself (frame/encoding.py)
    NATIVE_ENCODINGS = ("auto", "enum", "onehotinternal")

    def _encoding_scheme(self) -> str:
        """The effective categorical_encoding of this algorithm (validated)."""
        from ..frame.encoding import normalize_scheme

        return normalize_scheme(self.params.get("categorical_encoding"))

    def _encode_categoricals(self, train: Frame, valid: Frame | None):
        """Apply a frame-transform categorical_encoding (OneHotExplicit, Binary,
        Eigen, LabelEncoder, EnumLimited, SortByResponse where the algorithm
        has no native form) to the training / validation frames; the fitted
        encoder is kept for scoring (Model.adapt_frame)."""
        from ..frame.encoding import TRANSFORMS, CategoricalEncoder

        self.cat_encoder = None
        scheme = self._encoding_scheme()
        if scheme in self.NATIVE_ENCODINGS or scheme not in TRANSFORMS:
            return train, valid
        if not any(self.feature_types.get(c) == ENUM for c in self.x):
            return train, valid
        ce = CategoricalEncoder(scheme, self.x, self.feature_types, self.feature_domains,
                                max_levels=int(self.params.get("max_categorical_levels") or 10), y=self.y)
        ce.fit(train, self.comm)
        self.cat_encoder = ce
        self.x = list(ce.x_out)
        self.feature_types = dict(ce.out_types)
        self.feature_domains = dict(ce.out_domains)
        return ce.transform(train), (ce.transform(valid) if valid is not None else None)

    def fold_ids(self, frame: Frame, nfolds: int) -> torch.Tensor:
        fc = self.params.get("fold_column")
        if fc:
            return frame.vec(fc).as_float().long() % nfolds
        how = str(self.params.get("fold_assignment", "AUTO")).lower()
        n = frame.nrows
        if how == "modulo":
            return torch.arange(n, device=frame.device) % nfolds
        g = torch.Generator().manual_seed(self._seed() + 7)
        if how == "stratified" and self.y is not None and frame.vec(self.y).vtype == ENUM:
            yv = frame.vec(self.y).data.cpu()
            f = torch.empty(n, dtype=torch.long)
            for lvl in torch.unique(yv):
                idx = torch.nonzero(yv == lvl).flatten()
                perm = idx[torch.randperm(idx.numel(), generator=g)]
                f[perm] = torch.arange(perm.numel()) % nfolds
            return f.to(frame.device)
        return torch.randint(0, nfolds, (n,), generator=g).to(frame.device)

    def _cross_validate(self, frame: Frame, valid: Frame | None, nfolds: int, model_id: str):
        folds = self.fold_ids(frame, nfolds)
        holdout = None
        models = []
        for k in range(nfolds):
            sub = copy.copy(self)
            sub.params = dict(self.params, nfolds=0, model_id=f"{model_id}_cv_{k + 1}")
            tr = frame.rows(folds != k)
            ho_idx = torch.nonzero(folds == k).flatten()
            m = sub._fit(tr, None, sub.params["model_id"])
            m.comm = self.comm
            P = m.predict_raw(frame.rows(ho_idx))
            if holdout is None:
                holdout = torch.zeros((P.shape[0], frame.nrows), dtype=torch.float32, device=P.device)
            holdout[:, ho_idx.to(P.device)] = P.float()
            models.append(m)
            DKV.put(m.model_id, m)
        return models, holdout

    def _fit(self, train: Frame, valid: Frame | None, model_id: str) -> Model:
        raise NotImplementedError


def _as_enum_response(frame: Frame, y: str, domain: list) -> Frame:
    v = frame.vec(y)
    x = v.as_float()
    lut = {float(d): i for i, d in enumerate(domain)}
    codes = torch.full_like(x, -1, dtype=torch.int32)
    for val, i in lut.items():
        codes[x == val] = i
    nv = Vec(y, codes, ENUM, list(domain))
    return Frame([nv if u.name == y else u for u in frame.vecs], key=frame.key)


def response_codes(frame: Frame, y: str) -> torch.Tensor:
    return frame.vec(y).data
