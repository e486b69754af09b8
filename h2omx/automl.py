"""AutoML (H2O AutoML equivalent): trains a fixed sequence of algorithm
presets, then random-grid XGBoost / GBM / DeepLearning models (round-robin),
under a model-count / runtime budget (``max_runtime_secs_per_model`` caps
each model through its own ``max_runtime_secs``), optionally restricted by a
``modeling_plan``; re-running a ``project_name`` extends its leaderboard;
cross-validates every model with shared folds, and finishes with two
Stacked Ensembles (all models, best of family).  Models are ranked on a
leaderboard by the H2O default metric for the problem type.

Two schedulers (``parallelism``, an h2omx extension), picked
per run by ``"auto"`` (default): task-parallel when the replicated training
frame takes at most TASK_MEM_FRACTION of one device's memory, else data:

* ``"data"``: every model is data-parallel over all ranks (the row
  shards stay where they are and each model's collectives run over RCCL), so
  AutoML on 8 MI355X trains each model 8-way parallel in sequence.
* ``"task"``: the training frame is replicated on every GPU (all-gather; 288
  GB of HBM holds the AutoML shapes many times over) and the model plan is
  dealt round-robin to the ranks, each training its models on its own GPU
  with no collectives.  The models are then exchanged (MOJO bytes + metrics +
  cross-validation holdout predictions) so every rank holds the full set; the
  stacked ensembles and the leaderboard are computed identically everywhere.
  Small and medium models stop paying per-level collective latency.
"""
from __future__ import annotations

import time
import uuid

import numpy as np
import torch

from .frame.frame import DKV, Frame
from .models import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                     H2ORandomForestEstimator, H2OXGBoostEstimator)
from .frame.frame import ENUM, Vec
from .models.base import ModelCategory
from .models.ensemble import H2OStackedEnsembleEstimator
from .models.target_encoder import H2OTargetEncoderEstimator

ALGOS = ("GLM", "DRF", "GBM", "XGBoost", "DeepLearning", "StackedEnsemble")

# preprocessing=["target_encoding"] (H2O AutoML TargetEncoding step): categorical
# predictors with at least TE_CARDINALITY levels are replaced by their blended
# target means (inflection point 5, smoothing 10, no noise; out-of-fold means on
# the training rows when the run cross-validates) for the algos below.  The
# threshold / blending values follow H2O's AutoML step; h2o is not importable
# here, so parity with its encoded values is unpinned.
TE_CARDINALITY = 25
TE_ALGOS = ("gbm", "drf", "xgboost")
TE_FOLD = "__automl_te_fold"

# (algo, id suffix, estimator class, params) in H2O's default training order
PRESETS = [
    ("XGBoost", "1", H2OXGBoostEstimator, dict(max_depth=10, min_child_weight=5, sample_rate=0.6,
                                                col_sample_rate=0.8, col_sample_rate_per_tree=0.8)),
    ("GLM", "1", H2OGeneralizedLinearEstimator, dict(lambda_search=True)),
    ("DRF", "1", H2ORandomForestEstimator, dict()),
    ("GBM", "1", H2OGradientBoostingEstimator, dict(max_depth=6, min_rows=1, sample_rate=0.8, col_sample_rate=0.8,
                                                     col_sample_rate_per_tree=0.8)),
    ("GBM", "2", H2OGradientBoostingEstimator, dict(max_depth=7, min_rows=10, sample_rate=0.8,
                                                     col_sample_rate=0.8, col_sample_rate_per_tree=0.8)),
    ("GBM", "3", H2OGradientBoostingEstimator, dict(max_depth=8, min_rows=10, sample_rate=0.8,
                                                     col_sample_rate=0.8, col_sample_rate_per_tree=0.8)),
    ("GBM", "4", H2OGradientBoostingEstimator, dict(max_depth=10, min_rows=10, sample_rate=0.8,
                                                     col_sample_rate=0.8, col_sample_rate_per_tree=0.8)),
    ("GBM", "5", H2OGradientBoostingEstimator, dict(max_depth=15, min_rows=100, sample_rate=0.8,
                                                     col_sample_rate=0.8, col_sample_rate_per_tree=0.8)),
    ("XGBoost", "2", H2OXGBoostEstimator, dict(max_depth=20, min_child_weight=10, sample_rate=0.6,
                                                col_sample_rate=0.8, col_sample_rate_per_tree=0.8)),
    ("XGBoost", "3", H2OXGBoostEstimator, dict(max_depth=5, min_child_weight=3, sample_rate=0.8,
                                                col_sample_rate=0.8, col_sample_rate_per_tree=0.8)),
    ("DRF", "XRT", H2ORandomForestEstimator, dict(sample_rate=0.632, col_sample_rate_per_tree=0.8, nbins=10)),
    ("DeepLearning", "1", H2ODeepLearningEstimator, dict(hidden=[10, 10, 10], epochs=10)),
]

GRID = dict(max_depth=[3, 4, 5, 6, 7, 8, 9, 10, 12, 15], min_rows=[1, 5, 10, 15, 30, 100],
            sample_rate=[0.5, 0.6, 0.7, 0.8, 0.9, 1.0], col_sample_rate=[0.4, 0.7, 1.0],
            col_sample_rate_per_tree=[0.4, 0.7, 1.0], learn_rate=[0.05, 0.1])
# random-grid spaces after the presets (H2O AutoML's XGBoost / GBM / DeepLearning grids)
GRIDS = {
    "gbm": (H2OGradientBoostingEstimator, GRID),
    "xgboost": (H2OXGBoostEstimator, dict(max_depth=[3, 6, 9, 12, 15], min_child_weight=[1, 3, 5, 10, 15],
                                          sample_rate=[0.6, 0.8, 1.0], col_sample_rate=[0.6, 0.8, 1.0],
                                          col_sample_rate_per_tree=[0.7, 0.8, 0.9, 1.0],
                                          reg_lambda=[0.001, 0.01, 0.1, 1.0, 10.0], reg_alpha=[0.001, 0.01, 0.1, 0.5, 1.0],
                                          learn_rate=[0.05, 0.1, 0.3])),
    "deeplearning": (H2ODeepLearningEstimator, dict(hidden=[[20], [50], [100], [20, 20], [50, 50], [100, 100]],
                                                    epochs=[10], input_dropout_ratio=[0.0, 0.05, 0.1],
                                                    rho=[0.9, 0.95, 0.99], epsilon=[1e-6, 1e-7, 1e-8])),
}
_PROJECTS: dict = {}


def _metric_spec(category, sort_metric):
    sm = (sort_metric or "AUTO").lower()
    if sm == "auto":
        sm = {ModelCategory.BINOMIAL: "auc", ModelCategory.MULTINOMIAL: "mean_per_class_error"}.get(category,
                                                                                                  "mean_residual_deviance")
    key = {"auc": "AUC", "aucpr": "AUCPR", "logloss": "logloss", "rmse": "RMSE", "mse": "MSE", "mae": "mae",
           "mean_per_class_error": "mean_per_class_error", "mean_residual_deviance": "mean_residual_deviance",
           "rmsle": "rmsle"}[sm]
    return sm, key, sm in ("auc", "aucpr")


class H2OAutoML:
    def __init__(self, max_models=None, max_runtime_secs=None, max_runtime_secs_per_model=0.0, nfolds=-1, seed=-1,
                 project_name=None, include_algos=None, exclude_algos=None, sort_metric="AUTO",
                 keep_cross_validation_predictions=True, stopping_rounds=3, stopping_tolerance=None,
                 stopping_metric="AUTO", balance_classes=False, verbosity="warn", modeling_plan=None,
                 preprocessing=None, exploitation_ratio=-1.0, parallelism="auto", **_ignored):
        if parallelism not in ("auto", "data", "task"):
            raise ValueError("parallelism must be 'auto', 'data' or 'task'")
        self.parallelism = parallelism
        self.max_models = max_models
        self.max_runtime_secs = max_runtime_secs
        self.max_runtime_secs_per_model = float(max_runtime_secs_per_model or 0.0)
        self.nfolds = 5 if nfolds in (-1, None) else int(nfolds)
        self.seed = seed
        self.project_name = project_name or f"AutoML_{uuid.uuid4().hex[:8]}"
        inc = [a.lower() for a in include_algos] if include_algos else [a.lower() for a in ALGOS]
        exc = {a.lower() for a in (exclude_algos or [])}
        self.algos = [a for a in inc if a not in exc]
        self.plan = _parse_plan(modeling_plan) if modeling_plan else None
        # H2O exploitation phase: a share of the budget (time and models) refines the
        # best explored GBM with learning-rate annealing (-1 / 0: off)
        self.exploitation_ratio = float(exploitation_ratio or 0.0)
        if self.plan is not None:
            self.algos = [a for a in self.algos if a in self.plan or a == "stackedensemble"]
        self.sort_metric = sort_metric
        self.stopping = dict(stopping_rounds=int(stopping_rounds or 0), stopping_metric=stopping_metric,
                             stopping_tolerance=stopping_tolerance)
        self.preprocessing = preprocessing
        self.events: list[dict] = []
        self.models: list = []
        self.leaderboard: list[dict] = []
        self.leader = None
        self.training_info: dict = {}
        prev = _PROJECTS.get(self.project_name)
        if prev is not None:                      # H2O: same project_name -> extend its leaderboard
            self.models = list(prev.models)
            self.events = list(prev.events)
        _PROJECTS[self.project_name] = self

    def _log(self, stage, msg):
        self.events.append({"t": time.strftime("%H:%M:%S"), "stage": stage, "msg": msg})

    def train(self, x=None, y=None, training_frame: Frame | None = None, leaderboard_frame: Frame | None = None,
              validation_frame: Frame | None = None, comm=None):
        t0 = time.time()
        budget = self.max_runtime_secs
        if not budget and not self.max_models:
            budget = 3600.0
        seed = self.seed if self.seed is not None and self.seed >= 0 else 42
        rng = np.random.default_rng(seed)
        cv = dict(nfolds=self.nfolds, fold_assignment="Modulo", keep_cross_validation_predictions=True,
                  seed=seed) if self.nfolds > 1 else dict(seed=seed)
        category = None

        explo = min(max(self.exploitation_ratio, 0.0), 1.0)
        # model slots kept for the exploitation steps (GBM_lr_annealing_selection,
        # XGBoost_lr_search_selection)
        n_steps = sum(a in self.algos for a in ("gbm", "xgboost"))
        explo_models = min(n_steps, int(np.ceil(explo * int(self.max_models)))) if (explo and self.max_models) else 0

        def out_of_budget(phase="explore"):
            reserve = explo_models if phase == "explore" else 0
            if self.max_models and len(self.models) >= self.max_models - reserve:
                return True
            share = (1.0 - explo) if phase == "explore" else 1.0
            return bool(budget) and time.time() - t0 > budget * share

        def fit(name, cls, params):
            nonlocal category
            mid = f"{name}_AutoML_{self.project_name}"
            if any(m.model_id == mid for m in self.models):
                mid = f"{mid}_{len(self.models)}"
            rt = self.max_runtime_secs_per_model
            if budget:
                left = max(budget - (time.time() - t0), 1.0)
                rt = min(rt, left) if rt else left
            if rt:
                params = dict(params, max_runtime_secs=rt)
            try:
                est = cls(model_id=mid, **params, **cv)
                m = est.train(x=x, y=y, training_frame=training_frame, validation_frame=validation_frame, comm=comm)
            except Exception as e:  # noqa: BLE001
                self._log("ModelTraining", f"{name} failed: {type(e).__name__}: {e}")
                return None
            category = m.category
            self.models.append(m)
            self._log("ModelTraining", f"{mid} trained")
            return m

        self._log("Workflow", f"AutoML build started: {self.project_name}")
        task_mode = self._scheduler(training_frame, comm) == "task"
        # (task-parallel runs fit the step on the replicated frame, _train_task_parallel)
        te = None if task_mode else self._target_encoding(x, y, training_frame, validation_frame, seed, comm)
        if te is not None:
            fit_raw = fit

            def fit(name, cls, params):   # noqa: F811 - TE'd algos train on the encoded frames
                nonlocal x, training_frame, validation_frame
                if cls.algo not in TE_ALGOS:
                    return fit_raw(name, cls, params)
                saved = x, training_frame, validation_frame
                x, training_frame, validation_frame = te["x"], te["train"], te["valid"]
                try:
                    m = fit_raw(name, cls, params)
                finally:
                    x, training_frame, validation_frame = saved
                if m is not None:
                    m.preprocessors = (te["model"],)
                return m
        start_models = len(self.models)
        if self.max_models:
            self.max_models = int(self.max_models) + start_models
        if task_mode:
            category = self._train_task_parallel(x, y, training_frame, validation_frame, comm, cv, rng, budget, t0,
                                                 start_models, explo, explo_models)
            training_frame = self._local_frame
            comm_se = None
        else:
            category = self._train_sequential(fit, rng, out_of_budget)
            if explo > 0 and category is not None:
                self._exploit(fit, category, lambda: out_of_budget("exploit"))
            comm_se = comm
        base = [m for m in self.models if m.cross_validation_holdout is not None]
        if "stackedensemble" in self.algos and self.nfolds > 1 and len(base) >= 2 and category != ModelCategory.CLUSTERING:
            for name, members in (("StackedEnsemble_AllModels", base),
                                  ("StackedEnsemble_BestOfFamily", self._best_of_family(base, category))):
                if len(members) < 2:
                    continue
                try:
                    se = H2OStackedEnsembleEstimator(model_id=f"{name}_AutoML_{self.project_name}",
                                                     base_models=[m.model_id for m in members], seed=seed)
                    m = se.train(x=x, y=y, training_frame=training_frame, comm=comm_se)
                    m.cross_validation_metrics = None
                    self.models.append(m)
                    self._log("ModelTraining", f"{m.model_id} trained")
                except Exception as e:  # noqa: BLE001
                    self._log("ModelTraining", f"{name} failed: {type(e).__name__}: {e}")
        self._rank(category, leaderboard_frame, comm)
        self._log("Workflow", f"AutoML build done: {len(self.models)} models in {time.time() - t0:.1f}s")
        self.training_info = {"start_epoch": int(t0), "stop_epoch": int(time.time()),
                              "duration_secs": round(time.time() - t0, 3), "models": len(self.models),
                              "leader": self.leader.model_id if self.leader is not None else None,
                              "parallelism": self.parallelism}
        self._x, self._frame = x, training_frame
        return self

    def _plan_models(self, rng) -> list:
        """The ordered model plan: presets, then the round-robin random grids
        (identical on every rank for a given seed)."""
        out = [(f"{algo}_{suffix}", cls, dict(params)) for algo, suffix, cls, params in PRESETS
               if algo.lower() in self.algos and self._planned(algo, "defaults")]
        fams = [f for f in ("xgboost", "gbm", "deeplearning") if f in self.algos and self._planned(f, "grids")]
        name = {"xgboost": "XGBoost", "gbm": "GBM", "deeplearning": "DeepLearning"}
        cap = (self.max_models - len(self.models)) if self.max_models else 300
        counters = {f: 1 for f in fams}
        while fams and len(out) < cap and sum(counters.values()) < 300:
            for f in fams:
                cls, space = GRIDS[f]
                params = {k: v[int(rng.integers(len(v)))] for k, v in space.items()}
                if f != "deeplearning":
                    params.update({k: v for k, v in self.stopping.items() if v is not None})
                out.append((f"{name[f]}_grid_1_model_{counters[f]}", cls, params))
                counters[f] += 1
        return out[:cap] if self.max_models else out

    # "auto": replicate the frame (task-parallel) while it takes at most this share
    # of one device's memory (288 GB HBM per MI355X: AutoML's 10M x 100 frame is ~1.4 %)
    TASK_MEM_FRACTION = 0.25

    def _scheduler(self, frame, comm) -> str:
        if comm is None or comm.world_size <= 1:
            return "data"
        if self.parallelism != "auto":
            return self.parallelism
        rows = int(comm.all_reduce_numpy(np.array([float(frame.nrows)]))[0])
        need = rows * max(1, len(frame.names)) * 8          # float64-sized upper bound per cell
        if frame.device.type == "cuda":
            cap = torch.cuda.get_device_properties(frame.device).total_memory
        else:
            import psutil

            cap = psutil.virtual_memory().total // comm.world_size
        mode = "task" if need <= self.TASK_MEM_FRACTION * cap else "data"
        self._log("Workflow", f"parallelism auto -> {mode} ({need / 2**30:.2f} GiB replicated frame, "
                              f"{cap / 2**30:.0f} GiB per rank)")
        return mode

    def _target_encoding(self, x, y, frame, valid, seed, comm):
        """Fit the TargetEncoding preprocessing step (see TE_CARDINALITY) and
        return the encoded training / validation frames and predictor list,
        or None when the step is off or finds no high-cardinality predictor."""
        steps = [str(p).lower().replace("_", "") for p in (self.preprocessing or [])]
        if "targetencoding" not in steps or y is None:
            return None
        xs = list(x) if x else [n for n in frame.names if n != y]
        cols = [c for c in xs if frame.vec(c).vtype == ENUM and len(frame.vec(c).domain or []) >= TE_CARDINALITY]
        if not cols:
            self._log("Preprocessing", "target_encoding: no categorical predictor with >= "
                                       f"{TE_CARDINALITY} levels, step skipped")
            return None
        kfold = self.nfolds > 1
        fr = frame
        if kfold:
            # the same Modulo folds the cross-validated models use (global row index)
            from .models.tree.engine import global_row_base

            base = global_row_base(frame.nrows, comm)
            fid = (torch.arange(frame.nrows, device=frame.device) + base) % self.nfolds
            fr = Frame(list(frame.vecs) + [Vec(TE_FOLD, fid.to(torch.int32), "int")])
        te_model = H2OTargetEncoderEstimator(
            model_id=f"TargetEncoder_AutoML_{self.project_name}", blending=True, inflection_point=5.0,
            smoothing=10.0, noise=0.0, keep_original_categorical_columns=False, seed=seed,
            data_leakage_handling="KFold" if kfold else "None", fold_column=TE_FOLD if kfold else None,
        ).train(x=cols, y=y, training_frame=fr, comm=comm)
        train = te_model.transform(fr, as_training=True)
        if kfold:
            train = Frame([v for v in train.vecs if v.name != TE_FOLD])
        enc = [n for n in train.names if n not in frame.names]
        x_te = [c for c in xs if c not in cols] + enc
        self._log("Preprocessing", f"target_encoding: {len(cols)} column(s) encoded for "
                                   f"{', '.join(TE_ALGOS)}: {', '.join(cols)}")
        return {"model": te_model, "train": train, "x": x_te,
                "valid": te_model.transform(valid) if valid is not None else None}

    def _train_sequential(self, fit, rng, out_of_budget):
        category = None
        for algo, suffix, cls, params in PRESETS:
            if algo.lower() not in self.algos or not self._planned(algo, "defaults"):
                continue
            if out_of_budget():
                break
            m = fit(f"{algo}_{suffix}", cls, dict(params))
            category = m.category if m is not None else category
        # random grids, round-robin over the families still allowed
        fams = [f for f in ("xgboost", "gbm", "deeplearning") if f in self.algos and self._planned(f, "grids")]
        counters = {f: 1 for f in fams}
        name = {"xgboost": "XGBoost", "gbm": "GBM", "deeplearning": "DeepLearning"}
        while fams and not out_of_budget() and sum(counters.values()) < 300:
            for f in list(fams):
                if out_of_budget():
                    break
                cls, space = GRIDS[f]
                params = {k: v[int(rng.integers(len(v)))] for k, v in space.items()}
                if f != "deeplearning":
                    params.update({k: v for k, v in self.stopping.items() if v is not None})
                m = fit(f"{name[f]}_grid_1_model_{counters[f]}", cls, params)
                category = m.category if m is not None else category
                counters[f] += 1
        return category

    def _exploit_plan(self, category) -> list:
        """H2O AutoML's exploitation steps over the explored models, as a plan of
        (name, estimator class, params):

        * ``XGBoost_lr_search_selection``: the best XGBoost at half its learning
          rate over twice the trees;
        * ``GBM_lr_annealing_selection``: the best explored GBM retrained with its
          hyper-parameters and learning rate, decaying by 0.99 per tree
          (``learn_rate_annealing``) over twice the trees.

        Early stopping as configured; ranked like any other model.  Both
        schedulers run this plan (task-parallel: dealt over the ranks)."""
        out = []
        best_of = {m.algo: m for m in self._best_of_family(list(self.models), category)}
        xgb = best_of.get("xgboost")
        if xgb is not None:
            keep = ("max_depth", "min_rows", "min_child_weight", "sample_rate", "subsample", "col_sample_rate",
                    "colsample_bylevel", "col_sample_rate_per_tree", "colsample_bytree", "reg_lambda", "reg_alpha",
                    "gamma", "distribution")
            params = {k: xgb.params[k] for k in keep if xgb.params.get(k) is not None}
            lr = float(xgb.params.get("eta") or xgb.params.get("learn_rate") or 0.3)
            params.update(learn_rate=lr / 2, ntrees=int(xgb.params.get("ntrees", 50)) * 2, score_tree_interval=5)
            params.update({k: v for k, v in self.stopping.items() if v is not None})
            self._log("ModelTraining", f"exploitation: XGBoost_lr_search_selection from {xgb.model_id}")
            out.append(("XGBoost_lr_search_selection", H2OXGBoostEstimator, params))
        best = best_of.get("gbm")
        if best is not None:
            keep = ("max_depth", "min_rows", "sample_rate", "col_sample_rate", "col_sample_rate_per_tree",
                    "min_split_improvement", "distribution", "nbins")
            params = {k: best.params[k] for k in keep if k in best.params}
            lr = float(best.params.get("learn_rate", 0.1))
            params.update(learn_rate=lr, learn_rate_annealing=0.99, ntrees=int(best.params.get("ntrees", 50)) * 2,
                          score_tree_interval=5)
            params.update({k: v for k, v in self.stopping.items() if v is not None})
            self._log("ModelTraining", f"exploitation: GBM_lr_annealing_selection from {best.model_id}")
            out.append(("GBM_lr_annealing_selection", H2OGradientBoostingEstimator, params))
        return out

    def _exploit(self, fit, category, out_of_budget):
        """Sequential scheduler: the exploitation plan, one model at a time."""
        for name, cls, params in self._exploit_plan(category):
            if out_of_budget():
                break
            fit(name, cls, params)

    def _train_task_parallel(self, x, y, training_frame, validation_frame, comm, cv, rng, budget, t0, start_models,
                             explo=0.0, explo_models=0):
        """parallelism="task": replicate the frame, deal the plan round-robin to
        the ranks, train locally (comm=None), exchange the trained models.  With
        ``exploitation_ratio`` > 0 the exploration round keeps its share of the
        time / model budget and a second round deals the exploitation plan
        (built from the exchanged leaderboard, identical on every rank)."""
        from .frame.distributed import gather_frame

        local = gather_frame(training_frame, comm)
        valid = gather_frame(validation_frame, comm) if validation_frame is not None else None
        self._local_frame = local
        seed = self.seed if self.seed is not None and self.seed >= 0 else 42
        # every rank fits the same encoder on the same replicated rows (comm=None)
        te = self._target_encoding(x, y, local, valid, seed, None)
        plan = self._plan_models(rng)
        if explo_models:
            plan = plan[: max(0, len(plan) - explo_models)] if self.max_models else plan
        self._log("Workflow", f"task-parallel: {len(plan)} models over {comm.world_size} ranks "
                              f"({local.nrows} rows replicated per rank)")
        ctx = (x, y, local, valid, te, cv, budget, t0, comm)
        category = self._deal(plan, 0, ctx, budget * (1.0 - explo) if (budget and explo) else budget)
        if explo > 0 and category is not None:
            ex = self._exploit_plan(category)
            if ex:
                self._log("Workflow", f"task-parallel exploitation: {len(ex)} models over {comm.world_size} ranks")
                category = self._deal(ex, len(plan), ctx, budget) or category
        return category

    def _deal(self, plan, base, ctx, time_limit):
        """One task-parallel round: plan entry i trains on rank (base + i) % world;
        the trained models are exchanged (MOJO + metrics + CV holdout + params)
        and appended to the leaderboard in plan order on every rank."""
        from .frame.distributed import _gather_objects
        from .mojo import GenericModel, mojo_bytes

        x, y, local, valid, te, cv, budget, t0, comm = ctx
        mine = []
        for i in range(len(plan)):
            if (base + i) % comm.world_size != comm.rank:
                continue
            if time_limit and time.time() - t0 > time_limit:
                break
            name, cls, params = plan[i]
            mid = f"{name}_AutoML_{self.project_name}"
            rt = self.max_runtime_secs_per_model
            if budget:
                left = max(budget - (time.time() - t0), 1.0)
                rt = min(rt, left) if rt else left
            if rt:
                params = dict(params, max_runtime_secs=rt)
            use_te = te is not None and cls.algo in TE_ALGOS
            try:
                m = cls(model_id=mid, **params, **cv).train(
                    x=te["x"] if use_te else x, y=y, training_frame=te["train"] if use_te else local,
                    validation_frame=te["valid"] if use_te else valid, comm=None)
            except Exception as e:  # noqa: BLE001
                self._log("ModelTraining", f"{name} failed on rank {comm.rank}: {type(e).__name__}: {e}")
                continue
            h = m.cross_validation_holdout
            blob = mojo_bytes(m)   # the bare model (its encoder is refitted identically on every rank)
            if use_te:
                m.preprocessors = (te["model"],)
            mine.append((base + i, {"model_id": m.model_id, "algo": m.algo, "mojo": blob,
                                    "params": dict(m.params),
                                    "training_metrics": m.training_metrics, "validation_metrics": m.validation_metrics,
                                    "cross_validation_metrics": m.cross_validation_metrics,
                                    "holdout": None if h is None else h.detach().cpu().numpy(),
                                    "run_time_ms": getattr(m, "run_time_ms", 0), "rank": comm.rank}, m))
        payloads = _gather_objects(comm, [(i, pl) for i, pl, _ in mine])
        native = {i: m for i, _, m in mine}
        category = None
        for i, pl in sorted((e for lst in payloads for e in lst), key=lambda e: e[0]):
            m = native.get(i)
            if m is None:
                # trained on another rank: scoring model from its MOJO + the training-side metrics
                m = GenericModel(pl["mojo"], pl["model_id"])
                m.algo = pl["algo"]
                m.params = pl["params"]     # the exploitation plan reads the explored hyper-parameters
                if te is not None and pl["algo"] in TE_ALGOS:
                    m.preprocessors = (te["model"],)
                m.training_metrics = pl["training_metrics"]
                m.validation_metrics = pl["validation_metrics"]
                m.cross_validation_metrics = pl["cross_validation_metrics"]
                m.run_time_ms = pl["run_time_ms"]
                if pl["holdout"] is not None:
                    m.cross_validation_holdout = torch.from_numpy(pl["holdout"]).to(local.device)
                DKV.put(m.model_id, m)
            category = m.category
            self.models.append(m)
            self._log("ModelTraining", f"{pl['model_id']} trained on rank {pl['rank']}")
        return category

    def _planned(self, algo: str, kind: str) -> bool:
        if self.plan is None:
            return True
        steps = self.plan.get(algo.lower())
        return steps is not None and (kind in steps or "all" in steps)

    def get_best_model(self, algorithm: str | None = None, criterion: str | None = None):
        """Best model overall, or of one algorithm family, by ``criterion``
        (a leaderboard column; default: the sort metric)."""
        rows = self.leaderboard
        if algorithm:
            a = algorithm.lower()
            a = {"basemodel": None}.get(a, a)
            rows = [r for r in rows if (r["algo"] != "stackedensemble" if a is None else r["algo"] == a)]
        if not rows:
            return None
        if criterion:
            c = criterion.lower()
            higher = c in ("auc", "aucpr")
            rows = sorted(rows, key=lambda r: (np.isnan(r.get(c, np.nan)), -r.get(c, np.nan) if higher
                                               else r.get(c, np.nan)))
        return DKV.get(rows[0]["model_id"])

    def get_leaderboard(self, extra_columns=None) -> list[dict]:
        """Leaderboard rows; ``extra_columns="ALL"`` adds training_time_ms and
        predict_time_per_row_ms (timed on up to 10k training rows)."""
        import torch

        rows = [dict(r) for r in self.leaderboard]
        extra = extra_columns if isinstance(extra_columns, (list, tuple)) else \
            (["training_time_ms", "predict_time_per_row_ms"] if str(extra_columns).upper() == "ALL" else [])
        fr = getattr(self, "_frame", None)
        for r in rows:
            m = DKV.get(r["model_id"])
            if "training_time_ms" in extra:
                r["training_time_ms"] = int(getattr(m, "run_time_ms", 0))
            if "predict_time_per_row_ms" in extra and fr is not None:
                sub = fr.rows(torch.arange(min(fr.nrows, 10000), device=fr.device))
                t = time.perf_counter()
                m.predict_raw(sub)
                if sub.device.type == "cuda":
                    torch.cuda.synchronize(sub.device)
                r["predict_time_per_row_ms"] = (time.perf_counter() - t) * 1000 / max(sub.nrows, 1)
        return rows

    @property
    def event_log(self) -> Frame:
        import pandas as pd

        return Frame.from_pandas(pd.DataFrame(self.events or [{"t": "", "stage": "", "msg": ""}]))

    def _score(self, m, key, lb_frame, comm):
        if lb_frame is not None:
            mm = m._metrics(lb_frame, m.predict_raw(lb_frame), comm)
        else:
            mm = m.cross_validation_metrics or m.training_metrics
        return mm

    def _best_of_family(self, models, category):
        _, key, higher = _metric_spec(category, self.sort_metric)
        best = {}
        for m in models:
            mm = m.cross_validation_metrics or m.training_metrics or {}
            v = mm.get(key)
            if v is None:
                continue
            fam = m.algo
            if fam not in best or (v > best[fam][0] if higher else v < best[fam][0]):
                best[fam] = (v, m)
        return [m for _, m in best.values()]

    def _rank(self, category, lb_frame, comm):
        if category is None:
            return
        sm, key, higher = _metric_spec(category, self.sort_metric)
        rows = []
        for m in self.models:
            mm = self._score(m, key, lb_frame, comm) or {}
            r = {"model_id": m.model_id, "algo": m.algo}
            if category == ModelCategory.BINOMIAL:
                cols = [("auc", "AUC"), ("logloss", "logloss"), ("aucpr", "AUCPR"),
                        ("mean_per_class_error", "mean_per_class_error"), ("rmse", "RMSE"), ("mse", "MSE")]
            elif category == ModelCategory.MULTINOMIAL:
                cols = [("mean_per_class_error", "mean_per_class_error"), ("logloss", "logloss"), ("rmse", "RMSE"),
                        ("mse", "MSE")]
            else:
                cols = [("mean_residual_deviance", "mean_residual_deviance"), ("rmse", "RMSE"), ("mse", "MSE"),
                        ("mae", "mae"), ("rmsle", "rmsle")]
            for c, k in cols:
                v = mm.get(k)
                r[c] = float(v) if v is not None else float("nan")
            r["_sort"] = float(mm.get(key, float("nan")) or float("nan"))
            rows.append(r)
        rows.sort(key=lambda r: (np.isnan(r["_sort"]), -r["_sort"] if higher else r["_sort"]))
        for r in rows:
            r.pop("_sort")
        self.leaderboard = rows
        self.sort_metric_used = sm
        self.leader = DKV.get(rows[0]["model_id"]) if rows else None

    def leaderboard_frame(self) -> Frame:
        import pandas as pd

        return Frame.from_pandas(pd.DataFrame(self.leaderboard))


def _parse_plan(plan) -> dict:
    """modeling_plan: ["GBM", ("XGBoost", "grids"), {"name": "DRF", "alias": "defaults"}, ...]
    -> {algo: {"defaults", "grids", ...}}."""
    out: dict = {}
    for item in plan:
        if isinstance(item, str):
            out[item.lower()] = {"all"}
        elif isinstance(item, dict):
            steps = item.get("steps") or [item.get("alias", "all")]
            out[str(item["name"]).lower()] = {str(s.get("id", s) if isinstance(s, dict) else s).lower() for s in steps}
        else:
            out[str(item[0]).lower()] = {str(s).lower() for s in (item[1] if isinstance(item[1], (list, tuple))
                                                                  else [item[1]])}
    return out


def get_automl(project_name: str):
    return _PROJECTS.get(project_name)


def run_automl(spec: dict, comm=None) -> dict:
    """REST entry (/99/AutoMLBuilder JSON spec) executed on every rank."""
    bc = spec.get("build_control", {}) or {}
    isp = spec.get("input_spec", {}) or {}
    bm = spec.get("build_models", {}) or {}
    sc = bc.get("stopping_criteria", {}) or {}
    aml = H2OAutoML(max_models=sc.get("max_models"), max_runtime_secs=sc.get("max_runtime_secs"),
                    max_runtime_secs_per_model=sc.get("max_runtime_secs_per_model", 0.0),
                    seed=sc.get("seed", -1), nfolds=bc.get("nfolds", -1), project_name=bc.get("project_name"),
                    include_algos=bm.get("include_algos"), exclude_algos=bm.get("exclude_algos"),
                    sort_metric=isp.get("sort_metric", "AUTO"), modeling_plan=bm.get("modeling_plan"),
                    stopping_rounds=sc.get("stopping_rounds", 3), stopping_metric=sc.get("stopping_metric", "AUTO"),
                    stopping_tolerance=sc.get("stopping_tolerance"), preprocessing=bm.get("preprocessing"),
                    parallelism=bc.get("parallelism", "auto"))
    tf = DKV.get(_key(isp.get("training_frame")))
    lf = DKV.get(_key(isp.get("leaderboard_frame"))) if isp.get("leaderboard_frame") else None
    y = isp.get("response_column")
    y = _key(y)
    ignored = set(isp.get("ignored_columns") or [])
    x = [c for c in tf.names if c != y and c not in ignored]
    aml.train(x=x, y=y, training_frame=tf, leaderboard_frame=lf, comm=comm)
    return {"project_name": aml.project_name, "leaderboard": aml.leaderboard, "events": aml.events,
            "sort_metric": getattr(aml, "sort_metric_used", None)}


def _key(v):
    if isinstance(v, dict):
        return v.get("name") or v.get("column_name")
    return v
