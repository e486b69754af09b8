"""Hyper-parameter grid search (H2O ``H2OGridSearch`` / ``/99/Grid``).

A grid trains one model per hyper-parameter combination of a base
estimator.  Strategies, as in H2O:

* ``Cartesian`` (default): every combination, in lexicographic order of the
  hyper-parameter lists.
* ``RandomDiscrete``: combinations drawn without replacement from the
  Cartesian space with ``seed``, bounded by ``max_models`` /
  ``max_runtime_secs`` and optionally stopped early when the best value of
  ``stopping_metric`` over the last ``stopping_rounds`` models has not
  improved by ``stopping_tolerance`` (same moving-average rule as model
  early stopping, :mod:`h2omx.models.scoring`).

Every model is trained data-parallel over all ranks (the REST op runs the
same grid walk on every rank; the walk is deterministic so every rank
builds the same models in the same order).  Combinations that fail are
recorded in ``failed_params`` with their error, like H2O's
``failure_details``.
"""
from __future__ import annotations

import itertools
import time
import uuid

import numpy as np

from .frame.frame import DKV, Frame
from .models.base import ModelCategory
from .models.scoring import stop_early


def _metric_for(category, sort_by):
    s = (sort_by or "").lower()
    if not s or s == "auto":
        s = {ModelCategory.BINOMIAL: "logloss", ModelCategory.MULTINOMIAL: "logloss",
             ModelCategory.CLUSTERING: "tot_withinss"}.get(category, "residual_deviance")
    keys = {"auc": ("AUC", False), "aucpr": ("AUCPR", False), "logloss": ("logloss", True), "mse": ("MSE", True),
            "rmse": ("RMSE", True), "mae": ("mae", True), "rmsle": ("rmsle", True), "r2": ("r2", False),
            "residual_deviance": ("mean_residual_deviance", True),
            "mean_residual_deviance": ("mean_residual_deviance", True),
            "mean_per_class_error": ("mean_per_class_error", True), "err": ("err", True),
            "tot_withinss": ("tot_withinss", True), "betweenss": ("betweenss", False)}
    if s not in keys:
        raise ValueError(f"unsupported grid sort metric {sort_by!r}")
    key, lower = keys[s]
    return s, key, lower


def _model_metrics(m):
    if m.category == ModelCategory.CLUSTERING:
        return dict(getattr(m, "stats", {}) or {})
    return m.cross_validation_metrics or m.validation_metrics or m.training_metrics or {}


class H2OGridSearch:
    """``H2OGridSearch(model=H2OGradientBoostingEstimator, hyper_params={...},
    search_criteria={...})`` then ``.train(x=, y=, training_frame=, ...)``."""

    def __init__(self, model, hyper_params: dict, grid_id: str | None = None, search_criteria: dict | None = None,
                 parallelism: int = 1, **base_params):
        if isinstance(model, type):
            self.model_cls, self.base_params = model, dict(base_params)
        else:   # an estimator instance: its parameters are the base parameters
            self.model_cls, self.base_params = type(model), {**model.params, **base_params}
            self.base_params.pop("model_id", None)
        if not hyper_params:
            raise ValueError("hyper_params must name at least one parameter")
        self.hyper_params = {k: list(v) if isinstance(v, (list, tuple)) else [v] for k, v in hyper_params.items()}
        self.hyper_names = list(self.hyper_params)
        self.grid_id = grid_id or f"Grid_{self.model_cls.algo.upper()}_{uuid.uuid4().hex[:8]}"
        sc = dict(search_criteria or {})
        self.strategy = str(sc.get("strategy", "Cartesian"))
        if self.strategy not in ("Cartesian", "RandomDiscrete"):
            raise ValueError(f"unknown grid search strategy {self.strategy!r}")
        self.max_models = int(sc.get("max_models") or 0)
        self.max_runtime_secs = float(sc.get("max_runtime_secs") or 0.0)
        self.seed = int(sc.get("seed", -1) if sc.get("seed") is not None else -1)
        self.stopping_rounds = int(sc.get("stopping_rounds") or 0)
        self.stopping_metric = sc.get("stopping_metric", "AUTO")
        self.stopping_tolerance = float(sc.get("stopping_tolerance", 1e-3) or 1e-3)
        self.parallelism = int(parallelism or 1)
        self.models: list = []
        self.failed_params: list[dict] = []
        self.failure_details: list[str] = []
        self.category = None
        self.training_time_ms = 0

    # -- the search space ----------------------------------------------------
    def combinations(self) -> list[dict]:
        space = [dict(zip(self.hyper_names, vals)) for vals in itertools.product(*self.hyper_params.values())]
        if self.strategy == "RandomDiscrete":
            rng = np.random.default_rng(self.seed if self.seed >= 0 else 0xC0FFEE)
            space = [space[i] for i in rng.permutation(len(space))]
        return space

    def _budget_left(self, t0) -> bool:
        if self.max_models and len(self.models) + len(self.failed_params) >= self.max_models:
            return False
        return not (self.max_runtime_secs and time.time() - t0 >= self.max_runtime_secs)

    def train(self, x=None, y=None, training_frame: Frame | None = None, validation_frame: Frame | None = None,
              comm=None, **params):
        from .runtime.jobs import current_job

        t0 = time.time()
        job = current_job()
        combos = self.combinations()
        stop_values: list[float] = []
        for i, hp in enumerate(combos):
            if not self._budget_left(t0) or (job is not None and job.cancel_requested):
                break
            p = {**self.base_params, **params, **hp}
            p["model_id"] = f"{self.grid_id}_model_{len(self.models) + len(self.failed_params) + 1}"
            try:
                m = self.model_cls(**p).train(x=x, y=y, training_frame=training_frame,
                                              validation_frame=validation_frame, comm=comm)
            except Exception as e:  # noqa: BLE001 - recorded like H2O's failure_details
                self.failed_params.append(hp)
                self.failure_details.append(f"{type(e).__name__}: {e}")
                continue
            m.grid_hyper_params = hp
            self.models.append(m)
            self.category = m.category
            if job is not None:
                job.progress = min(0.99, (i + 1) / max(len(combos), 1))
            if self.strategy == "RandomDiscrete" and self.stopping_rounds > 0:
                _, key, lower = _metric_for(self.category, self.stopping_metric)
                stop_values.append(float(_model_metrics(m).get(key, float("nan")) or float("nan")))
                # best-so-far sequence: the grid stops when its best model stops improving
                best = (np.fmin if lower else np.fmax).accumulate(np.asarray(stop_values))
                if stop_early(list(best), self.stopping_rounds, lower, self.stopping_tolerance):
                    break
        self.training_time_ms = int((time.time() - t0) * 1000)
        DKV.put(self.grid_id, self)
        return self

    # -- results ---------------------------------------------------------------
    def get_grid(self, sort_by: str | None = None, decreasing: bool | None = None) -> "H2OGridSearch":
        if not self.models:
            return self
        metric, key, lower = _metric_for(self.category, sort_by)
        if decreasing is None:
            decreasing = not lower
        vals = [float(_model_metrics(m).get(key, float("nan")) or float("nan")) for m in self.models]
        order = sorted(range(len(vals)), key=lambda i: (np.isnan(vals[i]), -vals[i] if decreasing else vals[i]))
        self.models = [self.models[i] for i in order]
        self.sort_metric = metric
        return self

    @property
    def model_ids(self) -> list[str]:
        return [m.model_id for m in self.models]

    def summary_table(self, sort_by: str | None = None) -> list[dict]:
        if not self.models:
            return []
        metric, key, _ = _metric_for(self.category, sort_by or getattr(self, "sort_metric", None))
        rows = []
        for m in self.models:
            r = {k: m.grid_hyper_params.get(k) for k in self.hyper_names}
            r["model_ids"] = m.model_id
            r[metric] = _model_metrics(m).get(key)
            rows.append(r)
        return rows

    def to_json(self) -> dict:
        from .models.base import _jsonable

        return {"grid_id": {"name": self.grid_id, "type": "Key<Grid>", "URL": f"/99/Grids/{self.grid_id}"},
                "model_ids": [{"name": k, "type": "Key<Model>", "URL": f"/3/Models/{k}"} for k in self.model_ids],
                "hyper_names": self.hyper_names,
                "failed_params": [_jsonable(p) for p in self.failed_params],
                "failure_details": self.failure_details,
                "summary_table": _jsonable(self.summary_table()),
                "training_time_ms": self.training_time_ms,
                "search_criteria": {"strategy": self.strategy, "max_models": self.max_models,
                                    "max_runtime_secs": self.max_runtime_secs, "seed": self.seed,
                                    "stopping_rounds": self.stopping_rounds}}


def run_grid(algo: str, params: dict, hyper_params: dict, search_criteria: dict | None, x, y, training_frame: str,
             validation_frame: str | None, grid_id: str, comm=None) -> dict:
    """REST entry (/99/Grid/{algo}) executed on every rank."""
    from .models import ESTIMATORS

    cls = ESTIMATORS.get(algo)
    if cls is None:
        raise ValueError(f"unknown algorithm {algo!r}")
    grid = H2OGridSearch(cls, hyper_params, grid_id=grid_id, search_criteria=search_criteria, **params)
    tf = DKV.get(training_frame)
    vf = DKV.get(validation_frame) if validation_frame else None
    grid.train(x=x, y=y, training_frame=tf, validation_frame=vf, comm=comm)
    return grid.to_json()
