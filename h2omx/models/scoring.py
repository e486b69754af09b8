"""Scoring history and early stopping (H2O ScoreKeeper semantics).

Every ``score_interval`` iterations a model builder records training (and
validation) metrics; ``stopping_rounds = k > 0`` stops training when the
moving average (window k) of ``stopping_metric`` over the last k scoring
events has not improved on the best earlier moving average by at least the
relative ``stopping_tolerance``.  ``AUTO`` = logloss (classification),
deviance (regression).
"""
from __future__ import annotations

import math

import numpy as np
import torch

LOWER_IS_BETTER = {"logloss": True, "deviance": True, "mse": True, "rmse": True, "mae": True, "rmsle": True,
                   "mean_per_class_error": True, "misclassification": True, "auc": False, "aucpr": False,
                   "r2": False}

_METRIC_KEYS = {"logloss": "logloss", "deviance": "mean_residual_deviance", "mse": "MSE", "rmse": "RMSE",
                "mae": "mae", "rmsle": "rmsle", "mean_per_class_error": "mean_per_class_error", "auc": "AUC",
                "aucpr": "AUCPR", "r2": "r2"}


def resolve_metric(name: str, category: str) -> str:
    n = (name or "AUTO").lower()
    if n == "auto":
        return "logloss" if category in ("Binomial", "Multinomial") else "deviance"
    if n not in _METRIC_KEYS:
        raise ValueError(f"unsupported stopping_metric {name}")
    return n


def metric_value(metrics: dict, name: str) -> float:
    v = metrics.get(_METRIC_KEYS[name])
    return float("nan") if v is None else float(v)


def stop_early(values: list[float], k: int, lower_is_better: bool, tolerance: float) -> bool:
    v = [x for x in values if x is not None and math.isfinite(x)]
    if k <= 0 or len(v) < 2 * k:
        return False
    a = np.convolve(np.asarray(v, np.float64), np.ones(k) / k, mode="valid")   # moving averages
    last = a[-1]
    prev = a[: len(a) - k] if len(a) > k else a[:1]
    best = prev.min() if lower_is_better else prev.max()
    if best == 0:
        return False
    rel = (best - last) / abs(best) if lower_is_better else (last - best) / abs(best)
    return bool(rel < tolerance)


class ScoreKeeper:
    def __init__(self, metric: str, category: str, k: int, tolerance: float):
        self.metric = resolve_metric(metric, category)
        self.k = int(k or 0)
        self.tol = float(tolerance)
        self.lower = LOWER_IS_BETTER[self.metric]
        self.values: list[float] = []
        self.history: list[dict] = []

    def record(self, entry: dict, metrics: dict) -> bool:
        """Add one scoring event; returns True when training should stop."""
        self.history.append(entry)
        self.values.append(metric_value(metrics, self.metric))
        return stop_early(self.values, self.k, self.lower, self.tol)


def margins_to_scores(margin: torch.Tensor, dist: str, category: str, ntrees: int = 1) -> torch.Tensor:
    """Tree-ensemble margins [K][n] -> scores as TreeModel.predict_raw returns them."""
    if dist == "drf":
        m = margin / max(ntrees, 1)
        if category == "Binomial":
            p1 = m[0].clamp(0, 1)
            return torch.stack([1 - p1, p1])
        if category == "Multinomial":
            mm = m.clamp_min(0)
            s = mm.sum(0, keepdim=True)
            return torch.where(s > 0, mm / s.clamp_min(1e-30), torch.full_like(mm, 1.0 / mm.shape[0]))
        return m
    if category == "Binomial":
        p1 = torch.sigmoid(margin[0])
        return torch.stack([1 - p1, p1])
    if category == "Multinomial":
        return torch.softmax(margin, 0)
    if dist in ("poisson", "gamma", "tweedie"):
        return torch.exp(margin)
    return margin
