"""Model metrics (H2O ModelMetrics* equivalents)."""
from .core import (auc_from_scores, binomial_metrics, multinomial_metrics,  # noqa: F401
                   regression_metrics)
