"""Model builders (H2O estimator API)."""
from .base import Model, ModelBuilder, ModelCategory  # noqa: F401
from .tree_models import (H2OGradientBoostingEstimator, H2ORandomForestEstimator,  # noqa: F401
                          H2OXGBoostEstimator)
