"""Time the AutoML building blocks on the 10M x 100 AutoML shape (one fit each)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.synthetic import wide_gaussian  # noqa: E402
from h2omx.models import (H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,  # noqa: E402
                          H2ORandomForestEstimator, H2OXGBoostEstimator)

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
X, y = wide_gaussian(rows, 100, seed=5, device="cuda")
fr = Frame.from_tensor(X, y=y, y_categorical=True)
for name, est in [("glm", H2OGeneralizedLinearEstimator(family="binomial")),
                  ("drf", H2ORandomForestEstimator(ntrees=50, seed=1)),
                  ("gbm_d6", H2OGradientBoostingEstimator(ntrees=50, max_depth=6, seed=1)),
                  ("xgb", H2OXGBoostEstimator(ntrees=50, seed=1))]:
    torch.cuda.synchronize()
    t = time.time()
    m = est.train(y="response", training_frame=fr)
    torch.cuda.synchronize()
    tm = {k: round(v, 3) if isinstance(v, float) else v for k, v in (m.timings or {}).items()}
    print(f"{name}: {time.time() - t:.2f} s  AUC {m.training_metrics['AUC']:.4f}  timings {tm}", flush=True)
