"""One DRF (depth 20) and one GLM lambda-search fit on the AutoML shape, with engine phase timers."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.synthetic import wide_gaussian  # noqa: E402
from h2omx.models import H2OGeneralizedLinearEstimator, H2ORandomForestEstimator  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
which = sys.argv[2] if len(sys.argv) > 2 else "drf,glm"
X, y = wide_gaussian(rows, 100, seed=5, device="cuda")
fr = Frame.from_tensor(X, y=y, y_categorical=True)
if "drf" in which:
    for nt in (2, 10):
        torch.cuda.synchronize()
        t = time.time()
        m = H2ORandomForestEstimator(ntrees=nt, seed=1).train(y="response", training_frame=fr)
        torch.cuda.synchronize()
        print(f"DRF {nt} trees: {time.time() - t:.2f} s timings {m.timings}", flush=True)
if "glm" in which:
    for ls in (False, True):
        torch.cuda.synchronize()
        t = time.time()
        m = H2OGeneralizedLinearEstimator(family="binomial", lambda_search=ls).train(y="response", training_frame=fr)
        torch.cuda.synchronize()
        print(f"GLM lambda_search={ls}: {time.time() - t:.2f} s iterations {m.stats['iterations']}", flush=True)
