"""GPU fits of the main estimators must not import the CPU reference package
(h2omx.reference): run in a fresh interpreter, print the verdict as JSON."""
import json
import sys

import numpy as np
import pandas as pd
import torch

from h2omx.frame import Frame
from h2omx.models import (H2ODeepLearningEstimator, H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                          H2OKMeansEstimator, H2ORandomForestEstimator, H2OXGBoostEstimator)

rng = np.random.default_rng(0)
n = 20000
X = rng.normal(size=(n, 6))
df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
df["y"] = pd.Categorical(np.where(X[:, 0] + X[:, 1] * X[:, 2] > 0, "a", "b"))
fr = Frame.from_pandas(df, device=torch.device("cuda", 0))
for est in (H2OGradientBoostingEstimator(ntrees=5), H2OXGBoostEstimator(ntrees=5), H2ORandomForestEstimator(ntrees=3),
            H2OGeneralizedLinearEstimator(family="binomial"), H2ODeepLearningEstimator(hidden=[16], epochs=1)):
    est.train(y="y", training_frame=fr)
H2OKMeansEstimator(k=3).train(x=[f"x{i}" for i in range(6)], training_frame=fr)
print(json.dumps({"reference_loaded": sorted(m for m in sys.modules if m.startswith("h2omx.reference"))}))
