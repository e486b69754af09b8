"""AutoML's deep presets on 10M x 100 (XGBoost_2: depth 20, GBM_5: depth 15), 10 trees each,
wall time per engine setting given as KEY=VALUE overrides of HipTreeBuilder attributes."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.synthetic import wide_gaussian  # noqa: E402
from h2omx.models import H2OGradientBoostingEstimator, H2OXGBoostEstimator  # noqa: E402
import h2omx.models.tree.engine as E  # noqa: E402

X, y = wide_gaussian(10_000_000, 100, seed=5, device="cuda")
fr = Frame.from_tensor(X, y=y, y_categorical=True)
cfgs = [dict(a.split("=") for a in arg.split(",")) if arg != "default" else {} for arg in (sys.argv[1:] or ["default"])]
for cfg in cfgs:
    saved = {k: getattr(E.HipTreeBuilder, k) for k in cfg}
    for k, v in cfg.items():
        setattr(E.HipTreeBuilder, k, type(saved[k])(float(v)) if not isinstance(saved[k], bool) else v == "1")
    for name, cls, kw in (("XGBoost_2", H2OXGBoostEstimator, dict(max_depth=20, min_child_weight=10, sample_rate=0.6,
                                                                    col_sample_rate=0.8, col_sample_rate_per_tree=0.8)),
                          ("GBM_5", H2OGradientBoostingEstimator, dict(max_depth=15, min_rows=100, sample_rate=0.8,
                                                                        col_sample_rate=0.8,
                                                                        col_sample_rate_per_tree=0.8))):
        torch.cuda.synchronize()
        t = time.time()
        m = cls(ntrees=10, seed=1, **kw).train(y="response", training_frame=fr)
        torch.cuda.synchronize()
        print(f"{cfg or 'default'} {name} 10 trees: {time.time() - t:.2f} s (train {m.timings.get('train_s', 0):.2f})",
              flush=True)
    for k, v in saved.items():
        setattr(E.HipTreeBuilder, k, v)
