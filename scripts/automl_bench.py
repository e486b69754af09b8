#!/usr/bin/env python3
"""AutoML at scale on one GPU (BASELINE.md AutoML row): wide-Gaussian n x p
synthetic binomial data, GBM+GLM+XGB+DRF+SE, wall time + leaderboard."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--cols", type=int, default=100)
    ap.add_argument("--max-models", type=int, default=6)
    ap.add_argument("--nfolds", type=int, default=3)
    a = ap.parse_args()
    import torch

    from h2omx.automl import H2OAutoML
    from h2omx.frame import Frame
    from h2omx.frame.synthetic import wide_gaussian

    dev = torch.device("cuda", 0)
    t0 = time.time()
    X, y = wide_gaussian(a.rows, a.cols, seed=5, device=dev)
    fr = Frame.from_tensor(X, y=y, y_categorical=True)
    aml = H2OAutoML(max_models=a.max_models, nfolds=a.nfolds, seed=1,
                    include_algos=["GBM", "GLM", "XGBoost", "DRF", "StackedEnsemble"])
    t1 = time.time()
    aml.train(y="response", training_frame=fr)
    torch.cuda.synchronize()
    t2 = time.time()
    out = {"rows": a.rows, "cols": a.cols, "max_models": a.max_models, "nfolds": a.nfolds,
           "data_s": t1 - t0, "automl_wall_s": t2 - t1,
           "leaderboard": [{k: (round(v, 5) if isinstance(v, float) else v) for k, v in r.items()}
                           for r in aml.leaderboard],
           "model_run_ms": {m.model_id: m.run_time_ms for m in aml.models}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
