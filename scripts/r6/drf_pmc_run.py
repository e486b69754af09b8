#!/usr/bin/env python3
"""DRF depth 20 on wide-Gaussian 10M x 100 (estimator defaults), a short fit
for counter collection: drf_pmc_run.py [rows] [ntrees]."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from h2omx.frame import Frame
    from h2omx.frame.synthetic import wide_gaussian
    from h2omx.models import H2ORandomForestEstimator

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    ntrees = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = torch.device("cuda", 0)
    X, y = wide_gaussian(rows, 100, seed=5, device=dev)
    fr = Frame.from_tensor(X, y=y, y_categorical=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = H2ORandomForestEstimator(ntrees=ntrees, max_depth=20, seed=1).train(y="response", training_frame=fr)
    torch.cuda.synchronize()
    print(json.dumps({"fit_s": round(time.perf_counter() - t0, 3), "ntrees": ntrees,
                      "auc": round(float(m.training_metrics["AUC"]), 5)}), flush=True)


if __name__ == "__main__":
    main()
