#!/usr/bin/env python3
"""DRF depth 20 on 10M x 100 with an explicit nbins_top_level=1024 (the 255-bin
fine grid instead of the deep-tree default of 63): ms/tree and AUC, one JSON line
a fit - the price of the opt-out recorded in docs."""
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
    from h2omx.models.tree.engine import HipTreeBuilder

    if len(sys.argv) > 1:   # segmented-histogram LDS budget for the A/B
        HipTreeBuilder.SEG_LDS_BUDGET = int(sys.argv[1])

    dev = torch.device("cuda", 0)
    X, y = wide_gaussian(10_000_000, 100, seed=5, device=dev)
    fr = Frame.from_tensor(X, y=y, y_categorical=True)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = H2ORandomForestEstimator(ntrees=10, max_depth=20, seed=1, nbins_top_level=1024).train(
            y="response", training_frame=fr)
        torch.cuda.synchronize()
        print(json.dumps({"fine_bins": 255, "budget": HipTreeBuilder.SEG_LDS_BUDGET, "rep": rep, "fit_s": round(time.perf_counter() - t0, 3),
                          "ms_per_tree": round(1000 * float(m.timings.get("train_s", 0.0)) / 10, 2),
                          "auc": round(float(m.training_metrics["AUC"]), 5)}), flush=True)


if __name__ == "__main__":
    main()
