#!/usr/bin/env python3
"""Cost of the per-node histogram rule (histogram_type AUTO = UniformAdaptive)
against global QuantilesGlobal bins on the AutoML shapes: DRF depth 20 and
GBM on wide-Gaussian 10M x 100 (one GPU).  One JSON line per fit: wall time,
tree nodes, training AUC."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from h2omx.frame import Frame
    from h2omx.frame.synthetic import wide_gaussian
    from h2omx.models import H2OGradientBoostingEstimator, H2ORandomForestEstimator

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    dev = torch.device("cuda", 0)
    X, y = wide_gaussian(rows, 100, seed=5, device=dev)
    fr = Frame.from_tensor(X, y=y, y_categorical=True)
    cfgs = [("drf", H2ORandomForestEstimator, dict(ntrees=10, max_depth=20), ht, top)
            for ht, top in (("QuantilesGlobal", 1024), ("AUTO", 1024), ("AUTO", 127), ("AUTO", 63), ("AUTO", 31),
                            ("QuantilesGlobal", 1024), ("AUTO", 1024), ("AUTO", 63))]
    cfgs += [("gbm", H2OGradientBoostingEstimator, dict(ntrees=30, max_depth=6), ht, 1024)
             for ht in ("QuantilesGlobal", "AUTO", "QuantilesGlobal", "AUTO")]
    for algo, cls, kw, ht, top in cfgs:
        if True:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = cls(seed=1, histogram_type=ht, nbins_top_level=top, **kw).train(y="response", training_frame=fr)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            nodes = int(sum(len(c) for c in m.ens.compact()))
            print(json.dumps({"algo": algo, "histogram_type": ht, "nbins_top_level": top, "fit_s": round(dt, 3),
                              "train_s": round(float(m.timings.get("train_s", 0.0)), 3),
                              "nodes": nodes, "auc": round(float(m.training_metrics["AUC"]), 5)}), flush=True)


if __name__ == "__main__":
    main()
