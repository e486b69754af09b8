#!/usr/bin/env python3
"""Host-side profile (cProfile) of one DRF fit (depth 20, 10 trees, 10M x 100):
where the fixed per-fit time outside the tree kernels goes."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from h2omx.frame import Frame
    from h2omx.frame.synthetic import wide_gaussian
    from h2omx.models import H2ORandomForestEstimator

    dev = torch.device("cuda", 0)
    X, y = wide_gaussian(10_000_000, 100, seed=5, device=dev)
    fr = Frame.from_tensor(X, y=y, y_categorical=True)
    H2ORandomForestEstimator(ntrees=2, max_depth=20, seed=1).train(y="response", training_frame=fr)   # warm-up
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    ntrees = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    nfolds = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    m = H2ORandomForestEstimator(ntrees=ntrees, max_depth=20, seed=1, nfolds=nfolds).train(y="response",
                                                                                          training_frame=fr)
    torch.cuda.synchronize()
    pr.disable()
    print(f"DRF {ntrees} trees, nfolds {nfolds}: {time.perf_counter() - t:.3f} s, train_s {m.timings.get('train_s')}",
          flush=True)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(70)
    print(s.getvalue())


if __name__ == "__main__":
    main()
