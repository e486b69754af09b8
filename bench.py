#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): GBM binomial training throughput on
HIGGS-shape 11M x 28 synthetic data, one rank per MI355X.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

One *step* is one full boosting iteration: gradients + a depth-5 tree grown
level by level on the GPU (LDS histograms, fp64 reduce, RCCL all-reduce of
the level histograms when N > 1, split scan, partition) + margin update.
``value`` = total training rows x K / max-over-ranks wall time of the K timed
steps = aggregate row-trees per second.  Scaling is *weak* by default: every
rank holds its own 11M-row HIGGS-shape shard (global rows = N x 11M); use
``--scaling strong`` to split 11M rows over the ranks instead.  Training AUC
of the final model (all ranks) is reported next to the throughput.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

METRIC = "GBM train rows/sec on HIGGS-shape 11M×28 at 1/2/4/8 MI355X; AUC parity"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=11_000_000)
    ap.add_argument("--cols", type=int, default=28)
    ap.add_argument("--max-depth", type=int, default=5)
    ap.add_argument("--nbins", type=int, default=255)
    ap.add_argument("--learn-rate", type=float, default=0.1)
    ap.add_argument("--min-rows", type=float, default=10.0)
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-auc", action="store_true")
    ap.add_argument("--oracle-rows", type=int, default=0,
                    help="also fit sklearn HistGradientBoosting on this many rows for AUC parity")
    args = ap.parse_args(argv)

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from h2omx.frame.synthetic import higgs_like
    from h2omx.metrics.core import auc_from_scores
    from h2omx.models.tree import TreeParams, bin_matrix, compute_edges
    from h2omx.models.tree.boost import GpuBooster, TreeEnsemble, init_margin
    from h2omx.parallel.comm import Comm

    comm = Comm.from_env("cuda")
    dev = comm.device
    world, rank = comm.world_size, comm.rank
    if args.scaling == "weak":
        n_local = args.rows
    else:
        n_local = args.rows // world + (1 if rank < args.rows % world else 0)

    t_setup = time.perf_counter()
    X, y = higgs_like(n_local, seed=args.seed + 1000 * rank, device=dev)
    if args.cols != 28:
        X = X[: args.cols].contiguous() if args.cols < 28 else torch.cat(
            [X, torch.randn((args.cols - 28, n_local), device=dev)])
    edges, nvb, nbt = compute_edges(X, args.nbins, comm=comm)
    bm = bin_matrix(X, edges, nvb, nbt)
    tp = TreeParams(max_depth=args.max_depth, min_rows=args.min_rows, learn_rate=args.learn_rate, mode=0,
                    leaf_mode=0, min_split_improvement=1e-5, seed=args.seed)
    y_np = y.cpu().numpy()
    sums = comm.all_reduce_numpy(__import__("numpy").array([y_np.sum(), float(len(y_np))]))
    p0 = min(max(sums[0] / sums[1], 1e-6), 1 - 1e-6)
    import numpy as np

    ens = TreeEnsemble(trees=np.zeros((0, 1)), K=1, dist="bernoulli",
                       init_f=np.array([np.log(p0 / (1 - p0))]), nbt=nbt, feature_names=bm.names)
    gb = GpuBooster(bm, y_np, None, ens, tp, 1.0, args.seed, comm, {})
    torch.cuda.synchronize(dev)
    comm.barrier()
    setup_s = time.perf_counter() - t_setup

    for _ in range(args.warmup):
        gb.step()
    torch.cuda.synchronize(dev)
    comm.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        gb.step()
    torch.cuda.synchronize(dev)
    comm.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    elapsed = comm.max_scalar(elapsed)

    total_rows = int(comm.all_reduce_numpy(np.array([float(n_local)]))[0])
    value = total_rows * args.steps / elapsed
    auc = None
    if not args.no_auc:
        margin = gb.st.Fm[0, : bm.n]
        auc = auc_from_scores(margin, y, comm=comm)
    oracle = None
    if args.oracle_rows and rank == 0:
        from sklearn.ensemble import HistGradientBoostingClassifier
        from sklearn.metrics import roc_auc_score

        m = min(args.oracle_rows, n_local)
        Xs = X[:, :m].T.cpu().numpy()
        ys = y[:m].cpu().numpy()
        ntr = args.warmup + args.steps
        clf = HistGradientBoostingClassifier(max_iter=ntr, max_depth=args.max_depth, learning_rate=args.learn_rate,
                                             min_samples_leaf=int(args.min_rows), max_bins=min(args.nbins, 255),
                                             early_stopping=False, l2_regularization=0.0).fit(Xs, ys)
        oracle = {"rows": m, "sklearn_train_auc": float(roc_auc_score(ys, clf.decision_function(Xs))),
                  "h2omx_train_auc_same_rows": float(roc_auc_score(ys, gb.st.Fm[0, :m].cpu().numpy()))}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "rows/s (row-trees per second, all GPUs)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "fp32 (gradients/hessians), fp64 histogram reduce, uint8 bins",
            "data": "synthetic HIGGS-shape (28 cols) generated on device; random seed per rank",
            "config": {"model": "GBM bernoulli", "global_batch": total_rows, "seq_len": None,
                       "rows_per_gpu": n_local, "cols": args.cols, "max_depth": args.max_depth,
                       "nbins": args.nbins, "learn_rate": args.learn_rate, "min_rows": args.min_rows,
                       "parallelism": f"dp{world}"},
            "train_auc": auc,
            "setup_s": setup_s,
        }
        if oracle:
            out["oracle"] = oracle
        print(json.dumps(out), flush=True)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
