#!/usr/bin/env python3
"""Benchmarks (BASELINE.json / BASELINE.md), one rank per MI355X.

    python bench.py --gpus N --steps K --warmup W                 # headline (N > 1: one
                                                                  #   child rank per GPU)
    torchrun --nproc-per-node N bench.py --gpus N ...             # driver, N > 1
    python bench.py --model xgboost-airlines | dl-mlp ...         # other BASELINE configs

Headline (default, ``--model gbm-higgs``): GBM binomial training throughput
on HIGGS-shape 11M x 28 synthetic data.  One *step* is one full boosting
iteration: gradients + a depth-5 tree grown level by level on the GPU (LDS
histograms, exact integer reduce, RCCL all-reduce of the level histograms
when N > 1, split scan, partition, leaf values) + margin update.
``value`` = total training rows x K / max-over-ranks wall time of the K
timed steps = aggregate row-trees per second.  Scaling is *strong* by
default for the headline: the metric is "HIGGS-shape 11M x 28 at 1/2/4/8
MI355X", so the same 11M rows (same seed) are split over the N ranks and
N ranks grow the 1-rank trees; ``--scaling weak`` gives every rank its own
11M-row shard instead (global rows = N x 11M).  Each step is replayed as a
HIP graph when eligible (``--tree-graph``); after the timed steps a few
instrumented steps report the host-enqueue, per-phase and collective time
per tree.  Training AUC of the final model (all ranks) is reported;
``--oracle-rows R`` adds a scikit-learn HistGradientBoosting fit on R rows
for AUC parity.

``xgboost-airlines``: XGBoost-hist (second-order gain, depth 6, eta 0.3) on
Airlines-shape 31-column data, 150M rows over 8 GPUs = 18.75M rows per GPU
(weak).  ``dl-mlp``: H2O DeepLearning MLP 4x512 (Rectifier, ADADELTA,
softmax) on 200 features, 50M rows over 8 GPUs = 6.25M rows per GPU; one
step = one synchronous mini-batch (``--batch`` rows per GPU) forward +
backward + gradient all-reduce + update; value = samples/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

METRIC = "GBM train rows/sec on HIGGS-shape 11M×28 at 1/2/4/8 MI355X; AUC parity"


def _sync(torch, dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _timed(step, args, comm, torch, dev, finish=None):
    """W untimed + K timed steps; ``finish`` (inside both windows) completes
    work the step function may hold back (multi-tree graph replays)."""
    for _ in range(args.warmup):
        step()
    if finish is not None:
        finish()
    _sync(torch, dev)
    comm.barrier()
    _sync(torch, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if finish is not None:
        finish()
    _sync(torch, dev)
    comm.barrier()
    _sync(torch, dev)
    return comm.max_scalar(time.perf_counter() - t0)


def _trees(args, comm, torch, np, model):
    from h2omx.frame.synthetic import airlines_like, higgs_like
    from h2omx.metrics.core import auc_from_scores
    from h2omx.models.tree import TreeParams, bin_matrix, compute_edges
    from h2omx.models.tree.boost import GpuBooster, TreeEnsemble, train_ensemble

    dev = comm.device
    world, rank = comm.world_size, comm.rank
    rows = args.rows or (11_000_000 if model == "gbm-higgs" else 150_000_000 // 8)
    strong = args.scaling == "strong"
    # --loopback-ranks N (1 GPU): this process stands in for N ranks of the
    # strong-scaled job - `rows` is ONE rank's shard and the tree engine runs the
    # N-rank launch sequence (P2P exchanges against its own buffers), so the
    # timed step is the 8-GPU step minus only the xGMI link
    tcomm = comm
    if args.loopback_ranks > 1:
        if world != 1 or dev.type != "cuda":
            raise SystemExit("--loopback-ranks needs one rank on a GPU")
        from h2omx.parallel.comm import LoopbackComm

        tcomm = LoopbackComm(dev, args.loopback_ranks)
        strong = False
    t_setup = time.perf_counter()
    gen = higgs_like if model == "gbm-higgs" else airlines_like
    if strong:
        # strong scaling: the SAME global data set at every N (every rank generates
        # it with the global seed and keeps its contiguous row slice), so N ranks
        # train on exactly the rows of the 1-rank run and grow the same trees
        lo, hi = rows * rank // world, rows * (rank + 1) // world
        X, y = gen(rows, seed=args.seed, device=dev)
        X_full = X
        X, y = X[:, lo:hi].contiguous(), y[lo:hi].contiguous()
    else:
        X, y = gen(rows, seed=args.seed + 1000 * rank, device=dev)
        X_full = None
    n_local = X.shape[1]
    if model == "gbm-higgs":
        if args.cols != 28:
            X = X[: args.cols].contiguous() if args.cols < 28 else torch.cat(
                [X, torch.randn((args.cols - 28, n_local), device=dev)])
            X_full = None
        depth = args.max_depth or 5
        tp = TreeParams(max_depth=depth, min_rows=args.min_rows, learn_rate=args.learn_rate or 0.1, mode=0,
                        leaf_mode=0, min_split_improvement=1e-5, seed=args.seed)
    else:
        depth = args.max_depth or 6
        tp = TreeParams(max_depth=depth, min_rows=0.0, min_child_weight=1.0, reg_lambda=1.0, gamma=0.0,
                        learn_rate=args.learn_rate or 0.3, mode=1, leaf_mode=0, min_split_improvement=0.0,
                        seed=args.seed)
    if X_full is not None:
        # strong scaling: cut points of the global data (= the 1-rank run's)
        edges, nvb, nbt = compute_edges(X_full, args.nbins)
        del X_full
    else:
        edges, nvb, nbt = compute_edges(X, args.nbins, comm=comm)
    bm = bin_matrix(X, edges, nvb, nbt)
    y_np = y.cpu().numpy()
    sums = tcomm.all_reduce_numpy(np.array([y_np.sum(), float(len(y_np))]))
    p0 = min(max(sums[0] / sums[1], 1e-6), 1 - 1e-6)
    init = np.log(p0 / (1 - p0)) if model == "gbm-higgs" else 0.0   # XGBoost base_score 0.5
    ens = TreeEnsemble(trees=np.zeros((0, 1)), K=1, dist="bernoulli", init_f=np.array([init]), nbt=nbt,
                       feature_names=bm.names)
    gb = None
    if dev.type == "cuda":
        gb = GpuBooster(bm, y_np, None, ens, tp, 1.0, args.seed, tcomm, {})
        _sync(torch, dev)
        comm.barrier()
        setup_s = time.perf_counter() - t_setup
        tcomm.collective_stats(reset=True)
        elapsed = _timed(gb.step, args, comm, torch, dev, finish=gb.flush)
        coll = tcomm.collective_stats()
        gb.flush()   # fused mode: the last tree is applied inside the next step's level 0
        margin = gb.st.Fm[0, : bm.n]
        graph_used = gb.graph is not None
        graph_group = gb.graph.group if gb.graph is not None else 0
    else:
        # CPU rehearsal (reference tree builder): the boosting loop owns the
        # iterations, so the timed window is opened / closed from its callback
        setup_s = time.perf_counter() - t_setup
        clock = {}

        def cb(t, view):
            if t == args.warmup - 1 or (args.warmup == 0 and t == -1):
                comm.barrier()
                clock["t0"] = time.perf_counter()
            return None

        if args.warmup == 0:
            cb(-1, None)
        ens = train_ensemble(bm, y, dist="bernoulli",
                             ntrees=args.warmup + args.steps, tparams=tp, seed=args.seed, comm=comm,
                             init_f=np.array([init]), callback=cb)
        comm.barrier()
        elapsed = comm.max_scalar(time.perf_counter() - clock["t0"])
        margin = torch.from_numpy(ens._cpu_margin[0])
        coll, graph_used, graph_group = comm.collective_stats(), False, 0
    total_rows = int(comm.all_reduce_numpy(np.array([float(n_local)]))[0])
    if args.dump_trees:
        trees = gb.finish().trees if gb is not None else ens.trees
        if rank == 0:
            np.save(args.dump_trees, trees)
    auc = None
    if not args.no_auc:
        auc = auc_from_scores(margin, y, comm=comm)
    per_tree = None
    if gb is not None and args.instrument_steps > 0:
        per_tree = _instrument(gb, args, tcomm, torch, dev)
    fit = None
    fit_trees = args.fit_trees if args.fit_trees >= 0 else (50 if dev.type == "cuda" and tcomm is comm else 0)
    if fit_trees > 0:
        gb = None   # release the timed booster's buffers before the end-to-end fit
        fit = _fit_end_to_end(X, y, fit_trees, tp, args, comm, torch, dev, total_rows)
    out = {
        "metric": METRIC if model == "gbm-higgs" else
        "XGBoost-hist train rows/sec on Airlines-shape 150M×31 (18.75M rows per MI355X); AUC",
        "value": total_rows * args.steps / elapsed,
        "unit": "rows/s (row-trees per second, all GPUs)",
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True,
        "dtype": "fp32 gradients/hessians; histograms in fixed-point int32 (stochastic rounding) summed "
                 "exactly in int64; fp64 split gains; exact int64 leaf sums; uint8 bins",
        "data": f"synthetic {'HIGGS' if model == 'gbm-higgs' else 'Airlines'}-shape generated on device; "
                + ("one global data set (global seed), contiguous row slice per rank" if strong
                   else "own shard per rank (seed per rank)"),
        "config": {"model": "GBM bernoulli" if model == "gbm-higgs" else "XGBoost hist binary:logistic",
                   "global_batch": total_rows, "seq_len": None, "rows_per_gpu": n_local,
                   "cols": int(bm.F), "max_depth": depth, "nbins": args.nbins, "learn_rate": tp.learn_rate,
                   "min_rows": tp.min_rows, "parallelism": f"dp{world}"},
        "train_auc": auc,
        "setup_s": setup_s,
        "graph_replay": graph_used,
        "graph_trees_per_replay": graph_group,
        "collectives_per_tree": {"calls": coll["all_reduce_calls"] / max(args.steps, 1),
                                 "bytes": coll["all_reduce_bytes"] / max(args.steps, 1),
                                 "host_us": 1e6 * coll["all_reduce_s"] / max(args.steps, 1)},
        # collectives the host issued per timed tree (RCCL / gloo calls between graph
        # segments); 0 when the step graph carries its own P2P collectives
        "collectives_host_issued_per_tree": coll["all_reduce_calls"] / max(args.steps, 1),
        "collective_transport": _transport(tcomm),
    }
    if tcomm is not comm:
        out["metric"] += f" [LOOPBACK PROXY: 1 GPU standing in for {tcomm.world_size} ranks of {rows} rows each]"
        out["value"] = None
        out["loopback"] = {"ranks": tcomm.world_size, "rows_per_rank": n_local,
                           "note": "the N-rank launch sequence timed on one GPU (P2P exchanges read this GPU's own "
                                   "buffers N times); trees are those of N identical shards"}
        tcomm.shutdown()
    if per_tree is not None:
        out.update(per_tree)
    if fit is not None:
        out.update(fit)
    if args.oracle_rows and rank == 0:
        from sklearn.ensemble import HistGradientBoostingClassifier
        from sklearn.metrics import roc_auc_score

        m = min(args.oracle_rows, n_local)
        Xs = X[:, :m].T.cpu().numpy()
        ys = y[:m].cpu().numpy()
        clf = HistGradientBoostingClassifier(max_iter=args.warmup + args.steps, max_depth=depth,
                                             learning_rate=tp.learn_rate, min_samples_leaf=max(1, int(args.min_rows)),
                                             max_bins=min(args.nbins, 255), early_stopping=False,
                                             l2_regularization=0.0).fit(Xs, ys)
        out["oracle"] = {"rows": m, "sklearn_hgb_train_auc": float(roc_auc_score(ys, clf.decision_function(Xs))),
                         "h2omx_train_auc_same_rows": float(roc_auc_score(ys, margin[:m].cpu().numpy()))}
    return out


def _transport(comm):
    if comm.world_size == 1:
        return "none (1 rank)"
    if getattr(comm.p2p, "loopback", False):
        return f"p2p loopback ({comm.world_size} stand-in ranks, one GPU)"
    if comm.p2p is not None:
        return "p2p (one-shot IPC all-reduce kernels in the step graph)"
    import torch.distributed as dist

    be = dist.get_backend()
    return ("rccl" if be == "nccl" else be) + (f" (p2p off: {comm.p2p_error})" if comm.p2p_error else "")


def _instrument(gb, args, comm, torch, dev):
    """Per-tree cost structure, measured AFTER the timed steps on the same
    booster (extra trees; the reported model / AUC are taken before this):

    * ``host_enqueue_us_per_tree``: host time to enqueue one step with the GPU
      idle (synchronised before and after), with graph replay when the timed
      run used it and for the eager launch sequence;
    * ``phase_us_per_tree``: device time per phase (HIP events, eager steps);
      ``small_kernel_us_per_tree`` = hist_reduce + split + tree_begin + leaf,
      the launch-latency-bound part that does not shrink with rows per GPU;
    * ``allreduce_us_per_tree``: device time of the collectives (events around
      each RCCL call on the compute stream: includes waiting for the slowest
      rank) and their count / bytes."""
    b = gb.builder
    k = args.instrument_steps
    out = {}

    def enqueue_us(n):
        ts = []
        for _ in range(n):
            _sync(torch, dev)
            comm.barrier()
            t0 = time.perf_counter()
            gb.step()
            gb.flush()     # one step = one single-tree replay here
            ts.append(time.perf_counter() - t0)
            _sync(torch, dev)
        return 1e6 * float(np.median(ts))

    import numpy as np

    if gb.graph is not None:
        out["host_enqueue_us_per_tree_graph"] = enqueue_us(k)
    # eager launch sequence with per-phase device timers
    gb.graph, gb.use_graph = None, False
    b.tree_ctr = None
    out["host_enqueue_us_per_tree_eager"] = enqueue_us(k)
    b.timer.enabled = True
    comm.enable_timing(True)
    comm.collective_stats(reset=True)
    b.timer.acc.clear()
    for _ in range(k):
        gb.step()
    _sync(torch, dev)
    ph = {name: 1000.0 * v / k for name, v in b.timer.totals().items()}
    coll = comm.collective_stats()
    comm.enable_timing(False)
    b.timer.enabled = False
    ph["grad"] = ph.get("grad", 0.0)
    out["host_enqueue_us_per_tree"] = out.get("host_enqueue_us_per_tree_graph", out["host_enqueue_us_per_tree_eager"])
    out["phase_us_per_tree"] = {n: round(v, 1) for n, v in ph.items()}
    out["small_kernel_us_per_tree"] = round(sum(ph.get(n, 0.0) for n in ("hist_reduce", "split", "tree_begin",
                                                                         "leaf")), 1)
    out["allreduce_us_per_tree"] = round(ph.get("allreduce", 0.0), 1)
    out["allreduce_calls_per_tree"] = (coll["all_reduce_calls"] + coll.get("p2p_calls", 0)) / k
    out["allreduce_bytes_per_tree"] = coll["all_reduce_bytes"] / k
    out["instrument_note"] = (f"{k} extra eager trees after the timed run with HIP-event phase timers "
                              "(phase sums include event overhead); host enqueue = median over steps with the GPU idle")
    return out


def _fit_end_to_end(X, y, ntrees, tp, args, comm, torch, dev, total_rows):
    """Whole H2O-style fit on the raw feature matrix, timed wall-clock (max
    over ranks): quantile sketch + binning + initial margin + ``ntrees`` trees
    + final training AUC -> ``fit_rows_per_s`` = training rows / fit seconds
    (the per-tree ``value`` above is the steady-state boosting rate)."""
    from h2omx.metrics.core import auc_from_scores
    from h2omx.models.tree import bin_matrix, compute_edges
    from h2omx.models.tree.boost import train_ensemble

    _sync(torch, dev)
    comm.barrier()
    t0 = time.perf_counter()
    edges, nvb, nbt = compute_edges(X, args.nbins, comm=comm)
    bm = bin_matrix(X, edges, nvb, nbt)
    ens = train_ensemble(bm, y, dist="bernoulli", ntrees=ntrees, tparams=tp, seed=args.seed,
                         comm=comm if comm.world_size > 1 else None)
    auc = auc_from_scores(ens._state.Fm[0, : bm.n], y, comm=comm)
    _sync(torch, dev)
    comm.barrier()
    dt = comm.max_scalar(time.perf_counter() - t0)
    return {"fit_rows_per_s": total_rows / dt, "fit_s": dt, "fit_trees": ntrees, "fit_train_auc": auc,
            "fit_note": "end-to-end: quantile sketch + binning + init + trees + final AUC, wall clock"}


def _mlp(args, comm, torch, np):
    from h2omx.frame.synthetic import wide_gaussian
    from h2omx.models.deeplearning import H2ODeepLearningEstimator, _forward, _Net
    from h2omx.backend import dense as D

    dev = comm.device
    world, rank = comm.world_size, comm.rank
    rows = args.rows or 50_000_000 // 8
    n_local = rows if args.scaling == "weak" else rows // world
    t_setup = time.perf_counter()
    X, y = wide_gaussian(n_local, 200, seed=args.seed + 1000 * rank, device=dev)
    X = X.T.contiguous()                    # row-major [n][200]
    X = (X - X.mean(0)) / X.std(0).clamp_min(1e-6)
    yi = y.to(torch.int32)
    gen = torch.Generator().manual_seed(args.seed)
    net = _Net([200, 512, 512, 512, 512, 2], 1, dev, gen)
    comm.broadcast_(net.flat, 0)
    Eg2, Edx2 = torch.zeros_like(net.flat), torch.zeros_like(net.flat)
    B = args.batch
    nb = max(1, n_local // B)
    state = {"i": 0}
    bw = H2ODeepLearningEstimator._backward
    bf16 = args.precision == "bf16"
    graph = None
    if bf16:
        from h2omx.models.deeplearning import _Bf16Mlp

        mlp = _Bf16Mlp(net, 1, B, dev)
        yb = torch.zeros((B,), dtype=torch.int32, device=dev)

        def body():
            mlp.forward(mlp.Xb)
            mlp.loss_grad(yb)
            mlp.backward(None, mlp.Xbt, comm if world > 1 else None, world)
            D.adadelta_(net.flat, net.grad, Eg2, Edx2, 0.99, 1e-8, 0.0)
            mlp.refresh()

        if args.graph and world == 1 and dev.type == "cuda":
            # the step after the batch staging is one HIP graph (fixed buffers); warm-up
            # on a side stream first so every lazily allocated workspace exists
            mlp.load_batch(X[:B])
            yb.copy_(yi[:B])
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                body()
            torch.cuda.current_stream(dev).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                body()

    trainer = None
    if args.estimator_defaults:
        from h2omx.models.deeplearning import _DLTrainer

        p = dict(H2ODeepLearningEstimator.DEFAULTS)
        p.update(hidden=[512] * 4, activation="Rectifier", precision=args.precision)
        B = 256 if n_local >= 256 * 64 else max(16, n_local // 64)   # the estimator's mini_batch_size=1 mapping
        n_min = int(-comm.max_scalar(-float(n_local))) if world > 1 else n_local
        trainer = _DLTrainer(p, net, X, yi, 1, True, False, 0.0, [0.0] * 8, B, max(1, n_min // B),
                             comm if world > 1 else None, torch.Generator().manual_seed(args.seed),
                             None, 4, backward=bw)

    def step():
        if trainer is not None:
            trainer.step_deferred()     # (grouped graph replays; flushed inside the timed window)
            return
        i = state["i"] % nb
        state["i"] += 1
        if bf16:
            # stage the batch: bf16 row-major + transposed (+ ones row) and its labels
            mlp.load_batch(X[i * B:(i + 1) * B])
            yb.copy_(yi[i * B:(i + 1) * B])
            if graph is not None:
                graph.replay()
            else:
                body()
            return
        xb = X[i * B:(i + 1) * B]
        Hs, aux = _forward(net, xb, 1, True, 0.0, [0.0] * 8, None)
        dZ, _ = D.softmax_xent(Hs[-1], yi[i * B:(i + 1) * B], with_loss=False)
        bw(net, Hs, aux, dZ, 1, comm if world > 1 else None, world)
        D.adadelta_(net.flat, net.grad, Eg2, Edx2, 0.99, 1e-8, 0.0)

    _sync(torch, dev)
    comm.barrier()
    setup_s = time.perf_counter() - t_setup
    elapsed = _timed(step, args, comm, torch, dev, finish=trainer.flush if trainer is not None else None)
    if trainer is not None:
        trainer.sync()
    with torch.no_grad():
        xs, ys_ = X[:200_000], y[:200_000]
        from h2omx.metrics.core import auc_from_scores

        Z = _forward(net, xs, 1, False, 0.0, [0.0] * 8, None)[0][-1]
        auc = auc_from_scores(torch.softmax(Z, 1)[:, 1], ys_, comm=comm)
    flops_row = 6 * sum(a * b for a, b in zip([200, 512, 512, 512, 512], [512, 512, 512, 512, 2]))
    return {
        "metric": "H2O DeepLearning MLP 4×512 on 50M×200 synthetic (6.25M rows per MI355X): train samples/sec",
        "value": world * B * args.steps / elapsed,
        "unit": "samples/s (all GPUs)",
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True,
        "dtype": ("bf16 (bf16 MFMA GEMMs with fp32 accumulation; fp32 master weights, gradients and ADADELTA)"
                  if bf16 else "fp32 (fp32-accurate GEMMs: exact 3-piece bf16 split on MFMA for the large forward / "
                  "data-gradient products, fp32 MFMA weight gradients; fp32 ADADELTA)"),
        "data": "synthetic wide-Gaussian 200 features generated on device; random-init weights",
        "config": {"model": "MLP 200-512x4-2 Rectifier, ADADELTA(0.99,1e-8), softmax", "global_batch": world * B,
                   "seq_len": None, "rows_per_gpu": n_local, "batch_per_gpu": B,
                   "parallelism": f"dp{world} (" + ("model averaging per iteration" if trainer is not None
                                                     else "gradient all-reduce per step") + ")"},
        "train_auc_200k": auc,
        **({"estimator_defaults": {"mini_batch_rows_per_gpu": B, "replica_sync": "model averaging"
                                   if world > 1 else "none (1 GPU)",
                                   "train_samples_per_iteration": trainer.samples_per_iteration(),
                                   "steps_per_iteration": trainer.spi}} if trainer is not None else {}),
        "achieved_tflops_per_gpu": flops_row * B * args.steps / elapsed / 1e12,
        "setup_s": setup_s,
    }


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", choices=["gbm-higgs", "xgboost-airlines", "dl-mlp"], default="gbm-higgs")
    ap.add_argument("--rows", type=int, default=0, help="rows per GPU (weak) / total (strong); 0 = config default")
    ap.add_argument("--cols", type=int, default=28)
    ap.add_argument("--max-depth", type=int, default=0)
    ap.add_argument("--nbins", type=int, default=255)
    ap.add_argument("--learn-rate", type=float, default=0.0)
    ap.add_argument("--min-rows", type=float, default=10.0)
    ap.add_argument("--batch", type=int, default=8192, help="dl-mlp rows per GPU per step")
    ap.add_argument("--graph", type=int, default=0,
                    help="dl-mlp bf16, 1 GPU: replay each step as a HIP graph (measured no faster: GPU-bound)")
    ap.add_argument("--precision", choices=["bf16", "fp32"], default="fp32",
                    help="dl-mlp GEMM operand precision: fp32 (default, H2O DeepLearning trains in fp32) or bf16 "
                         "(h2omx extension; fp32 accumulation and master weights either way)")
    ap.add_argument("--estimator-defaults", action="store_true",
                    help="dl-mlp: one step = one mini-batch of H2ODeepLearningEstimator's shipped defaults "
                         "(mini_batch_size=1 -> 256 rows per GPU, train_samples_per_iteration=-2 model averaging, "
                         "ADADELTA) through the estimator's own trainer")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="gbm-higgs default strong (11M rows in total, split over the ranks: the headline metric's "
                         "config at every N); xgboost-airlines / dl-mlp default weak (their configs are per-GPU)")
    ap.add_argument("--dump-trees", default="", help="tree models: rank 0 saves the trained trees (.npy)")
    ap.add_argument("--instrument-steps", type=int, default=-1,
                    help="tree models: extra steps measuring host enqueue / per-phase / collective time; "
                         "-1 = 5 on GPU, 0 on CPU")
    ap.add_argument("--tree-graph", choices=["auto", "0", "1"], default="auto",
                    help="tree models: HIP-graph replay of each boosting step (H2OMX_TREE_GRAPH)")
    ap.add_argument("--loopback-ranks", type=int, default=0,
                    help="tree models, 1 GPU: run the N-rank step (fused P2P exchanges against this GPU's own "
                         "buffers) on --rows rows = one rank's shard; a timing proxy of the N-GPU step")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--device", choices=["auto", "cuda", "cpu"], default="auto",
                    help="cpu: the torch reference paths (multi-rank rehearsal of this script over gloo)")
    ap.add_argument("--no-auc", action="store_true")
    ap.add_argument("--fit-trees", type=int, default=-1,
                    help="tree models: also time a whole fit (sketch + binning + N trees + AUC) -> fit_rows_per_s; "
                         "-1 = 50 on GPU, 0 on CPU")
    ap.add_argument("--oracle-rows", type=int, default=0,
                    help="also fit sklearn HistGradientBoosting on this many rows for AUC parity")
    args = ap.parse_args(argv)
    if args.scaling is None:
        args.scaling = "strong" if args.model == "gbm-higgs" else "weak"
    os.environ["H2OMX_TREE_GRAPH"] = args.tree_graph

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not under torchrun: start one rank per GPU here (fresh child processes;
        # this parent never touches the GPU) and exit with the first failure
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from h2omx.runtime.launch import spawn_ranks

        cmd = [sys.executable, os.path.abspath(__file__), *(sys.argv[1:] if argv is None else argv)]
        return spawn_ranks(cmd, args.gpus)

    import numpy as np
    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from h2omx.parallel.comm import Comm

    device = args.device if args.device != "auto" else ("cuda" if torch.cuda.device_count() > 0 else "cpu")
    if args.instrument_steps < 0:
        args.instrument_steps = 5 if device == "cuda" else 0
    comm = Comm.from_env(device)
    topo = None
    if comm.world_size > 1:
        from h2omx.runtime.topology import check_cloud

        topo = check_cloud(comm)
    if args.model == "dl-mlp":
        out = _mlp(args, comm, torch, np)
    else:
        out = _trees(args, comm, torch, np, args.model)
    if comm.rank == 0:
        res = {"metric": out.pop("metric"), "value": out.pop("value"), "unit": out.pop("unit"),
               "n_gpus": comm.world_size, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": out.pop("ms_per_step"), "higher_is_better": out.pop("higher_is_better"),
               "scaling": args.scaling, "vs_baseline": None}
        res.update(out)
        if topo is not None:
            res["topology"] = {"p2p": {h: e["p2p"] for h, e in topo["hosts"].items()}, "problems": topo["problems"]}
        print(json.dumps(res), flush=True)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
