#!/usr/bin/env python3
"""Attribute the GBM AUC gap: fixed-point GPU histograms vs the fp64 oracle vs sklearn.

Same 1M-row HIGGS-shape data (generated on the CPU with a fixed seed, binned
once with the same 255 quantile bins) is trained three ways, 50 trees,
depth 5, learn_rate 0.1, min_rows 10:

  * ``--part cpu``: ``RefTreeBuilder`` (h2omx/reference/tree.py: fp64
    histograms, exact sums - the "exact" mode) and scikit-learn
    HistGradientBoosting (max_bins 255, no regularisation) -> margins + AUCs
  * ``--part gpu``: the HIP engine (int32 fixed-point rows with stochastic
    rounding, exact int64 sums; what bench.py times) -> margins + AUC
  * ``--part compare``: AUCs, |margin| differences, identical-split fractions

    python scripts/precision_parity.py --part cpu  --out /tmp/prec     # here
    gpurun ... python scripts/precision_parity.py --part gpu --out gpurun_out/prec
    python scripts/precision_parity.py --part compare --out /tmp/prec --gpu gpurun_out/prec
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _data(rows, seed):
    import torch

    from h2omx.frame.synthetic import higgs_like
    from h2omx.models.tree import bin_matrix, compute_edges

    X, y = higgs_like(rows, seed=seed, device=torch.device("cpu"))
    e, nv, nbt = compute_edges(X, 255)
    return X, y, bin_matrix(X, e, nv, nbt), (e, nv, nbt)


def _auc(m, y):
    from sklearn.metrics import roc_auc_score

    return float(roc_auc_score(y, m))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", choices=["cpu", "gpu", "compare"], required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--gpu", default=None, help="compare: directory of the gpu part")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--trees", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import torch

    from h2omx.models.tree import TreeParams, bin_matrix, train_ensemble

    tp = TreeParams(max_depth=5, min_rows=10.0, learn_rate=0.1, min_split_improvement=1e-5)
    if a.part in ("cpu", "gpu"):
        X, y, bm, (e, nv, nbt) = _data(a.rows, a.seed)
        yn = y.numpy()
    if a.part == "cpu":
        t = time.time()
        ens = train_ensemble(bm, y, dist="bernoulli", ntrees=a.trees, tparams=tp, seed=a.seed)
        t_ref = time.time() - t
        m_ref = ens._cpu_margin[0][: a.rows].astype(np.float64)
        np.save(os.path.join(a.out, "margin_ref.npy"), m_ref.astype(np.float32))
        np.save(os.path.join(a.out, "trees_ref.npy"), ens.trees)
        from sklearn.ensemble import HistGradientBoostingClassifier

        Xs = X.T.numpy()
        t = time.time()
        clf = HistGradientBoostingClassifier(max_iter=a.trees, max_depth=5, learning_rate=0.1, min_samples_leaf=10,
                                             max_bins=255, early_stopping=False, l2_regularization=0.0).fit(Xs, yn)
        t_sk = time.time() - t
        m_sk = clf.decision_function(Xs)
        out = {"rows": a.rows, "trees": a.trees, "auc_fp64_oracle": _auc(m_ref, yn), "auc_sklearn_hgb": _auc(m_sk, yn),
               "fit_s_fp64_oracle_cpu": t_ref, "fit_s_sklearn_cpu": t_sk}
        json.dump(out, open(os.path.join(a.out, "cpu.json"), "w"), indent=1)
        print(json.dumps(out))
    elif a.part == "gpu":
        dev = torch.device("cuda", 0)
        bmg = bin_matrix(X.to(dev), e, nv, nbt)
        yg = y.to(dev)
        train_ensemble(bmg, yg, dist="bernoulli", ntrees=2, tparams=tp, seed=a.seed)   # warm-up
        torch.cuda.synchronize()
        t = time.time()
        ens = train_ensemble(bmg, yg, dist="bernoulli", ntrees=a.trees, tparams=tp, seed=a.seed)
        torch.cuda.synchronize()
        t_gpu = time.time() - t
        m = ens._state.Fm[0, : a.rows].double().cpu().numpy()
        np.save(os.path.join(a.out, "margin_gpu.npy"), m.astype(np.float32))
        np.save(os.path.join(a.out, "trees_gpu.npy"), ens.trees)
        out = {"rows": a.rows, "trees": a.trees, "auc_gpu_fixed_point": _auc(m, yn), "fit_s_gpu": t_gpu}
        json.dump(out, open(os.path.join(a.out, "gpu.json"), "w"), indent=1)
        print(json.dumps(out))
    else:
        c = json.load(open(os.path.join(a.out, "cpu.json")))
        g = json.load(open(os.path.join(a.gpu, "gpu.json")))
        mr = np.load(os.path.join(a.out, "margin_ref.npy")).astype(np.float64)
        mg = np.load(os.path.join(a.gpu, "margin_gpu.npy")).astype(np.float64)
        tr = np.load(os.path.join(a.out, "trees_ref.npy"))
        tg = np.load(os.path.join(a.gpu, "trees_gpu.npy"))
        same_tree = 0
        first_diff = None
        for t in range(min(len(tr), len(tg))):
            ok = True
            stack = [0]
            while stack:
                i = stack.pop()
                if tr[t][i]["feat"] != tg[t][i]["feat"] or (tr[t][i]["feat"] >= 0 and tr[t][i]["bin"] != tg[t][i]["bin"]):
                    ok = False
                    break
                if tr[t][i]["feat"] >= 0:
                    stack += [int(tr[t][i]["left"]), int(tr[t][i]["left"]) + 1]
            same_tree += ok
            if not ok and first_diff is None:
                first_diff = t
        d = np.abs(mr - mg)
        res = dict(c, **g)
        res.update({"auc_gap_gpu_minus_fp64": g["auc_gpu_fixed_point"] - c["auc_fp64_oracle"],
                    "auc_gap_fp64_minus_sklearn": c["auc_fp64_oracle"] - c["auc_sklearn_hgb"],
                    "trees_with_identical_splits": same_tree, "first_tree_that_differs": first_diff,
                    "margin_absdiff_max": float(d.max()), "margin_absdiff_mean": float(d.mean()),
                    "margin_absdiff_p99": float(np.quantile(d, 0.99))})
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
