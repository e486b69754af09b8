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


def _data(rows, seed, kind="portable"):
    """``portable`` (default): higgs_like_portable - bit-identical on every
    host, so the GPU box and the oracle host bin the same values (torch's
    vectorised exp / log in higgs_like differ in the last bit between host
    CPUs, which moved a few rows across cut points: the r3 0.0896 margin gap,
    profiles/r4/precision_pin_r4.md)."""
    import torch

    from h2omx.frame.synthetic import higgs_like, higgs_like_portable
    from h2omx.models.tree import bin_matrix, compute_edges

    if kind == "portable":
        X, y = higgs_like_portable(rows, seed=seed)
    else:
        X, y = higgs_like(rows, seed=seed, device=torch.device("cpu"))
    e, nv, nbt = compute_edges(X, 255)
    return X, y, bin_matrix(X, e, nv, nbt), (e, nv, nbt)


def _hashes(X, y, e, bm) -> dict:
    import hashlib

    h = lambda a: hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]   # noqa: E731
    return {"x": h(X.numpy()), "y": h(y.numpy()), "edges": h(e), "codes": h(bm.codes.cpu().numpy())}


def _reach(tr):
    keep, stack = [], [0]
    while stack:
        i = stack.pop()
        keep.append(i)
        if tr[i]["feat"] >= 0:
            stack += [int(tr[i]["left"]), int(tr[i]["left"]) + 1]
    return sorted(keep)


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
    ap.add_argument("--data", choices=["portable", "higgs"], default="portable")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import torch

    from h2omx.models.tree import TreeParams, bin_matrix, train_ensemble

    tp = TreeParams(max_depth=5, min_rows=10.0, learn_rate=0.1, min_split_improvement=1e-5)
    if a.part in ("cpu", "gpu"):
        X, y, bm, (e, nv, nbt) = _data(a.rows, a.seed, a.data)
        yn = y.numpy()
        hashes = _hashes(X, y, e, bm)
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
        out = {"rows": a.rows, "trees": a.trees, "data": a.data, "auc_fp64_oracle": _auc(m_ref, yn),
               "auc_sklearn_hgb": _auc(m_sk, yn), "fit_s_fp64_oracle_cpu": t_ref, "fit_s_sklearn_cpu": t_sk,
               "hashes_cpu": hashes}
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
        if a.rows <= 2_000_000:   # (11M margins: 44 MB; compare re-applies the trees instead)
            np.save(os.path.join(a.out, "margin_gpu.npy"), m.astype(np.float32))
        np.save(os.path.join(a.out, "init_f.npy"), np.asarray(ens.init_f, np.float64))
        np.save(os.path.join(a.out, "trees_gpu.npy"), ens.trees)
        out = {"rows": a.rows, "trees": a.trees, "data": a.data, "auc_gpu_fixed_point": _auc(m, yn),
               "fit_s_gpu": t_gpu, "hashes_gpu_box": hashes}
        json.dump(out, open(os.path.join(a.out, "gpu.json"), "w"), indent=1)
        print(json.dumps(out))
    else:
        c = json.load(open(os.path.join(a.out, "cpu.json")))
        g = json.load(open(os.path.join(a.gpu, "gpu.json")))
        mr = np.load(os.path.join(a.out, "margin_ref.npy")).astype(np.float64)
        tr = np.load(os.path.join(a.out, "trees_ref.npy"))
        tg = np.load(os.path.join(a.gpu, "trees_gpu.npy"))
        mpath = os.path.join(a.gpu, "margin_gpu.npy")
        if os.path.exists(mpath):
            mg = np.load(mpath).astype(np.float64)
        else:
            # GPU margins = init + every GPU tree applied through its thresholds
            # (training routing == threshold routing on the device, route_check)
            from h2omx.reference.tree import predict_tree_numpy

            X, _, _, _ = _data(c["rows"], a.seed, c.get("data", "portable"))
            Xn = X.numpy()
            mg = np.full(c["rows"], float(np.load(os.path.join(a.gpu, "init_f.npy"))[0]), np.float64)
            for t in range(tg.shape[0]):
                mg += predict_tree_numpy(tg[t], Xn)
        # every field of every reachable node: split feature / bin, NA
        # direction, raw threshold, child ids, leaf values
        same_tree, first_diff, nodes, diff = 0, None, 0, {"feat": 0, "bin": 0, "na_left": 0, "thr": 0, "left": 0}
        leaf_dv = 0.0
        for t in range(min(len(tr), len(tg))):
            kr, kg = _reach(tr[t]), _reach(tg[t])
            ok = kr == kg
            if ok:
                a_, b_ = tr[t][kr], tg[t][kr]
                inner = a_["feat"] >= 0
                nodes += len(kr)
                for f in ("feat", "bin", "left"):
                    diff[f] += int((a_[f] != b_[f])[inner].sum())
                diff["na_left"] += int(((a_["na_left"] & 1) != (b_["na_left"] & 1))[inner].sum())
                diff["thr"] += int((a_["thr"] != b_["thr"])[inner].sum())
                ok = not any(int((a_[f] != b_[f])[inner].sum()) for f in ("feat", "bin", "thr"))
                leaf_dv = max(leaf_dv, float(np.abs(a_["value"].astype(np.float64)
                                                    - b_["value"].astype(np.float64))[~inner].max()))
            same_tree += ok
            if not ok and first_diff is None:
                first_diff = t
        d = np.abs(mr - mg)
        res = dict(c, **g)
        res.update({"same_data_on_both_hosts": c.get("hashes_cpu") == g.get("hashes_gpu_box"),
                    "auc_gap_gpu_minus_fp64": g["auc_gpu_fixed_point"] - c["auc_fp64_oracle"],
                    "auc_gap_fp64_minus_sklearn": c["auc_fp64_oracle"] - c["auc_sklearn_hgb"],
                    "trees_with_identical_splits": same_tree, "first_tree_that_differs": first_diff,
                    "reachable_nodes_compared": nodes, "node_field_differences": diff,
                    "leaf_value_absdiff_max": leaf_dv,
                    "margin_absdiff_max": float(d.max()), "margin_absdiff_mean": float(d.mean()),
                    "margin_absdiff_p99": float(np.quantile(d, 0.99)),
                    "rows_margin_absdiff_gt_1e-5": int((d > 1e-5).sum())})
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
