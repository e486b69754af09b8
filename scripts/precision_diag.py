#!/usr/bin/env python3
"""Precision-pin divergence, CPU half: train the fp64
oracle (RefTreeBuilder) on the same HIGGS-shape rows as a GPU run
(scripts/route_check.py saved its trees) and compare EVERY field of every
reachable node (feat, bin, na_left, child ids, leaf values), then the
margins row by row: which tree / leaf puts the largest margin gap on which
rows, and how many rows that leaf holds.

    python scripts/precision_diag.py --gpu-trees gpurun_out/r4b/route/trees.npy --out /tmp/pdiag
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def reach(tr):
    keep, stack = [], [0]
    while stack:
        i = stack.pop()
        keep.append(i)
        if tr[i]["feat"] >= 0:
            stack += [int(tr[i]["left"]), int(tr[i]["left"]) + 1]
    return sorted(keep)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu-trees", required=True)
    ap.add_argument("--rows", type=int, default=11_000_000)
    ap.add_argument("--trees", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="/tmp/pdiag")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import torch

    from h2omx.frame.synthetic import higgs_like
    from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble
    from h2omx.reference.tree import predict_tree_numpy

    X, y = higgs_like(a.rows, seed=a.seed, device=torch.device("cpu"))
    e, nv, nbt = compute_edges(X, 255)
    bm = bin_matrix(X, e, nv, nbt)
    tp = TreeParams(max_depth=5, min_rows=10.0, learn_rate=0.1, min_split_improvement=1e-5)
    ref_path = os.path.join(a.out, "trees_ref.npy")
    if os.path.exists(ref_path):
        tr_ref = np.load(ref_path)
        m_ref = np.load(os.path.join(a.out, "margin_ref.npy"))
    else:
        t0 = time.time()
        ens = train_ensemble(bm, y, dist="bernoulli", ntrees=a.trees, tparams=tp, seed=a.seed)
        print(f"oracle fit {time.time() - t0:.0f} s", flush=True)
        tr_ref = ens.trees
        m_ref = ens._cpu_margin[0][: a.rows].astype(np.float32)
        np.save(ref_path, tr_ref)
        np.save(os.path.join(a.out, "margin_ref.npy"), m_ref)
        np.save(os.path.join(a.out, "init_f.npy"), ens.init_f)
    tr_gpu = np.load(a.gpu_trees)
    init_f = float(np.load(os.path.join(a.out, "init_f.npy"))[0])
    Xn = X.numpy()
    report = {"trees": []}
    m_gpu = np.full(a.rows, init_f, np.float64)
    worst = []
    for t in range(min(len(tr_ref), len(tr_gpu))):
        r, g = tr_ref[t], tr_gpu[t]
        rr, rg = reach(r), reach(g)
        ent = {"tree": t, "same_shape": rr == rg}
        if rr == rg:
            for f in ("feat", "bin", "left"):
                ent[f"diff_{f}"] = int((r[rr][f] != g[rg][f]).sum())
            inner = r[rr]["feat"] >= 0
            ent["diff_na_left"] = int(((r[rr]["na_left"] & 1) != (g[rg]["na_left"] & 1))[inner].sum())
            leaves = ~inner
            dv = np.abs(r[rr]["value"].astype(np.float64) - g[rg]["value"].astype(np.float64))[leaves]
            ent["max_leaf_value_diff"] = float(dv.max()) if dv.size else 0.0
            if dv.size and dv.max() > 1e-4:
                li = np.array(rr)[leaves][int(np.argmax(dv))]
                ent["worst_leaf"] = {"node": int(li), "ref": float(r[li]["value"]), "gpu": float(g[li]["value"]),
                                     "ref_weight": float(r[li]["weight"]), "gpu_weight": float(g[li]["weight"])}
        vr = predict_tree_numpy(r, Xn)
        vg = predict_tree_numpy(g, Xn)
        m_gpu += vg
        d = np.abs(vr - vg)
        ent["rows_leaf_value_diff_gt_1e-4"] = int((d > 1e-4).sum())
        if d.max() > 1e-4:
            rows = np.nonzero(d > 1e-4)[0][:5]
            ent["example_rows"] = rows.tolist()
            worst.append((float(d.max()), t))
        report["trees"].append(ent)
    dm = np.abs(m_gpu - m_ref.astype(np.float64))
    report["margin_absdiff_max"] = float(dm.max())
    report["margin_absdiff_rows_gt_1e-5"] = int((dm > 1e-5).sum())
    report["worst_trees"] = sorted(worst, reverse=True)[:10]
    json.dump(report, open(os.path.join(a.out, "precision_diag.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in report.items() if k != "trees"}))
    for ent in report["trees"]:
        if not ent["same_shape"] or ent.get("max_leaf_value_diff", 0) > 1e-4 or ent["rows_leaf_value_diff_gt_1e-4"]:
            print(json.dumps(ent))


if __name__ == "__main__":
    main()
