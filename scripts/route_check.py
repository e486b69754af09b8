#!/usr/bin/env python3
"""Precision-pin divergence probe: does the GPU training
route every row like the exported trees do?

Trains the HIGGS-shape GBM on the GPU (same settings as precision_parity.py),
then compares the training margin ``Fm`` (accumulated from the per-row leaf
ids of the training partitions) with ``raw_margin`` (every tree re-applied to
the raw features through its thresholds).  Rows where they differ were routed
differently during training; the script reports them tree by tree (training
leaf vs threshold leaf, the row's values on the split features) and dumps the
worst rows' trees + values for the CPU oracle comparison.

    python scripts/route_check.py --rows 11000000 --trees 50 --out gpurun_out/route
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=11_000_000)
    ap.add_argument("--trees", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/route")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import torch

    from h2omx.frame.synthetic import higgs_like
    from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble
    from h2omx.reference.tree import predict_tree_numpy

    dev = torch.device("cuda", 0)
    X, y = higgs_like(a.rows, seed=a.seed, device=torch.device("cpu"))
    e, nv, nbt = compute_edges(X, 255)
    Xg = X.to(dev)
    bm = bin_matrix(Xg, e, nv, nbt)
    tp = TreeParams(max_depth=5, min_rows=10.0, learn_rate=0.1, min_split_improvement=1e-5)
    ens = train_ensemble(bm, y.to(dev), dist="bernoulli", ntrees=a.trees, tparams=tp, seed=a.seed)
    torch.cuda.synchronize()
    fm = ens._state.Fm[0, : a.rows].double()
    rm = ens.raw_margin(Xg)[0].double()
    d = (fm - rm).abs()
    out = {"rows": a.rows, "trees": a.trees, "max_abs_fm_minus_raw": float(d.max()),
           "rows_over_1e-5": int((d > 1e-5).sum()), "rows_over_1e-3": int((d > 1e-3).sum())}
    bad = torch.nonzero(d > 1e-5).flatten()[:64].cpu().numpy()
    out["bad_rows"] = bad.tolist()
    # per-tree attribution for the bad rows: threshold routing vs binned routing
    codes = bm.codes[:, bad].cpu().numpy() if bad.size else None
    Xb = X[:, bad].numpy() if bad.size else None
    per = []
    if bad.size:
        for t in range(ens.trees.shape[0]):
            tr = ens.trees[t]
            v_raw = predict_tree_numpy(tr, Xb)
            # binned routing: b <= bin
            idx = np.zeros(bad.size, np.int64)
            for _ in range(64):
                f = tr["feat"][idx]
                inner = f >= 0
                if not inner.any():
                    break
                r = np.nonzero(inner)[0]
                b = codes[f[r], r].astype(np.int64)
                nd = tr[idx[r]]
                left = np.where(b == nbt - 1, nd["na_left"] & 1, b <= nd["bin"]).astype(bool)
                idx[r] = np.where(left, nd["left"], nd["left"] + 1)
            v_bin = tr["value"][idx].astype(np.float64)
            diff = np.nonzero(np.abs(v_raw - v_bin) > 0)[0]
            if diff.size:
                per.append({"tree": t, "rows": bad[diff].tolist()[:8]})
    out["trees_where_threshold_and_bin_routing_differ"] = per[:20]
    # edge cases: values equal to a cut point, and bin codes inconsistent with the edges
    if bad.size:
        eq = []
        for j, r in enumerate(bad[:16]):
            for f in range(X.shape[0]):
                m = int(nv[f]) - 1
                v = float(X[f, r])
                c = int(codes[f, j])
                want = int(np.searchsorted(e[f, :m], np.float32(v), side="left")) if not np.isnan(v) else nbt - 1
                if c != want:
                    eq.append({"row": int(r), "feat": f, "value": v, "code_gpu": c, "code_numpy": want})
        out["code_mismatches"] = eq[:32]
    np.save(os.path.join(a.out, "trees.npy"), ens.trees)
    json.dump(out, open(os.path.join(a.out, "route_check.json"), "w"), indent=1)
    print(json.dumps(out)[:4000])


if __name__ == "__main__":
    main()
