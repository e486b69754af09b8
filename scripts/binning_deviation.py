#!/usr/bin/env python3
"""How far h2omx's per-node UniformAdaptive rule is from H2O's (CPU, numpy).

H2O (hex/tree/DHistogram, histogram_type AUTO = UniformAdaptive) re-bins every
node's own [min, max] of each column into nb = max(nbins_top_level >> depth,
nbins) equal-width bins and splits at those bin boundaries.  h2omx keeps uint8
fine quantile bins per column (255, or 63 for trees deeper than 12 levels with
the default nbins_top_level) and lets a node split only at the fine edges
nearest H2O's cut points (csrc/tree_kernels.hip adaptive_candidates; CPU mirror
reference/tree.adaptive_mask).  So a split can differ from H2O's in two ways:
  1. the threshold: H2O's cut c_k vs the snapped fine edge - the rows between
     the two change sides;
  2. the candidate set: where a node holds fewer fine edges than H2O has cuts
     (nb > interior fine edges in the node's range), several cuts snap to one
     edge and the node has fewer candidates than H2O.
For nodes of random axis-aligned boxes (depth 0..5) of HIGGS-shape data this
script measures, per (node, feature): the fraction of the node's rows whose
side differs between each H2O cut and the closest split h2omx can make there
(max and mean over the cuts), distinct candidates h2omx / H2O, and the best squared-error gain of
the feature under each rule (relative shortfall), plus how often the best
feature of a node differs.  Output: one JSON document (profiles/r6/).

    python scripts/binning_deviation.py [rows] [fine_bins] > out.json
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from h2omx.frame.synthetic import higgs_like  # noqa: E402
from h2omx.models.tree import TreeParams, bin_matrix, compute_edges  # noqa: E402
from h2omx.models.tree.binning import adaptive_ranges, node_bins  # noqa: E402
from h2omx.reference.tree import adaptive_mask  # noqa: E402


def se_gain(gl, wl, g, w):
    gr, wr = g - gl, w - wl
    ok = (wl > 0) & (wr > 0)
    out = np.full(gl.shape, -np.inf)
    out[ok] = gl[ok] ** 2 / wl[ok] + gr[ok] ** 2 / wr[ok] - g * g / w
    return out


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    fine = int(sys.argv[2]) if len(sys.argv) > 2 else 255
    X, y = higgs_like(rows, seed=3)
    Xn, yn = X.numpy().astype(np.float64), y.numpy().astype(np.float64)
    e, nv, nbt = compute_edges(X, fine, histogram_type="QuantilesGlobal")
    bm = bin_matrix(X, e, nv, nbt)
    fr = adaptive_ranges(X, bm).numpy()
    codes = bm.codes.numpy()[:, :rows]
    edges = bm.edges.numpy()
    nvb = bm.nvb.numpy()
    F = Xn.shape[0]
    g = yn - yn.mean()             # first-tree squared-error residuals
    tp = TreeParams(hist_mode=1, hist_top=1024, hist_nbins=20)
    rng = np.random.default_rng(0)
    per_depth = {}
    for depth in range(6):
        nb = node_bins(1024, 20, depth)
        flips_max, flips_mean, cand_ratio, gain_short, best_diff, nodes = [], [], [], [], 0, 0
        for trial in range(40 if depth else 1):
            # a node at `depth`: a random axis-aligned box of `depth` splits
            sel = np.ones(rows, bool)
            for _ in range(depth):
                f0 = int(rng.integers(F))
                q = np.quantile(Xn[f0, sel], rng.uniform(0.2, 0.8)) if sel.any() else 0.0
                sel &= (Xn[f0] <= q) if rng.random() < 0.5 else (Xn[f0] > q)
            idx = np.nonzero(sel)[0]
            if idx.size < 200:
                continue
            nodes += 1
            best_h2o, best_mx = (-np.inf, -1), (-np.inf, -1)
            for f in range(F):
                x, c = Xn[f, idx], codes[f, idx]
                live = ~np.isnan(x)
                x, c, gf = x[live], c[live], g[idx][live]
                lo, hi = x.min(), x.max()
                if not hi > lo:
                    continue
                # H2O: equal-width cuts of the node's own range, left = x < cut
                cuts = lo + (hi - lo) * np.arange(1, nb) / nb
                order = np.argsort(x)
                xs, gs = x[order], gf[order]
                cg = np.concatenate([[0.0], np.cumsum(gs)])
                k = np.searchsorted(xs, cuts, side="left")          # rows with x < cut
                gain_h = se_gain(cg[k], k.astype(float), cg[-1], float(len(xs)))
                # h2omx: fine-bin histogram of the node, candidates = snapped edges
                m = int(nvb[f]) + 1
                S = np.bincount(c, minlength=nbt).astype(np.float64)
                keep = adaptive_mask(tp, edges[f], fr[f], S, m, nbt, 0, f, depth, 0)
                T = min(m, nbt - 1)
                allowed = np.arange(T) if keep is None else np.nonzero(keep)[0]
                G = np.bincount(c, weights=gf, minlength=nbt)
                cgb, cwb = np.cumsum(G), np.cumsum(S)
                gain_m = se_gain(cgb[allowed], cwb[allowed], cg[-1], float(len(xs)))
                # every H2O cut vs the closest partition h2omx can make: both are
                # thresholds in the same row order (monotone bins), so the rows that
                # change sides are |left fraction (H2O cut) - left fraction (candidate)|
                e_f = edges[f][:T].astype(np.float64)
                near = allowed[np.argmin(np.abs(e_f[allowed][None, :] - cuts[:, None]), axis=1)] if allowed.size else None
                if near is not None:
                    nl = len(xs)
                    frac_h = k / nl
                    frac_m = cwb[allowed] / nl
                    fl = np.abs(frac_h[:, None] - frac_m[None, :]).min(axis=1)
                    flips_max.append(float(fl.max()))
                    flips_mean.append(float(fl.mean()))
                    cand_ratio.append(np.unique(near).size / float(nb - 1))
                bh, bmx = float(np.max(gain_h)), float(np.max(gain_m)) if gain_m.size else -np.inf
                if bh > 0:
                    gain_short.append(max(0.0, (bh - bmx) / bh))
                if bh > best_h2o[0]:
                    best_h2o = (bh, f)
                if bmx > best_mx[0]:
                    best_mx = (bmx, f)
            best_diff += int(best_h2o[1] != best_mx[1])
        per_depth[depth] = {
            "h2o_bins_per_node": nb, "nodes": nodes,
            "row_side_flip_max_p50": float(np.median(flips_max)), "row_side_flip_max_p99": float(np.quantile(flips_max, 0.99)),
            "row_side_flip_mean": float(np.mean(flips_mean)),
            "distinct_candidates_vs_h2o_p50": float(np.median(cand_ratio)),
            "best_gain_shortfall_p50": float(np.median(gain_short)), "best_gain_shortfall_p99": float(np.quantile(gain_short, 0.99)),
            "best_feature_differs": f"{best_diff}/{nodes}",
        }
    print(json.dumps({"rows": rows, "fine_bins": fine, "data": "higgs_like(seed=3)", "per_depth": per_depth}, indent=1))


if __name__ == "__main__":
    main()
