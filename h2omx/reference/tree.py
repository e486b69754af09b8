"""CPU (NumPy) implementation of the level-wise histogram tree algorithm.

This mirrors ``csrc/tree_kernels.hip`` decision for decision (same gain
formulas, constraints, tie-breaking, child numbering, hashing for sampling)
and serves two purposes:

* the **numerics oracle** for the HIP kernels in ``tests/`` (GPU results are
  compared against it), and
* the CPU plumbing path (e.g. the "1-replica H2O CR on kind (CPU)" config),
  so the REST/operator stack is testable on machines without an MI355X.

It is not a performance path.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..models.tree.binning import BinnedMatrix
from ..models.tree.engine import TreeParams, tree_capacity
from ..models.tree.hashing import M32, _mix32, hash4, u01  # noqa: F401
from ..models.tree.structs import (CAT_SPLIT_BIT, CAT_WORDS, DIST_CODES, NA_LEFT_BIT, TREE_NODE_DTYPE,
                                   bitset_has, bitset_words, interaction_allowed, interaction_child,
                                   interaction_masks)




def _l1(g, a):
    if a <= 0:
        return g
    return np.where(g > a, g - a, np.where(g < -a, g + a, 0.0))


def split_gain(GL, HL, WL, G, H, W, p: TreeParams):
    """mode 0 (H2O): squared-error gain on (G, W) with min_rows on W;
    mode 1 (XGBoost): second-order gain on (G, H) with min_child_weight on H."""
    GR, HR, WR = G - GL, H - HL, W - WL
    with np.errstate(divide="ignore", invalid="ignore"):
        if p.mode == 0:
            ok = (WL >= p.min_rows) & (WR >= p.min_rows) & (WL > 0) & (WR > 0)
            gain = GL * GL / WL + GR * GR / WR - G * G / W
        else:
            ok = (HL >= p.min_child_weight) & (HR >= p.min_child_weight) & (HL > 0) & (HR > 0)
            lam = p.reg_lambda
            tl, tr, tt = _l1(GL, p.reg_alpha), _l1(GR, p.reg_alpha), _l1(G, p.reg_alpha)
            gain = 0.5 * (tl * tl / (HL + lam) + tr * tr / (HR + lam) - tt * tt / (H + lam)) - p.gamma
    return np.where(ok, gain, -np.inf)


def leaf_value(G, H, W, p: TreeParams):
    if p.leaf_mode == 1:
        v = -G / W if W > 0 else 0.0
    else:
        g = float(_l1(np.float64(G), p.reg_alpha))
        den = H + p.reg_lambda
        v = -g / den if den > 1e-12 else 0.0
    v *= p.learn_rate
    if p.max_abs_leaf > 0:
        v = min(max(v, -p.max_abs_leaf), p.max_abs_leaf)
    return v


def feature_allowed(p: TreeParams, F: int, tree_index: int, depth: int, node: int, tree_fmask=None):
    allowed = np.ones(F, bool) if tree_fmask is None else np.asarray(tree_fmask, bool).copy()
    if p.mtries > 0 or p.col_sample_rate < 1.0:
        key = (tree_index * 131 + depth) & 0xFFFFFFFF
        hs = hash4(p.seed & 0xFFFFFFFF, key, node, np.arange(F))
        if p.mtries > 0:
            order = np.lexsort((np.arange(F), hs))
            rank = np.empty(F, np.int64)
            rank[order] = np.arange(F)
            allowed &= rank < p.mtries
        else:
            allowed &= u01(hs) < np.float32(p.col_sample_rate)
    return allowed


def _ua_count(x: float, lo: float, span: float, nb: int) -> int:
    """Uniform cuts lo + span k / nb (k = 1 .. nb - 1) at or below x (mirror of ua_count)."""
    if x == -np.inf:
        return 0
    if x == np.inf:
        return nb - 1
    r = (x - lo) * float(nb) / span
    k = 0 if r < 0.0 else (nb - 1 if r >= float(nb - 1) else int(r))
    while k < nb - 1 and lo + (span * float(k + 1)) / float(nb) <= x:
        k += 1
    while k > 0 and lo + (span * float(k)) / float(nb) > x:
        k -= 1
    return k


def adaptive_mask(p: TreeParams, edges_f: np.ndarray, frange_f: np.ndarray, S: np.ndarray, m: int, nbt: int,
                  node: int, f: int, depth: int, tree_index: int) -> np.ndarray | None:
    """Candidate thresholds of (node, f) under the per-node histogram rule
    (mirror of adaptive_candidates in csrc/tree_kernels.hip): bool over the
    scanned thresholds t < min(m, nbt - 1), or None when every one is kept.
    ``S``: the node's per-bin weight (mode 0) / hessian (mode 1) sums."""
    mode = p.hist_mode
    if mode == 3:
        mode = (1, 1, 2, 0)[tree_index & 3]      # UniformAdaptive, UniformAdaptive, Random, QuantilesGlobal
    if mode == 0:
        return None
    T = min(m, nbt - 1)
    ne = np.nonzero(S[:T] > 0)[0]
    if ne.size == 0 or ne[-1] - ne[0] < 1:
        return None
    lo, hi = int(ne[0]), int(ne[-1])
    e = edges_f
    fmin, fmax, exact, isint = (float(v) for v in frange_f)
    if exact:
        lo_v = float(e[lo]) if lo < m - 1 else fmax
        hi_v = float(e[hi]) if hi < m - 1 else fmax
    else:
        lo_v = fmin if lo == 0 else float(e[lo - 1])
        hi_v = fmax if hi == m - 1 else float(e[hi])
    span = hi_v - lo_v
    if not (span > 0.0) or not (span < np.inf):
        return None
    top = (int(p.hist_top) >> depth) if depth < 31 else 0
    nb = max(top, int(p.hist_nbins), 2)
    if isint and span + 1.0 <= float(nb):
        return None
    keep = np.ones(T, bool)
    ts = np.arange(lo, hi)
    x = e[ts].astype(np.float64)
    mL = np.full(ts.size, -np.inf)
    mR = np.full(ts.size, np.inf)
    mL[1:] = 0.5 * (e[ts[1:] - 1].astype(np.float64) + x[1:])
    mR[:-1] = 0.5 * (x[:-1] + e[ts[:-1] + 1].astype(np.float64))
    if mode == 1:
        hit = np.array([_ua_count(b, lo_v, span, nb) > _ua_count(a, lo_v, span, nb) for a, b in zip(mL, mR)])
    else:
        key = (((tree_index * 131 + depth) & 0xFFFFFFFF) ^ ((f * 0x9E3779B1) & 0xFFFFFFFF))
        s2 = (p.seed & 0xFFFFFFFF) ^ 0x52414E44
        c = lo_v + span * u01(hash4(s2, key, node, np.arange(1, nb)))
        hit = ((mL[:, None] < c[None, :]) & (c[None, :] <= mR[:, None])).any(axis=1)
    keep[lo:hi] = hit
    return keep


class RefTreeBuilder:
    def __init__(self, bm: BinnedMatrix, params: TreeParams, comm=None):
        self.bm = bm
        self.p = params
        self.comm = comm
        self.codes = bm.codes.numpy() if hasattr(bm.codes, "numpy") else np.asarray(bm.codes)
        self.nvb = np.asarray(bm.nvb.cpu().numpy() if hasattr(bm.nvb, "cpu") else bm.nvb)
        self.edges = np.asarray(bm.edges.cpu().numpy() if hasattr(bm.edges, "cpu") else bm.edges)
        self.capacity = tree_capacity(min(params.max_depth, 24))
        self.nid = np.full(bm.npad, -1, np.int64)
        self.n_nodes_total = 0
        # categorical group splits (mirror of feat_best_cat_wave / part_right)
        self.cat = None if getattr(bm, "cat", None) is None or not np.any(bm.cat) else np.asarray(bm.cat, bool)
        self.catbits = None
        self.frange = None
        if params.hist_mode:
            if getattr(bm, "frange", None) is None:
                raise ValueError("TreeParams.hist_mode needs BinnedMatrix.frange (binning.adaptive_ranges)")
            self.frange = np.asarray(bm.frange.cpu().numpy(), np.float32)

    def _hist(self, rows_node, g, h, w, n_nodes):
        """Full histograms [n_nodes][F][3][nbt] (float64) of active rows."""
        F, nbt = self.bm.F, self.bm.nbt
        out = np.zeros((n_nodes, F, 3, nbt), np.float64)
        act = np.nonzero(rows_node >= 0)[0]
        if act.size:
            nn = rows_node[act]
            gw, hw, ww = g[act].astype(np.float64), h[act].astype(np.float64), w[act].astype(np.float64)
            for f in range(F):
                key = nn * nbt + self.codes[f, act]
                out[:, f, 0, :] = np.bincount(key, gw, n_nodes * nbt).reshape(n_nodes, nbt)
                out[:, f, 1, :] = np.bincount(key, hw, n_nodes * nbt).reshape(n_nodes, nbt)
                out[:, f, 2, :] = np.bincount(key, ww, n_nodes * nbt).reshape(n_nodes, nbt)
        if self.comm is not None and self.comm.world_size > 1:
            out = self.comm.all_reduce_numpy(out)
        return out

    def build(self, g, h, w, tree_index: int, tree_fmask=None) -> np.ndarray:
        p, bm = self.p, self.bm
        F, nbt = bm.F, bm.nbt
        g = np.asarray(g, np.float32)
        h = np.asarray(h, np.float32)
        w = np.ones_like(g) if w is None else np.asarray(w, np.float32)
        tree = np.zeros(self.capacity, TREE_NODE_DTYPE)
        catbits = np.zeros((self.capacity, CAT_WORDS), np.uint32) if self.cat is not None else None
        self.catbits = catbits
        nid = self.nid
        # rows of weight zero still get routed but do not contribute
        contrib = np.where((nid >= 0) & (w != 0), nid, -1)
        n_nodes, base = 1, 0
        # monotone constraints (mirror of mono_ok / SplitParams::gbound): sign per
        # feature, [lo, hi] value interval per node id set by the parent's split
        mono = None
        if p.monotone is not None and any(int(m) != 0 for m in p.monotone):
            mono = np.sign(np.asarray(p.monotone, np.int64))
            bounds = {}

        def clip(v, gid):
            if mono is None or gid == 0 or gid not in bounds:
                return v
            lo, hi = bounds[gid]
            return min(max(v, lo), hi)

        def lv_vec(Gv, Sv):
            # leaf_value(G, S, S) over arrays (leaf_mode 0, S = W or H by mode)
            with np.errstate(divide="ignore", invalid="ignore"):
                if p.leaf_mode == 1:
                    v = np.where(Sv > 0, -Gv / Sv, 0.0)
                else:
                    den = Sv + p.reg_lambda
                    v = np.where(den > 1e-12, -_l1(Gv, p.reg_alpha) / den, 0.0)
            v = v * p.learn_rate
            if p.max_abs_leaf > 0:
                v = np.clip(v, -p.max_abs_leaf, p.max_abs_leaf)
            return v

        # interaction constraints (mirror of inter_ok / inter_children): state per node id
        fsets = istate = None
        if p.interactions:
            fsets = interaction_masks(p.interactions, F)
            istate = {0: ((1 << 64) - 1, -2)}

        def mono_mask(mf, GLv, SLv, Gs, Ss):
            wl, wr = lv_vec(GLv, SLv), lv_vec(Gs - GLv, Ss - SLv)
            return wl <= wr if mf > 0 else wl >= wr

        leaf_gh = {}     # gid -> (G, H) of every node created as a leaf (Newton mono refine)
        for d in range(p.max_depth):
            last = d == p.max_depth - 1
            contrib = np.where((nid >= 0) & (w != 0), nid, -1)
            H = self._hist(contrib, g, h, w, n_nodes)
            next_base = base + n_nodes
            k = 0
            child_of = np.full(n_nodes, -1, np.int64)
            feat_of = np.zeros(n_nodes, np.int64)
            bin_of = np.zeros(n_nodes, np.int64)
            naleft_of = np.zeros(n_nodes, np.int64)
            leafkids = np.zeros(n_nodes, bool)
            catleft_of = {}      # node -> bool [nbt] left set of a categorical split
            for i in range(n_nodes):
                hist = H[i]
                tot = hist[0].sum(axis=1)  # feature 0 totals [3]
                Gt, Ht, Wt = tot
                allowed = feature_allowed(p, F, tree_index, d, i, tree_fmask)
                if fsets is not None:
                    st = istate[base + i]
                    allowed &= np.array([interaction_allowed(st, fsets, f) for f in range(F)])
                best = (-np.inf, None)
                for f in range(F):
                    if not allowed[f]:
                        continue
                    m = int(self.nvb[f])
                    hv = hist[f]
                    tg, th, tw = hv.sum(axis=1)
                    is_cat = self.cat is not None and self.cat[f]
                    if is_cat:
                        # levels ordered by G / S inside the node (S = W or H by mode), ties by
                        # level code, empty levels dropped; candidate left sets = prefixes
                        vals = hv[:, : min(m, nbt - 1)]
                        S = vals[2] if p.mode == 0 else vals[1]
                        ne = S > 0
                        with np.errstate(divide="ignore", invalid="ignore"):
                            key = np.where(ne, vals[0] / np.where(ne, S, 1.0), np.inf)
                        order = np.lexsort((np.arange(key.size), key))
                        order = order[ne[order]]
                        if order.size == 0:
                            continue
                        cs = np.cumsum(vals[:, order], axis=1)
                    else:
                        cs = np.cumsum(hv[:, : nbt - 1], axis=1)[:, : min(m, nbt - 1)]
                    na = hv[:, nbt - 1]
                    gA = split_gain(cs[0], cs[1], cs[2], tg, th, tw, p)
                    if na[2] > 0:
                        gB = split_gain(cs[0] + na[0], cs[1] + na[1], cs[2] + na[2], tg, th, tw, p)
                    else:
                        gB = np.full_like(gA, -np.inf)
                    if self.frange is not None and not is_cat:
                        keep = adaptive_mask(p, self.edges[f], self.frange[f], hv[2] if p.mode == 0 else hv[1],
                                             m, nbt, i, f, d, tree_index)
                        if keep is not None:
                            gA = np.where(keep, gA, -np.inf)
                            gB = np.where(keep, gB, -np.inf)
                    if mono is not None and mono[f] != 0:
                        si, ts = (2, tw) if p.mode == 0 else (1, th)
                        gA = np.where(mono_mask(mono[f], cs[0], cs[si], tg, ts), gA, -np.inf)
                        if na[2] > 0:
                            gB = np.where(mono_mask(mono[f], cs[0] + na[0], cs[si] + na[si], tg, ts), gB, -np.inf)
                    # codes 2t (NA right) / 2t+1 (NA left); best = max gain, min code
                    both = np.stack([gA, gB], axis=1).reshape(-1)
                    if not np.any(both > -np.inf):
                        continue
                    if is_cat:
                        # positions in sorted order; ties broken by the code 2 * level + na
                        codes = np.stack([2 * order, 2 * order + 1], axis=1).reshape(-1)
                        gmax = both.max()
                        cand = np.nonzero(both == gmax)[0]
                        c = int(cand[np.argmin(codes[cand])])
                    else:
                        c = int(np.argmax(both))  # first max = smallest code
                    gval = both[c]
                    if gval > best[0]:
                        t, na_left = c // 2, c % 2
                        GL, HL, WL = cs[0, t], cs[1, t], cs[2, t]
                        if na_left:
                            GL, HL, WL = GL + na[0], HL + na[1], WL + na[2]
                        if is_cat:
                            left = np.zeros(nbt, bool)
                            left[order[: t + 1]] = True
                            best = (gval, (f, int(order[t]), na_left, GL, HL, WL, left))
                        else:
                            best = (gval, (f, t, na_left, GL, HL, WL, None))
                do_split = (not False) and best[1] is not None and np.isfinite(best[0]) and best[0] > 0
                if do_split and p.mode == 0 and p.min_split_improvement > 0:
                    base_term = Gt * Gt / Wt if Wt > 0 else 0.0
                    do_split = best[0] > p.min_split_improvement * max(base_term, 1e-12)
                gid = base + i
                rec = tree[gid] if gid < self.capacity else np.zeros((), TREE_NODE_DTYPE)
                rec["value"] = clip(leaf_value(Gt, Ht, Wt, p), gid)
                rec["weight"] = Wt
                leaf_gh[gid] = (Gt, Ht)
                if do_split:
                    f, t, na_left, GL, HL, WL, catleft = best[1]
                    if fsets is not None:
                        cs_ = interaction_child(istate[gid], fsets, f)
                        istate[next_base + 2 * k] = istate[next_base + 2 * k + 1] = cs_
                    if mono is not None:
                        cg = next_base + 2 * k
                        lo, hi = bounds.get(gid, (-np.inf, np.inf)) if gid else (-np.inf, np.inf)
                        llo, lhi, rlo, rhi = lo, hi, lo, hi
                        if mono[f] != 0:
                            SL, St = (WL, Wt) if p.mode == 0 else (HL, Ht)
                            wl = min(max(leaf_value(GL, SL, SL, p), lo), hi)
                            wr = min(max(leaf_value(Gt - GL, St - SL, St - SL, p), lo), hi)
                            mid = 0.5 * (wl + wr)
                            if mono[f] > 0:
                                lhi = rlo = mid
                            else:
                                llo = rhi = mid
                        bounds[cg], bounds[cg + 1] = (llo, lhi), (rlo, rhi)
                    m = int(self.nvb[f])
                    rec["feat"], rec["bin"], rec["na_left"] = f, t, na_left
                    rec["left"] = next_base + 2 * k
                    rec["gain"] = best[0]
                    rec["thr"] = self.edges[f, t] if t < m - 1 else np.inf
                    if catleft is not None:
                        rec["na_left"] = na_left | CAT_SPLIT_BIT
                        rec["thr"] = np.nan
                        catleft_of[i] = catleft
                        if gid < self.capacity:
                            catbits[gid] = bitset_words(np.nonzero(catleft)[0])
                    child_of[i], feat_of[i], bin_of[i], naleft_of[i] = 2 * k, f, t, na_left
                    if last:
                        leafkids[i] = True
                        lc = tree[next_base + 2 * k]
                        rc = tree[next_base + 2 * k + 1]
                        lc["feat"] = rc["feat"] = -1
                        lc["left"] = rc["left"] = -1
                        lc["value"] = clip(leaf_value(GL, HL, WL, p), next_base + 2 * k)
                        rc["value"] = clip(leaf_value(Gt - GL, Ht - HL, Wt - WL, p), next_base + 2 * k + 1)
                        lc["weight"], rc["weight"] = WL, Wt - WL
                        leaf_gh[next_base + 2 * k], leaf_gh[next_base + 2 * k + 1] = (GL, HL), (Gt - GL, Ht - HL)
                    k += 1
                else:
                    rec["feat"], rec["left"] = -1, -1
            # partition
            act = np.nonzero(nid >= 0)[0]
            if act.size:
                nn = nid[act]
                ch = child_of[nn]
                leaf = ch < 0
                new = np.empty_like(nn)
                new[leaf] = ~(base + nn[leaf])
                sp = ~leaf
                if np.any(sp):
                    a_sp = act[sp]
                    nsp = nn[sp]
                    b = self.codes[feat_of[nsp], a_sp].astype(np.int64)
                    right = np.where(b == nbt - 1, 1 - naleft_of[nsp], (b > bin_of[nsp]).astype(np.int64))
                    for ci, cl in catleft_of.items():
                        sel = (nsp == ci) & (b != nbt - 1)
                        right[sel] = (~cl[b[sel]]).astype(np.int64)
                    lk = leafkids[nsp]
                    new_sp = np.where(lk, ~(next_base + ch[sp] + right), ch[sp] + right)
                    new[sp] = new_sp
                nid[act] = new
            base = next_base
            n_nodes = 2 * k
            self.n_nodes_total = base + n_nodes
            if n_nodes == 0:
                break
        if mono is not None and p.mode == 0 and p.leaf_mode == 0:
            _mono_newton_refine(tree, mono, leaf_gh, p)
        return tree


def _mono_newton_refine(tree, mono, leaf_gh, p):
    """Mirror of mono_newton_kernel: node intervals re-derived on the Newton
    (-G/H) scale of the leaf values from the subtree (G, H) sums, leaves
    clamped into them (squared-error splits carry W, not H)."""
    sums = {}

    def gh(gid):
        if gid not in sums:
            rec = tree[gid]
            if rec["feat"] < 0:
                sums[gid] = leaf_gh.get(gid, (0.0, 0.0))
            else:
                a, b = gh(int(rec["left"])), gh(int(rec["left"]) + 1)
                sums[gid] = (a[0] + b[0], a[1] + b[1])
        return sums[gid]

    stack = [(0, -np.inf, np.inf)]
    while stack:
        gid, lo, hi = stack.pop()
        rec = tree[gid]
        if rec["feat"] < 0:
            G, H = gh(gid)
            rec["value"] = min(max(leaf_value(G, H, H, p), lo), hi)
            continue
        l = int(rec["left"])
        llo, lhi, rlo, rhi = lo, hi, lo, hi
        mf = int(mono[int(rec["feat"])])
        if mf != 0:
            (GL, HL), (GR, HR) = gh(l), gh(l + 1)
            wl = min(max(leaf_value(GL, HL, HL, p), lo), hi)
            wr = min(max(leaf_value(GR, HR, HR, p), lo), hi)
            mid = 0.5 * (wl + wr)
            if mf > 0:
                lhi = rlo = mid
            else:
                llo = rhi = mid
        stack += [(l, llo, lhi), (l + 1, rlo, rhi)]


# ---------------------------------------------------------------------------
# gradients (mirror of boost_update_kernel / softmax_grad_kernel)
# ---------------------------------------------------------------------------
def bag_weights(n: int, sample_rate: float, seed: int, tree_index: int, row_base: int = 0) -> np.ndarray:
    if sample_rate >= 1.0:
        return np.ones(n, np.float32)
    rows = (np.arange(n, dtype=np.int64) + row_base).astype(np.uint32)
    u = u01(hash4(seed & 0xFFFFFFFF, tree_index, rows, 0x5BD1E995))
    return (u < np.float32(sample_rate)).astype(np.float32)


def dist_grad(dist: str, F, y, tweedie_power=1.5, quantile_alpha=0.5, huber_delta=1.0):
    F = np.asarray(F, np.float64)
    y = np.asarray(y, np.float64)
    code = DIST_CODES[dist]
    if code == 0:
        return F - y, np.ones_like(F)
    if code == 1:
        pr = 1.0 / (1.0 + np.exp(-F))
        return pr - y, np.maximum(pr * (1 - pr), 1e-16)
    if code == 2:
        mu = np.exp(F)
        return mu - y, np.maximum(mu, 1e-16)
    if code == 3:
        e = y * np.exp(-F)
        return 1 - e, np.maximum(e, 1e-16)
    if code == 4:
        rho = tweedie_power
        a, b = y * np.exp((1 - rho) * F), np.exp((2 - rho) * F)
        return -a + b, np.maximum(-(1 - rho) * a + (2 - rho) * b, 1e-16)
    if code == 5:
        return np.sign(F - y), np.ones_like(F)
    if code == 6:
        return np.where(y > F, -quantile_alpha, 1 - quantile_alpha), np.ones_like(F)
    if code == 7:
        r = F - y
        return np.where(np.abs(r) <= huber_delta, r, np.sign(r) * huber_delta), np.ones_like(F)
    return -y, np.ones_like(F)


# ---- CPU boosting loop and scoring (moved out of models/tree/boost.py) ----
def predict_tree_numpy(tree: np.ndarray, Xn: np.ndarray, catbits: np.ndarray | None = None) -> np.ndarray:
    """Leaf values of one tree for raw feature-major ``Xn``; ``catbits``
    [nodes][8]: left sets of categorical splits (raw value = level code)."""
    n = Xn.shape[1]
    idx = np.zeros(n, np.int64)
    for _ in range(64):
        feat = tree["feat"][idx]
        inner = feat >= 0
        if not inner.any():
            break
        r = np.nonzero(inner)[0]
        v = Xn[feat[r], r]
        nd = tree[idx[r]]
        nal = (nd["na_left"] & NA_LEFT_BIT) != 0
        with np.errstate(invalid="ignore"):
            left = np.where(np.isnan(v), nal, v <= nd["thr"])
        iscat = (nd["na_left"] & CAT_SPLIT_BIT) != 0
        if catbits is not None and iscat.any():
            c = np.where(np.isnan(v), -1, v).astype(np.int64)
            inset = bitset_has(catbits[np.minimum(idx[r], len(catbits) - 1)], c)
            oor = (c < 0) | (c > 255)
            left = np.where(iscat & ~np.isnan(v), np.where(oor, nal, inset), left)
        idx[r] = np.where(left, nd["left"], nd["left"] + 1)
    return tree["value"][idx].astype(np.float64)


def raw_margin_cpu(ens, X, nt: int):
    """TreeEnsemble.raw_margin for host tensors: margins [K][n] in fp64 NumPy."""
    import torch

    T = nt * ens.K
    n = X.shape[1]
    Xn = X.float().numpy()
    out = np.zeros((ens.K, n), np.float64) if ens.average else np.repeat(ens.init_f[:, None], n, 1).astype(np.float64)
    cb = getattr(ens, "catbits", None)
    for t in range(T):
        out[t % ens.K] += predict_tree_numpy(ens.trees[t], Xn, None if cb is None else cb[t])
    if ens.average and nt > 0:
        out /= nt
    return torch.from_numpy(out.astype(np.float32))


class _CpuView:
    def __init__(self, Fm, trees, K, init_f, cats=None):
        self.Fm, self._trees, self.K, self.init_f = Fm, trees, K, init_f
        self._cats = cats or []

    def catbits(self, lo: int, hi: int):
        sel = self._cats[lo * self.K: hi * self.K]
        if not sel:
            return None
        width = max(len(t) for t in self._trees[lo * self.K: hi * self.K])
        out = np.zeros((len(sel), width, CAT_WORDS), np.uint32)
        for i, c in enumerate(sel):
            out[i, : c.shape[0]] = c
        return out

    @property
    def margin(self) -> torch.Tensor:
        return torch.from_numpy(self.Fm)

    def trees(self, lo: int, hi: int) -> np.ndarray:
        from ..models.tree.boost import concat_trees

        sel = self._trees[lo * self.K: hi * self.K]
        return concat_trees(*[t[None] for t in sel]) if sel else np.zeros((0, 1), TREE_NODE_DTYPE)


def train_cpu(bm, y_np, w_np, ens, ntrees, tp, sample_rate, seed, comm, callback, dist_kw, tree_offset=0):
    K, dist, n = ens.K, ens.dist, bm.n
    builder = RefTreeBuilder(bm, tp, comm)
    from ..models.tree.boost import _tree_fmask
    from ..models.tree.engine import global_row_base

    row_base = global_row_base(n, comm)
    bmg = getattr(ens, "_base_margin", None)
    Fm = (bmg.cpu().numpy().astype(np.float32).copy() if bmg is not None
          else np.repeat(ens.init_f[:, None], n, 1).astype(np.float32))
    wobs = np.ones(n, np.float32) if w_np is None else w_np.astype(np.float32)
    trees = []
    cats = []      # categorical left-set bitsets per tree (builder.catbits)
    # DRF out-of-bag sums (GPU: oob_accumulate_kernel)
    oob = (np.zeros((K, n), np.float64), np.zeros(n, np.float64)) if (dist == "drf" and sample_rate < 1.0) else None
    t0 = time.perf_counter()
    lr0, ann = tp.learn_rate, getattr(tp, "learn_rate_annealing", 1.0)
    for t in range(ntrees):
        ti = tree_offset + t      # global iteration index (checkpoint continuation)
        builder.p.learn_rate = lr0 * ann ** ti
        wb = wobs * bag_weights(n, sample_rate, seed, ti, row_base)
        if K == 1:
            gr, hs = dist_grad(dist, Fm[0], y_np, **dist_kw)
            grads = [(gr, hs)]
        elif dist == "drf":
            grads = [(-(y_np == k).astype(np.float64), np.ones(n)) for k in range(K)]
        else:
            z = Fm - Fm.max(axis=0, keepdims=True)
            pr = np.exp(z)
            pr /= pr.sum(axis=0, keepdims=True)
            grads = [(pr[k] - (y_np == k), np.maximum(pr[k] * (1 - pr[k]), 1e-16)) for k in range(K)]
        fmask = _tree_fmask(tp, bm.F, ti, None)
        for k in range(K):
            gr, hs = grads[k]
            pad = bm.npad - n
            builder.nid[:] = -1
            builder.nid[:n] = 0
            g32 = np.concatenate([(gr * wb).astype(np.float32), np.zeros(pad, np.float32)])
            h32 = np.concatenate([(hs * wb).astype(np.float32), np.zeros(pad, np.float32)])
            w32 = np.concatenate([wb, np.zeros(pad, np.float32)])
            tree = builder.build(g32, h32, w32, ti * K + k, fmask)
            leaf = ~builder.nid[:n]
            Fm[k] += tree["value"][leaf]
            # keep the used prefix only (deep trees: capacity 2^(d+1) - 1 slots)
            used = max(1, min(builder.n_nodes_total, builder.capacity))
            trees.append(tree[:used].copy())
            if builder.catbits is not None:
                cats.append(builder.catbits[:used].copy())
            if oob is not None:
                out_of_bag = (wb == 0) & (wobs != 0)
                oob[0][k][out_of_bag] += tree["value"][leaf[out_of_bag]].astype(np.float32)
                if k == 0:
                    oob[1][out_of_bag] += 1.0
        if callback is not None and callback(t, _CpuView(Fm, trees, K, ens.init_f, cats)) is True:
            break
    ens.timings["train_s"] = time.perf_counter() - t0
    builder.p.learn_rate = lr0
    if trees:
        from ..models.tree.boost import concat_trees

        ens.trees = concat_trees(*[t[None] for t in trees])
        if cats:
            width = ens.trees.shape[1]
            ens.catbits = np.zeros((len(cats), width, CAT_WORDS), np.uint32)
            for i, c in enumerate(cats):
                ens.catbits[i, : c.shape[0]] = c
    ens._cpu_margin = Fm
    if oob is not None:
        import torch

        ens._oob = (torch.from_numpy(oob[0].astype(np.float32)), torch.from_numpy(oob[1].astype(np.float32)))
