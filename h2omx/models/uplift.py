"""Uplift Distributed Random Forest (H2O ``H2OUpliftRandomForestEstimator``).

Uplift modelling estimates the causal effect of a binary treatment on a
binary response: for each row, uplift = P(y=1 | treated, x) - P(y=1 | control, x).
Every tree is grown on a bagged row sample.  Each node split maximises the
divergence gain between the treatment and control response distributions
(Rzepakowski & Jaroszewicz 2012): for p = P(y=1 | T), q = P(y=1 | C)

    KL:          p log(p/q) + (1-p) log((1-p)/(1-q))
    Euclidean:   (p - q)^2 + ((1-p) - (1-q))^2
    ChiSquared:  (p - q)^2 / q + ((1-p) - (1-q))^2 / (1-q)

    gain = n_L/n D(L) + n_R/n D(R) - D(node)

Trees are built level-wise on the same uint8 binned matrix as the other tree
models (``tree.binning``: device quantile sketch plus the HIP binning
kernel).  Per level, one device histogram holds four statistics per
(node, feature, bin): treated count, treated responders, control count and
control responders.  Each histogram is a float64 bincount; across ranks they
are summed with one all-reduce.  The split scan runs as vectorised tensor ops
over every (node, feature, bin, NA direction).  A child needs ``min_rows`` rows
and at least one treated and one control row.  Leaves store (p_t, p_c).
Prediction averages both over the trees.

Output columns match H2O: ``uplift_predict``, ``p_y1_with_treatment`` and
``p_y1_without_treatment``.

Metrics (``uplift_metrics``): rows are ranked by predicted uplift and cut at
``auuc_nbins`` quantile thresholds.  At each cut the cumulative treated and
control counts and responders give three curves:
    qini = y_t - y_c n_t / n_c
    lift = y_t / n_t - y_c / n_c
    gain = lift (n_t + n_c)
AUUC is the trapezoid area under the ``auuc_type`` curve over the population
fraction.  ``qini`` is the Qini coefficient: AUUC(qini) minus the random-targeting
triangle.  ``ate`` / ``att`` / ``atc`` are the mean predicted uplift over all,
treated and control rows.  H2O's exact AUUC binning is not reproduced
byte-for-byte ("parity unpinned"; there is no H2O runtime here to compare against).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame, Vec
from .base import Model, ModelBuilder, ModelCategory
from .tree import bin_matrix, compute_edges

UPLIFT_CATEGORY = "BinomialUplift"
_EPS = 1e-6


def divergence(p: torch.Tensor, q: torch.Tensor, metric: str) -> torch.Tensor:
    metric = metric.lower()
    if metric in ("auto", "kl"):
        p_ = p.clamp(_EPS, 1 - _EPS)
        q_ = q.clamp(_EPS, 1 - _EPS)
        return p_ * torch.log(p_ / q_) + (1 - p_) * torch.log((1 - p_) / (1 - q_))
    if metric == "euclidean":
        return 2.0 * (p - q) ** 2
    if metric in ("chisquared", "chi_squared"):
        q_ = q.clamp(_EPS, 1 - _EPS)
        return (p - q) ** 2 / q_ + (p - q) ** 2 / (1 - q_)
    raise ValueError(f"uplift_metric {metric!r} (AUTO, KL, Euclidean, ChiSquared)")


def _ratio(y, n, fallback):
    return torch.where(n > 0, y / n.clamp_min(1e-300), fallback)


class UpliftTree:
    """Flat arrays of one tree: feat (-1 = leaf), bin, na_left, left child
    (right = left + 1), leaf (p_t, p_c) for every node."""

    def __init__(self):
        self.feat, self.bin, self.na_left, self.left, self.pt, self.pc = [], [], [], [], [], []

    def add(self, pt, pc) -> int:
        self.feat.append(-1)
        self.bin.append(0)
        self.na_left.append(0)
        self.left.append(-1)
        self.pt.append(float(pt))
        self.pc.append(float(pc))
        return len(self.feat) - 1

    def arrays(self):
        return {"feat": np.array(self.feat, np.int32), "bin": np.array(self.bin, np.int32),
                "na_left": np.array(self.na_left, np.int8), "left": np.array(self.left, np.int32),
                "pt": np.array(self.pt, np.float64), "pc": np.array(self.pc, np.float64)}


def predict_tree(tr: dict, codes: torch.Tensor, n: int, nbt: int):
    """Route binned rows (uint8 [F][npad]) through one tree -> (p_t, p_c) [n]."""
    dev = codes.device
    feat = torch.from_numpy(tr["feat"]).to(dev).long()
    binv = torch.from_numpy(tr["bin"]).to(dev).long()
    nal = torch.from_numpy(tr["na_left"]).to(dev).bool()
    left = torch.from_numpy(tr["left"]).to(dev).long()
    nid = torch.zeros(n, dtype=torch.long, device=dev)
    rows = torch.arange(n, device=dev)
    for _ in range(64):
        f = feat[nid]
        live = f >= 0
        if not bool(live.any()):
            break
        c = codes[f.clamp_min(0), rows].long()
        right = torch.where(c == nbt - 1, ~nal[nid], c > binv[nid])
        nid = torch.where(live, left[nid] + right.long(), nid)
    pt = torch.from_numpy(tr["pt"]).to(dev)[nid]
    pc = torch.from_numpy(tr["pc"]).to(dev)[nid]
    return pt, pc


def uplift_metrics(uplift: torch.Tensor, y: torch.Tensor, treat: torch.Tensor, nbins: int = 1000,
                   auuc_type: str = "qini", comm=None) -> dict:
    """AUUC / Qini / ATE metrics of predicted uplift against (y, treatment).
    Multi-rank: the per-threshold counts are all-reduced, and the thresholds
    are quantiles of the pooled predictions."""
    u = uplift.double().flatten()
    yv = y.double().flatten()
    tv = treat.double().flatten()
    if comm is not None and comm.world_size > 1:
        pool = comm.all_gather_cat(u[torch.randperm(u.numel(), device=u.device)[:100_000]])
    else:
        pool = u
    nb = int(nbins) if nbins and int(nbins) > 0 else 1000
    qs = torch.linspace(1, 0, nb + 1, dtype=torch.float64, device=u.device)[1:]
    thr = torch.quantile(pool.cpu(), qs.cpu()).to(u.device) if pool.numel() > 0 else torch.zeros(nb)
    thr = torch.unique(thr).flip(0)                        # descending distinct thresholds
    # rows with u >= thr[k] -> bucket of the first threshold they pass
    b = torch.searchsorted(-thr, -u, right=True).clamp(max=thr.numel() - 1)
    K = thr.numel()
    cnt = torch.zeros((4, K), dtype=torch.float64, device=u.device)
    cnt[0].index_add_(0, b, tv)
    cnt[1].index_add_(0, b, tv * yv)
    cnt[2].index_add_(0, b, 1 - tv)
    cnt[3].index_add_(0, b, (1 - tv) * yv)
    tot = torch.stack([u.sum(), (u * tv).sum(), tv.sum(), ((1 - tv) * u).sum(), (1 - tv).sum(),
                       torch.tensor(float(u.numel()), dtype=torch.float64, device=u.device)])
    if comm is not None and comm.world_size > 1:
        comm.all_reduce_(cnt)
        comm.all_reduce_(tot)
    c = torch.cumsum(cnt, 1).cpu().numpy()
    nt, yt, nc, yc = c
    with np.errstate(divide="ignore", invalid="ignore"):
        qini = np.where(nc > 0, yt - yc * nt / np.maximum(nc, 1e-300), yt)
        lift = np.where((nt > 0) & (nc > 0), yt / np.maximum(nt, 1e-300) - yc / np.maximum(nc, 1e-300), 0.0)
    gain = lift * (nt + nc)
    frac = (nt + nc) / max(float(nt[-1] + nc[-1]), 1e-300)
    x = np.concatenate([[0.0], frac])
    curves = {"qini": qini, "lift": lift, "gain": gain}

    def area(cv):
        yy = np.concatenate([[0.0], cv])
        return float(np.sum((x[1:] - x[:-1]) * (yy[1:] + yy[:-1]) / 2))

    kind = "qini" if str(auuc_type).lower() == "auto" else str(auuc_type).lower()
    aucs = {k: area(v) for k, v in curves.items()}
    final = float(curves[kind][-1])
    t = tot.cpu().numpy()
    out = {
        "auuc": aucs[kind], "auuc_type": kind,
        "auuc_normalized": aucs[kind] / abs(final) if final != 0 else 0.0,
        "auuc_table": aucs,
        "qini": aucs["qini"] - float(qini[-1]) / 2.0,
        "ate": float(t[0] / max(t[5], 1)), "att": float(t[1] / max(t[2], 1)), "atc": float(t[3] / max(t[4], 1)),
        "thresholds_and_metric_scores": [
            {"threshold": float(thr[k]), "n_treatment": float(nt[k]), "n_control": float(nc[k]),
             "y_treatment": float(yt[k]), "y_control": float(yc[k]), "qini": float(qini[k]),
             "lift": float(lift[k]), "gain": float(gain[k])} for k in range(K)],
        "nobs": int(t[5]),
    }
    return out


class UpliftDRFModel(Model):
    algo = "upliftdrf"
    algo_full_name = "Uplift Distributed Random Forest"

    def __init__(self, builder, model_id, trees, edges, nvb, nbt, treatment_column):
        super().__init__(builder, model_id)
        self.trees = trees
        self.edges = edges
        self.nvb = nvb
        self.nbt = nbt
        self.treatment_column = treatment_column
        self.category = UPLIFT_CATEGORY

    def _codes(self, frame: Frame):
        X = frame.feature_matrix(self.x)
        return bin_matrix(X, self.edges, self.nvb, self.nbt, names=self.x)

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        bm = self._codes(frame)
        n = frame.nrows
        pt = torch.zeros(n, dtype=torch.float64, device=bm.device)
        pc = torch.zeros_like(pt)
        for tr in self.trees:
            a, b = predict_tree(tr, bm.codes, n, self.nbt)
            pt += a
            pc += b
        k = max(len(self.trees), 1)
        pt, pc = (pt / k).float(), (pc / k).float()
        return torch.stack([pt - pc, pt, pc]).to(frame.device)

    def predict(self, frame: Frame) -> Frame:
        P = self.predict_raw(frame)
        return Frame([Vec("uplift_predict", P[0], "real"), Vec("p_y1_with_treatment", P[1], "real"),
                      Vec("p_y1_without_treatment", P[2], "real")])

    def _metrics(self, frame: Frame, P: torch.Tensor, comm=None) -> dict:
        frame = self.adapt_frame(frame)
        y = frame.vec(self.y).data.double()
        t = _treatment(frame, self.treatment_column, self.params.get("_treatment_domain"))
        ok = (y >= 0) & (t >= 0)
        return uplift_metrics(P[0][ok], y[ok], t[ok], int(self.params.get("auuc_nbins") or -1),
                              str(self.params.get("auuc_type", "AUTO")), comm)

    def varimp(self):
        g = np.zeros(len(self.x))
        for tr in self.trees:
            for f, gn in zip(tr["feat"], tr.get("gain", np.zeros(len(tr["feat"])))):
                if f >= 0:
                    g[f] += max(float(gn), 0.0)
        if g.max() <= 0:
            return [(c, 0.0, 0.0, 0.0) for c in self.x]
        order = np.argsort(-g, kind="stable")
        return [(self.x[i], float(g[i]), float(g[i] / g.max()), float(g[i] / g.sum())) for i in order]

    def summary(self):
        nl = [int((tr["feat"] < 0).sum()) for tr in self.trees]
        return {"model_id": self.model_id, "algo": self.algo, "number_of_trees": len(self.trees),
                "min_leaves": min(nl) if nl else 0, "max_leaves": max(nl) if nl else 0,
                "mean_leaves": float(np.mean(nl)) if nl else 0.0}


def _treatment(frame: Frame, col: str, domain=None) -> torch.Tensor:
    """Treatment indicator as float64 (1 treated, 0 control, -1 NA).  Categorical
    columns use their second level as the treatment (H2O: domain ["0", "1"])."""
    v = frame.vec(col)
    if v.vtype == ENUM:
        dom = list(v.domain or [])
        ref = list(domain) if domain else dom
        if len(ref) != 2:
            raise ValueError(f"upliftdrf: treatment_column {col!r} must have exactly 2 levels")
        lut = torch.tensor([ref.index(d) if d in ref else -1 for d in dom] + [-1], dtype=torch.float64,
                           device=v.data.device)
        c = v.data.long()
        return lut[torch.where(c >= 0, c, torch.full_like(c, len(dom)))]
    x = v.as_float().double()
    return torch.where(torch.isnan(x), torch.full_like(x, -1.0), (x != 0).double())


class H2OUpliftRandomForestEstimator(ModelBuilder):
    algo = "upliftdrf"
    DEFAULTS = dict(treatment_column="treatment", uplift_metric="AUTO", auuc_type="AUTO", auuc_nbins=-1,
                    ntrees=50, max_depth=20, min_rows=10.0, nbins=20, nbins_top_level=1024, nbins_cats=1024,
                    sample_rate=0.632, mtries=-2, col_sample_rate_per_tree=1.0, min_split_improvement=1e-5,
                    histogram_type="AUTO", stopping_rounds=0, stopping_metric="AUTO", score_each_iteration=False,
                    score_tree_interval=0, _treatment_domain=None)

    def _resolve_columns(self, frame, x, y):
        x, y = super()._resolve_columns(frame, x, y)
        tc = self.params["treatment_column"]
        if tc not in frame.names:
            raise ValueError(f"upliftdrf: treatment_column {tc!r} not in the frame")
        return [c for c in x if c != tc], y

    def _fit(self, train: Frame, valid, model_id):
        if self.category != ModelCategory.BINOMIAL:
            raise ValueError("upliftdrf needs a binary (two-level) response")
        p_ = self.params
        comm = self.comm
        world = comm.world_size if comm is not None else 1
        tc = p_["treatment_column"]
        tv = train.vec(tc)
        if tv.vtype == ENUM:
            p_["_treatment_domain"] = list(tv.domain)
        treat = _treatment(train, tc, p_["_treatment_domain"])
        y = train.vec(self.y).data.double()
        ok = (y >= 0) & (treat >= 0)
        X = train.feature_matrix(self.x)
        if not bool(ok.all()):
            X, y, treat = X[:, ok], y[ok], treat[ok]
        n = y.numel()
        dev = X.device
        nbins = max(2, min(int(p_["nbins"]), 254))
        seed = self._seed()
        edges, nvb, nbt = compute_edges(X, nbins, seed=seed, comm=comm, histogram_type=p_.get("histogram_type"))
        bm = bin_matrix(X, edges, nvb, nbt, names=self.x)
        codes = bm.codes[:, :n]
        F = len(self.x)
        nvb_np = np.asarray(nvb, np.int64)
        metric = str(p_["uplift_metric"])
        min_rows = float(p_["min_rows"])
        msi = float(p_["min_split_improvement"])
        mt = int(p_["mtries"])
        mtries = F if mt in (-2, 0) or mt >= F else (max(1, int(math.sqrt(F))) if mt == -1 else max(1, mt))
        rank = comm.rank if comm is not None else 0
        g_rows = torch.Generator(device=dev).manual_seed(seed * 7919 + rank)
        g_feat = torch.Generator().manual_seed(seed)           # identical on every rank
        # bins beyond a feature's value bins are never split points
        bin_ok = torch.zeros((F, nbt - 1), dtype=torch.bool, device=dev)
        for f in range(F):
            bin_ok[f, : max(int(nvb_np[f]) - 1, 0)] = True
        trees = []
        # row category (treated/control x y=0/1): every statistic is a count of one of them
        cat = ((1 - treat) * 2 + y).long()
        for t in range(int(p_["ntrees"])):
            sr = float(p_["sample_rate"])
            rc = cat.clone()
            if sr < 1:
                rc[torch.rand(n, generator=g_rows, device=dev) >= sr] = -1
            csr = float(p_["col_sample_rate_per_tree"])
            tree_cols = torch.ones(F, dtype=torch.bool)
            if csr < 1:
                k = max(1, int(round(csr * F)))
                tree_cols[:] = False
                tree_cols[torch.randperm(F, generator=g_feat)[:k]] = True
            trees.append(self._grow(codes, rc, F, nbt, bin_ok, tree_cols, mtries, g_feat, metric, min_rows, msi,
                                    comm))
        model = UpliftDRFModel(self, model_id, trees, np.asarray(edges), nvb_np, nbt, tc)
        return model

    @staticmethod
    def _hist(codes, rc, slot, S, F, nbt, comm):
        """Category counts [S][F][nbt][4] of the rows with slot >= 0: one
        unweighted bincount over (slot, feature, bin, category) keys."""
        dev = codes.device
        rows = torch.nonzero((slot >= 0) & (rc >= 0)).flatten()
        H = torch.zeros(S * F * nbt * 4, dtype=torch.float64, device=dev)
        if rows.numel():
            base = (slot[rows] * (F * nbt * 4) + rc[rows])[None, :]
            fchunk = max(1, (1 << 26) // rows.numel())
            for f0 in range(0, F, fchunk):
                f1 = min(F, f0 + fchunk)
                fi = torch.arange(f0, f1, device=dev)[:, None]
                key = base + (fi * nbt + codes[f0:f1][:, rows].long()) * 4
                H += torch.bincount(key.flatten(), minlength=H.numel()).double()
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(H)
        return H.view(S, F, nbt, 4)

    def _grow(self, codes, rc, F, nbt, bin_ok, tree_cols, mtries, g_feat, metric, min_rows, msi, comm):
        """Level-wise tree on category counts; each level builds the histogram
        of the smaller child of every split and derives its sibling by
        subtraction from the parent."""
        dev = codes.device
        n = codes.shape[1]
        max_depth = int(self.params["max_depth"])
        tree = UpliftTree()
        gains = [0.0]
        nid = torch.where(rc >= 0, torch.zeros_like(rc), torch.full_like(rc, -1))   # level-local node, -1 = done
        Hc = self._hist(codes, rc, nid, 1, F, nbt, comm)                   # [K][F][nbt][4 categories]
        tot0 = Hc[0, 0].sum(0).cpu().numpy()
        root_t = tot0[0] + tot0[1]
        root_c = tot0[2] + tot0[3]
        tree.add(tot0[1] / root_t if root_t > 0 else 0.0, tot0[3] / root_c if root_c > 0 else 0.0)
        level_nodes = [0]
        for depth in range(max_depth):              # max_depth levels of splits (as the GBM/DRF engine)
            K = len(level_nodes)
            # statistics [4][K][F][nbt]: nt, yt, nc, yc
            H = torch.stack([Hc[..., 0] + Hc[..., 1], Hc[..., 1], Hc[..., 2] + Hc[..., 3], Hc[..., 3]])
            na = H[..., nbt - 1]
            cum = torch.cumsum(H[..., : nbt - 1], -1)
            node_tot = H[:, :, 0, :].sum(-1)                               # [4][K]
            T = node_tot[:, :, None, None]
            zero = torch.zeros(K, dtype=torch.float64, device=dev)
            pn = _ratio(node_tot[1], node_tot[0], zero)
            qn = _ratio(node_tot[3], node_tot[2], zero)
            d_node = divergence(pn, qn, metric)
            ntot = (node_tot[0] + node_tot[2]).clamp_min(1e-300)
            fmask = tree_cols.clone()[None, :].repeat(K, 1)
            if mtries < F:
                r = torch.rand((K, F), generator=g_feat)
                r[~fmask] = 2.0
                kth = torch.topk(r, mtries, dim=1, largest=False).values[:, -1:]
                fmask = r <= kth
            fmask = fmask.to(dev)
            best_gain = torch.full((K,), -math.inf, dtype=torch.float64, device=dev)
            best = torch.zeros((K, 3), dtype=torch.long, device=dev)         # feat, bin, na_left
            for na_left in (0, 1):
                L = cum + (na[..., None] if na_left else 0.0)
                R = T - L
                nL, nR = L[0] + L[2], R[0] + R[2]
                valid = ((nL >= min_rows) & (nR >= min_rows) & (L[0] > 0) & (L[2] > 0) & (R[0] > 0) & (R[2] > 0)
                         & bin_ok[None] & fmask[:, :, None])
                dL = divergence(_ratio(L[1], L[0], pn[:, None, None]), _ratio(L[3], L[2], qn[:, None, None]), metric)
                dR = divergence(_ratio(R[1], R[0], pn[:, None, None]), _ratio(R[3], R[2], qn[:, None, None]), metric)
                gain = (nL * dL + nR * dR) / ntot[:, None, None] - d_node[:, None, None]
                gain = torch.where(valid, gain, torch.full_like(gain, -math.inf))
                gv, gi = gain.view(K, -1).max(1)
                upd = gv > best_gain
                best_gain = torch.where(upd, gv, best_gain)
                fb = torch.stack([gi // (nbt - 1), gi % (nbt - 1), torch.full_like(gi, na_left)], 1)
                best = torch.where(upd[:, None], fb, best)
            split = torch.isfinite(best_gain) & (best_gain > msi)
            kk = torch.arange(K, device=dev)
            Lk = cum[:, kk, best[:, 0], best[:, 1]] + na[:, kk, best[:, 0]] * best[:, 2][None, :]
            Rk = node_tot - Lk
            split_c = split.cpu().numpy()
            if not split_c.any():
                break
            best_c, gain_c = best.cpu().numpy(), best_gain.cpu().numpy()
            Lc, Rc, tot_c = Lk.cpu().numpy(), Rk.cpu().numpy(), node_tot.cpu().numpy()
            new_nodes, parent, built_right = [], [], []
            remap = np.full(K, -1, np.int64)
            for k in np.nonzero(split_c)[0]:
                node = level_nodes[k]
                pt, pc = tree.pt[node], tree.pc[node]
                lt, lc = Lc[:, k], Rc[:, k]
                li = tree.add(lt[1] / lt[0] if lt[0] > 0 else pt, lt[3] / lt[2] if lt[2] > 0 else pc)
                tree.add(lc[1] / lc[0] if lc[0] > 0 else pt, lc[3] / lc[2] if lc[2] > 0 else pc)
                gains += [0.0, 0.0]
                f, b, nl = (int(v) for v in best_c[k])
                tree.feat[node], tree.bin[node], tree.na_left[node], tree.left[node] = f, b, nl, li
                gains[node] = float(gain_c[k]) * float(tot_c[0, k] + tot_c[2, k])
                remap[k] = len(parent)
                parent.append(k)
                built_right.append(bool(lc[0] + lc[2] < lt[0] + lt[2]))       # build the smaller child
                new_nodes += [li, li + 1]
            # route the rows of split nodes to their children (level-local ids 2 * remap + right)
            remap_d = torch.from_numpy(remap).to(dev)
            rows = torch.nonzero(nid >= 0).flatten()
            k = nid[rows]
            rk = remap_d[k]
            c = codes[best[k, 0], rows].long()
            right = torch.where(c == nbt - 1, best[k, 2] == 0, c > best[k, 1])
            nid[rows] = torch.where(rk >= 0, 2 * rk + right.long(), torch.full_like(rk, -1))
            P = len(parent)
            br = torch.tensor(built_right, dtype=torch.long, device=dev)
            # build slot of a row: its pair index when it sits in the built child
            slot = torch.where((nid >= 0) & ((nid & 1) == br[(nid >> 1).clamp_min(0)]), nid >> 1,
                               torch.full_like(nid, -1))
            Hb = self._hist(codes, rc, slot, P, F, nbt, comm)
            Hpar = Hc[torch.tensor(parent, dtype=torch.long, device=dev)]
            Hs = Hpar - Hb
            Hn = torch.empty((2 * P, F, nbt, 4), dtype=torch.float64, device=dev)
            pidx = torch.arange(P, device=dev)
            Hn[2 * pidx + br] = Hb
            Hn[2 * pidx + 1 - br] = Hs
            Hc = Hn
            level_nodes = new_nodes
        arr = tree.arrays()
        arr["gain"] = np.array(gains, np.float64)
        return arr
