"""Distributed model metrics.

Every metric is computed from per-shard sufficient statistics that are
all-reduced once (sums, or a fine score histogram for AUC / thresholds), so
training metrics of a multi-GPU model cost one small collective.  H2O's
``AUC2`` uses a 400-bin histogram; we use 2^16 bins over the observed score
range, which puts the AUC error well below 1e-4.
"""
from __future__ import annotations

import math

import numpy as np
import torch

AUC_BINS = 1 << 16


def _reduce(comm, t: torch.Tensor, op="sum") -> torch.Tensor:
    if comm is not None and comm.world_size > 1:
        comm.all_reduce_(t, op)
    return t


def score_histograms(score: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None = None, comm=None,
                     nbins: int = AUC_BINS):
    """Weighted histograms of scores for positives / negatives over [lo, hi]."""
    s = score.detach().double()
    lohi = torch.stack([s.min(), -s.max()]) if s.numel() else torch.tensor([0.0, 0.0], device=s.device, dtype=torch.float64)
    lohi = _reduce(comm, lohi.clone(), "min")
    lo, hi = float(lohi[0]), float(-lohi[1])
    span = max(hi - lo, 1e-300)
    yy = y.detach().double()
    if s.is_cuda:
        # HIP kernel (csrc/metrics_kernels.hip): fixed-point integer atomics ->
        # deterministic histograms, then one all-reduce
        from .. import ops

        lib = ops.metrics_lib()
        Hq = torch.zeros((2, nbins), dtype=torch.int64, device=s.device)
        sc, yc = s.contiguous(), yy.contiguous()
        wc = None if w is None else w.detach().double().contiguous()
        ops.check(lib.h2omx_auc_hist(ops.P(sc), ops.P(yc), ops.P(wc), sc.numel(), nbins, lo, hi, ops.P(Hq),
                                     ops.stream(s.device)), "auc_hist")
        Hq = _reduce(comm, Hq)
        return Hq.cpu().numpy().astype(np.float64) / 16777216.0, lo, hi
    idx = ((s - lo) / span * (nbins - 1)).round().clamp_(0, nbins - 1).long()
    ww = torch.ones_like(yy) if w is None else w.detach().double()
    pos = torch.bincount(idx, weights=ww * yy, minlength=nbins)
    neg = torch.bincount(idx, weights=ww * (1 - yy), minlength=nbins)
    H = torch.stack([pos, neg])
    H = _reduce(comm, H)
    return H.cpu().numpy(), lo, hi


def auc_from_hist(pos: np.ndarray, neg: np.ndarray) -> float:
    # sweep thresholds from high to low score
    p = pos[::-1].astype(np.float64)
    q = neg[::-1].astype(np.float64)
    P, N = p.sum(), q.sum()
    if P <= 0 or N <= 0:
        return float("nan")
    tp = np.cumsum(p)
    fp = np.cumsum(q)
    tp0 = np.concatenate([[0.0], tp[:-1]])
    # trapezoid: within a bin ties count half
    return float(((fp - np.concatenate([[0.0], fp[:-1]])) * (tp0 + tp) * 0.5).sum() / (P * N))


def auc_from_scores(score, y, w=None, comm=None) -> float:
    H, _, _ = score_histograms(score, y, w, comm)
    return auc_from_hist(H[0], H[1])


def binomial_metrics(prob: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None = None, comm=None) -> dict:
    """H2O ModelMetricsBinomial: AUC, AUCPR, logloss, MSE, RMSE, gini, max-F1 threshold, confusion matrix."""
    p = prob.detach().double().clamp(1e-15, 1 - 1e-15)
    yy = y.detach().double()
    ww = torch.ones_like(yy) if w is None else w.detach().double()
    sums = torch.stack([
        (ww * -(yy * torch.log(p) + (1 - yy) * torch.log1p(-p))).sum(),
        (ww * (yy - p) ** 2).sum(),
        ww.sum(),
    ])
    sums = _reduce(comm, sums).cpu().numpy()
    H, lo, hi = score_histograms(p, yy, ww, comm)
    auc = auc_from_hist(H[0], H[1])
    pos, neg = H[0][::-1], H[1][::-1]
    tp, fp = np.cumsum(pos), np.cumsum(neg)
    P, N = pos.sum(), neg.sum()
    fn, tn = P - tp, N - fp
    prec = np.where(tp + fp > 0, tp / np.maximum(tp + fp, 1e-300), 1.0)
    rec = tp / max(P, 1e-300)
    f1 = np.where(prec + rec > 0, 2 * prec * rec / np.maximum(prec + rec, 1e-300), 0.0)
    k = int(np.argmax(f1))
    nb = len(pos)
    thr = hi - (hi - lo) * k / max(nb - 1, 1)
    rec_prev = np.concatenate([[0.0], rec[:-1]])
    aucpr = float(((rec - rec_prev) * prec).sum())
    mpce = 0.5 * ((fn[k] / max(P, 1e-300)) + (fp[k] / max(N, 1e-300)))
    n = sums[2]
    mse = sums[1] / n
    return {
        "AUC": auc, "AUCPR": aucpr, "Gini": 2 * auc - 1, "logloss": sums[0] / n, "MSE": mse,
        "RMSE": math.sqrt(mse), "nobs": float(n), "max_f1_threshold": float(thr), "max_f1": float(f1[k]),
        "mean_per_class_error": float(mpce),
        "confusion_matrix": [[float(tn[k]), float(fp[k])], [float(fn[k]), float(tp[k])]],
    }


def regression_metrics(pred: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None = None, comm=None,
                       dist: str = "gaussian") -> dict:
    pr = pred.detach().double()
    yy = y.detach().double()
    ww = torch.ones_like(yy) if w is None else w.detach().double()
    r = yy - pr
    rmsle_ok = (pr > -1) & (yy > -1)
    dev = _deviance(dist, yy, pr)
    sums = torch.stack([(ww * r * r).sum(), (ww * r.abs()).sum(), ww.sum(), (ww * yy).sum(), (ww * yy * yy).sum(),
                        (ww * torch.where(rmsle_ok, (torch.log1p(pr.clamp_min(-0.999999)) - torch.log1p(yy.clamp_min(-0.999999))) ** 2, torch.zeros_like(pr))).sum(),
                        (ww * dev).sum()])
    s = _reduce(comm, sums).cpu().numpy()
    n = s[2]
    mse = s[0] / n
    var = s[4] / n - (s[3] / n) ** 2
    return {"MSE": mse, "RMSE": math.sqrt(mse), "mae": s[1] / n, "rmsle": math.sqrt(max(s[5] / n, 0.0)),
            "mean_residual_deviance": s[6] / n, "r2": 1 - mse / var if var > 0 else float("nan"), "nobs": float(n)}


def _deviance(dist, y, mu):
    if dist == "poisson":
        mu = mu.clamp_min(1e-15)
        return 2 * (torch.where(y > 0, y * torch.log(y.clamp_min(1e-300) / mu), torch.zeros_like(y)) - (y - mu))
    if dist == "gamma":
        mu = mu.clamp_min(1e-15)
        return 2 * (-torch.log(y.clamp_min(1e-300) / mu) + (y - mu) / mu)
    if dist == "laplace":
        return (y - mu).abs()
    return (y - mu) ** 2


def multinomial_metrics(prob: torch.Tensor, y: torch.Tensor, w: torch.Tensor | None = None, comm=None) -> dict:
    """prob [K][n]; y class indices."""
    K = prob.shape[0]
    p = prob.detach().double().clamp(1e-15, 1.0)
    yi = y.detach().long()
    ww = torch.ones(yi.shape, dtype=torch.float64, device=p.device) if w is None else w.detach().double()
    py = p.gather(0, yi[None, :])[0]
    onehot = torch.nn.functional.one_hot(yi, K).double().T
    pred = p.argmax(0)
    cm = torch.zeros((K, K), dtype=torch.float64, device=p.device)
    cm.index_put_((yi, pred), ww, accumulate=True)
    top = p.topk(min(K, 10), dim=0).indices  # [k][n]
    hits = (top == yi[None, :]).double().cumsum(0)
    sums = torch.cat([torch.stack([(ww * -torch.log(py)).sum(), (ww * ((onehot - p) ** 2).sum(0)).sum(), ww.sum()]),
                      cm.reshape(-1), (hits * ww[None, :]).sum(1)])
    s = _reduce(comm, sums).cpu().numpy()
    n = s[2]
    cmn = s[3:3 + K * K].reshape(K, K)
    per_class_err = [1 - cmn[k, k] / cmn[k].sum() if cmn[k].sum() > 0 else 0.0 for k in range(K)]
    mse = s[1] / n
    return {"logloss": s[0] / n, "MSE": mse, "RMSE": math.sqrt(mse), "nobs": float(n),
            "mean_per_class_error": float(np.mean(per_class_err)), "confusion_matrix": cmn.tolist(),
            "hit_ratio_table": (s[3 + K * K:] / n).tolist()}
