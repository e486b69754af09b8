"""GLM extensions: interaction columns (``interactions`` /
``interaction_pairs``) and the ordinal family (proportional-odds cumulative
logit).

Interactions follow H2O's expansion.  For a pair (a, b):
  * numeric x numeric    -> one product column "a_b";
  * categorical x numeric -> one column per level of the categorical,
    "a.level_b" = [a == level] * b (a level-specific slope);
  * categorical x categorical -> one combined factor "a_b", with levels
    "la_lb" seen in training (counted over all ranks).  The design matrix
    one-hot expands it like any factor.
The spec is stored on the model, and scoring frames are augmented the same way.

Ordinal: P(y <= k | x) = sigmoid(theta_k - x.beta) for k = 0 .. K-2, with
increasing thresholds theta (parameterised as theta_0 plus cumulative exp
increments).  The negative log-likelihood plus lambda (1 - alpha) / 2 |beta|^2
is minimised with L-BFGS.  Every loss / gradient evaluation is one fp64
pass on the device; multi-rank runs all-reduce the loss and gradient.
"""
from __future__ import annotations

import itertools

import numpy as np
import torch

from ..frame.distributed import _gather_objects
from ..frame.frame import ENUM, Frame, Vec


def interaction_pairs(params: dict, x: list, frame: Frame) -> list:
    pairs = []
    cols = params.get("interactions") or []
    for a, b in itertools.combinations([c for c in cols if c in frame.names], 2):
        pairs.append((a, b))
    for pr in params.get("interaction_pairs") or []:
        a, b = (pr[0], pr[1]) if isinstance(pr, (list, tuple)) else tuple(str(pr).split(":"))
        if (a, b) not in pairs and (b, a) not in pairs:
            pairs.append((a, b))
    return pairs


def build_interaction_spec(frame: Frame, pairs: list, comm=None) -> list:
    spec = []
    for a, b in pairs:
        va, vb = frame.vec(a), frame.vec(b)
        ea, eb = va.vtype == ENUM, vb.vtype == ENUM
        if ea and eb:
            ca, cb = va.data.long(), vb.data.long()
            ok = (ca >= 0) & (cb >= 0)
            La = len(vb.domain or [])
            u = torch.unique(ca[ok] * max(La, 1) + cb[ok]).cpu().tolist()
            seen = sorted(set().union(*[set(s) for s in _gather_objects(comm, u)]))
            levels = [f"{va.domain[k // max(La, 1)]}_{vb.domain[k % max(La, 1)]}" for k in seen]
            spec.append(("ee", a, b, levels))
        elif ea or eb:
            cat, num = (a, b) if ea else (b, a)
            spec.append(("en", cat, num, list(frame.vec(cat).domain or [])))
        else:
            spec.append(("nn", a, b, None))
    return spec


def interaction_columns(spec: list) -> list:
    out = []
    for kind, a, b, lv in spec:
        if kind == "en":
            out += [f"{a}.{level}_{b}" for level in lv]
        else:
            out.append(f"{a}_{b}")
    return out


def apply_interactions(frame: Frame, spec: list) -> Frame:
    if not spec:
        return frame
    have = set(frame.names)
    vecs = list(frame.vecs)
    for kind, a, b, lv in spec:
        if kind == "nn":
            if f"{a}_{b}" not in have:
                vecs.append(Vec(f"{a}_{b}", frame.vec(a).as_float() * frame.vec(b).as_float(), "real"))
        elif kind == "en":
            c = frame.vec(a)
            codes = c.data.long()
            dom = list(c.domain or [])
            x = frame.vec(b).as_float()
            for level in lv:
                name = f"{a}.{level}_{b}"
                if name in have:
                    continue
                j = dom.index(level) if level in dom else -2
                ind = torch.where(codes < 0, torch.full_like(x, float("nan")), (codes == j).float())
                vecs.append(Vec(name, ind * x, "real"))
        else:
            name = f"{a}_{b}"
            if name in have:
                continue
            va, vb = frame.vec(a), frame.vec(b)
            pos = {s: i for i, s in enumerate(lv)}
            da, db = list(va.domain or []), list(vb.domain or [])
            lut = torch.tensor([pos.get(f"{x}_{y}", -1) for x in da for y in db] + [-1], dtype=torch.int64)
            ca, cb = va.data.long().cpu(), vb.data.long().cpu()
            idx = torch.where((ca >= 0) & (cb >= 0), ca * max(len(db), 1) + cb, torch.full_like(ca, lut.numel() - 1))
            vecs.append(Vec(name, lut[idx].to(torch.int32).to(frame.device), ENUM, list(lv)))
    return Frame(vecs, key=frame.key)


# ---------------------------------------------------------------------------
# ordinal
# ---------------------------------------------------------------------------
def _ordinal_params(v: torch.Tensor, p: int, K: int):
    beta = v[:p]
    th = torch.cumsum(torch.cat([v[p:p + 1], torch.exp(v[p + 1:])]), 0)     # K-1 increasing thresholds
    return beta, th


def ordinal_probs(X: torch.Tensor, beta: torch.Tensor, th: torch.Tensor) -> torch.Tensor:
    """Class probabilities [K][n] from standardised X [p][n]."""
    eta = beta @ X
    cum = torch.sigmoid(th[:, None] - eta[None, :])                          # [K-1][n]
    ones = torch.ones((1, eta.numel()), dtype=cum.dtype, device=cum.device)
    zeros = torch.zeros_like(ones)
    c = torch.cat([zeros, cum, ones])
    return (c[1:] - c[:-1]).clamp_min(1e-15)


def fit_ordinal(X: torch.Tensor, y: torch.Tensor, w, K: int, lam: float, alpha: float, comm=None,
                max_iter: int = 200, tol: float = 1e-8):
    """Returns (beta [p] fp64 numpy, thresholds [K-1] numpy, neg-log-lik)."""
    from scipy.optimize import minimize

    Xd = X.double()
    p = Xd.shape[0]
    yi = y.long()
    wd = w.double() if w is not None else torch.ones(yi.numel(), dtype=torch.float64, device=Xd.device)
    cnt = torch.bincount(yi, weights=wd, minlength=K).double()
    if comm is not None and comm.world_size > 1:
        comm.all_reduce_(cnt)
    N = float(cnt.sum())
    cum = (torch.cumsum(cnt, 0)[:-1] / max(N, 1e-300)).clamp(1e-6, 1 - 1e-6).cpu().numpy()
    th0 = np.log(cum / (1 - cum))
    v0 = np.concatenate([np.zeros(p), [th0[0]], np.log(np.maximum(np.diff(th0), 1e-3))])
    l2 = lam * (1 - alpha)

    def fg(v_np):
        v = torch.tensor(v_np, dtype=torch.float64, device=Xd.device, requires_grad=True)
        beta, th = _ordinal_params(v, p, K)
        P = ordinal_probs(Xd, beta, th)
        nll = -(wd * torch.log(P.gather(0, yi[None, :])[0])).sum()
        g = torch.autograd.grad(nll, v)[0]
        out = torch.cat([nll.detach()[None], g])
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(out)
        f = float(out[0]) / N + 0.5 * l2 * float((v_np[:p] ** 2).sum())
        grad = out[1:].cpu().numpy() / N
        grad[:p] += l2 * v_np[:p]
        return f, grad

    res = minimize(fg, v0, jac=True, method="L-BFGS-B", options={"maxiter": max_iter, "gtol": tol})
    v = torch.tensor(res.x, dtype=torch.float64)
    beta, th = _ordinal_params(v, p, K)
    return beta.numpy(), th.numpy(), float(res.fun) * N, int(res.nit)
