"""GLM solvers besides IRLSM (H2O ``solver``: AUTO, IRLSM, L_BFGS,
COORDINATE_DESCENT, COORDINATE_DESCENT_NAIVE, GRADIENT_DESCENT_LH,
GRADIENT_DESCENT_SQERR).

``L_BFGS`` minimises the same objective as IRLSM,

    f(b) = deviance(b) / (2 N) + lambda (alpha |b|_1 + (1 - alpha) / 2 |b|^2)  (+ 1/2 bᵀ P b, GAM)

(intercepts unpenalised), from gradient passes only: one HIP pass over the
design per function evaluation (``ops.dense.glm_grad_pass``: linear
predictors -> per-row gradient weights -> Xᵀr), no p x p Gram, which is why
H2O picks it for wide data and many-class multinomials.  The L1 part uses
orthant-wise limited-memory quasi-Newton (OWL-QN: pseudo-gradient, orthant
projection of the step, Armijo backtracking); with alpha = 0 it is plain
L-BFGS.  The two-loop recursion and line search run on the host on vectors of
K (p + 1) doubles; every function/gradient evaluation is one device pass (and
one fused all-reduce of [gradient | deviance] across ranks).
"""
from __future__ import annotations

import numpy as np

SOLVERS = ("AUTO", "IRLSM", "L_BFGS", "COORDINATE_DESCENT", "COORDINATE_DESCENT_NAIVE", "GRADIENT_DESCENT_LH",
           "GRADIENT_DESCENT_SQERR")

# AUTO picks L_BFGS above these sizes (the Gram / Cholesky path stops paying)
AUTO_LBFGS_P = 5000
AUTO_LBFGS_KP = 10000


def resolve_solver(solver, family: str, p: int, K: int) -> str:
    """Validate ``solver`` and resolve AUTO (H2O GLM semantics)."""
    s = str(solver or "AUTO").upper()
    if s not in SOLVERS:
        raise ValueError(f"glm: unknown solver {solver!r} (one of {', '.join(SOLVERS)})")
    if s.startswith("GRADIENT_DESCENT") and family != "ordinal":
        raise ValueError(f"glm: solver {s} is only supported for family='ordinal' (as in H2O)")
    if family == "ordinal":
        if s in ("AUTO", "GRADIENT_DESCENT_LH", "GRADIENT_DESCENT_SQERR"):
            return "GRADIENT_DESCENT_LH" if s == "AUTO" else s
        raise ValueError(f"glm: family='ordinal' supports solver GRADIENT_DESCENT_LH / GRADIENT_DESCENT_SQERR, not {s}")
    if s == "AUTO":
        return "L_BFGS" if (p + 1 > AUTO_LBFGS_P or (family == "multinomial" and K * (p + 1) > AUTO_LBFGS_KP)) \
            else "IRLSM"
    return s


class LbfgsResult:
    def __init__(self, beta, f, dev, iters, evals, converged, stop_reason=""):
        self.beta, self.f, self.dev, self.iters, self.evals, self.converged = beta, f, dev, iters, evals, converged
        # "gradient" / "objective" (converged), "line_search_failed", "max_iterations"
        self.stop_reason = stop_reason


def owlqn(fg, b0: np.ndarray, pen_mask: np.ndarray, l1: float, max_iter: int = 500, m: int = 10,
          grad_eps: float = 1e-6, obj_eps: float = 1e-10, non_negative: bool = False) -> LbfgsResult:
    """Minimise smooth(b) + l1 * |b[pen_mask]|_1.

    ``fg(b) -> (smooth value, smooth gradient, deviance)``.  Returns the final
    point; ``converged`` when the pseudo-gradient's max-norm <= grad_eps or the
    relative objective change <= obj_eps."""
    b = np.asarray(b0, np.float64).copy()
    pen = pen_mask.astype(bool)
    if non_negative:
        b[pen] = np.maximum(b[pen], 0.0)
    fs, g, dev = fg(b)
    evals = 1

    def total(fs_, b_):
        return fs_ + l1 * np.abs(b_[pen]).sum()

    def pseudo(b_, g_):
        pg = g_.copy()
        if l1 > 0:
            bp, gp = b_[pen], g_[pen]
            out = np.where(bp > 0, gp + l1, np.where(bp < 0, gp - l1,
                                                    np.where(gp + l1 < 0, gp + l1, np.where(gp - l1 > 0, gp - l1, 0.0))))
            pg[pen] = out
        if non_negative:
            # at the bound b = 0 only an increase is feasible
            z = pen & (b_ <= 0) & (pg > 0)
            pg[z] = 0.0
        return pg

    S, Y, RHO = [], [], []
    f = total(fs, b)
    converged = False
    stop = "max_iterations"
    it = 0
    retried = False     # steepest-descent retry after a failed line search
    for it in range(1, max_iter + 1):
        pg = pseudo(b, g)
        if np.abs(pg).max() <= grad_eps:
            converged, stop = True, "gradient"
            break
        # two-loop recursion on the pseudo-gradient
        q = pg.copy()
        alphas = []
        for s_, y_, r_ in reversed(list(zip(S, Y, RHO))):
            a = r_ * s_.dot(q)
            alphas.append(a)
            q -= a * y_
        if S:
            q *= S[-1].dot(Y[-1]) / max(Y[-1].dot(Y[-1]), 1e-300)
        else:
            q /= max(np.abs(pg).max(), 1.0)
        for (s_, y_, r_), a in zip(zip(S, Y, RHO), reversed(alphas)):
            bb = r_ * y_.dot(q)
            q += s_ * (a - bb)
        d = -q
        # keep only descent coordinates of the pseudo-gradient (OWL-QN)
        if l1 > 0 or non_negative:
            d = np.where(d * pg < 0, d, 0.0)
        if d.dot(pg) >= 0:          # not a descent direction: restart from steepest descent
            S, Y, RHO = [], [], []
            d = -pg / max(np.abs(pg).max(), 1.0)
        xi = np.where(b != 0, np.sign(b), -np.sign(pg))
        t = 1.0
        accepted = False
        for _ in range(40):
            bn = b + t * d
            if l1 > 0:
                bn[pen] = np.where(np.sign(bn[pen]) == xi[pen], bn[pen], 0.0)
            if non_negative:
                bn[pen] = np.maximum(bn[pen], 0.0)
            fsn, gn, devn = fg(bn)
            evals += 1
            fn = total(fsn, bn)
            if fn <= f + 1e-4 * pg.dot(bn - b):
                accepted = True
                break
            t *= 0.5
        if not accepted:
            # no Armijo step along the quasi-Newton direction: drop the curvature
            # history and retry once from steepest descent; a second failure stops
            # WITHOUT claiming convergence (fp32 gradients of the HIP pass can stall
            # the search well before grad_eps / obj_eps are met)
            if S and not retried:
                S, Y, RHO = [], [], []
                retried = True
                continue
            stop = "line_search_failed"
            break
        retried = False
        s_, y_ = bn - b, gn - g
        sy = s_.dot(y_)
        if sy > 1e-12 * max(1.0, np.abs(s_).max() * np.abs(y_).max()):
            S.append(s_)
            Y.append(y_)
            RHO.append(1.0 / sy)
            if len(S) > m:
                S.pop(0)
                Y.pop(0)
                RHO.pop(0)
        rel = abs(f - fn) / max(abs(f), abs(fn), 1e-300)
        b, g, f, dev = bn, gn, fn, devn
        if rel <= obj_eps:
            converged, stop = True, "objective"
            break
    return LbfgsResult(b, f, dev, it, evals, converged, stop)
