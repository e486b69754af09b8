"""Generalized Linear Models (H2O GLM equivalent) with IRLS on the GPU.

Every IRLS iteration is ONE fused pass over the rows (csrc/dense_kernels.hip
glm_irls_kernel): eta = X beta, IRLS weights / working response and the
weighted Gram of [X | 1 | z] on the fp32 matrix cores, reduced in fp64 and
(for multi-rank clusters) all-reduced once.  The tiny (p+1)x(p+1) elastic-net
sub-problem is solved on the host by Cholesky (ridge) or cyclic coordinate
descent on the Gram (lasso / elastic net), like H2O's IRLSM solver.
``solver``: AUTO (IRLSM; L_BFGS for > 5000 columns or wide multinomials),
IRLSM, COORDINATE_DESCENT(_NAIVE) (IRLS with the coordinate-descent inner
solver every iteration), L_BFGS (OWL-QN over Gram-free gradient passes,
models/glm_solvers.py); GRADIENT_DESCENT_LH is the ordinal family's solver.
Unknown values raise.

Families: gaussian, binomial, quasibinomial, fractionalbinomial, poisson,
gamma, tweedie, negativebinomial (fixed ``theta``), multinomial (per-class
cyclic IRLS) and ordinal (cumulative logit, L-BFGS; models/glm_extras.py).
``interactions`` / ``interaction_pairs`` add H2O-style interaction columns.  Standardization, one-hot categorical
expansion (first level dropped, H2O's use_all_factor_levels=False), mean
imputation of NAs, lambda search, p-values (lambda = 0) and the H2O output
fields (coefficients, standardized coefficients, deviances, AIC) are
supported.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory
from .glm_solvers import owlqn, resolve_solver


class DesignInfo:
    """How frame columns expand into standardized numeric predictors."""

    def __init__(self, x, types, domains, use_all_levels=False):
        self.x = list(x)
        self.types = types
        self.domains = domains
        self.use_all_levels = use_all_levels
        self.names = []
        self.spec = []  # (col, level or None)
        for c in self.x:
            if types[c] == ENUM:
                dom = domains[c] or []
                lv = range(len(dom)) if use_all_levels else range(1, len(dom))
                for k in lv:
                    self.names.append(f"{c}.{dom[k]}")
                    self.spec.append((c, k))
            else:
                self.names.append(c)
                self.spec.append((c, None))
        self.means = None
        self.sds = None

    def raw_matrix(self, frame: Frame) -> torch.Tensor:
        cols = []
        for c, k in self.spec:
            v = frame.vec(c)
            if k is None:
                cols.append(v.as_float())
            else:
                codes = v.data
                col = (codes == k).float()
                cols.append(torch.where(codes < 0, torch.full_like(col, float("nan")), col))
        if not cols:
            return torch.zeros((0, frame.nrows), device=frame.device)
        return torch.stack(cols)

    def fit_standardization(self, Xraw: torch.Tensor, standardize: bool, comm=None):
        p, n = Xraw.shape
        ok = ~torch.isnan(Xraw)
        s1 = torch.where(ok, Xraw, torch.zeros_like(Xraw)).double().sum(1)
        s2 = torch.where(ok, Xraw, torch.zeros_like(Xraw)).double().pow(2).sum(1)
        cnt = ok.double().sum(1)
        stats = torch.stack([s1, s2, cnt])
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(stats)
        s1, s2, cnt = stats
        mean = (s1 / cnt.clamp_min(1)).cpu().numpy()
        var = (s2 / cnt.clamp_min(1) - (s1 / cnt.clamp_min(1)) ** 2).clamp_min(0).cpu().numpy()
        sd = np.sqrt(var * (cnt.cpu().numpy() / np.maximum(cnt.cpu().numpy() - 1, 1)))
        self.means = mean
        self.sds = np.where(sd > 0, sd, 1.0) if standardize else np.ones_like(sd)
        if not standardize:
            self.center = np.zeros_like(mean)
        else:
            self.center = mean

    def transform(self, Xraw: torch.Tensor) -> torch.Tensor:
        """Mean-impute NAs then standardize (float32, feature-major)."""
        m = torch.from_numpy(self.means.astype(np.float32)).to(Xraw.device)[:, None]
        c = torch.from_numpy(self.center.astype(np.float32)).to(Xraw.device)[:, None]
        s = torch.from_numpy(self.sds.astype(np.float32)).to(Xraw.device)[:, None]
        X = torch.where(torch.isnan(Xraw), m.expand_as(Xraw), Xraw)
        return ((X - c) / s).contiguous()


def _soft(x, t):
    return np.sign(x) * max(abs(x) - t, 0.0)


def _enet_cd(A, r, pen, l1, free_idx, non_negative, b, max_iter, tol) -> int:
    """Covariance-update cyclic coordinate descent in C++ (csrc/host/solvers.cpp)."""
    import ctypes

    from .._native import require

    lib = require("host")
    fn = lib.h2omx_enet_cd
    fn.restype = ctypes.c_int
    dp = ctypes.POINTER(ctypes.c_double)
    fn.argtypes = [dp, ctypes.c_int, dp, dp, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int, dp,
                   ctypes.c_int, ctypes.c_double]
    k = len(r)
    it = fn(A.ctypes.data_as(dp), A.shape[1], r.ctypes.data_as(dp), pen.ctypes.data_as(dp), k, float(l1),
            int(free_idx), int(bool(non_negative)), b.ctypes.data_as(dp), int(max_iter), float(tol))
    if it < 0:
        raise RuntimeError("h2omx_enet_cd: bad arguments")
    return it


def solve_enet(G: np.ndarray, p: int, N: float, lam: float, alpha: float, beta0: np.ndarray, intercept: bool,
               non_negative: bool = False, max_iter: int = 500, tol: float = 1e-9, penalty: np.ndarray | None = None,
               force_cd: bool = False):
    """Minimise (1/2N) sum w (z - x.b)^2 + lam (alpha |b|_1 + (1-alpha)/2 |b|^2)
    (+ 1/2 bᵀ P b for a quadratic ``penalty`` P on the p coefficients, GAM
    smoothness) given the augmented Gram G of [x | 1 | z].  Returns beta (p
    coefficients + intercept).  Ridge / unpenalised problems take a Cholesky
    solve unless ``force_cd`` (solver COORDINATE_DESCENT) asks for the
    covariance-update coordinate descent every time."""
    XtX = G[: p + 1, : p + 1] / N
    if penalty is not None:
        XtX = XtX.copy()
        XtX[:p, :p] += penalty
    Xtz = G[: p + 1, p + 1] / N
    l1 = lam * alpha
    l2 = lam * (1 - alpha)
    pen = np.full(p + 1, l2)
    pen[p] = 0.0
    if not intercept:
        XtX = XtX[:p, :p]
        Xtz = Xtz[:p]
        pen = pen[:p]
    k = len(Xtz)
    if l1 == 0 and not non_negative and not force_cd:
        A = XtX + np.diag(pen)
        try:
            L = np.linalg.cholesky(A + 1e-12 * np.eye(k) * max(1.0, np.abs(A).max()))
            b = np.linalg.solve(L.T, np.linalg.solve(L, Xtz))
        except np.linalg.LinAlgError:
            b = np.linalg.lstsq(A, Xtz, rcond=None)[0]
    else:
        b = np.ascontiguousarray(beta0[:k] if beta0 is not None else np.zeros(k), np.float64).copy()
        _enet_cd(np.ascontiguousarray(XtX, np.float64), np.ascontiguousarray(Xtz, np.float64),
                 np.ascontiguousarray(pen, np.float64), l1, p if intercept else -1, non_negative, b, max_iter, tol)
    if not intercept:
        b = np.concatenate([b, [0.0]])
    return b


class GLMModel(Model):
    algo = "glm"
    algo_full_name = "Generalized Linear Modeling"

    def __init__(self, builder, model_id, design, beta_std, family, link, stats):
        super().__init__(builder, model_id)
        self.design = design
        self.family = family
        self.link = link
        self.beta_std = beta_std            # [K][p+1] standardized space
        self.stats = stats
        K, p1 = beta_std.shape
        p = p1 - 1
        s = design.sds
        c = design.center
        self.beta = np.zeros_like(beta_std)  # raw scale
        for k in range(K):
            self.beta[k, :p] = beta_std[k, :p] / s
            self.beta[k, p] = beta_std[k, p] - float((beta_std[k, :p] * c / s).sum())

    def coef(self, k: int = 0) -> dict:
        out = {"Intercept": float(self.beta[k, -1])}
        out.update({n: float(v) for n, v in zip(self.design.names, self.beta[k, :-1])})
        return out

    def coef_norm(self, k: int = 0) -> dict:
        out = {"Intercept": float(self.beta_std[k, -1])}
        out.update({n: float(v) for n, v in zip(self.design.names, self.beta_std[k, :-1])})
        return out

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        spec = getattr(self, "interaction_spec", None)
        if spec:
            from .glm_extras import apply_interactions

            frame = apply_interactions(frame, spec)
        Xs = self.design.transform(self.design.raw_matrix(frame))
        b = torch.from_numpy(self.beta_std.astype(np.float64)).to(Xs.device)
        p = Xs.shape[0]
        if self.family == "ordinal":
            from .glm_extras import ordinal_probs

            th = torch.tensor(self.stats["ordinal_thresholds"], dtype=torch.float64, device=Xs.device)
            return ordinal_probs(Xs.double(), b[0, :p], th).float()
        eta = b[:, :p] @ Xs.double() + b[:, p:p + 1]
        if self.params.get("offset_column"):
            eta = eta + frame.vec(self.params["offset_column"]).as_float().double()[None, :]
        if self.family == "multinomial":
            return torch.softmax(eta, 0).float()
        mu = _torch_linkinv(eta[0], self.link, self.params.get("tweedie_link_power", 0.0))
        if self.category == ModelCategory.BINOMIAL:
            return torch.stack([1 - mu, mu]).float()
        return mu[None, :].float()

    def predict_contributions(self, frame: Frame) -> Frame:
        """Exact linear SHAP values in link space (explain_more.glm_contributions)."""
        from ..explain_more import glm_contributions

        return glm_contributions(self, frame)

    def varimp(self):
        b = np.abs(self.beta_std[:, :-1]).sum(0)
        if b.max() <= 0:
            return [(n, 0.0, 0.0, 0.0) for n in self.design.names]
        order = np.argsort(-b, kind="stable")
        return [(self.design.names[i], float(b[i]), float(b[i] / b.max()), float(b[i] / b.sum())) for i in order]

    def summary(self):
        return {"model_id": self.model_id, "family": self.family, "link": self.link,
                "regularization": f"Elastic Net (alpha = {self.params['alpha']}, lambda = {self.stats['lambda']:.4g})",
                "number_of_predictors_total": len(self.design.names),
                "number_of_active_predictors": int((np.abs(self.beta[:, :-1]) > 0).any(0).sum()),
                "number_of_iterations": self.stats["iterations"]}

    def to_json(self):
        j = super().to_json()
        out = j["output"]
        names = ["Intercept"] + self.design.names
        if self.family == "multinomial":
            out["coefficients_table"] = {"names": names, "coefficients": [
                [float(self.beta[k, -1])] + self.beta[k, :-1].tolist() for k in range(self.beta.shape[0])]}
        else:
            out["coefficients_table"] = {"names": names,
                                         "coefficients": [float(self.beta[0, -1])] + self.beta[0, :-1].tolist(),
                                         "standardized_coefficients": [float(self.beta_std[0, -1])] +
                                         self.beta_std[0, :-1].tolist()}
            if self.stats.get("std_errors") is not None:
                out["coefficients_table"].update(std_error=self.stats["std_errors"], z_value=self.stats["z_values"],
                                                 p_value=self.stats["p_values"])
        out["null_deviance"] = self.stats["null_deviance"]
        out["residual_deviance"] = self.stats["residual_deviance"]
        out["AIC"] = self.stats.get("aic")
        out["lambda_best"] = self.stats["lambda"]
        return j


def _torch_linkinv(eta, link, link_power=0.0):
    if link == "logit":
        return torch.sigmoid(eta)
    if link == "log":
        return torch.exp(eta.clamp(max=700))
    if link == "inverse":
        return 1 / eta
    if link == "tweedie":
        return torch.exp(eta) if link_power == 0 else eta.clamp_min(1e-10) ** (1 / link_power)
    return eta


class H2OGeneralizedLinearEstimator(ModelBuilder):
    algo = "glm"
    DEFAULTS = dict(family="AUTO", link="family_default", solver="AUTO", alpha=None, lambda_=None, Lambda=None,
                    lambda_search=False, nlambdas=-1, lambda_min_ratio=-1.0, standardize=True, intercept=True,
                    max_iterations=-1, beta_epsilon=1e-4, objective_epsilon=-1.0, gradient_epsilon=-1.0,
                    non_negative=False, compute_p_values=False, remove_collinear_columns=False,
                    missing_values_handling="MeanImputation", tweedie_variance_power=0.0, tweedie_link_power=1.0,
                    use_all_factor_levels=False, offset_column=None, prior=-1.0, balance_classes=False,
                    theta=1e-10, interactions=None, interaction_pairs=None)

    def __init__(self, **params):
        if "lambda" in params:
            params["lambda_"] = params.pop("lambda")
        super().__init__(**params)

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        """``interactions`` / ``interaction_pairs``: the frames gain the
        interaction columns (glm_extras) before the usual fit; the spec is kept
        on the model so scoring frames are augmented identically."""
        from .glm_extras import apply_interactions, build_interaction_spec, interaction_columns, interaction_pairs

        self.params.update(kw)
        pairs = interaction_pairs(self.params, x, training_frame) if training_frame is not None else []
        if not pairs:
            return super().train(x=x, y=y, training_frame=training_frame, validation_frame=validation_frame,
                                 comm=comm)
        spec = build_interaction_spec(training_frame, pairs, comm)
        aug = apply_interactions(training_frame, spec)
        vaug = apply_interactions(validation_frame, spec) if validation_frame is not None else None
        special = {y, self.params.get("weights_column"), self.params.get("fold_column"),
                   self.params.get("offset_column")}
        ign = set(self.params.get("ignored_columns") or [])
        base_x = list(x) if x is not None else [n for n in training_frame.names if n not in special and n not in ign]
        model = super().train(x=base_x + interaction_columns(spec), y=y, training_frame=aug, validation_frame=vaug,
                              comm=comm)
        model.interaction_spec = spec
        return model

    def _family(self):
        fam = str(self.params["family"]).lower()
        if fam == "auto":
            return {ModelCategory.BINOMIAL: "binomial", ModelCategory.MULTINOMIAL: "multinomial"}.get(
                self.category, "gaussian")
        return fam

    def _fit_ordinal(self, X, y, w, N, design, lam_param, alpha, model_id):
        return _fit_ordinal_impl(self, X, y, w, N, design, lam_param, alpha, model_id)

    def _fit_lbfgs(self, *a):
        return _fit_lbfgs_impl(self, *a)

    def _penalty_matrix(self, design):
        """Quadratic coefficient penalty (raw scale, p×p) added to the IRLS normal
        equations; None for plain GLM (overridden by GAM)."""
        return None

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        family = self._family()
        link = str(p_["link"]).lower()
        if link in ("family_default", "auto"):
            link = D.DEFAULT_LINK[family]
        comm = self.comm
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, p_["use_all_factor_levels"])
        Xraw = design.raw_matrix(train)
        yv = train.vec(self.y)
        y = yv.data.float() if yv.vtype == ENUM else yv.as_float()
        ok = (y >= 0) if yv.vtype == ENUM else ~torch.isnan(y)
        w = train.vec(p_["weights_column"]).as_float() if p_.get("weights_column") else None
        off = train.vec(p_["offset_column"]).as_float() if p_.get("offset_column") else None
        if not bool(ok.all()):
            Xraw, y = Xraw[:, ok], y[ok]
            w = None if w is None else w[ok]
            off = None if off is None else off[ok]
        design.fit_standardization(Xraw, bool(p_["standardize"]), comm)
        X = design.transform(Xraw)
        del Xraw
        p = X.shape[0]
        K = len(self.response_domain) if family == "multinomial" else 1
        if family == "ordinal" and not self.response_domain:
            raise ValueError("glm: family='ordinal' needs a categorical response")
        # optional quadratic penalty on the raw-scale coefficients (GAM), moved to the
        # standardised scale: b_raw = b_std / sd  ->  P_std = D⁻¹ P D⁻¹
        pen_raw = self._penalty_matrix(design)
        pen_std = None if pen_raw is None else pen_raw / np.outer(design.sds, design.sds)
        solver = resolve_solver(p_["solver"], family, p, K)
        if solver == "GRADIENT_DESCENT_SQERR":
            raise ValueError("glm: solver GRADIENT_DESCENT_SQERR (ordinal squared-error objective) is not supported; "
                             "use GRADIENT_DESCENT_LH")
        alpha = p_["alpha"]
        alpha = (0.0 if solver == "L_BFGS" else 0.5) if alpha is None else float(alpha[0] if isinstance(alpha, (list, tuple)) else alpha)
        lam_param = p_["lambda_"] if p_["lambda_"] is not None else p_["Lambda"]
        var_power = float(p_["theta"]) if family == "negativebinomial" else float(p_["tweedie_variance_power"] or 1.5)
        link_power = float(p_["tweedie_link_power"]) if family == "tweedie" else 0.0
        if family == "tweedie" and link_power != 0.0 and link == "tweedie":
            pass
        intercept = bool(p_["intercept"])
        max_iter = int(p_["max_iterations"]) if int(p_["max_iterations"]) > 0 else (50 if family != "multinomial" else 100)
        beps = float(p_["beta_epsilon"])

        def allreduce(G, dev):
            if comm is not None and comm.world_size > 1:
                arr = comm.all_reduce_numpy(np.concatenate([G.ravel(), [dev]]))
                return arr[:-1].reshape(G.shape), float(arr[-1])
            return G, dev

        # intercept-only (null) model and lambda_max
        ysum = torch.stack([(y * (w if w is not None else 1)).double().sum(),
                            (w.double().sum() if w is not None else torch.tensor(float(y.numel()), dtype=torch.float64,
                                                                                  device=y.device))])
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(ysum)
        N = float(ysum[1])
        ybar = float(ysum[0]) / max(N, 1e-300)
        beta = np.zeros((K, p + 1))
        if family == "ordinal":
            return self._fit_ordinal(X, y, w, N, design, lam_param, alpha, model_id)
        if family in ("binomial", "quasibinomial", "fractionalbinomial"):
            pb = min(max(ybar, 1e-10), 1 - 1e-10)
            beta[0, p] = math.log(pb / (1 - pb))
        elif family in ("poisson", "gamma", "negativebinomial") or (family == "tweedie" and link_power == 0.0):
            beta[0, p] = math.log(max(ybar, 1e-10)) if link in ("log", "tweedie") else (1.0 / ybar if link == "inverse" else ybar)
        elif family == "multinomial":
            ycpu = y.long()
            cnt = torch.bincount(ycpu, minlength=K).double()
            if comm is not None and comm.world_size > 1:
                comm.all_reduce_(cnt)
            pr = (cnt / cnt.sum()).clamp_min(1e-10).cpu().numpy()
            beta[:, p] = np.log(pr) - np.log(pr).mean()
        else:
            beta[0, p] = ybar if link == "identity" else beta[0, p]
        G0, null_dev = allreduce(*D.glm_irls_pass(X, y, w, off, beta, family, link, 0, var_power, link_power))
        for k in range(1, K):
            null_dev += allreduce(*D.glm_irls_pass(X, y, w, off, beta, family, link, k, var_power, link_power))[1]
        lam_max = float(np.abs(G0[:p, p + 1]).max() / N / max(alpha, 1e-3)) if p > 0 else 0.0
        if lam_param is not None:
            lambdas = [float(v) for v in (lam_param if isinstance(lam_param, (list, tuple)) else [lam_param])]
        elif p_["lambda_search"]:
            nl = int(p_["nlambdas"]) if int(p_["nlambdas"]) > 0 else 100
            ratio = float(p_["lambda_min_ratio"]) if float(p_["lambda_min_ratio"]) > 0 else (1e-4 if N > p else 1e-2)
            lambdas = list(lam_max * ratio ** (np.arange(nl) / max(nl - 1, 1)))
        else:
            lambdas = [lam_max * 1e-3]
        iters_total = 0
        dev = null_dev
        history = []
        best = None
        lam_devs = []
        if solver == "L_BFGS":
            return self._fit_lbfgs(X, y, w, off, beta, family, link, var_power, link_power, N, null_dev, lam_max,
                                   lambdas, alpha, intercept, pen_std, design, model_id)
        force_cd = solver in ("COORDINATE_DESCENT", "COORDINATE_DESCENT_NAIVE")
        for lam in lambdas:
            for it in range(max_iter):
                iters_total += 1
                old = beta.copy()
                dev_k = 0.0
                for k in range(K):
                    G, dev = allreduce(*D.glm_irls_pass(X, y, w, off, beta, family, link, k, var_power, link_power))
                    dev_k += dev    # multinomial: pass k carries the rows of class k
                    beta[k] = solve_enet(G, p, N, lam, alpha, beta[k], intercept, bool(p_["non_negative"]),
                                         penalty=pen_std, force_cd=force_cd)
                dev = dev_k
                history.append({"iteration": iters_total, "lambda": lam, "deviance": dev})
                if np.abs(beta - old).max() < beps:
                    break
            if best is None or p_["lambda_search"]:
                best = (lam, beta.copy(), dev)
            if p_["lambda_search"]:
                # H2O-style early exit: the path stops once the last few lambdas no
                # longer reduce the deviance noticeably (relative to the null deviance)
                lam_devs.append(dev)
                if len(lam_devs) >= 4 and lam_devs[-4] - lam_devs[-1] < 1e-4 * max(null_dev, 1e-300):
                    break
        lam, beta, _ = best
        # final deviance at the chosen beta (multinomial: every class's pass)
        G, dev = allreduce(*D.glm_irls_pass(X, y, w, off, beta, family, link, 0, var_power, link_power))
        for k in range(1, K):
            dev += allreduce(*D.glm_irls_pass(X, y, w, off, beta, family, link, k, var_power, link_power))[1]
        stats = {"lambda": lam, "iterations": iters_total, "null_deviance": null_dev, "residual_deviance": dev,
                 "lambda_max": lam_max, "nobs": N, "solver": solver}
        k_active = int((np.abs(beta[:, :p]) > 0).sum()) + (K if intercept else 0)
        if family in ("binomial", "poisson", "multinomial"):
            stats["aic"] = dev + 2 * k_active
        if p_["compute_p_values"] and family != "multinomial" and lam == 0.0:
            stats.update(_p_values(G, p, family, dev, N, k_active, design, beta[0]))
        model = GLMModel(self, model_id, design, beta, family, link, stats)
        model.scoring_history = history
        return model


def _fit_lbfgs_impl(est, X, y, w, off, beta, family, link, var_power, link_power, N, null_dev, lam_max, lambdas,
                    alpha, intercept, pen_std, design, model_id):
    """solver=L_BFGS: OWL-QN over the gradient passes (glm_solvers.owlqn),
    warm-started along the lambda list; lambda_search keeps the last lambda
    (as the IRLSM path does)."""
    p_ = est.params
    comm = est.comm
    K, p1 = beta.shape
    p = p1 - 1
    pen_mask = np.zeros((K, p1), bool)
    pen_mask[:, :p] = True
    free = np.ones((K, p1), bool)
    if not intercept:
        beta[:, p] = 0.0
        free[:, p] = False
    fam_grad = "multinomial" if family == "multinomial" else family

    def fg_at(l2):
        def fg(bflat):
            B = bflat.reshape(K, p1)
            g, dv = D.glm_grad_pass(X, y, w, off, B, fam_grad, link, var_power, link_power)
            if comm is not None and comm.world_size > 1:
                arr = comm.all_reduce_numpy(np.concatenate([g.ravel(), [dv]]))
                g, dv = arr[:-1].reshape(K, p1), float(arr[-1])
            Bp = np.where(pen_mask, B, 0.0)
            fs = dv / (2 * N) + 0.5 * l2 * float((Bp * Bp).sum())
            grad = g / N + l2 * Bp
            if pen_std is not None:
                fs += 0.5 * float(B[0, :p] @ pen_std @ B[0, :p])
                grad[0, :p] += pen_std @ B[0, :p]
            grad = np.where(free, grad, 0.0)
            return fs, grad.ravel(), dv
        return fg

    max_iter = int(p_["max_iterations"]) if int(p_["max_iterations"]) > 0 else 500
    geps = float(p_["gradient_epsilon"]) if float(p_["gradient_epsilon"]) > 0 else 1e-6
    oeps = float(p_["objective_epsilon"]) if float(p_["objective_epsilon"]) > 0 else 1e-10
    history, best, iters = [], None, 0
    for lam in lambdas:
        res = owlqn(fg_at(lam * (1 - alpha)), beta.ravel(), pen_mask.ravel(), lam * alpha, max_iter=max_iter,
                    grad_eps=geps, obj_eps=oeps, non_negative=bool(p_["non_negative"]))
        beta = res.beta.reshape(K, p1)
        iters += res.iters
        history.append({"iteration": iters, "lambda": lam, "deviance": res.dev, "objective": res.f,
                        "function_evaluations": res.evals, "converged": res.converged,
                        "stop_reason": res.stop_reason})
        best = (lam, beta.copy(), res.dev, res)
    lam, beta, dev, last = best
    stats = {"lambda": lam, "iterations": iters, "null_deviance": null_dev, "residual_deviance": dev,
             "lambda_max": lam_max, "nobs": N, "solver": "L_BFGS", "converged": bool(last.converged),
             "stop_reason": last.stop_reason}
    k_active = int((np.abs(beta[:, :p]) > 0).sum()) + (K if intercept else 0)
    if family in ("binomial", "poisson", "multinomial"):
        stats["aic"] = dev + 2 * k_active
    if p_["compute_p_values"] and family != "multinomial" and lam == 0.0:
        G, _ = D.glm_irls_pass(X, y, w, off, beta, family, link, 0, var_power, link_power)
        if comm is not None and comm.world_size > 1:
            G = comm.all_reduce_numpy(G)
        stats.update(_p_values(G, p, family, dev, N, k_active, design, beta[0]))
    model = GLMModel(est, model_id, design, beta, family, link, stats)
    model.scoring_history = history
    return model


def _fit_ordinal_impl(est, X, y, w, N, design, lam_param, alpha, model_id):
    from .glm_extras import fit_ordinal

    K = len(est.response_domain)
    lam = 0.0 if lam_param is None else float(lam_param[0] if isinstance(lam_param, (list, tuple)) else lam_param)
    b, th, nll, nit = fit_ordinal(X, y, w, K, lam, alpha, est.comm,
                                  max_iter=int(est.params["max_iterations"]) if int(est.params["max_iterations"]) > 0
                                  else 200)
    p = X.shape[0]
    beta = np.zeros((1, p + 1))
    beta[0, :p] = b
    wd = w.double() if w is not None else torch.ones(y.numel(), dtype=torch.float64, device=y.device)
    cnt = torch.bincount(y.long(), weights=wd, minlength=K).double()
    if est.comm is not None and est.comm.world_size > 1:
        est.comm.all_reduce_(cnt)
    pr = (cnt / cnt.sum()).clamp_min(1e-15)
    null_dev = float(-2 * (cnt * torch.log(pr)).sum())
    stats = {"lambda": lam, "iterations": nit, "null_deviance": null_dev, "residual_deviance": 2 * nll,
             "lambda_max": 0.0, "nobs": N, "ordinal_thresholds": th.tolist(),
             "aic": 2 * nll + 2 * (p + K - 1)}
    return GLMModel(est, model_id, design, beta, "ordinal", "ologit", stats)


def _p_values(G, p, family, dev, N, k_active, design, beta_std):
    from scipy import stats as sst

    A = G[: p + 1, : p + 1]
    try:
        inv = np.linalg.inv(A)
    except np.linalg.LinAlgError:
        return {"std_errors": None}
    disp = 1.0 if family in ("binomial", "poisson") else dev / max(N - k_active, 1)
    se_std = np.sqrt(np.maximum(np.diag(inv) * disp, 0))
    # report in raw scale: se_raw_j = se_std_j / sd_j (intercept approximated by its std-space value)
    se = np.concatenate([[se_std[p]], se_std[:p] / design.sds])
    z = np.concatenate([[beta_std[p]], beta_std[:p]]) / np.maximum(np.concatenate([[se_std[p]], se_std[:p]]), 1e-300)
    if family in ("binomial", "poisson"):
        pv = 2 * sst.norm.sf(np.abs(z))
    else:
        pv = 2 * sst.t.sf(np.abs(z), df=max(N - k_active, 1))
    return {"std_errors": se.tolist(), "z_values": z.tolist(), "p_values": pv.tolist()}
