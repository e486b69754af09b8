"""K-Means clustering (H2O KMeans equivalent).

Lloyd iterations run one fused HIP pass each (csrc/dense_kernels.hip
kmeans_kernel): distances on the fp32 matrix cores, arg-min in registers,
per-workgroup cluster sums / counts / SSE without atomics, then one small
all-reduce of the [k][d] sums per iteration across ranks (SURVEY.md §2.5
K12/K13, collective C5).  Initialisation: Furthest (H2O default),
PlusPlus, Random or User points; categorical columns are one-hot encoded.
"""
from __future__ import annotations

import numpy as np
import torch

from ..frame.frame import ENUM, Frame
from ..backend import dense as D
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo


class KMeansModel(Model):
    algo = "kmeans"
    algo_full_name = "K-means"

    def __init__(self, builder, model_id, design, centers_std, stats):
        super().__init__(builder, model_id)
        self.design = design
        self.centers_std = centers_std          # [k][d] standardized
        self.centers = centers_std * design.sds[None, :] + design.center[None, :]
        self.stats = stats

    def _X(self, frame):
        return self.design.transform(self.design.raw_matrix(frame))

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        X = self._X(frame)
        a, _, _, _ = D.kmeans_step(X, self.centers_std.astype(np.float32), na_free=True)
        return a.to(X.device).float()[None, :]

    def model_performance(self, frame: Frame | None = None):
        if frame is None:
            return self.training_metrics
        X = self._X(frame)
        _, _, cnt, sse = D.kmeans_step(X, self.centers_std.astype(np.float32), na_free=True)
        totss = float((X.double() - X.double().mean(1, keepdim=True)).pow(2).sum())
        return {"tot_withinss": float(sse.sum()), "totss": totss, "betweenss": totss - float(sse.sum()),
                "size": cnt.tolist(), "withinss": sse.tolist()}

    def summary(self):
        return {"model_id": self.model_id, "number_of_clusters": int(self.centers.shape[0]),
                "number_of_iterations": self.stats["iterations"], "within_cluster_sum_of_squares": self.stats["tot_withinss"],
                "total_sum_of_squares": self.stats["totss"], "between_cluster_sum_of_squares": self.stats["betweenss"]}

    def to_json(self):
        j = super().to_json()
        out = j["output"]
        out["centers"] = {"names": self.design.names, "data": self.centers.tolist()}
        out["centers_std"] = {"names": self.design.names, "data": self.centers_std.tolist()}
        out["training_metrics"] = {k: v for k, v in self.stats.items()}
        return j


class H2OKMeansEstimator(ModelBuilder):
    algo = "kmeans"
    DEFAULTS = dict(k=1, max_iterations=10, standardize=True, init="Furthest", user_points=None,
                    estimate_k=False, cluster_size_constraints=None, categorical_encoding="AUTO")

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        k = int(p_["k"])
        comm = self.comm
        design = DesignInfo(self.x, self.feature_types, self.feature_domains, use_all_levels=True)
        Xraw = design.raw_matrix(train)
        design.fit_standardization(Xraw, bool(p_["standardize"]), comm)
        X = design.transform(Xraw)
        del Xraw
        d, n = X.shape
        g = torch.Generator().manual_seed(self._seed())
        if p_.get("estimate_k") and p_.get("user_points") is None:
            C = self._estimate_k(X, k, str(p_["init"]).lower(), g, design)
            k = C.shape[0]
        else:
            C = self._init(X, k, str(p_["init"]).lower(), g, design)
        it = 0
        prev = None
        stats = {}
        for it in range(1, int(p_["max_iterations"]) + 1):
            assign, sums, cnt, sse = D.kmeans_step(X, C.astype(np.float32), na_free=True)
            if comm is not None and comm.world_size > 1:
                red = comm.all_reduce_numpy(np.concatenate([sums.ravel(), cnt, sse]))
                sums, cnt, sse = red[: k * d].reshape(k, d), red[k * d: k * d + k], red[k * d + k:]
            newC = C.copy()
            nz = cnt > 0
            newC[nz] = sums[nz] / cnt[nz, None]
            if (~nz).any():  # re-seed empty clusters at the farthest points
                far = self._farthest(X, C, int((~nz).sum()))
                newC[~nz] = far
            changed = None if prev is None else int((assign != prev).sum().item())
            if comm is not None and comm.world_size > 1 and changed is not None:
                changed = int(comm.all_reduce_numpy(np.array([float(changed)]))[0])
            prev = assign
            C = newC
            stats = {"tot_withinss": float(sse.sum()), "withinss": sse.tolist(), "size": cnt.tolist()}
            if changed == 0:
                break
        # final statistics at the converged centers
        assign, sums, cnt, sse = D.kmeans_step(X, C.astype(np.float32), na_free=True)
        tot = torch.stack([X.double().sum(1), X.double().pow(2).sum(1)])
        nn = float(n)
        if comm is not None and comm.world_size > 1:
            red = comm.all_reduce_numpy(np.concatenate([cnt, sse, tot.cpu().numpy().ravel(), [nn]]))
            cnt, sse = red[:k], red[k:2 * k]
            tot = torch.from_numpy(red[2 * k: 2 * k + 2 * d].reshape(2, d))
            nn = red[-1]
        totss = float((tot[1] - tot[0] ** 2 / nn).sum())
        stats = {"iterations": it, "tot_withinss": float(sse.sum()), "withinss": sse.tolist(), "size": cnt.tolist(),
                 "totss": totss, "betweenss": totss - float(sse.sum())}
        model = KMeansModel(self, model_id, design, C, stats)
        model.training_metrics = stats
        return model

    # estimate_k: stop adding centers once the proportional reduction in the
    # within-cluster sum of squares falls below this (H2O's PRE rule; the
    # threshold is unpinned: the reference holds no estimate_k output, see
    # docs/PARITY.md)
    PRE_MIN = 0.1

    def _estimate_k(self, X, kmax, how, g, design):
        """H2O ``estimate_k``: grow k from 1 up to ``k`` (the maximum), each step
        seeding the new center at the point farthest from the current centers
        and running Lloyd iterations; keep the last k whose step still reduced
        the total within-cluster SS by at least PRE_MIN."""
        comm = self.comm
        C = self._init(X, 1, how, g, design)
        prev_ss, best = None, C
        for kk in range(1, kmax + 1):
            if kk > 1:
                far, dist2 = self._farthest(X, C, 1, with_dist=True)
                if comm is not None and comm.world_size > 1:
                    # the GLOBAL farthest point: every rank offers its local candidate
                    # and distance; the largest distance wins (lowest rank on a tie)
                    cands = comm.all_gather_object((float(dist2[0]), comm.rank, far[0].tolist()))
                    best_c = max(cands, key=lambda c: (c[0], -c[1]))
                    far = np.asarray([best_c[2]], np.float64)
                C = np.concatenate([C, far])
            for _ in range(int(self.params["max_iterations"])):
                assign, sums, cnt, sse = D.kmeans_step(X, C.astype(np.float32), na_free=True)
                if comm is not None and comm.world_size > 1:
                    red = comm.all_reduce_numpy(np.concatenate([sums.ravel(), cnt, sse]))
                    d = X.shape[0]
                    sums, cnt, sse = red[: kk * d].reshape(kk, d), red[kk * d: kk * d + kk], red[kk * d + kk:]
                nz = cnt > 0
                newC = C.copy()
                newC[nz] = sums[nz] / cnt[nz, None]
                if np.allclose(newC, C, rtol=0, atol=1e-9):
                    C = newC
                    break
                C = newC
            ss = float(sse.sum())
            if prev_ss is not None and (prev_ss <= 0 or (prev_ss - ss) / prev_ss < self.PRE_MIN):
                break
            best, prev_ss = C.copy(), ss
        return best

    def _init(self, X, k, how, g, design):
        d, n = X.shape
        up = self.params.get("user_points")
        if up is not None:
            pts = np.asarray(up.to_pandas().values if isinstance(up, Frame) else up, np.float64)[:k]
            return (pts - design.center[None, :]) / design.sds[None, :]
        if how == "random":
            idx = torch.randint(0, n, (k,), generator=g)
            return X[:, idx.to(X.device)].T.double().cpu().numpy()
        first = int(torch.randint(0, n, (1,), generator=g))
        C = [X[:, first].double().cpu().numpy()]
        mind = ((X.double() - torch.from_numpy(C[0]).to(X.device)[:, None]) ** 2).sum(0)
        for _ in range(1, k):
            if how == "plusplus":
                pr = (mind / mind.sum()).cpu()
                j = int(torch.multinomial(pr.float(), 1, generator=g))
            else:  # furthest
                j = int(torch.argmax(mind))
            c = X[:, j].double()
            C.append(c.cpu().numpy())
            mind = torch.minimum(mind, ((X.double() - c[:, None]) ** 2).sum(0))
        return np.stack(C)

    def _farthest(self, X, C, m, with_dist: bool = False):
        Ct = torch.from_numpy(C).to(X.device)
        d2 = (X.double().pow(2).sum(0)[None, :] - 2 * Ct @ X.double() + Ct.pow(2).sum(1)[:, None]).min(0).values
        top = torch.topk(d2, m)
        pts = X[:, top.indices].T.double().cpu().numpy()
        return (pts, top.values.cpu().numpy()) if with_dist else pts

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        return super().train(x=x, y=None, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)
