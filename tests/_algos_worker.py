"""Worker for tests/test_algos_multirank.py: one rank of a gloo world holding
a row shard; trains the newer estimators and writes their key outputs (JSON)."""
import json
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.distributed import unify_domains  # noqa: E402
from h2omx.models import (H2OANOVAGLMEstimator, H2OCoxProportionalHazardsEstimator,  # noqa: E402
                          H2OGeneralizedAdditiveEstimator, H2OGeneralizedLowRankEstimator,
                          H2OIsotonicRegressionEstimator, H2OModelSelectionEstimator,
                          H2OSingularValueDecompositionEstimator, H2OTargetEncoderEstimator,
                          H2OHGLMEstimator, H2OSupportVectorMachineEstimator,
                          H2OUpliftRandomForestEstimator)
from h2omx.parallel.comm import Comm  # noqa: E402


def data(n=1200):
    rng = np.random.default_rng(11)
    X = rng.normal(size=(n, 4))
    df = pd.DataFrame(X, columns=["a", "b", "c", "d"])
    df["g"] = pd.Categorical(rng.choice(list("pqrs"), n))
    df["y"] = np.sin(X[:, 0]) + X[:, 1] - 0.5 * X[:, 2] + rng.normal(scale=0.3, size=n)
    df["t"] = np.ceil(rng.exponential(np.exp(-0.5 * X[:, 0])) * 10) / 10
    df["ev"] = (rng.random(n) < 0.7).astype(float)
    trt = rng.random(n) < 0.5
    df["trt"] = pd.Categorical(np.where(trt, "treatment", "control"), categories=["control", "treatment"])
    p = np.clip(0.3 + 0.1 * X[:, 1] + trt * np.where(X[:, 0] > 0, 0.3, -0.1), 0.02, 0.98)
    df["yb"] = pd.Categorical(np.where(rng.random(n) < p, "1", "0"), categories=["0", "1"])
    return df


def main():
    out_path = sys.argv[1]
    device = os.environ.get("H2OMX_WORKER_DEVICE", "cpu")    # "cuda": ranks share the GPU over gloo
    comm = Comm.from_env(device=device)
    c = comm if comm.world_size > 1 else None
    df = data()
    n = len(df)
    lo, hi = n * comm.rank // comm.world_size, n * (comm.rank + 1) // comm.world_size
    fr = unify_domains(Frame.from_pandas(df.iloc[lo:hi].reset_index(drop=True), device=comm.device), c)
    res = {}
    te = H2OTargetEncoderEstimator(noise=0.0, blending=True).train(x=["g"], y="y", training_frame=fr, comm=c)
    res["te"] = te.transform(fr).to_pandas()["g_te"].tolist()
    svd = H2OSingularValueDecompositionEstimator(nv=3).train(x=["a", "b", "c", "d"], training_frame=fr, comm=c)
    res["svd_d"] = svd.d.tolist()
    gl = H2OGeneralizedLowRankEstimator(k=2, init="SVD", max_iterations=30, min_step_size=0.0).train(
        x=["a", "b", "c", "d"], training_frame=fr, comm=c)
    res["glrm_obj"] = gl.objective
    iso = H2OIsotonicRegressionEstimator().train(x=["a"], y="y", training_frame=fr, comm=c)
    res["iso"] = [iso.thresholds_x.tolist(), iso.thresholds_y.tolist()]
    cox = H2OCoxProportionalHazardsEstimator(stop_column="t").train(x=["a", "b"], y="ev", training_frame=fr, comm=c)
    res["cox"] = cox.beta.tolist()
    ms = H2OModelSelectionEstimator(mode="maxr", max_predictor_number=2).train(
        x=["a", "b", "c", "d"], y="y", training_frame=fr, comm=c)
    res["ms"] = [[r["predictors"], r["best_r2_value"]] for r in ms.result()]
    gam = H2OGeneralizedAdditiveEstimator(family="gaussian", gam_columns=["a"], num_knots=[6], lambda_=0.0).train(
        x=["a", "b", "c"], y="y", training_frame=fr, comm=c)
    res["gam"] = gam.coef()
    an = H2OANOVAGLMEstimator(family="gaussian", highest_interaction_term=1).train(
        x=["a", "b", "d"], y="y", training_frame=fr, comm=c)
    res["anova"] = [r["deviance_difference"] for r in an.result()]
    up = H2OUpliftRandomForestEstimator(ntrees=3, max_depth=4, sample_rate=1.0, treatment_column="trt", seed=3).train(
        x=["a", "b", "c"], y="yb", training_frame=fr, comm=c)
    res["uplift"] = up.predict(fr).to_pandas()["uplift_predict"].tolist()
    res["auuc"] = up.training_metrics["auuc"]
    sv = H2OSupportVectorMachineEstimator(gamma=0.5).train(x=["a", "b"], y="yb", training_frame=fr, comm=c)
    res["svm"] = sv.decision_function(fr).tolist()
    hg = H2OHGLMEstimator(group_column="g", random_columns=["b"]).train(x=["a", "b"], y="y", training_frame=fr,
                                                                      comm=c)
    res["hglm"] = list(hg.coef().values()) + [hg.sigma2] + hg.T.ravel().tolist()
    from h2omx.frame.tools import interaction

    ia = interaction(fr, ["g", "trt"], max_factors=5, comm=c).vecs[0]
    res["inter"] = [ia.domain[i] if i >= 0 else None for i in ia.data.tolist()]
    # calibration on a row-sharded calibration frame: Platt's Newton steps and the
    # isotonic PAV fit see the whole frame (all-reduce / all-gather), and the
    # laplace / quantile initial margins are the weighted quantiles over all ranks
    from h2omx.models import H2OGradientBoostingEstimator, H2OKMeansEstimator

    for meth in ("PlattScaling", "IsotonicRegression"):
        gb = H2OGradientBoostingEstimator(ntrees=3, max_depth=3, seed=1, calibrate_model=True, calibration_frame=fr,
                                          calibration_method=meth).train(x=["a", "b", "c"], y="yb",
                                                                         training_frame=fr, comm=c)
        cal = gb.calibration
        res[f"cal_{meth}"] = ([cal["intercept"], cal["slope"]] if meth == "PlattScaling"
                              else [cal["x"], cal["y"], cal["x_min"]])
    for dist in ("laplace", "quantile"):
        gq = H2OGradientBoostingEstimator(ntrees=2, max_depth=2, seed=1, distribution=dist, quantile_alpha=0.3).train(
            x=["a", "b"], y="y", training_frame=fr, comm=c)
        res[f"init_{dist}"] = float(gq.ens.init_f[0])
    km = H2OKMeansEstimator(k=6, estimate_k=True, standardize=True, seed=4, max_iterations=20).train(
        x=["a", "b", "c"], training_frame=fr, comm=c)
    res["km_k"] = int(km.centers.shape[0])
    with open(out_path, "w") as f:
        json.dump(res, f)
    comm.barrier()


if __name__ == "__main__":
    main()
