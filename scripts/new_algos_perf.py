"""Timing of the newer estimators on the GPU (uplift DRF, PSVM, infogram)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from h2omx.frame.frame import ENUM, Frame, Vec  # noqa: E402
from h2omx.models import (H2OInfogram, H2OSupportVectorMachineEstimator,  # noqa: E402
                          H2OUpliftRandomForestEstimator)

dev = torch.device("cuda", 0)
out = {}
g = torch.Generator(device=dev).manual_seed(0)
n, F = 1_000_000, 20
X = torch.randn((F, n), generator=g, device=dev)
t = (torch.rand(n, generator=g, device=dev) < 0.5)
p = (0.3 + 0.1 * X[1].clamp(-2, 2) + t * torch.where(X[0] > 0, 0.2, -0.05)).clamp(0.02, 0.98)
y = (torch.rand(n, generator=g, device=dev) < p).int()
fr = Frame([Vec(f"x{i}", X[i], "real") for i in range(F)] + [Vec("trt", t.int(), ENUM, ["c", "t"]),
                                                              Vec("y", y, ENUM, ["0", "1"])])
for trees, depth in ((1, 10), (10, 10)):
    torch.cuda.synchronize()
    t0 = time.time()
    m = H2OUpliftRandomForestEstimator(ntrees=trees, max_depth=depth, treatment_column="trt", seed=1).train(
        y="y", training_frame=fr)
    torch.cuda.synchronize()
    out[f"uplift_1Mx20_{trees}trees_d{depth}_s"] = time.time() - t0
out["uplift_auuc"] = m.training_metrics["auuc"]
print(json.dumps(out), flush=True)
ns = 50_000
Xs = torch.randn((2, ns), generator=g, device=dev)
ys = ((Xs ** 2).sum(0) < 1.4).int()
frs = Frame([Vec("a", Xs[0], "real"), Vec("b", Xs[1], "real"), Vec("y", ys, ENUM, ["0", "1"])])
torch.cuda.synchronize()
t0 = time.time()
sv = H2OSupportVectorMachineEstimator(gamma=0.5).train(y="y", training_frame=frs)
torch.cuda.synchronize()
out["psvm_50k_s"] = time.time() - t0
out["psvm_nsv"] = int(sv.sv.shape[0])
out["psvm_timings"] = sv.timings
t0 = time.time()
P = sv.predict(frs)
torch.cuda.synchronize()
out["psvm_score_50k_s"] = time.time() - t0
out["psvm_acc"] = float((P.vec("predict").data == ys).float().mean())
print(json.dumps(out), flush=True)
t0 = time.time()
ig = H2OInfogram(algorithm_params=dict(ntrees=20, max_depth=4), seed=1).train(
    x=[f"x{i}" for i in range(F)], y="y", training_frame=fr)
torch.cuda.synchronize()
out["infogram_1Mx20_s"] = time.time() - t0
out["infogram_admissible"] = ig.get_admissible_features()
print(json.dumps(out), flush=True)
