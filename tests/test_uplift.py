"""Uplift DRF: recovers a known heterogeneous treatment effect, H2O's output
columns and metrics, divergence formulas, and AUUC ordering (a perfect
ranking beats a random one)."""
import numpy as np
import pytest
import torch

from h2omx.frame.frame import ENUM, Frame, Vec
from h2omx.models import H2OUpliftRandomForestEstimator
from h2omx.models.uplift import divergence, uplift_metrics


def _data(n=20000, seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn((4, n), generator=g)
    t = (torch.rand(n, generator=g) < 0.5).float()
    eff = torch.where(X[0] > 0, 0.3, -0.1)
    p = (torch.sigmoid(X[1] * 0.5) * 0.6 + t * eff).clamp(0.02, 0.98)
    y = (torch.rand(n, generator=g) < p).int()
    vecs = [Vec(f"x{i}", X[i].to(device), "real") for i in range(4)]
    vecs += [Vec("treatment", t.int().to(device), ENUM, ["control", "treatment"]),
             Vec("y", y.to(device), ENUM, ["0", "1"])]
    return Frame(vecs), eff


def _check(fr, eff, metric="AUTO"):
    m = H2OUpliftRandomForestEstimator(ntrees=8, max_depth=5, seed=1, treatment_column="treatment",
                                       uplift_metric=metric).train(y="y", training_frame=fr)
    P = m.predict(fr)
    assert P.names == ["uplift_predict", "p_y1_with_treatment", "p_y1_without_treatment"]
    up = P.vec("uplift_predict").data.cpu().numpy()
    np.testing.assert_allclose(up, P.vec("p_y1_with_treatment").data.cpu().numpy()
                               - P.vec("p_y1_without_treatment").data.cpu().numpy(), atol=1e-6)
    assert np.corrcoef(up, eff.numpy())[0, 1] > 0.9
    tm = m.training_metrics
    assert abs(tm["ate"] - 0.1) < 0.03
    assert tm["qini"] > 0 and tm["auuc"] > 0
    assert "x0" in [v[0] for v in m.varimp()[:2]]     # ChiSquared also rewards splits that move q
    assert m.category == "BinomialUplift"
    return m


@pytest.mark.parametrize("metric", ["KL", "Euclidean", "ChiSquared"])
def test_uplift_recovers_effect(metric):
    fr, eff = _data()
    _check(fr, eff, metric)


def test_divergences():
    p, q = torch.tensor([0.3, 0.5]), torch.tensor([0.1, 0.5])
    kl = divergence(p, q, "KL")
    ref = p * torch.log(p / q) + (1 - p) * torch.log((1 - p) / (1 - q))
    torch.testing.assert_close(kl, ref)
    torch.testing.assert_close(divergence(p, q, "Euclidean"), 2 * (p - q) ** 2)
    torch.testing.assert_close(divergence(p, q, "ChiSquared"), (p - q) ** 2 / q + (p - q) ** 2 / (1 - q))
    assert float(kl[1]) == 0.0


def test_auuc_ranks_perfect_above_random():
    g = torch.Generator().manual_seed(3)
    n = 40000
    t = (torch.rand(n, generator=g) < 0.5).double()
    tau = torch.rand(n, generator=g) * 0.6 - 0.2
    y = (torch.rand(n, generator=g) < (0.3 + t * tau).clamp(0, 1)).double()
    good = uplift_metrics(tau, y, t, 100)
    rand = uplift_metrics(torch.rand(n, generator=g), y, t, 100)
    assert good["auuc"] > rand["auuc"] + 100
    assert good["qini"] > 0 > rand["qini"] - 200
    assert {"qini", "lift", "gain"} == set(good["auuc_table"])
    assert len(good["thresholds_and_metric_scores"]) <= 100


def test_uplift_requires_treatment_column():
    fr, _ = _data(500)
    with pytest.raises(ValueError):
        H2OUpliftRandomForestEstimator(treatment_column="nope", ntrees=1).train(y="y", training_frame=fr)


@pytest.mark.gpu
def test_uplift_gpu_matches_cpu(cuda_dev):
    fr, eff = _data(8000)
    frg, _ = _data(8000, device=cuda_dev)
    kw = dict(ntrees=3, max_depth=4, seed=1, treatment_column="treatment", sample_rate=1.0)
    a = H2OUpliftRandomForestEstimator(**kw).train(y="y", training_frame=fr).predict(fr)
    b = H2OUpliftRandomForestEstimator(**kw).train(y="y", training_frame=frg).predict(frg)
    np.testing.assert_allclose(b.vec("uplift_predict").data.cpu().numpy(), a.vec("uplift_predict").data.numpy(),
                               atol=1e-5)
