"""PSVM (ICF + interior point) against scikit-learn's exact SVC on a
non-linearly separable problem: same decision function, support vectors and
accuracy; GPU scoring path."""
import numpy as np
import pytest
import torch

from h2omx.frame.frame import ENUM, Frame, Vec
from h2omx.models import H2OSupportVectorMachineEstimator
from h2omx.models.psvm import icf


def _frame(n=2000, device="cpu"):
    g = torch.Generator().manual_seed(0)
    X = torch.randn((2, n), generator=g)
    y = ((X ** 2).sum(0) < 1.4).int()
    return Frame([Vec("a", X[0].to(device), "real"), Vec("b", X[1].to(device), "real"),
                  Vec("y", y.to(device), ENUM, ["0", "1"])]), X, y


def test_psvm_matches_sklearn_svc():
    from sklearn.svm import SVC

    fr, X, y = _frame()
    m = H2OSupportVectorMachineEstimator(gamma=0.5, hyper_param=1.0).train(y="y", training_frame=fr)
    ref = SVC(C=1.0, gamma=0.5).fit(X.T.numpy(), y.numpy())
    f = m.decision_function(fr).numpy()
    fs = ref.decision_function(X.T.numpy())
    assert np.corrcoef(f, fs)[0, 1] > 0.9999
    assert np.abs(f - fs).max() < 0.05 * np.abs(fs).max()        # rank-sqrt(n) ICF vs the exact kernel
    assert (np.sign(f) == np.sign(fs)).mean() > 0.995
    assert abs(m.sv.shape[0] - ref.n_support_.sum()) <= 0.02 * ref.n_support_.sum() + 2
    P = m.predict(fr)
    assert P.names == ["predict", "decision_function"]
    assert float((P.vec("predict").data == y).float().mean()) > 0.99


def test_icf_reconstructs_kernel():
    g = torch.Generator().manual_seed(1)
    X = torch.randn((300, 3), generator=g, dtype=torch.float64)
    H = icf(X, 0.3, 300, 1e-10)
    K = torch.exp(-0.3 * torch.cdist(X, X) ** 2)
    assert float((H @ H.T - K).abs().max()) < 1e-6


@pytest.mark.gpu
def test_psvm_gpu_matches_cpu(cuda_dev):
    fr, _, _ = _frame(1500)
    frg, _, _ = _frame(1500, device=cuda_dev)
    a = H2OSupportVectorMachineEstimator(gamma=0.5).train(y="y", training_frame=fr).decision_function(fr)
    b = H2OSupportVectorMachineEstimator(gamma=0.5).train(y="y", training_frame=frg).decision_function(frg)
    np.testing.assert_allclose(b.cpu().numpy(), a.numpy(), atol=2e-3)
