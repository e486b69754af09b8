"""One fp32 DeepLearning training step on the GPU against autograd.

The reference is the same update computed by torch autograd in float64 on the
CPU (forward, softmax cross-entropy / squared loss averaged over the batch,
backward) followed by H2O's ADADELTA (``reference/dense.py adadelta_``).
Both GPU paths of ``models/deeplearning._DLTrainer`` are pinned:

* the fused small-batch chain (``ops/mlp.py`` / ``csrc/mlp_kernels.hip``:
  forward, loss gradient, backward and ADADELTA in 2 L - 1 launches);
* the per-op path (GEMM kernels, fused activation backward, the bias /
  output-layer gradient folds inside the ADADELTA kernel).

Gradients, updated weights and both ADADELTA accumulators must match at
rtol 1e-4 (fp32 MFMA accumulation vs float64)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [
    # sizes, act (1 relu, 2 tanh), M, regression, l2
    ([200, 512, 512, 512, 512, 2], 1, 256, False, 0.0),     # estimator-default shape of the DL bench
    ([37, 48, 40, 3], 2, 50, False, 1e-4),                  # ragged dims, tanh, 3 classes, L2
    ([21, 64, 1], 1, 100, True, 0.0),                       # one hidden layer (ADADELTA tail launch), regression
    ([16, 32, 32, 8], 1, 7, False, 0.0),                    # 8 classes, a batch smaller than one MFMA block
]


def _reference(sizes, act, W0, X, y, regression, rho, eps, l2, Eg2_0, Edx2_0, layers):
    """float64 autograd step: returns (grad, new flat, Eg2, Edx2)."""
    flat = torch.from_numpy(W0).double().requires_grad_(True)
    H = torch.from_numpy(X).double()
    L = len(layers)
    for i, (off, w, f) in enumerate(layers):
        Wl = flat[off: off + w * f].view(w, f)
        bl = flat[off + w * f: off + w * f + w]
        Z = H @ Wl.T + bl
        if i < L - 1:
            H = torch.relu(Z) if act == 1 else torch.tanh(Z)
        else:
            H = Z
    if regression:
        loss = 0.5 * ((H[:, 0] - torch.from_numpy(y).double()) ** 2).mean()
    else:
        loss = torch.nn.functional.cross_entropy(H, torch.from_numpy(y).long())
    loss.backward()
    G = flat.grad.detach().clone()
    Wn = flat.detach().clone()
    g = G + l2 * Wn
    Eg2 = rho * torch.from_numpy(Eg2_0).double() + (1 - rho) * g * g
    Edx2 = torch.from_numpy(Edx2_0).double()
    dx = -torch.sqrt(Edx2 + eps) / torch.sqrt(Eg2 + eps) * g
    Edx2 = rho * Edx2 + (1 - rho) * dx * dx
    return G.numpy(), (Wn + dx).numpy(), Eg2.numpy(), Edx2.numpy()


def _close(name, got, want, rtol=1e-4):
    scale = np.abs(want).max() + 1e-30
    err = np.abs(got - want) / (np.abs(want) + 1e-3 * scale)
    assert err.max() <= rtol, f"{name}: max rel err {err.max():.3g} at {int(err.argmax())}"


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_one_training_step_matches_autograd(case, fused, monkeypatch):
    from h2omx.models.deeplearning import H2ODeepLearningEstimator, _DLTrainer, _Net

    sizes, act, M, regression, l2 = CASES[case]
    monkeypatch.setattr(_DLTrainer, "FUSED", fused)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(case)
    X = rng.normal(size=(M * 3, sizes[0])).astype(np.float32)
    y = (rng.normal(size=M * 3).astype(np.float32) if regression
         else rng.integers(0, sizes[-1], size=M * 3).astype(np.int32))
    gen = torch.Generator().manual_seed(case)
    net = _Net(sizes, act, dev, gen)
    p = dict(H2ODeepLearningEstimator.DEFAULTS)
    p.update(l2=l2, loss="Automatic")
    Xd = torch.from_numpy(X).to(dev)
    Yd = torch.from_numpy(y).to(dev)
    tr = _DLTrainer(p, net, Xd, Yd, act, not regression, False, 0.0, [0.0] * 8, M, 3, None,
                    torch.Generator().manual_seed(1), None, len(sizes) - 2, backward=H2ODeepLearningEstimator._backward)
    assert (tr.fused is not None) == fused
    # non-trivial ADADELTA state (as after a few steps)
    P = net.flat.numel()
    Eg2_0 = (rng.random(P) * 1e-4).astype(np.float32)
    Edx2_0 = (rng.random(P) * 1e-6).astype(np.float32)
    tr.Eg2.copy_(torch.from_numpy(Eg2_0))
    tr.Edx2.copy_(torch.from_numpy(Edx2_0))
    W0 = net.flat.cpu().numpy().copy()
    idx = torch.arange(M, 2 * M, device=dev)
    tr._body(idx)
    torch.cuda.synchronize()
    G, Wn, E1, E2 = _reference(sizes, act, W0, X[M:2 * M], y[M:2 * M], regression, float(p["rho"]),
                               float(p["epsilon"]), l2, Eg2_0, Edx2_0, net.layers)
    _close("grad", net.grad.cpu().numpy(), G)
    _close("weights", net.flat.cpu().numpy(), Wn)
    _close("Eg2", tr.Eg2.cpu().numpy(), E1)
    _close("Edx2", tr.Edx2.cpu().numpy(), E2)


def test_fused_chain_is_the_estimator_default_path():
    """The estimator's defaults (Rectifier, ADADELTA, 256-row batches) train on the
    fused chain: 2 L - 1 launches per update (L = 3 layers here)."""
    from h2omx.frame import Frame
    from h2omx.models import H2ODeepLearningEstimator
    from h2omx.frame.synthetic import higgs_like

    dev = torch.device("cuda", 0)
    X, y = higgs_like(40000, seed=3, device=dev)
    fr = Frame.from_tensor(X.contiguous(), y=y, y_categorical=True)
    est = H2ODeepLearningEstimator(hidden=[64, 64], epochs=1, seed=1)
    m = est.train(y="response", training_frame=fr)
    tr = getattr(est, "_last_trainer", None)
    assert tr is not None and tr.fused is not None and tr.fused.launches == 5
    assert m.training_metrics["AUC"] > 0.7
