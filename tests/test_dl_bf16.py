"""bf16 MLP path (ops.dense.gemm_bf16_nt / cvt_bf16 / rowsum_bf16 and
models.deeplearning._Bf16Mlp): CPU contract vs fp32 autograd, HIP kernels vs
the CPU contract on the same bf16 operands."""
import numpy as np
import pytest
import torch

from h2omx.models.deeplearning import _Bf16Mlp, _Net
from h2omx.backend import dense as D


def _net(sizes, act, dev, seed=0):
    return _Net(sizes, act, dev, torch.Generator().manual_seed(seed))


def _autograd_grads(net, X, y, act):
    """fp32 reference gradients of mean softmax cross-entropy."""
    Ws = [net.W(i).detach().clone().requires_grad_(True) for i in range(len(net.layers))]
    bs = [net.b(i).detach().clone().requires_grad_(True) for i in range(len(net.layers))]
    H = X
    for i in range(len(Ws)):
        Z = H @ Ws[i].T + bs[i]
        H = Z if i == len(Ws) - 1 else (torch.relu(Z) if act == 1 else torch.tanh(Z))
    loss = torch.nn.functional.cross_entropy(H, y.long())
    loss.backward()
    return [w.grad for w in Ws], [b.grad for b in bs], H.detach()


@pytest.mark.parametrize("act", [1, 2])
def test_bf16_mlp_cpu_contract_matches_fp32_autograd(act):
    torch.manual_seed(0)
    sizes = [20, 48, 24, 3]
    B = 64
    net = _net(sizes, act, "cpu")
    X = torch.randn(B, sizes[0])
    y = torch.randint(0, 3, (B,), dtype=torch.int32)
    m = _Bf16Mlp(net, act, B, "cpu")
    xb, xbt = m.load_batch(X)
    Z = m.forward(xb)
    dZ, _ = D.softmax_xent(Z.clone(), y)
    net.grad.zero_()
    m.backward(dZ, xbt)
    gW, gb, Zref = _autograd_grads(net, X, y, act)
    np.testing.assert_allclose(Z.numpy(), Zref.numpy(), rtol=0.05, atol=0.05)
    for i in range(len(sizes) - 1):
        a, r = net.W(i, net.grad), gW[i]
        assert float((a - r).norm() / r.norm()) < 0.05, i
        a, r = net.b(i, net.grad), gb[i]
        assert float((a - r).norm() / r.norm().clamp_min(1e-6)) < 0.05, i


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,splitk", [(300, 200, 136, 1), (128, 128, 64, 1), (1000, 70, 520, 1),
                                          (96, 260, 4096, 8), (2, 512, 8192, 32)])
@pytest.mark.parametrize("epi", ["plain", "bias_relu_both", "mask_tanh_t", "c_last"])
def test_gemm_bf16_nt_matches_reference(cuda_dev, M, N, K, splitk, epi):
    if splitk > 1 and epi not in ("plain", "c_last"):
        pytest.skip("split-K writes fp32 only")
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K + 8, generator=g).to(torch.bfloat16)
    Bm = torch.randn(N, K, generator=g).to(torch.bfloat16)
    bias = torch.randn(N, generator=g)
    Y = torch.randn(M, N + 8, generator=g).clamp(-0.99, 0.99).to(torch.bfloat16)
    kw = {}
    if epi == "bias_relu_both":
        kw = dict(bias=bias, act=1)
    elif epi == "mask_tanh_t":
        kw = dict(mask_act=2, ymask=Y)
    ld = N + (8 - N % 8) % 8
    outs = {}
    for dev in ("cpu", cuda_dev):
        f32 = torch.zeros(M, N, device=dev)
        bf = torch.zeros(M, ld, dtype=torch.bfloat16, device=dev) if splitk == 1 else None
        bft = torch.zeros(N, M + (8 - M % 8) % 8, dtype=torch.bfloat16, device=dev) if splitk == 1 else None
        kk = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in kw.items()}
        if epi == "c_last":
            last = torch.zeros(M, device=dev)
            f32w = torch.zeros(M, N - 1, device=dev)
            D.gemm_bf16_nt(A.to(dev), Bm.to(dev), M, N, K, out_f32=f32w, splitk=splitk, c_last=last)
            f32 = torch.cat([f32w, last[:, None]], 1)
            outs[str(dev)] = (f32.cpu(), None, None)
            continue
        D.gemm_bf16_nt(A.to(dev), Bm.to(dev), M, N, K, out_f32=f32, splitk=splitk, **kk)
        if splitk == 1 and epi != "c_last":
            D.gemm_bf16_nt(A.to(dev), Bm.to(dev), M, N, K, out_bf16=bf, out_bf16_t=bft, **kk)
        outs[str(dev)] = (f32.cpu(), None if bf is None else bf.cpu().float(), None if bft is None else bft.cpu().float())
    ref, got = outs["cpu"], outs[str(cuda_dev)]
    scale = float(ref[0].abs().max()) + 1e-6
    assert float((ref[0] - got[0]).abs().max()) / scale < 2e-3
    if ref[1] is not None:
        assert float((ref[1] - got[1]).abs().max()) / scale < 1e-2
        assert float((ref[2] - got[2]).abs().max()) / scale < 1e-2
        assert float(got[1][:, N:].abs().max() if ld > N else 0.0) == 0.0   # pad columns untouched (zero)


@pytest.mark.gpu
def test_cvt_rowsum_bf16(cuda_dev):
    g = torch.Generator().manual_seed(3)
    X = torch.randn(77, 203, generator=g)
    out = torch.full((77, 208), 5.0).to(torch.bfloat16).to(cuda_dev)
    out_t = torch.zeros(203, 80, dtype=torch.bfloat16, device=cuda_dev)
    D.cvt_bf16(X.to(cuda_dev), out=out, out_t=out_t)
    np.testing.assert_array_equal(out[:, :203].float().cpu().numpy(), X.to(torch.bfloat16).float().numpy())
    assert float(out[:, 203:].float().abs().max()) == 0.0
    np.testing.assert_array_equal(out_t[:, :77].float().cpu().numpy(), X.T.to(torch.bfloat16).float().numpy())
    s = torch.zeros(203, device=cuda_dev)
    D.rowsum_bf16(out_t, 203, 77, s)
    np.testing.assert_allclose(s.cpu().numpy(), X.T.to(torch.bfloat16).float().sum(1).numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("act", [1, 2])
def test_bf16_mlp_gpu_step_matches_cpu_contract(cuda_dev, act):
    torch.manual_seed(1)
    sizes = [200, 512, 512, 2]
    B = 512
    nets = {d: _net(sizes, act, d, seed=5) for d in ("cpu", cuda_dev)}
    X = torch.randn(B, sizes[0])
    y = torch.randint(0, 2, (B,), dtype=torch.int32)
    res = {}
    for d, net in nets.items():
        m = _Bf16Mlp(net, act, B, d)
        xb, xbt = m.load_batch(X.to(d))
        Z = m.forward(xb).clone()
        dZ, _ = D.softmax_xent(Z.clone(), y.to(d))
        net.grad.zero_()
        m.backward(dZ, xbt)
        res[str(d)] = (Z.cpu(), net.grad.cpu())
    (zc, gc), (zg, gg) = res["cpu"], res[str(cuda_dev)]
    assert float((zc - zg).abs().max()) < 2e-2 * (float(zc.abs().max()) + 1e-3)
    assert float((gc - gg).norm() / gc.norm()) < 2e-2
