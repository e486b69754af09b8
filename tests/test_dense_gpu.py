"""HIP dense kernels (fp32 MFMA) vs fp64/fp32 PyTorch references."""
import numpy as np
import pytest
import torch

from h2omx.backend import dense as D

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fp32_gemm_kernels(monkeypatch):
    """These tests pin the fp32 MFMA GEMM kernels (large NT GEMMs otherwise go
    to the x3 kernel, pinned by test_x3_gemm_matches_fp64)."""
    from h2omx.ops import dense as OD

    monkeypatch.setattr(OD, "X3_GEMM", False)


@pytest.mark.parametrize("M,N,K,act,bias", [(8192, 512, 512, 1, True), (8192, 512, 200, 1, True),
                                            (4097, 300, 516, 2, True), (1000, 130, 64, 0, False),
                                            (50, 2048, 1024, 1, True)])
def test_x3_gemm_matches_fp64(cuda_dev, monkeypatch, M, N, K, act, bias):
    """The x3 bf16-split GEMM (exact 3-piece operand split, six products,
    fp32 accumulation) has fp32 accuracy against float64; ops.dense.gemm
    routes large NT GEMMs to it."""
    from h2omx.ops import dense as OD
    from h2omx.ops.mlp import gemm_x3

    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn((M, K), generator=g).cuda()
    W = torch.randn((N, K), generator=g).cuda() * 0.05
    b = torch.randn((N,), generator=g).cuda() if bias else None
    Z = A.double() @ W.double().t() + (b.double() if bias else 0.0)
    ref = torch.relu(Z) if act == 1 else (torch.tanh(Z) if act == 2 else Z)
    got = gemm_x3(A, W, b, act)
    # fp32-equivalent: no worse than twice the fp32 MFMA kernel's error (and
    # within a few fp32 roundings of the pre-activation magnitude)
    f32 = OD.gemm_fp32(A, W, b, act, tb=True)
    err32 = (f32.double() - ref).abs().max().item()
    tol = max(2.0 * err32, 2e-6 * Z.abs().max().item())
    assert (got.double() - ref).abs().max().item() <= tol
    monkeypatch.setattr(OD, "X3_GEMM", True)
    routed = D.gemm(A, W, b, act, False, True)
    assert (routed.double() - ref).abs().max().item() <= tol
    if M * N * K >= OD.X3_MIN_MNK:
        assert torch.equal(routed, got)


@pytest.mark.parametrize("M,K,N,act", [(8192, 512, 512, 1), (8192, 512, 512, 2), (4100, 516, 300, 2),
                                       (8000, 1024, 200, 1)])
def test_x3_dact_matches_fp64(cuda_dev, monkeypatch, M, K, N, act):
    """Hidden-layer data gradient on the x3 GEMM (W transposed into scratch,
    act'(Y) and the 64-row bias partials in the epilogue) against float64,
    with fp32-kernel accuracy."""
    from h2omx.ops import dense as OD

    g = torch.Generator(device="cpu").manual_seed(M + K + N + act)
    dZ = torch.randn((M, K), generator=g).cuda()
    W = torch.randn((K, N), generator=g).cuda() * 0.05
    Y = torch.randn((M, N), generator=g).cuda()
    Y = Y.clamp_min(0) if act == 1 else torch.tanh(Y)
    dH = dZ.double() @ W.double()
    ref = dH * ((Y > 0).double() if act == 1 else (1 - Y.double() ** 2))
    f32, _ = OD.gemm_dact(dZ, W, Y, act)                 # fp32 MFMA route (X3_GEMM off)
    err32 = (f32.double() - ref).abs().max().item()
    monkeypatch.setattr(OD, "X3_GEMM", True)
    out, (ws, splits) = OD.gemm_dact(dZ, W, Y, act)
    assert splits == -(-M // 64)                        # the x3 route ran
    tol = max(2.0 * err32, 2e-6 * dH.abs().max().item())
    assert (out.double() - ref).abs().max().item() <= tol
    colsum = ws[: splits * N].view(splits, N).double().sum(0)
    assert torch.allclose(colsum, ref.sum(0), rtol=1e-5, atol=1e-3)
    for s in (0, splits - 1):   # each slice is its own 64 rows
        assert torch.allclose(ws[s * N:(s + 1) * N].double(), out[s * 64:(s + 1) * 64].double().sum(0),
                              rtol=1e-5, atol=1e-4)
    # batched transposes (one launch for several layers) feed the same bits
    W2 = torch.randn((N, 3 * K // 4 if K % 16 == 0 else K), generator=g).cuda()
    Wt, W2t = OD.transpose_weights([W, W2])
    assert torch.equal(Wt, W.t()) and torch.equal(W2t, W2.t())
    out2, _ = OD.gemm_dact(dZ, W, Y, act, Wt=Wt)
    assert torch.equal(out2, out)


@pytest.mark.parametrize("p,family,link", [(5, "binomial", "logit"), (30, "gaussian", "identity"),
                                           (61, "poisson", "log"), (100, "binomial", "logit"),
                                           (300, "binomial", "logit"), (700, "gaussian", "identity")])
def test_glm_irls_gram_matches_reference(cuda_dev, p, family, link):
    rng = np.random.default_rng(p)
    n = 20_011
    X = rng.normal(size=(p, n)).astype(np.float32)
    beta = np.zeros((1, p + 1))
    beta[0, :p] = rng.normal(scale=0.1, size=p)
    beta[0, p] = 0.2
    eta = beta[0, :p] @ X + beta[0, p]
    if family == "binomial":
        y = (rng.random(n) < 1 / (1 + np.exp(-eta))).astype(np.float32)
    elif family == "poisson":
        y = rng.poisson(np.exp(eta)).astype(np.float32)
    else:
        y = (eta + rng.normal(size=n)).astype(np.float32)
    w = rng.uniform(0.5, 2.0, n).astype(np.float32)
    Xt, yt, wt = torch.from_numpy(X), torch.from_numpy(y), torch.from_numpy(w)
    Gr, dr = D.glm_irls_pass(Xt, yt, wt, None, beta, family, link)
    Gg, dg = D.glm_irls_pass(Xt.to(cuda_dev), yt.to(cuda_dev), wt.to(cuda_dev), None, beta, family, link)
    scale = np.abs(Gr).max()
    assert np.abs(Gg - Gr).max() / scale < 2e-5
    assert abs(dg - dr) / abs(dr) < 1e-5


@pytest.mark.parametrize("p", [12, 290])
def test_glm_multinomial_gram(cuda_dev, p):
    """p = 290 runs the wide path (eta GEMM + glm_wz / glm_aug + Gram GEMM)."""
    rng = np.random.default_rng(1)
    n, K = 9001, 3
    X = rng.normal(size=(p, n)).astype(np.float32)
    y = rng.integers(0, K, n).astype(np.float32)
    beta = rng.normal(scale=0.1, size=(K, p + 1))
    Xt, yt = torch.from_numpy(X), torch.from_numpy(y)
    for c in range(K):
        Gr, dr = D.glm_irls_pass(Xt, yt, None, None, beta, "multinomial", "logit", cls=c)
        Gg, dg = D.glm_irls_pass(Xt.to(cuda_dev), yt.to(cuda_dev), None, None, beta, "multinomial", "logit", cls=c)
        assert np.abs(Gg - Gr).max() / np.abs(Gr).max() < 2e-5
        assert abs(dg - dr) / abs(dr) < 1e-5


@pytest.mark.parametrize("d,k", [(4, 3), (28, 10), (64, 40), (100, 17), (200, 8)])
def test_kmeans_step_matches_reference(cuda_dev, d, k):
    rng = np.random.default_rng(d)
    n = 30_000
    X = rng.normal(size=(d, n)).astype(np.float32)
    C = rng.normal(size=(k, d)).astype(np.float32)
    ar, sr, cr, er = D.kmeans_step(torch.from_numpy(X), torch.from_numpy(C))
    ag, sg, cg, eg = D.kmeans_step(torch.from_numpy(X).to(cuda_dev), torch.from_numpy(C).to(cuda_dev))
    agree = (ag.cpu().numpy() == ar.numpy()).mean()
    assert agree > 0.999  # fp32 near-ties may flip
    if agree == 1.0:
        np.testing.assert_allclose(cg, cr)
        np.testing.assert_allclose(sg, sr, rtol=1e-4, atol=1e-3)
        np.testing.assert_allclose(eg, er, rtol=1e-3)


@pytest.mark.parametrize("mfma", [True, False])
@pytest.mark.parametrize("d,k", [(4, 3), (33, 16), (64, 17), (64, 32), (100, 10), (128, 16), (96, 5), (14, 12),
                                 (110, 16), (126, 4), (30, 29)])
def test_kmeans_wave_kernel_matches_reference(cuda_dev, monkeypatch, d, k, mfma):
    """Wave-unit Lloyd passes (csrc/kmeans_wave.hip: MFMA cluster sums, or the
    LDS-tile row walk) against the fp64 NumPy oracle and the workgroup-tile
    kernel: tail chunk (n % 64 != 0), NA cells, empty clusters, the count / SSE
    columns at the end of a 16-feature block (d = 14, 30, 110, 126)."""
    rng = np.random.default_rng(100 + d + k)
    n = 40_003
    X = rng.normal(size=(d, n)).astype(np.float32)
    X[rng.integers(0, d, 50), rng.integers(0, n, 50)] = np.nan
    C = rng.normal(size=(k, d)).astype(np.float32)
    C[-1] += 50.0   # far away: empty cluster
    Xc = np.nan_to_num(X, nan=0.0)
    ar, sr, cr, er = D.kmeans_step(torch.from_numpy(Xc), torch.from_numpy(C))
    outs = {}
    import h2omx.ops.dense as OD

    for wave in (True, False):
        monkeypatch.setattr(OD, "KM_WAVE", wave)
        monkeypatch.setattr(OD, "KM_MFMA", wave and mfma)
        outs[wave] = D.kmeans_step(torch.from_numpy(X).to(cuda_dev), torch.from_numpy(C).to(cuda_dev))
    if mfma:   # the NA-free variant on the imputed design gives the same pass
        monkeypatch.setattr(OD, "KM_MFMA", True)
        monkeypatch.setattr(OD, "KM_WAVE", True)
        a2, s2, c2, e2 = D.kmeans_step(torch.from_numpy(Xc).to(cuda_dev), torch.from_numpy(C).to(cuda_dev), na_free=True)
        assert torch.equal(a2, outs[True][0]) and np.array_equal(c2, outs[True][2])
        np.testing.assert_allclose(s2, outs[True][1], rtol=1e-6, atol=1e-5)
    ag, sg, cg, eg = outs[True]
    agree = (ag.cpu().numpy() == ar.numpy()).mean()
    assert agree > 0.999
    assert cg[-1] == 0 and cg.sum() == n
    if agree == 1.0:
        np.testing.assert_array_equal(cg, cr)
        np.testing.assert_allclose(sg, sr, rtol=1e-4, atol=2e-3)
        np.testing.assert_allclose(eg, er, rtol=1e-4)
    # same assignment as the tile kernel up to fp32 near-ties
    assert (outs[False][0].cpu().numpy() == ag.cpu().numpy()).mean() > 0.999


@pytest.mark.parametrize("M,N,K,ta,tb,act", [(1000, 512, 200, False, False, 1), (513, 257, 129, False, True, 2),
                                             (200, 512, 1000, True, False, 0), (64, 64, 64, True, True, 1)])
def test_gemm_matches_torch(cuda_dev, M, N, K, ta, tb, act):
    torch.manual_seed(0)
    A = torch.randn((K, M) if ta else (M, K), device=cuda_dev)
    B = torch.randn((N, K) if tb else (K, N), device=cuda_dev)
    bias = torch.randn(N, device=cuda_dev)
    C = D.gemm(A, B, bias, act, ta, tb)
    ref = D.gemm(A.cpu().double().float(), B.cpu().float(), bias.cpu(), act, ta, tb)
    assert torch.allclose(C.cpu(), ref, rtol=1e-4, atol=1e-3)


def test_mlp_elementwise(cuda_dev):
    torch.manual_seed(1)
    Z = torch.randn(300, 5, device=cuda_dev)
    y = torch.randint(0, 5, (300,), device=cuda_dev, dtype=torch.int32)
    dZ, loss = D.softmax_xent(Z, y)
    dZr, lr = D.softmax_xent(Z.cpu(), y.cpu())
    assert torch.allclose(dZ.cpu(), dZr, atol=1e-6) and abs(loss.item() - lr.item()) < 1e-5
    W = torch.randn(1000, device=cuda_dev)
    G = torch.randn(1000, device=cuda_dev)
    e1, e2 = torch.zeros_like(W), torch.zeros_like(W)
    Wc, e1c, e2c = W.cpu().clone(), e1.cpu().clone(), e2.cpu().clone()
    D.adadelta_(W, G, e1, e2, 0.99, 1e-8, 1e-5)
    D.adadelta_(Wc, G.cpu(), e1c, e2c, 0.99, 1e-8, 1e-5)
    assert torch.allclose(W.cpu(), Wc, atol=1e-6)


@pytest.mark.parametrize("M,N,K,ta,tb", [(512, 200, 8192, True, False), (512, 512, 8192, True, False),
                                         (2, 512, 8192, True, False), (130, 70, 5000, False, True)])
def test_gemm_splitk_matches_torch(cuda_dev, M, N, K, ta, tb):
    """Weight-gradient shaped GEMMs (small output, long K) take the split-K path."""
    torch.manual_seed(2)
    A = torch.randn((K, M) if ta else (M, K), device=cuda_dev)
    B = torch.randn((N, K) if tb else (K, N), device=cuda_dev)
    C = D.gemm(A, B, None, 0, ta, tb)
    ref = (A.T if ta else A).double() @ (B.T if tb else B).double()
    assert torch.allclose(C.double(), ref, rtol=1e-4, atol=2e-2)
    C2 = D.gemm(A, B, None, 0, ta, tb)
    assert torch.equal(C, C2)   # deterministic


def test_bias_grad_split(cuda_dev):
    dY = torch.randn(8192, 300, device=cuda_dev)
    db = D.bias_grad(dY)
    assert torch.allclose(db.double(), dY.double().sum(0), atol=1e-3)


def test_auc_hist_kernel_matches_cpu(cuda_dev):
    from h2omx.metrics.core import score_histograms
    from sklearn.metrics import roc_auc_score
    from h2omx.metrics import auc_from_scores

    torch.manual_seed(3)
    s = torch.rand(200000, dtype=torch.float64)
    y = (torch.rand(200000) < s).double()
    w = torch.rand(200000, dtype=torch.float64)
    Hc, lo, hi = score_histograms(s, y, w)
    Hg, lo2, hi2 = score_histograms(s.to(cuda_dev), y.to(cuda_dev), w.to(cuda_dev))
    assert lo == lo2 and hi == hi2
    np.testing.assert_allclose(Hg, Hc, rtol=1e-6, atol=1e-6)
    a = auc_from_scores(s.to(cuda_dev), y.to(cuda_dev))
    assert abs(a - roc_auc_score(y.numpy(), s.numpy())) < 1e-4


@pytest.mark.parametrize("M,N,K,act", [(8192, 2, 512, 0), (1000, 3, 200, 1), (777, 8, 37, 2), (64, 1, 16, 0)])
def test_gemm_skinny_output_matches_torch(cuda_dev, M, N, K, act):
    """Classifier-layer shapes (N <= 8) take the one-wave-per-row kernel."""
    torch.manual_seed(3)
    A = torch.randn((M, K), device=cuda_dev)
    B = torch.randn((N, K), device=cuda_dev)
    bias = torch.randn(N, device=cuda_dev)
    C = D.gemm(A, B, bias, act, False, True)
    ref = D.gemm(A.cpu(), B.cpu(), bias.cpu(), act, False, True)
    assert torch.allclose(C.cpu(), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K", [(8192, 512, 2), (333, 100, 5)])
def test_gemm_thin_k_matches_torch(cuda_dev, M, N, K):
    torch.manual_seed(4)
    A = torch.randn((M, K), device=cuda_dev)
    B = torch.randn((K, N), device=cuda_dev)
    C = D.gemm(A, B)
    assert torch.allclose(C.cpu(), A.cpu() @ B.cpu(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,out,inp,act", [(8192, 512, 512, 1), (8192, 512, 200, 2), (300, 64, 40, 0), (300, 30, 40, 1)])
def test_act_backward_bias_and_wgrad(cuda_dev, M, out, inp, act):
    """Fused activation backward + bias-gradient slices, and the weight-gradient
    GEMM whose split-K reduce also folds the bias slices (fp64 reference)."""
    torch.manual_seed(5)
    Y = torch.randn((M, out), device=cuda_dev)
    if act == 1:
        Y = Y.clamp_min(0)
    elif act == 2:
        Y = torch.tanh(Y)
    dY = torch.randn((M, out), device=cuda_dev)
    H = torch.randn((M, inp), device=cuda_dev)
    dYr = dY.double().cpu()
    if act == 1:
        dZr = dYr * (Y.cpu() > 0).double()
    elif act == 2:
        dZr = dYr * (1 - Y.cpu().double() ** 2)
    else:
        dZr = dYr
    dZ, bpart = D.act_backward_bias(Y, dY.clone(), act)
    assert torch.allclose(dZ.double().cpu(), dZr, atol=1e-6)
    dW = torch.empty((out, inp), device=cuda_dev)
    db = torch.empty((out,), device=cuda_dev)
    D.wgrad_bias(dZ, H, dW, db, bpart)
    assert torch.allclose(dW.double().cpu(), dZr.T @ H.double().cpu(), rtol=1e-4, atol=2e-2)
    assert torch.allclose(db.double().cpu(), dZr.sum(0), atol=1e-3)


@pytest.mark.parametrize("M,N,K,ta,tb", [(8192, 512, 512, False, True), (8192, 512, 512, False, False),
                                         (512, 512, 8192, True, False), (1000, 300, 77, False, False),
                                         (130, 70, 5000, True, True), (8192, 512, 200, False, True),
                                         (256, 512, 512, False, True), (512, 200, 8192, True, False)])
def test_gemm_64_tiles_bit_identical_to_128(cuda_dev, M, N, K, ta, tb):
    """The 64 x 64-tile kernel keeps each element's k-ordered fmaf chain (and
    the split-K chunking) of the 128 x 128 one: bit-identical outputs."""
    from h2omx.ops import dense as OD

    torch.manual_seed(6)
    A = torch.randn((K, M) if ta else (M, K), device=cuda_dev)
    B = torch.randn((N, K) if tb else (K, N), device=cuda_dev)
    bias = None if ta else torch.randn(N, device=cuda_dev)
    out = {}
    try:
        for tile in (128, 64, 1, 2, 0):  # 1 / 2: 64 x 64 wave tiles on 128 x 128 / 128 x 64 blocks; 0 = auto
            OD.set_gemm_tile(tile)
            out[tile] = D.gemm(A, B, bias, 0 if ta else 1, ta, tb)
    finally:
        OD.set_gemm_tile(0)
    assert torch.equal(out[0], out[128])
    assert torch.equal(out[64], out[128])
    assert torch.equal(out[1], out[128]) and torch.equal(out[2], out[128])
    ref = (A.T if ta else A).double() @ (B.T if tb else B).double()
    if bias is not None:
        ref = (ref + bias.double()).clamp_min(0)
    assert torch.allclose(out[64].double(), ref, rtol=1e-4, atol=2e-2)


@pytest.mark.parametrize("p,family,link,n,off", [(5, "binomial", "logit", 20_000, False),
                                                 (100, "binomial", "logit", 40_000, True),
                                                 (14, "poisson", "log", 3_001, True),
                                                 (126, "gamma", "inverse", 8_000, False)])
def test_glm_wave_kernel_matches_workgroup_kernel_and_reference(cuda_dev, monkeypatch, p, family, link, n, off):
    """Wave-unit IRLS kernel (register-resident chunks, 16x16 Gram tiles; 16-byte
    column loads when n % 4 == 0) vs the workgroup kernel and the fp64 oracle;
    offsets, prior weights and NaN imputation (means) included."""
    from h2omx.ops import dense as DD

    rng = np.random.default_rng(p + n)
    X = rng.normal(size=(p, n)).astype(np.float32)
    beta = np.zeros((1, p + 1))
    beta[0, :p] = rng.normal(scale=0.05, size=p)
    beta[0, p] = 0.3 if family != "gamma" else 2.0
    eta = beta[0, :p] @ X + beta[0, p]
    if family == "binomial":
        y = (rng.random(n) < 1 / (1 + np.exp(-eta))).astype(np.float32)
    elif family == "poisson":
        y = rng.poisson(np.exp(eta)).astype(np.float32)
    else:
        y = rng.gamma(2.0, 1.0 / np.maximum(eta, 0.2) / 2.0).astype(np.float32)
    w = rng.uniform(0.5, 2.0, n).astype(np.float32)
    o = (0.1 * rng.normal(size=n)).astype(np.float32) if off else None
    Xt, yt, wt = torch.from_numpy(X), torch.from_numpy(y), torch.from_numpy(w)
    ot = None if o is None else torch.from_numpy(o)
    Gr, dr = D.glm_irls_pass(Xt, yt, wt, ot, beta, family, link)
    g = lambda: DD.glm_irls_pass(Xt.to(cuda_dev), yt.to(cuda_dev), wt.to(cuda_dev),
                                 None if ot is None else ot.to(cuda_dev), beta, family, link)
    monkeypatch.setattr(DD, "GLM_WAVE", True)
    Gw, dw = g()
    monkeypatch.setattr(DD, "GLM_WAVE", False)
    Gk, dk = g()
    scale = np.abs(Gr).max()
    assert np.abs(Gw - Gr).max() / scale < 2e-5
    assert np.abs(Gw - Gk).max() / scale < 2e-5
    assert abs(dw - dr) / abs(dr) < 1e-5


@pytest.mark.parametrize("p,family,link,n,off", [(100, "binomial", "logit", 100_003, True),
                                                 (15, "gaussian", "identity", 4_096, False),
                                                 (14, "poisson", "log", 777, True),
                                                 (30, "binomial", "logit", 65_536, False),
                                                 (1, "gamma", "inverse", 5_000, False),
                                                 (126, "tweedie", "tweedie", 9_000, True)])
def test_glm_split_gram_matches_f32_and_reference(cuda_dev, monkeypatch, p, family, link, n, off):
    """glm_irls_split_kernel (exact 3-way bf16 split, 6 bf16 MFMAs per tile) vs
    the fp32-MFMA wave kernel and the fp64 oracle: tails (n % 32 != 0),
    unaligned columns (n % 4 != 0 -> scalar loads), the intercept at the end of
    block NB-2 (p = 15) and alone in a block (p = 14, p = 126), one feature."""
    from h2omx.ops import dense as DD

    rng = np.random.default_rng(3 * p + n)
    X = rng.normal(size=(p, n)).astype(np.float32)
    X[0] *= 50.0                     # a wide dynamic range across columns
    beta = np.zeros((1, p + 1))
    beta[0, :p] = rng.normal(scale=0.05, size=p)
    beta[0, p] = 0.3 if family not in ("gamma", "tweedie") else 2.0
    beta[0, 0] *= 0.02
    eta = beta[0, :p] @ X + beta[0, p]
    if family == "binomial":
        y = (rng.random(n) < 1 / (1 + np.exp(-eta))).astype(np.float32)
    elif family == "poisson":
        y = rng.poisson(np.exp(eta)).astype(np.float32)
    elif family == "gaussian":
        y = (eta + rng.normal(size=n)).astype(np.float32)
    else:
        y = rng.gamma(2.0, 1.0 / np.maximum(eta, 0.2) / 2.0).astype(np.float32)
    w = rng.uniform(0.5, 2.0, n).astype(np.float32)
    o = (0.1 * rng.normal(size=n)).astype(np.float32) if off else None
    Xt, yt, wt = torch.from_numpy(X), torch.from_numpy(y), torch.from_numpy(w)
    ot = None if o is None else torch.from_numpy(o)
    kw = dict(var_power=1.5, link_power=0.0) if family == "tweedie" else {}
    Gr, dr = D.glm_irls_pass(Xt, yt, wt, ot, beta, family, link, **kw)
    g = lambda: DD.glm_irls_pass(Xt.to(cuda_dev), yt.to(cuda_dev), wt.to(cuda_dev),
                                 None if ot is None else ot.to(cuda_dev), beta, family, link, **kw)
    monkeypatch.setattr(DD, "GLM_WAVE", True)
    monkeypatch.setattr(DD, "GLM_GRAM", "split")
    Gs, ds = g()
    monkeypatch.setattr(DD, "GLM_GRAM", "f32")
    Gf, df = g()
    scale = np.abs(Gr).max()
    es, ef = np.abs(Gs - Gr).max() / scale, np.abs(Gf - Gr).max() / scale
    assert es < 2e-6 and ef < 2e-6, (es, ef)
    # entry-wise on the significant entries: the split is as accurate as fp32 MFMA
    big = np.abs(Gr) > 1e-4 * scale
    rs = (np.abs(Gs - Gr) / np.abs(Gr))[big].max()
    rf = (np.abs(Gf - Gr) / np.abs(Gr))[big].max()
    assert rs < 1e-5 and rs < 4 * rf + 1e-6, (rs, rf)
    assert abs(ds - dr) / abs(dr) < 1e-5 and abs(ds - df) / abs(df) < 1e-6


def test_glm_gram_ill_conditioned_collinear_design(cuda_dev):
    """Near-collinear columns (x2 = x1 + 1e-3 noise) with a 1e4 dynamic range of
    column scales: the fp32-per-unit / fp64-across-units Gram stays within 2e-6
    of the fp64 oracle entry-wise, and the gaussian GLM fitted on it reproduces
    the fp64 least-squares fitted values to 1e-4."""
    import pandas as pd

    from h2omx.frame import Frame
    from h2omx.models import H2OGeneralizedLinearEstimator

    rng = np.random.default_rng(7)
    n = 200_000
    x1 = rng.normal(size=n)
    cols = {"x1": x1, "x2": x1 + 1e-3 * rng.normal(size=n), "x3": 100.0 * rng.normal(size=n),
            "x4": 0.01 * rng.normal(size=n), "x5": 0.5 * x1 + rng.normal(size=n)}
    X = np.stack(list(cols.values())).astype(np.float32)
    beta = np.zeros((1, 6))
    y = (2 * x1 - x1 + 0.003 * cols["x3"] + 40 * cols["x4"] + rng.normal(size=n)).astype(np.float32)
    Gr, _ = D.glm_irls_pass(torch.from_numpy(X), torch.from_numpy(y), None, None, beta, "gaussian", "identity")
    Gg, _ = D.glm_irls_pass(torch.from_numpy(X).to(cuda_dev), torch.from_numpy(y).to(cuda_dev), None, None, beta,
                            "gaussian", "identity")
    rel = np.abs(Gg - Gr) / np.maximum(np.abs(Gr), 1e-30)
    big = np.abs(Gr) > 1e-6 * np.abs(Gr).max()
    assert rel[big].max() < 2e-6, rel[big].max()
    df = pd.DataFrame({k: v.astype(np.float32) for k, v in cols.items()})
    df["y"] = y
    fr = Frame.from_pandas(df, device=cuda_dev)
    m = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0.0, standardize=True).train(
        x=list(cols), y="y", training_frame=fr)
    A = np.column_stack([X.T.astype(np.float64), np.ones(n)])
    coef, *_ = np.linalg.lstsq(A, y.astype(np.float64), rcond=None)
    fitted_ref = A @ coef
    fitted = m.predict(fr).to_pandas()["predict"].to_numpy(np.float64)
    assert np.abs(fitted - fitted_ref).max() < 1e-4 * np.abs(fitted_ref).max()


@pytest.mark.parametrize("M,K,N,act,tile", [(8192, 512, 512, 1, 1), (8192, 512, 512, 2, 2), (1000, 77, 300, 1, 1),
                                            (333, 130, 70, 2, 2)])
def test_gemm_dact_matches_reference(cuda_dev, M, K, N, act, tile):
    """dZ_prev = (dZ W) * act'(Y) in the GEMM epilogue + per-128-row bias partials,
    folded by the weight-gradient reduce (fp64 reference)."""
    from h2omx.ops import dense as OD

    torch.manual_seed(7)
    dZ = torch.randn((M, K), device=cuda_dev)
    W = torch.randn((K, N), device=cuda_dev)
    Y = torch.randn((M, N), device=cuda_dev)
    Y = Y.clamp_min(0) if act == 1 else torch.tanh(Y)
    out, bpart = OD.gemm_dact(dZ, W, Y, act, tile=tile)
    dH = dZ.double() @ W.double()
    ref = dH * ((Y > 0).double() if act == 1 else (1 - Y.double() ** 2))
    assert torch.allclose(out.double(), ref, rtol=1e-4, atol=2e-3)
    ws, splits = bpart
    assert splits == -(-M // 128)
    assert torch.allclose(ws[: splits * N].view(splits, N).double().sum(0), ref.sum(0), atol=2e-2)
    # the unfused pair gives the same dZ_prev bits (same k-ordered fmaf chain)
    OD.set_gemm_tile(tile)
    try:
        dH32 = D.gemm(dZ, W)
    finally:
        OD.set_gemm_tile(0)
    dZ2, _ = D.act_backward_bias(Y, dH32, act)
    assert torch.equal(out, dZ2)


@pytest.mark.parametrize("M,N,C,act", [(8192, 512, 2, 1), (1000, 300, 3, 2), (333, 64, 8, 1), (8192, 200, 1, 2)])
def test_output_layer_streaming_kernels(cuda_dev, M, N, C, act):
    """few-class output layer: dW = dZ^T H, db = sum dZ (out_wgrad) and
    dZ_prev = (dZ W) * act'(H) with its bias partials (thin_dact), fp64 reference"""
    from h2omx.ops import dense as OD

    torch.manual_seed(8)
    dZ = torch.randn((M, C), device=cuda_dev)
    H = torch.randn((M, N), device=cuda_dev)
    H = H.clamp_min(0) if act == 1 else torch.tanh(H)
    W = torch.randn((C, N), device=cuda_dev)
    dW = torch.empty((C, N), device=cuda_dev)
    db = torch.empty((C,), device=cuda_dev)
    OD.out_wgrad(dZ, H, dW, db)
    assert torch.allclose(dW.double(), dZ.double().T @ H.double(), rtol=1e-4, atol=1e-3)
    assert torch.allclose(db.double(), dZ.double().sum(0), atol=1e-3)
    out, (ws, S) = OD.thin_dact(dZ, W, H, act)
    ref = (dZ.double() @ W.double()) * ((H > 0).double() if act == 1 else (1 - H.double() ** 2))
    assert torch.allclose(out.double(), ref, rtol=1e-5, atol=1e-5)
    assert torch.allclose(ws[: S * N].view(S, N).double().sum(0), ref.sum(0), atol=1e-3)
