"""Quantile sketch helpers on the CPU (the same torch code runs on the GPU)."""
import numpy as np
import torch

from h2omx.models.tree.binning import _edges_device, sort_rows


def test_sort_rows_matches_torch_sort():
    """One int64 radix sort of (row, order-preserving float bits) keys sorts
    every row like torch.sort(dim=1): NaNs (either sign) last, infinities,
    signed zeros, duplicates."""
    torch.manual_seed(0)
    S = torch.randn(6, 3000)
    S[0, ::7] = float("nan")
    S[1, ::3] = -0.0
    S[1, 1::3] = 0.0
    S[2, :5] = float("inf")
    S[2, 5:9] = -float("inf")
    S[3] = torch.randint(0, 4, (3000,)).float()
    S[4, ::11] = -float("nan")
    S[5] = float("nan")
    a, b = sort_rows(S), torch.sort(S, dim=1).values
    assert torch.equal(torch.isnan(a), torch.isnan(b))
    assert torch.equal(torch.nan_to_num(a, nan=0.0), torch.nan_to_num(b, nan=0.0))
    for nb in (20, 255):
        for x, y in zip(_edges_device(a, nb), _edges_device(b, nb)):
            np.testing.assert_array_equal(x, y)


def test_histogram_types():
    """histogram_type: quantile vs equal-width vs robust vs random cut points;
    few-valued columns keep one bin per value; unknown rejected.  (The per-node
    rules UniformAdaptive / Random / RoundRobin of GBM / DRF are in
    test_hist_adaptive.py; these are the global grids.)"""
    import numpy as np
    import pytest
    import torch

    from h2omx.models.tree.binning import compute_edges

    g = torch.Generator().manual_seed(0)
    X = torch.randn((3, 20000), generator=g)
    X[1] = X[1] ** 3                       # heavy tails
    X[2] = torch.randint(0, 6, (20000,), generator=g).float()
    eq, nvq, _ = compute_edges(X, 32, histogram_type="QuantilesGlobal")
    eu, nvu, _ = compute_edges(X, 32, histogram_type="UniformAdaptive")
    er, nvr, _ = compute_edges(X, 32, histogram_type="UniformRobust")
    ex, nvx, _ = compute_edges(X, 32, histogram_type="Random")
    ea, _, _ = compute_edges(X, 32, histogram_type="AUTO")
    np.testing.assert_array_equal(ea, eq)
    for e, nv in ((eu, nvu), (er, nvr), (ex, nvx)):
        np.testing.assert_array_equal(e[2, : nv[2] - 1], np.arange(5, dtype=np.float32))   # value bins
    d = np.diff(eu[0, : nvu[0] - 1])
    assert np.allclose(d, d[0], rtol=1e-3)                                  # equal width
    assert eu[1, 0] < er[1, 0] and er[1, nvr[1] - 2] < eu[1, nvu[1] - 2]     # robust range inside the full one
    assert not np.allclose(np.diff(ex[0, : nvx[0] - 1]), d[0], rtol=1e-2)   # random spacing
    er2, _, _ = compute_edges(X, 32, histogram_type="RoundRobin")      # global grid: the quantile one
    np.testing.assert_array_equal(er2, eq)
    with pytest.raises(ValueError, match="unknown histogram_type"):
        compute_edges(X, 32, histogram_type="Sturges")


def test_row_major_codes_line_aligned(monkeypatch):
    """Row-major code rows have power-of-two strides up to 128 bytes and
    multiples of 128 above (no row straddles a 128-byte line), zero pad bytes
    and the same codes as the feature-major matrix; ROW_ALIGN off keeps the
    4-byte strides."""
    from h2omx.models.tree import bin_matrix, compute_edges
    from h2omx.models.tree.binning import BinnedMatrix

    rng = np.random.default_rng(3)
    for F, want in ((3, 4), (13, 16), (28, 32), (100, 128), (130, 256)):
        X = torch.from_numpy(rng.normal(size=(F, 257)).astype(np.float32))
        e, nv, nbt = compute_edges(X, 63)
        bm = bin_matrix(X, e, nv, nbt)
        assert bm.fp == want
        rm = bm.codes_rm
        assert rm.shape == (257, want)
        assert torch.equal(rm[:, :F], bm.codes[:, :257].t())
        assert int(rm[:, F:].abs().sum()) == 0
    monkeypatch.setattr(BinnedMatrix, "ROW_ALIGN", False)
    X = torch.from_numpy(rng.normal(size=(100, 50)).astype(np.float32))
    e, nv, nbt = compute_edges(X, 63)
    assert bin_matrix(X, e, nv, nbt).fp == 100
