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
