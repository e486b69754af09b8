"""K1 device quantile sketch (csrc/sketch_kernels.hip) against the sort path:
identical cut points for continuous, heavy-tailed, low-cardinality,
integer-valued (values sharing a radix bin), constant, NaN-heavy and
all-NaN features."""
import numpy as np
import pytest
import torch

from h2omx.models.tree import binning as B


def _cols(n, seed=0):
    rng = np.random.default_rng(seed)
    cols = [
        rng.normal(size=n),                                   # continuous
        rng.standard_cauchy(size=n),                          # heavy tails
        rng.integers(0, 2, n).astype(float),                  # binary
        rng.integers(0, 7, n) * 0.5 - 1.0,                    # few levels
        1000.0 + rng.integers(0, 120, n),                     # integers sharing top-16 key bits
        np.full(n, 3.25),                                     # constant
        np.where(rng.random(n) < 0.6, np.nan, rng.uniform(-2, 2, n)),  # NaN heavy
        np.full(n, np.nan),                                   # all NaN
        np.round(rng.exponential(1.0, n), 2),                 # many ties, > 255 distinct
        np.round(rng.normal(size=n), 1),                      # -0.0 and +0.0 (one value)
        np.round(rng.normal(size=n) * 30, 0),                 # signed zeros, > 255 distinct
        rng.uniform(0, 1, n).astype(np.float32).astype(float) * 1e-30,   # tiny magnitudes
    ]
    return np.stack(cols).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("n,nbins", [(300_000, 255), (50_000, 20), (1_500_000, 63)])
def test_sketch_matches_sort(cuda_dev, monkeypatch, n, nbins):
    X = torch.from_numpy(_cols(n, seed=n % 97)).to(cuda_dev)
    monkeypatch.setattr(B, "SKETCH", True)
    e1, v1, nb1 = B.compute_edges(X, nbins)
    monkeypatch.setattr(B, "SKETCH", False)
    e2, v2, nb2 = B.compute_edges(X, nbins)
    assert nb1 == nb2
    np.testing.assert_array_equal(v1, v2)
    np.testing.assert_array_equal(e1, e2)
    # ... and the host oracle on the same sample
    m = min(n, 1 << 20)
    if n <= m:
        e3, v3, _ = B.compute_edges(X.cpu(), nbins)
        np.testing.assert_array_equal(v1, v3)
        np.testing.assert_array_equal(e1, e3)
