"""K-Means estimate_k (H2O): k grows from 1 up to the given maximum while each
added center still reduces the within-cluster sum of squares by >= 10 %."""
import numpy as np
import pandas as pd

from h2omx.frame import Frame
from h2omx.models import H2OKMeansEstimator


def test_estimate_k_finds_the_blob_count():
    rng = np.random.default_rng(0)
    centers = np.array([[0, 0], [8, 0], [0, 8], [8, 8]], float)
    X = np.concatenate([c + 0.5 * rng.normal(size=(400, 2)) for c in centers])
    fr = Frame.from_pandas(pd.DataFrame(X, columns=["a", "b"]))
    m = H2OKMeansEstimator(k=10, estimate_k=True, standardize=False, seed=1).train(training_frame=fr)
    assert len(m.training_metrics["size"]) == 4
    got = np.asarray(m.centers)
    # every true blob center has a fitted center within 0.3
    assert all(np.min(np.linalg.norm(got - c, axis=1)) < 0.3 for c in centers)
    fixed = H2OKMeansEstimator(k=6, standardize=False, seed=1).train(training_frame=fr)
    assert len(fixed.training_metrics["size"]) == 6


import pytest  # noqa: E402


@pytest.mark.gpu
def test_estimate_k_gpu(cuda_dev):
    rng = np.random.default_rng(1)
    centers = np.array([[0, 0, 0], [6, 0, 0], [0, 6, 0]], float)
    X = np.concatenate([c + 0.4 * rng.normal(size=(3000, 3)) for c in centers])
    fr = Frame.from_pandas(pd.DataFrame(X, columns=["a", "b", "c"]), device=cuda_dev)
    m = H2OKMeansEstimator(k=8, estimate_k=True, standardize=False, seed=1).train(training_frame=fr)
    assert len(m.training_metrics["size"]) == 3
    assert all(np.min(np.linalg.norm(np.asarray(m.centers) - c, axis=1)) < 0.2 for c in centers)
