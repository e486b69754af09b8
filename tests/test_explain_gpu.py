"""TreeSHAP HIP kernel (csrc/explain_kernels.hip) vs the NumPy path
formula and additivity on the device."""
import numpy as np
import pytest
import torch

from h2omx import _native
from h2omx.explain import _shap_numpy, predict_contributions, tree_paths
from h2omx.frame import Frame
from h2omx.models import H2OGradientBoostingEstimator, H2ORandomForestEstimator, H2OXGBoostEstimator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cls,kw,F", [(H2OGradientBoostingEstimator, dict(ntrees=20, max_depth=5), 6),
                                      (H2OXGBoostEstimator, dict(ntrees=10, max_depth=8), 70),
                                      (H2ORandomForestEstimator, dict(ntrees=5, max_depth=12), 10)])
def test_tree_shap_kernel(cuda_dev, cls, kw, F):
    rng = np.random.default_rng(F)
    n = 20000
    X = rng.normal(size=(n, F)).astype(np.float32)
    X[::13, 0] = np.nan
    y = (np.nan_to_num(X[:, 0]) + X[:, 1] * X[:, 2] + rng.normal(size=n) > 0).astype(np.float32)
    names = [f"f{i}" for i in range(F)]
    fr = Frame.from_numpy(np.c_[X, y], names=names + ["y"], device=cuda_dev)
    m = cls(seed=1, **kw).train(y="y", training_frame=fr)
    C = predict_contributions(m, fr)
    out = torch.stack([v.data for v in C.vecs])
    assert out.is_cuda
    margin = m.ens.raw_margin(fr.feature_matrix(m.x))[0]
    assert torch.allclose(out.sum(0), margin, atol=5e-4 * max(1.0, float(margin.abs().max())))
    nt = m.ens.ntrees
    lv, el, _, maxm, sets = tree_paths(m.ens.trees[:nt], 1.0 / nt if m.ens.average else 1.0)
    ref = _shap_numpy(X[:300].T.astype(np.float64), lv, el, maxm, sets)
    np.testing.assert_allclose(out[:F, :300].cpu().numpy(), ref, atol=2e-4 * max(1.0, np.abs(ref).max()))
    assert "explain" in " ".join(_native.loaded_libraries())
