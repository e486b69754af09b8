"""learn_rate_annealing (H2O GBM): tree t is grown with learn_rate x annealing^t.
With an annealing factor the leaf values of tree t shrink by annealing^t
relative to the un-annealed model (same residuals, same splits at tree 1)."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models import H2OGradientBoostingEstimator


def _frame(device="cpu"):
    rng = np.random.default_rng(0)
    df = pd.DataFrame({"a": rng.normal(size=3000), "b": rng.normal(size=3000)})
    df["y"] = np.sin(df.a) + 0.5 * df.b + 0.1 * rng.normal(size=3000)
    return Frame.from_pandas(df, device=device)


def _values(m, t):
    from h2omx.models.tree_models import _reachable

    tr = m.ens.trees[t]
    return np.array([tr[i]["value"] for i in _reachable(tr)], np.float64)


def _leaf_scale(m, t):
    return float(np.abs(_values(m, t)).max())


def _check(fr):
    kw = dict(ntrees=4, max_depth=3, seed=1, learn_rate=0.5)
    ann = H2OGradientBoostingEstimator(learn_rate_annealing=0.5, **kw).train(x=["a", "b"], y="y", training_frame=fr)
    # tree 0 is identical to the un-annealed model's tree 0 (rate 0.5 both)
    base = H2OGradientBoostingEstimator(**kw).train(x=["a", "b"], y="y", training_frame=fr)
    np.testing.assert_allclose(_leaf_scale(ann, 0), _leaf_scale(base, 0), rtol=1e-6)
    # tree 1 sees the same residuals in both models (tree 0 identical), so it has
    # the same splits and leaf values scaled by 0.25 / 0.5
    np.testing.assert_allclose(_values(ann, 1), 0.5 * _values(base, 1), rtol=1e-5, atol=1e-7)
    assert _leaf_scale(ann, 3) < _leaf_scale(base, 3)
    assert ann.training_metrics["MSE"] < float(np.var(fr.to_pandas().y))


def test_learn_rate_annealing_cpu():
    _check(_frame())


@pytest.mark.gpu
def test_learn_rate_annealing_gpu(cuda_dev):
    _check(_frame(cuda_dev))


def test_checkpoint_continues_annealing_and_hashes():
    """A model continued from a checkpoint keeps counting iterations: tree t of
    the continuation uses learn_rate x annealing^(t0 + t) and the same bagging
    hashes as one long run, so 4 + 4 trees equal 8 trees."""
    fr = _frame()
    kw = dict(max_depth=3, seed=1, learn_rate=0.5, learn_rate_annealing=0.7, sample_rate=0.8)
    full = H2OGradientBoostingEstimator(ntrees=8, **kw).train(x=["a", "b"], y="y", training_frame=fr)
    half = H2OGradientBoostingEstimator(ntrees=4, model_id="half_ann", **kw).train(x=["a", "b"], y="y",
                                                                                  training_frame=fr)
    cont = H2OGradientBoostingEstimator(ntrees=8, checkpoint=half, **kw).train(x=["a", "b"], y="y",
                                                                             training_frame=fr)
    for t in range(8):
        np.testing.assert_allclose(_values(cont, t), _values(full, t), rtol=1e-4, atol=1e-6, err_msg=f"tree {t}")
