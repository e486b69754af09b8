"""Infogram: redundant predictors lose net information (core), proxies of a
protected attribute lose safety (fair); H2O accessors."""
import torch

from h2omx.frame.frame import ENUM, Frame, Vec
from h2omx.models import H2OInfogram

AP = dict(ntrees=15, max_depth=3, learn_rate=0.2)


def _frame(n=4000):
    g = torch.Generator().manual_seed(0)
    X = torch.randn((5, n), generator=g)
    X[2] = X[0] + 0.05 * torch.randn(n, generator=g)        # near copy of x0
    A = (torch.rand(n, generator=g) < 0.5).float()
    X[3] = A + 0.3 * torch.randn(n, generator=g)            # proxy of the protected attribute
    y = (torch.rand(n, generator=g) < torch.sigmoid(1.5 * X[0] + X[1] + A)).int()
    vecs = [Vec(f"x{i}", X[i], "real") for i in range(5)] + [Vec("a", A, "real"), Vec("y", y, ENUM, ["0", "1"])]
    return Frame(vecs)


def test_core_infogram():
    fr = _frame()
    m = H2OInfogram(algorithm_params=AP, seed=1).train(x=[f"x{i}" for i in range(5)], y="y", training_frame=fr)
    rows = {r["column"]: r for r in m.table}
    assert "x1" in m.get_admissible_features()
    assert "x4" not in m.get_admissible_features()
    # x0 / x2 carry the same information: neither adds much given the other
    assert rows["x0"]["net_information"] < 0.2 and rows["x2"]["net_information"] < 0.2
    assert rows["x0"]["total_information"] == 1.0
    sf = m.get_admissible_score_frame()
    assert sf.names == ["column", "admissible", "admissible_index", "total_information", "net_information", "cmi_raw"]
    assert len(m.get_admissible_cmi()) == len(m.get_admissible_features())


def test_fair_infogram():
    fr = _frame()
    m = H2OInfogram(algorithm_params=AP, seed=1, protected_columns=["a"]).train(
        x=[f"x{i}" for i in range(5)] + ["a"], y="y", training_frame=fr)
    adm = m.get_admissible_features()
    assert "x0" in adm and "x1" in adm
    assert "x3" not in adm and "a" not in [r["column"] for r in m.table]
    assert {"relevance_index", "safety_index"} <= set(m.table[0])
