"""Cloud-formation peer / transport check (h2omx/runtime/topology.py)."""
import pytest

from h2omx.runtime.topology import assess, check_cloud


def _r(host, dev, visible, row=None):
    return {"host": host, "device": dev, "visible": visible, "peer_row": row if row is not None else [True] * visible}


def test_one_pod_eight_ranks_all_peers():
    rep = assess([_r("n0", i, 8) for i in range(8)])
    assert rep["ok"] and rep["hosts"]["n0"]["p2p"] == "all pairs peer-accessible"


def test_pod_per_gpu_without_peer_visibility_is_flagged():
    rep = assess([_r(f"n0", 0, 1) for _ in range(4)])
    assert not rep["ok"]
    assert rep["hosts"]["n0"]["p2p"] == "not visible"
    assert "pod-per-GPU" in rep["problems"][0]


def test_partial_peer_access_is_flagged():
    rows = [[True, True, False, True], [True, True, True, True], [False, True, True, True], [True] * 4]
    rep = assess([_r("n0", i, 4, rows[i]) for i in range(4)])
    assert rep["hosts"]["n0"]["p2p"] == "partial" and not rep["ok"]


def test_single_rank_per_host_and_cpu_ranks():
    rep = assess([_r("a", 0, 1), _r("b", 0, 1), {"host": "c", "device": None, "visible": 0}])
    assert rep["ok"]
    assert all(e["p2p"].startswith("n/a") for e in rep["hosts"].values())


class _FakeComm:
    def __init__(self, infos):
        self.world_size, self.rank, self.device, self._infos = len(infos), 0, None, infos

    def all_gather_object(self, obj):
        return self._infos


def test_required_p2p_fails_formation_loudly():
    comm = _FakeComm([_r("n0", 0, 1), _r("n0", 0, 1)])
    logs = []
    rep = check_cloud(comm, require=False, probe_mb=0, log=logs.append)
    assert not rep["ok"] and any("WARNING" in m for m in logs)
    with pytest.raises(RuntimeError, match="H2OMX_REQUIRE_P2P"):
        check_cloud(comm, require=True, probe_mb=0, log=logs.append)


def test_ranks_sharing_one_gpu_are_reported_as_such():
    infos = [dict(_r("n0", 0, 1), gpu_id="GPU-A") for _ in range(2)]
    rep = assess(infos)
    assert rep["hosts"]["n0"]["p2p"] == "shared device"


def test_cloud_summary_for_rest_and_operator():
    from h2omx.parallel.comm import Comm
    from h2omx.runtime.topology import cloud_summary

    rep = assess([_r("n0", 0, 1) for _ in range(2)])
    out = cloud_summary(rep, Comm(0, 1))
    assert out["world"] == 2 and out["ok"] is False and out["p2p"] == {"n0": "not visible"}
    assert out["problems"] and out["collectives"] == "none (1 rank)"
    assert cloud_summary(None)["ok"] is True
