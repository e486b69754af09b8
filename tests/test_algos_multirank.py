"""The newer estimators give the same model on 2 gloo ranks (row shards) as on
one rank: every statistic is combined with collectives."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, tmp_path, gpu=False):
    port = _port()
    procs, outs = [], []
    for r in range(world):
        out = tmp_path / f"alg{world}_{r}{'_gpu' if gpu else ''}.json"
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        if gpu:      # both ranks on the one GPU; gloo carries the collectives (RCCL needs one GPU per rank)
            env.update(H2OMX_WORKER_DEVICE="cuda", H2OMX_DIST_BACKEND="gloo", LOCAL_RANK="0")
        else:
            env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_algos_worker.py"), str(out)], env=env))
        outs.append(out)
    for p in procs:
        assert p.wait(timeout=300) == 0
    return [json.load(open(o)) for o in outs]


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    t = tmp_path_factory.mktemp("algos")
    return _run(1, t)[0], _run(2, t)


def test_two_ranks_match_one_rank(results):
    _compare(*results)


@pytest.mark.gpu
def test_two_ranks_match_one_rank_gpu(tmp_path):
    """Same estimators on the GPU: one rank vs two ranks sharing it (device tensors through the collectives)."""
    # fp32 device reductions see different row sets per rank: looser tolerances than the fp64 CPU run
    _compare(_run(1, tmp_path, gpu=True)[0], _run(2, tmp_path, gpu=True), f=1000.0)


def _compare(one, two, f=1.0):
    np.testing.assert_allclose(two[0]["te"] + two[1]["te"], one["te"], rtol=1e-6 * f)
    for r in two:
        np.testing.assert_allclose(r["svd_d"], one["svd_d"], rtol=1e-5 * f)
        np.testing.assert_allclose(r["glrm_obj"], one["glrm_obj"], rtol=1e-4 * f)
        np.testing.assert_allclose(r["iso"][0], one["iso"][0])
        np.testing.assert_allclose(r["iso"][1], one["iso"][1], rtol=1e-9 * f)
        np.testing.assert_allclose(r["cox"], one["cox"], rtol=1e-7 * f)
        assert [m[0] for m in r["ms"]] == [m[0] for m in one["ms"]]
        np.testing.assert_allclose([m[1] for m in r["ms"]], [m[1] for m in one["ms"]], rtol=1e-6 * f)
        for k, v in one["gam"].items():
            assert abs(r["gam"][k] - v) < 1e-3 * f * max(1.0, abs(v)), k
        np.testing.assert_allclose(r["anova"], one["anova"], rtol=1e-4 * f)
        np.testing.assert_allclose(r["auuc"], one["auuc"], rtol=1e-9 * f)
    np.testing.assert_allclose(two[0]["uplift"] + two[1]["uplift"], one["uplift"], rtol=1e-6 * f)
    np.testing.assert_allclose(two[0]["svm"] + two[1]["svm"], one["svm"], rtol=1e-4 * f, atol=1e-4 * f)
    assert two[0]["inter"] + two[1]["inter"] == one["inter"]
    for r in two:
        np.testing.assert_allclose(r["hglm"], one["hglm"], rtol=1e-7 * f, atol=1e-9 * f)
        np.testing.assert_allclose(r["cal_PlattScaling"], one["cal_PlattScaling"], rtol=1e-5 * f)
        xs, ys, xmin = r["cal_IsotonicRegression"]
        assert len(xs) == len(one["cal_IsotonicRegression"][0])
        np.testing.assert_allclose(xs, one["cal_IsotonicRegression"][0], rtol=1e-5 * f)
        # p1 of the 1- and 2-rank models agree to rounding, which can move a row
        # across a PAV block boundary: the fitted step values agree to ~1e-3
        np.testing.assert_allclose(ys, one["cal_IsotonicRegression"][1], atol=5e-3)
        for dist in ("laplace", "quantile"):
            assert r[f"init_{dist}"] == one[f"init_{dist}"], dist
        assert r["km_k"] == one["km_k"]
