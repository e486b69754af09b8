"""BASELINE config #1 end to end: an ``H2O`` custom resource (nodes: 1, CPU)
-> the operator renders Service + StatefulSet -> the fake kubelet runs the
RENDERED container command with the RENDERED env (POD_NAME from the
downward API, the H2O_* clustering contract, H2OMX_GPUS_PER_NODE) -> the pod
forms its cloud and answers ``/kubernetes/isLeaderNode`` -> the operator
reports the CR Ready -> a client imports iris over REST and trains GLM
binomial (versicolor vs the rest, unpenalised) and multinomial (ridge):
coefficients agree with scikit-learn's LogisticRegression to 1e-4.

The reference runs its deploy test against a live cluster
(``/root/reference/.github/workflows/rust.yml:18-25``,
``/root/reference/src/k8s/mod.rs:218-239``); the same flow on kind runs in
CI (.github/workflows/ci.yml, job ``kind-e2e``)."""
import os
import subprocess
import time
import urllib.request

import numpy as np
import pandas as pd
import pytest

from tests.fake_k8s import FakeK8s
from tests.fake_kubelet import FakeKubelet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTROL = os.path.join(ROOT, "control")
OPERATOR = os.path.join(CONTROL, "build", "h2omx-operator")


@pytest.fixture(scope="module")
def cloud(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("e2e")
    subprocess.run(["make", "-C", CONTROL, "-j8"], check=True, capture_output=True)
    k8s = FakeK8s(token="t0k").start()
    cfg = k8s.kubeconfig(str(tmp / "kubeconfig"), namespace="default")
    kubelet = FakeKubelet(str(tmp))
    k8s.kubelet = kubelet
    cr = {"apiVersion": "h2o.ai/v1beta", "kind": "H2O", "metadata": {"name": "iris"},
          "spec": {"nodes": 1, "version": "latest",
                   "resources": {"cpu": 2, "memory": "4Gi", "memoryPercentage": 50, "gpu": 0}}}
    k8s.put("h2os", "default", cr)
    try:
        r = subprocess.run([OPERATOR, "--kubeconfig", cfg, "--once"], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        info = kubelet.wait_ready("iris-stateful-set-0", timeout=240)
        yield {"k8s": k8s, "cfg": cfg, "kubelet": kubelet, "pod": info, "tmp": tmp}
    finally:
        kubelet.stop()
        k8s.stop()


def test_rendered_pod_runs_and_leader_probe(cloud):
    k8s, info = cloud["k8s"], cloud["pod"]
    sts = k8s.get("statefulsets", "default", "iris-stateful-set")
    c = sts["spec"]["template"]["spec"]["containers"][0]
    assert c["command"] == ["python3", "-m", "h2omx.runtime.node"]
    env = info["env"]
    # the env the process got is the rendered contract (ports remapped for localhost)
    assert env["POD_NAME"] == "iris-stateful-set-0"
    assert env["H2O_KUBERNETES_SERVICE_DNS"] == "iris-service.default.svc.cluster.local"
    assert env["H2O_NODE_EXPECTED_COUNT"] == "1" and env["H2OMX_GPUS_PER_NODE"] == "1"
    probe = c["readinessProbe"]["httpGet"]
    port = info["ports"][probe["port"]]
    with urllib.request.urlopen(f"http://127.0.0.1:{port}{probe['path']}", timeout=5) as r:
        assert r.status == 200
    # second operator pass: pod Ready -> CR Ready with the leader pod, and the
    # cloud's GPU topology / collective transport from the leader's /3/Cloud
    rest = info["ports"][54321]
    subprocess.run([OPERATOR, "--kubeconfig", cloud["cfg"], "--once"], check=True, capture_output=True, timeout=60,
                   env=dict(os.environ, H2OMX_OPERATOR_CLOUD_URL=f"http://127.0.0.1:{rest}"))
    st = k8s.get("h2os", "default", "iris")["status"]
    assert st["phase"] == "Ready" and st["leaderPod"] == "iris-stateful-set-0" and st["readyNodes"] == 1
    assert st["topology"]["world"] == 1 and st["topology"]["ok"] is True


def _iris_csv(tmp):
    from sklearn.datasets import load_iris

    d = load_iris(as_frame=True)
    df = d.frame.rename(columns={"sepal length (cm)": "sepal_len", "sepal width (cm)": "sepal_wid",
                                 "petal length (cm)": "petal_len", "petal width (cm)": "petal_wid"})
    df["species"] = np.array(d.target_names)[d.target]
    df["versicolor"] = np.where(df.species == "versicolor", "versicolor", "other")
    df = df.drop(columns=["target"])
    p = os.path.join(str(tmp), "iris.csv")
    df.to_csv(p, index=False)
    return p, df


X_COLS = ["sepal_len", "sepal_wid", "petal_len", "petal_wid"]


def test_glm_on_iris_over_rest_matches_sklearn(cloud):
    from sklearn.linear_model import LogisticRegression

    from h2omx.client import H2OConnection

    rest = cloud["pod"]["ports"][54321]
    conn = H2OConnection(f"http://127.0.0.1:{rest}")
    assert conn.connect()["cloud_size"] == 1
    path, df = _iris_csv(cloud["tmp"])
    key = conn.upload_file(path, destination_frame="iris.hex")
    fr = conn.frame(key)
    assert fr["rows"] == 150
    X = df[X_COLS].to_numpy(float)

    # binomial, unpenalised: versicolor vs the rest (not separable -> finite MLE)
    m = conn.train("glm", key, y="versicolor", x=X_COLS, family="binomial", **{"lambda": 0},
                   beta_epsilon=1e-12, objective_epsilon=1e-14, max_iterations=200)
    tab = m["output"]["coefficients_table"]
    coef = dict(zip(tab["names"], tab["coefficients"]))
    yb = (df.versicolor == "versicolor").to_numpy(int)
    sk = LogisticRegression(penalty=None, tol=1e-12, max_iter=100000).fit(X, yb)
    got = np.array([coef["Intercept"]] + [coef[c] for c in X_COLS])
    want = np.concatenate([sk.intercept_, sk.coef_[0]])
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-4)

    # multinomial, ridge: H2O's lambda (1 - alpha) / 2 ||b||^2 on the log-likelihood / N
    # equals sklearn's ||w||^2 / (2 C N) at lambda = 1 / (C N); raw (unstandardised) scale
    C, n = 1.0, len(df)
    m = conn.train("glm", key, y="species", x=X_COLS, family="multinomial", alpha=0.0,
                   **{"lambda": 1.0 / (C * n)}, standardize=False, beta_epsilon=1e-12, objective_epsilon=1e-14,
                   max_iterations=500)
    tab = m["output"]["coefficients_table"]
    B = np.array(tab["coefficients"])          # [K][1 + p]: intercept first
    sk = LogisticRegression(C=C, tol=1e-12, max_iter=100000).fit(X, df.species.to_numpy())
    want = np.concatenate([sk.intercept_[:, None], sk.coef_], 1)
    # the unpenalised intercepts are identified only up to a common shift
    # (softmax invariance); sklearn returns the zero-sum representative
    B[:, 0] -= B[:, 0].mean()
    np.testing.assert_allclose(B, want, rtol=1e-4, atol=1e-4)
    # the model scores through the same cloud
    pred = conn.predict(m["model_id"]["name"], key)
    acc = np.mean(np.array([c for c in conn.frame(pred, rows=150)["columns"][0]["data"]]) ==
                  np.searchsorted(sorted(df.species.unique()), df.species.to_numpy()))
    assert acc > 0.9
