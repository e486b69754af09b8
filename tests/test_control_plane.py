"""h2ok CLI + operator tests against the in-process fake Kubernetes API.

Ports every test of the reference (src/cli/mod.rs:282-329,
src/k8s/mod.rs:201-240, tests/integration_tests.rs of isgasho/h2o-kubernetes)
with the live K3s cluster replaced by tests/fake_k8s.py, plus coverage the
reference lacked (rollback, descriptor de-duplication, namespaces, TLS, the
operator).
"""
import json
import os
import re
import subprocess
import sys
import time

import pytest

from tests.fake_k8s import FakeK8s

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTROL = os.path.join(ROOT, "control")
H2OK = os.path.join(CONTROL, "build", "h2ok")
OPERATOR = os.path.join(CONTROL, "build", "h2omx-operator")
GENERAL_HELP = r"H2O Kubernetes CLI \d+.\d+.\d+.*"


@pytest.fixture(scope="session", autouse=True)
def built():
    subprocess.run(["make", "-C", CONTROL, "-j8"], check=True, capture_output=True)
    assert os.path.exists(H2OK) and os.path.exists(OPERATOR)


@pytest.fixture()
def k8s(tmp_path):
    srv = FakeK8s(token="s3cr3t").start()
    cfg = srv.kubeconfig(str(tmp_path / "kubeconfig"), namespace="default")
    srv.cfg = cfg
    yield srv
    srv.stop()


def run(args, cwd, stdin=None, env=None, timeout=60):
    e = dict(os.environ)
    e.pop("KUBECONFIG", None)
    e["HOME"] = str(cwd)
    if env:
        e.update(env)
    return subprocess.run([H2OK] + args, cwd=cwd, input=stdin, capture_output=True, text=True, timeout=timeout,
                          env=e)


# ---- tests/integration_tests.rs -------------------------------------------
def test_general_help(tmp_path):
    r = run(["-h"], tmp_path)
    assert r.returncode == 0
    assert re.match(GENERAL_HELP, r.stdout)


def test_general_help_no_flag(tmp_path):
    r = run([], tmp_path)
    assert r.returncode != 0
    assert re.match(GENERAL_HELP, r.stderr)


def test_deployment_help(tmp_path):
    r = run(["deploy", "-h"], tmp_path)
    assert r.returncode == 0
    assert re.match(r"h2ok-deploy.*", r.stdout)
    assert "--cluster_size <cluster_size>" in r.stdout and "[default: 50]" in r.stdout


def test_undeploy_help(tmp_path):
    r = run(["undeploy", "-h"], tmp_path)
    assert r.returncode == 0
    assert re.match(r"h2ok-undeploy.*\nUndeploys an existing H2O cluster from Kubernetes.*", r.stdout)


def test_deploy_undeploy(k8s, tmp_path):
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", k8s.cfg], tmp_path)
    assert r.returncode == 0, r.stderr
    assert re.match(r".*\.h2ok", r.stdout)
    descriptor = os.path.join(tmp_path, r.stdout.strip())
    r = run(["ingress", "-f", descriptor], tmp_path)
    assert r.returncode == 0, r.stderr
    assert len(k8s.list("ingresses")) == 1
    r = run(["undeploy", "-f", descriptor], tmp_path)
    assert r.returncode == 0, r.stderr
    assert re.match(r"Removed deployment 'h2o-.*", r.stdout)
    assert not os.path.exists(descriptor)
    assert k8s.list("services") == [] and k8s.list("statefulsets") == [] and k8s.list("ingresses") == []


def test_undeploy_piping(k8s, tmp_path):
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", k8s.cfg], tmp_path)
    assert r.returncode == 0, r.stderr
    r2 = run(["undeploy"], tmp_path, stdin=r.stdout)
    assert r2.returncode == 0, r2.stderr
    assert re.match(r"Removed deployment 'h2o-.*", r2.stdout)
    # trailing newline from `echo` is tolerated (Q8)
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", k8s.cfg], tmp_path)
    r2 = run(["undeploy"], tmp_path, stdin=r.stdout + "\n")
    assert r2.returncode == 0, r2.stderr


def test_undeploy_missing_deployment_descriptor(tmp_path):
    r = run(["undeploy"], tmp_path, stdin="nonexistent_file")
    assert r.returncode == 1
    assert re.search(r"Unable to process user input: UserInputError \{ kind: UnreachableDeploymentDescriptor \}",
                     r.stderr)
    r = run(["undeploy"], tmp_path, stdin="")
    assert r.returncode == 1
    assert "MissingDeploymentDescriptor" in r.stderr


# ---- src/cli/mod.rs unit tests -------------------------------------------------
def test_kubeconfig_path_and_namespace(k8s, tmp_path):
    r = run(["deploy", "--kubeconfig", k8s.cfg, "--cluster_size", "1", "--dry-run"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "namespace: default" in r.stdout  # kubeconfig default namespace
    r = run(["deploy", "--namespace", "non-default", "--cluster_size", "1", "--dry-run", "--kubeconfig", k8s.cfg],
            tmp_path)
    assert r.returncode == 0
    assert "namespace: non-default" in r.stdout
    r = run(["deploy", "--kubeconfig", str(tmp_path / "missing.yaml"), "--cluster_size", "1"], tmp_path)
    assert r.returncode == 1 and "Invalid file path" in r.stderr


def test_validate_number_range(tmp_path):
    base = ["deploy", "--cluster_size", "1", "--dry-run", "--cluster_name", "x1"]
    assert run(base + ["--memory_percentage", "10"], tmp_path).returncode == 0
    r = run(base + ["--memory_percentage", "101"], tmp_path)
    assert r.returncode == 1 and "withing range <0,100>" in r.stderr
    r = run(["deploy", "--cluster_size", "0"], tmp_path)
    assert r.returncode == 1 and "greater than zero" in r.stderr
    r = run(["deploy", "--cluster_size", "abc"], tmp_path)  # Q10: no panic
    assert r.returncode == 1 and "not an integer" in r.stderr
    r = run(["deploy", "--cluster_size", "1", "--memory", "1 GB"], tmp_path)
    assert r.returncode == 1 and "Memory requirement" in r.stderr
    r = run(["deploy"], tmp_path)
    assert r.returncode == 1 and "--cluster_size <cluster_size>" in r.stderr


# ---- src/k8s/mod.rs::test_deploy_h2o ---------------------------------------------
def test_deploy_h2o_objects(k8s, tmp_path):
    r = run(["deploy", "--kubeconfig", k8s.cfg, "--cluster_name", "h2o-k8s-test-cluster", "-p", "80", "-m",
             "256Mi", "--cpus", "2", "-s", "2"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert r.stdout == "h2o-k8s-test-cluster.h2ok"
    svcs, stss = k8s.list("services"), k8s.list("statefulsets")
    assert len(svcs) == 1 and len(stss) == 1 and k8s.list("ingresses") == []
    svc, sts = svcs[0], stss[0]
    assert svc["metadata"]["name"] == "h2o-k8s-test-cluster-service"
    assert svc["spec"]["clusterIP"] == "None" and svc["spec"]["publishNotReadyAddresses"] is True
    assert svc["spec"]["ports"][0]["port"] == 80 and svc["spec"]["ports"][0]["targetPort"] == 54321
    spec = sts["spec"]
    assert sts["metadata"]["name"] == "h2o-k8s-test-cluster-stateful-set"
    assert spec["serviceName"] == "h2o-k8s-test-cluster-service"
    assert spec["replicas"] == 2 and spec["podManagementPolicy"] == "Parallel"
    c = spec["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"] == {"cpu": "2", "memory": "256Mi", "amd.com/gpu": "1"}
    assert c["resources"]["requests"] == c["resources"]["limits"]
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["H2O_KUBERNETES_SERVICE_DNS"] == "h2o-k8s-test-cluster-service.default.svc.cluster.local"
    assert env["H2O_NODE_LOOKUP_TIMEOUT"] == "180" and env["H2O_NODE_EXPECTED_COUNT"] == "2"
    assert env["H2O_KUBERNETES_API_PORT"] == "8081" and env["H2OMX_MEMORY_PERCENTAGE"] == "80"
    probe = c["readinessProbe"]
    assert probe["httpGet"] == {"path": "/kubernetes/isLeaderNode", "port": 8081}
    assert (probe["initialDelaySeconds"], probe["periodSeconds"], probe["failureThreshold"]) == (5, 5, 1)
    desc = json.load(open(tmp_path / "h2o-k8s-test-cluster.h2ok"))
    assert list(desc) == ["specification", "ingresses", "stateful_sets", "services"]
    sp = desc["specification"]
    assert (sp["name"], sp["namespace"], sp["memory_percentage"], sp["memory"], sp["num_cpu"], sp["num_h2o_nodes"]) == \
        ("h2o-k8s-test-cluster", "default", 80, "256Mi", 2, 2)
    assert sp["kubeconfig_path"] == k8s.cfg
    # ingress with a load-balancer IP (watch loop), connection hints in the object
    r = run(["ingress", "-f", str(tmp_path / "h2o-k8s-test-cluster.h2ok")], tmp_path)
    assert r.returncode == 0
    desc = json.load(open(tmp_path / "h2o-k8s-test-cluster.h2ok"))
    assert len(desc["ingresses"]) == 1
    ing = desc["ingresses"][0]
    assert ing["status"]["loadBalancer"]["ingress"][0]["ip"] == "10.43.0.7"
    assert ing["spec"]["rules"][0]["http"]["paths"][0]["backend"]["service"]["name"] == "h2o-k8s-test-cluster-service"
    r = run(["status", "-f", str(tmp_path / "h2o-k8s-test-cluster.h2ok")], tmp_path)
    assert r.returncode == 0 and "2/2 pods, leader h2o-k8s-test-cluster-stateful-set-0" in r.stdout
    r = run(["undeploy", "-f", str(tmp_path / "h2o-k8s-test-cluster.h2ok")], tmp_path)
    assert r.returncode == 0
    assert k8s.list("services") == [] and k8s.list("statefulsets") == [] and k8s.list("ingresses") == []


def test_single_pod_eight_gpu_topology(tmp_path):
    """--cluster_size 1 --gpus_per_node 8: one pod holding the node's eight
    GPUs and eight ranks (the node entry point forks one per GPU); nothing is
    mounted over /dev/shm, so the host's shared memory stays visible to RCCL."""
    r = run(["deploy", "--cluster_size", "1", "--gpus_per_node", "8", "--dry-run", "-c", "single"], tmp_path)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "replicas: 1" in out and 'amd.com/gpu: "8"' in out
    assert "- name: H2OMX_GPUS_PER_NODE\n          value: \"8\"" in out
    assert "hostIPC: true" in out
    assert "/dev/shm" not in out and "emptyDir" not in out
    r = run(["deploy", "--cluster_size", "8", "--dry-run", "-c", "per-gpu"], tmp_path)
    assert "replicas: 8" in r.stdout and 'amd.com/gpu: "1"' in r.stdout and "/dev/shm" not in r.stdout


def test_rollback_on_statefulset_failure(k8s, tmp_path):
    k8s.fail[("POST", "statefulsets")] = 500
    r = run(["deploy", "--kubeconfig", k8s.cfg, "-c", "rb", "-s", "1"], tmp_path)
    assert r.returncode == 101
    assert "Rewinding existing deployment" in r.stderr
    assert k8s.list("services") == []  # service rolled back
    assert not os.path.exists(tmp_path / "rb.h2ok")


def test_descriptor_dedup_and_namespace(k8s, tmp_path):
    r1 = run(["deploy", "--kubeconfig", k8s.cfg, "-c", "dup", "-s", "1", "-n", "team-a"], tmp_path)
    r2 = run(["deploy", "--kubeconfig", k8s.cfg, "-c", "dup", "-s", "1", "-n", "team-b"], tmp_path)
    assert r1.returncode == 0 and r2.returncode == 0
    assert r1.stdout == "dup.h2ok" and r2.stdout == "dup(1).h2ok"  # Q4: real file name
    assert "Writing file" in r2.stderr  # Q5: diagnostics never pollute the pipe
    assert k8s.get("services", "team-a", "dup-service") and k8s.get("services", "team-b", "dup-service")
    assert run(["undeploy", "-f", str(tmp_path / "dup(1).h2ok")], tmp_path).returncode == 0
    assert k8s.get("services", "team-b", "dup-service") is None
    assert k8s.get("services", "team-a", "dup-service")


def test_partial_undeploy_keeps_descriptor(k8s, tmp_path):
    run(["deploy", "--kubeconfig", k8s.cfg, "-c", "part", "-s", "1"], tmp_path)
    k8s.fail[("DELETE", "statefulsets")] = 500
    r = run(["undeploy", "-f", str(tmp_path / "part.h2ok")], tmp_path)
    assert r.returncode == 2
    assert "Unable to undeploy 'part-stateful-set' - skipping." in r.stdout
    assert os.path.exists(tmp_path / "part.h2ok")  # Q7
    del k8s.fail[("DELETE", "statefulsets")]
    assert run(["undeploy", "-f", str(tmp_path / "part.h2ok")], tmp_path).returncode == 0


def test_kubeconfig_inference_and_bad_token(k8s, tmp_path):
    env = {"KUBECONFIG": k8s.cfg}
    r = run(["deploy", "-c", "infer", "-s", "1"], tmp_path, env=env)
    assert r.returncode == 0, r.stderr
    bad = k8s.kubeconfig(str(tmp_path / "bad"), token="wrong")
    r = run(["deploy", "-c", "nope", "-s", "1", "-k", bad], tmp_path)
    assert r.returncode == 101 and "401" in r.stderr
    r = run(["deploy", "-c", "nocfg", "-s", "1"], tmp_path)
    assert r.returncode == 101 and "No kubeconfig provided" in r.stderr


def test_tls_cluster(tmp_path):
    srv = FakeK8s(token="t", tls=True, tmpdir=str(tmp_path)).start()
    try:
        cfg = srv.kubeconfig(str(tmp_path / "kc"))
        r = run(["deploy", "-k", cfg, "-c", "tls", "-s", "1"], tmp_path)
        assert r.returncode == 0, r.stderr
        assert srv.get("statefulsets", "default", "tls-stateful-set")
        assert run(["undeploy", "-f", str(tmp_path / "tls.h2ok")], tmp_path).returncode == 0
    finally:
        srv.stop()


# ---- operator ------------------------------------------------------------------
def _cr(name, nodes=2, **spec):
    s = {"nodes": nodes, "version": "latest", "resources": {"cpu": 4, "memory": "64Gi", "memoryPercentage": 60,
                                                            "gpu": 1}}
    s.update(spec)
    return {"apiVersion": "h2o.ai/v1beta", "kind": "H2O", "metadata": {"name": name}, "spec": s}


def test_operator_reconcile(k8s, tmp_path):
    k8s.put("h2os", "default", _cr("h2o-op", nodes=3))
    r = subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    sts = k8s.get("statefulsets", "default", "h2o-op-stateful-set")
    svc = k8s.get("services", "default", "h2o-op-service")
    assert sts and svc
    assert sts["spec"]["replicas"] == 3
    cr = k8s.get("h2os", "default", "h2o-op")
    assert sts["metadata"]["ownerReferences"][0]["uid"] == cr["metadata"]["uid"]
    limits = sts["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]
    assert limits == {"cpu": "4", "memory": "64Gi", "amd.com/gpu": "1"}
    # second pass: pods exist (fake controller) -> status Ready with the leader
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    st = k8s.get("h2os", "default", "h2o-op")["status"]
    assert st["phase"] == "Ready" and st["readyNodes"] == 1 and st["leaderPod"] == "h2o-op-stateful-set-0"
    # spec change -> the fixed-size cloud is replaced.  The fake keeps a
    # foreground-deleted StatefulSet terminating for a while (409 on create),
    # like a real apiserver: the pass deletes it and reports Replacing ...
    cr = k8s.get("h2os", "default", "h2o-op")
    cr["spec"]["nodes"] = 5
    k8s.put("h2os", "default", cr, "MODIFIED")
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    old = k8s.get("statefulsets", "default", "h2o-op-stateful-set")
    assert old["spec"]["replicas"] == 3 and old["metadata"]["deletionTimestamp"]
    st = k8s.get("h2os", "default", "h2o-op")["status"]
    assert st["phase"] == "Replacing" and "terminate" in st["message"]
    # ... a pass while it is still terminating changes nothing (no 409 -> Failed)
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    assert k8s.get("h2os", "default", "h2o-op")["status"]["phase"] == "Replacing"
    # ... and once it is gone the new one is created; the stale message is cleared
    for _ in range(50):
        if k8s.get("statefulsets", "default", "h2o-op-stateful-set") is None:
            break
        time.sleep(0.05)
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    assert k8s.get("statefulsets", "default", "h2o-op-stateful-set")["spec"]["replicas"] == 5
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    st = k8s.get("h2os", "default", "h2o-op")["status"]
    assert st["phase"] == "Ready" and "message" not in st


def test_operator_watch_loop_replaces_statefulset(k8s, tmp_path):
    """The long-running operator requeues a CR whose StatefulSet is still
    terminating and converges without a spec event."""
    k8s.foreground_delay = 1.5
    p = subprocess.Popen([OPERATOR, "--kubeconfig", k8s.cfg, "--resync", "60", "--requeue", "1"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        k8s.put("h2os", "default", _cr("h2o-rq", nodes=2))
        for _ in range(100):
            if k8s.get("statefulsets", "default", "h2o-rq-stateful-set"):
                break
            time.sleep(0.05)
        cr = k8s.get("h2os", "default", "h2o-rq")
        cr["spec"]["nodes"] = 4
        k8s.put("h2os", "default", cr, "MODIFIED")
        for _ in range(200):
            s = k8s.get("statefulsets", "default", "h2o-rq-stateful-set")
            if s and s["spec"]["replicas"] == 4:
                break
            time.sleep(0.05)
        assert k8s.get("statefulsets", "default", "h2o-rq-stateful-set")["spec"]["replicas"] == 4
    finally:
        p.terminate()
        p.wait(timeout=10)


def test_operator_repairs_service_drift(k8s, tmp_path):
    k8s.put("h2os", "default", _cr("h2o-dr", nodes=1))
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    svc = k8s.get("services", "default", "h2o-dr-service")
    want_ports, want_sel = svc["spec"]["ports"], svc["spec"]["selector"]
    svc["spec"]["ports"] = [{"port": 8080, "targetPort": 1234, "protocol": "TCP"}]
    svc["spec"]["selector"] = {"app": "someone-else"}
    k8s.put("services", "default", svc, "MODIFIED")
    r = subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], capture_output=True, text=True, timeout=60)
    assert "drifted" in r.stdout
    svc = k8s.get("services", "default", "h2o-dr-service")
    assert svc["spec"]["ports"] == want_ports and svc["spec"]["selector"] == want_sel
    # an unchanged service is left alone
    n = len(k8s.requests)
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    assert not any(m == "PATCH" and "/services/" in path for m, path in k8s.requests[n:])


@pytest.mark.parametrize("api", ["networking.k8s.io/v1", "networking.k8s.io/v1beta1"])
def test_operator_ingress_from_cr(k8s, tmp_path, api):
    """spec.ingress: the operator owns <name>-ingress (h2ok's ingress verb) and
    publishes the load-balancer address in status; disabling removes it."""
    plural = "ingresses"
    k8s.put("h2os", "default", _cr("h2o-in", nodes=1, ingress={"enabled": True, "apiVersion": api}))
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    ing = k8s.get(plural, "default", "h2o-in-ingress")
    assert ing and ing["apiVersion"] == api
    cr = k8s.get("h2os", "default", "h2o-in")
    assert ing["metadata"]["ownerReferences"][0]["uid"] == cr["metadata"]["uid"]
    assert cr["status"]["ingressIP"] == ""            # load balancer not there yet
    time.sleep(0.6)                                   # fake LB assigns 10.43.0.7
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    st = k8s.get("h2os", "default", "h2o-in")["status"]
    assert st["ingressIP"] == "10.43.0.7" and st["connectURL"] == "http://10.43.0.7:80/h2o-in"
    assert st["ingressPath"].startswith("/h2o-in")
    cr = k8s.get("h2os", "default", "h2o-in")
    cr["spec"]["ingress"]["enabled"] = False
    k8s.put("h2os", "default", cr, "MODIFIED")
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    assert k8s.get(plural, "default", "h2o-in-ingress") is None
    assert "ingressIP" not in k8s.get("h2os", "default", "h2o-in")["status"]


def test_operator_watch_loop(k8s, tmp_path):
    p = subprocess.Popen([OPERATOR, "--kubeconfig", k8s.cfg, "--resync", "2"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        k8s.put("h2os", "default", _cr("h2o-w", nodes=1))
        for _ in range(50):
            if k8s.get("statefulsets", "default", "h2o-w-stateful-set"):
                break
            time.sleep(0.1)
        assert k8s.get("statefulsets", "default", "h2o-w-stateful-set")
        k8s.delete("h2os", "default", "h2o-w")
        for _ in range(50):
            if not k8s.get("statefulsets", "default", "h2o-w-stateful-set"):
                break
            time.sleep(0.1)
        assert k8s.get("statefulsets", "default", "h2o-w-stateful-set") is None
    finally:
        p.terminate()
        p.wait(timeout=10)


def test_crd_manifest_matches_operator():
    from tests.yamlio import load_all

    docs = load_all(os.path.join(ROOT, "deploy", "crd.yaml"))
    crd = docs[0]
    assert crd["spec"]["group"] == "h2o.ai" and crd["spec"]["names"]["plural"] == "h2os"
    v = crd["spec"]["versions"][0]
    assert v["name"] == "v1beta" and "status" in v["subresources"]
    props = v["schema"]["openAPIV3Schema"]["properties"]
    assert set(props["spec"]["properties"]["ingress"]["properties"]) == {"enabled", "apiVersion", "className"}
    for k in ("ingressIP", "ingressPath", "connectURL", "message"):
        assert k in props["status"]["properties"]
    # a structural schema prunes undeclared status fields on a real apiserver:
    # every key the operator writes must be declared, the free-form topology
    # object with preserve-unknown-fields
    import re

    src = open(os.path.join(ROOT, "control", "src", "operator_main.cpp")).read()
    written = set(re.findall(r'st\["(\w+)"\]', src))
    assert written and written <= set(props["status"]["properties"]), written - set(props["status"]["properties"])
    topo = props["status"]["properties"]["topology"]
    assert topo["type"] == "object" and topo["x-kubernetes-preserve-unknown-fields"] is True


# ---- kubeconfig credential plugins (kube-rs Config::infer parity) ---------------
_PLUGIN = r'''
import json, os, sys
state = sys.argv[1]
n = int(open(state).read()) if os.path.exists(state) else 0
open(state, "w").write(str(n + 1))
info = json.loads(os.environ["KUBERNETES_EXEC_INFO"])
open(state + ".info", "w").write(json.dumps(info))
if os.environ.get("PLUGIN_FAIL"):
    sys.stderr.write("token service unreachable\n")
    sys.exit(3)
tokens = os.environ["PLUGIN_TOKENS"].split(",")
print(json.dumps({"apiVersion": info["apiVersion"], "kind": "ExecCredential",
                  "status": {"token": tokens[min(n, len(tokens) - 1)],
                             "expirationTimestamp": "2099-01-01T00:00:00Z"}}))
'''


def _exec_kubeconfig(k8s, tmp_path, tokens, fail=False):
    plugin = tmp_path / "plugin.py"
    plugin.write_text(_PLUGIN)
    state = tmp_path / "calls"
    env = [("PLUGIN_TOKENS", ",".join(tokens))] + ([("PLUGIN_FAIL", "1")] if fail else [])
    lines = ["apiVersion: v1", "kind: Config", "clusters:", "- cluster:", f"    server: {k8s.url}", "  name: fake",
             "contexts:", "- context:", "    cluster: fake", "    user: eks-user", "    namespace: default",
             "  name: ctx", "current-context: ctx", "users:", "- name: eks-user", "  user:", "    exec:",
             "      apiVersion: client.authentication.k8s.io/v1beta1", f"      command: {sys.executable}",
             "      args:", f"      - {plugin}", f"      - {state}", "      env:"]
    for k, v in env:
        lines += [f"      - name: {k}", f"        value: \"{v}\""]
    lines += ["      provideClusterInfo: true", "      installHint: install the fake plugin"]
    cfg = tmp_path / "exec-kubeconfig"
    cfg.write_text("\n".join(lines) + "\n")
    return str(cfg), state


def test_exec_plugin_credentials(k8s, tmp_path):
    cfg, state = _exec_kubeconfig(k8s, tmp_path, ["s3cr3t"])
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", cfg], tmp_path)
    assert r.returncode == 0, r.stderr
    assert len(k8s.list("statefulsets")) == 1
    assert int(state.read_text()) == 1                # cached for the whole run (expiry 2099)
    info = json.loads(open(str(state) + ".info").read())
    assert info["kind"] == "ExecCredential" and info["apiVersion"] == "client.authentication.k8s.io/v1beta1"
    assert info["spec"]["interactive"] is False and info["spec"]["cluster"]["server"] == k8s.url


def test_exec_plugin_refreshes_after_401(k8s, tmp_path):
    cfg, state = _exec_kubeconfig(k8s, tmp_path, ["stale-token", "s3cr3t"])
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", cfg], tmp_path)
    assert r.returncode == 0, r.stderr
    assert int(state.read_text()) == 2


def test_exec_plugin_failure_is_reported(k8s, tmp_path):
    cfg, _ = _exec_kubeconfig(k8s, tmp_path, ["x"], fail=True)
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", cfg], tmp_path)
    assert r.returncode != 0
    assert "token service unreachable" in r.stderr and "status 3" in r.stderr
    assert k8s.list("statefulsets") == []


def test_auth_provider_oidc_token(k8s, tmp_path):
    lines = ["apiVersion: v1", "kind: Config", "clusters:", "- cluster:", f"    server: {k8s.url}", "  name: fake",
             "contexts:", "- context:", "    cluster: fake", "    user: oidc", "  name: ctx", "current-context: ctx",
             "users:", "- name: oidc", "  user:", "    auth-provider:", "      name: oidc", "      config:",
             "        id-token: s3cr3t", "        idp-issuer-url: https://issuer"]
    cfg = tmp_path / "oidc-kubeconfig"
    cfg.write_text("\n".join(lines) + "\n")
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", str(cfg)], tmp_path)
    assert r.returncode == 0, r.stderr


# ---- sanitizers: the control plane under ASan + UBSan -------------
def test_control_plane_under_asan_ubsan(k8s, tmp_path):
    """`make -C control asan` builds h2ok / h2omx-operator with
    -fsanitize=address,undefined; the deploy -> ingress -> undeploy flow, an
    exec-plugin login and an operator pass run clean (no sanitizer report,
    leak checking on)."""
    subprocess.run(["make", "-C", CONTROL, "asan", "-j8"], check=True, capture_output=True, timeout=900)
    h2ok = os.path.join(CONTROL, "build-asan", "h2ok")
    op = os.path.join(CONTROL, "build-asan", "h2omx-operator")
    env = dict(os.environ, HOME=str(tmp_path), ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("KUBECONFIG", None)

    def go(args, **kw):
        r = subprocess.run(args, cwd=tmp_path, capture_output=True, text=True, timeout=120, env=env, **kw)
        for bad in ("AddressSanitizer", "LeakSanitizer", "runtime error:"):
            assert bad not in r.stderr, r.stderr[-4000:]
        return r

    r = go([h2ok, "deploy", "--cluster_size", "2", "--kubeconfig", k8s.cfg])
    assert r.returncode == 0, r.stderr
    d = os.path.join(tmp_path, r.stdout.strip())
    assert go([h2ok, "ingress", "-f", d]).returncode == 0
    assert go([h2ok, "undeploy"], input=d).returncode == 0
    assert go([h2ok, "deploy", "--cluster_size", "x"]).returncode == 1        # validator error path
    cfg, _ = _exec_kubeconfig(k8s, tmp_path, ["s3cr3t"])
    assert go([h2ok, "deploy", "--cluster_size", "1", "--kubeconfig", cfg]).returncode == 0
    k8s.put("h2os", "default", _cr("h2o-asan", nodes=2, ingress={"enabled": True}))
    assert go([op, "--kubeconfig", k8s.cfg, "--once"]).returncode == 0
    assert k8s.get("statefulsets", "default", "h2o-asan-stateful-set")


def test_ci_and_release_workflows():
    """CI builds + tests the control plane (also under ASan/UBSan) and the CPU
    suite with gfx950 kernels; tags produce packaged binaries (reference
    .github/workflows/rust.yml, release.yml)."""
    from tests.yamlio import load_all

    ci = load_all(os.path.join(ROOT, ".github", "workflows", "ci.yml"))[0]
    steps = " ".join(str(s.get("run", "")) for j in ci["jobs"].values() for s in j["steps"])
    assert "make -C control asan" in steps and 'pytest tests -x -q -m "not gpu"' in steps
    assert "-m gpu" in steps and "bench.py" in steps
    rel = load_all(os.path.join(ROOT, ".github", "workflows", "release.yml"))[0]
    trigger = rel.get("on", rel.get(True))          # YAML 1.1 reads the key `on` as true
    assert trigger["push"]["tags"] == ["v*"]
    rsteps = " ".join(str(s.get("run", "")) for j in rel["jobs"].values() for s in j["steps"])
    assert "make -C control package" in rsteps and "gh release create" in rsteps
    # BASELINE config #1 on a kind cluster; h2ok also ships for macOS
    assert "scripts/e2e/iris_glm_rest.py" in steps and "kind load docker-image" in steps
    assert any("macos" in str(j.get("runs-on", "")) or "macos" in str(j.get("strategy", ""))
               for j in rel["jobs"].values())


# ---- Traefik v2 ingress (K3s, the reference CI's cluster: rust.yml:18-20) -----------
def test_traefik_v2_ingress(k8s, tmp_path):
    """--ingress_class traefik: a Prefix route on /<name> plus a StripPrefix
    Middleware CR referenced by the router annotation (Traefik v2 ignores v1's
    PathPrefixStrip annotation and takes a regex path literally); undeploy
    removes the middleware too."""
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", k8s.cfg, "-c", "h2o-tr", "--ingress_class", "traefik"],
            tmp_path)
    assert r.returncode == 0, r.stderr
    desc = str(tmp_path / "h2o-tr.h2ok")
    r = run(["ingress", "-f", desc], tmp_path)
    assert r.returncode == 0, r.stderr
    mws = k8s.list("middlewares")
    assert len(mws) == 1
    mw = mws[0]
    assert mw["apiVersion"] == "traefik.io/v1alpha1" and mw["metadata"]["name"] == "h2o-tr-stripprefix"
    assert mw["spec"] == {"stripPrefix": {"prefixes": ["/h2o-tr"]}}
    assert any(m == "POST" and p.startswith("/apis/traefik.io/v1alpha1/namespaces/default/middlewares")
               for m, p in k8s.requests)
    ing = k8s.list("ingresses")[0]
    path = ing["spec"]["rules"][0]["http"]["paths"][0]
    assert path["path"] == "/h2o-tr" and path["pathType"] == "Prefix"
    assert ing["spec"]["ingressClassName"] == "traefik"
    ann = ing["metadata"]["annotations"]
    assert ann == {"traefik.ingress.kubernetes.io/router.middlewares": "default-h2o-tr-stripprefix@kubernetescrd"}
    d = json.load(open(desc))
    assert d["specification"]["ingress_class"] == "traefik" and len(d["middlewares"]) == 1
    r = run(["undeploy", "-f", desc], tmp_path)
    assert r.returncode == 0, r.stderr
    assert k8s.list("middlewares") == [] and k8s.list("ingresses") == []
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", k8s.cfg, "--ingress_class", "haproxy"], tmp_path)
    assert r.returncode != 0 and "ingress class" in r.stderr


def test_nginx_ingress_class_keeps_regex_route(k8s, tmp_path):
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", k8s.cfg, "-c", "h2o-nx", "--ingress_class", "nginx"],
            tmp_path)
    assert r.returncode == 0, r.stderr
    r = run(["ingress", "-f", str(tmp_path / "h2o-nx.h2ok")], tmp_path)
    assert r.returncode == 0, r.stderr
    ing = k8s.list("ingresses")[0]
    assert ing["spec"]["ingressClassName"] == "nginx"
    assert ing["spec"]["rules"][0]["http"]["paths"][0]["path"] == "/h2o-nx(/|$)(.*)"
    assert k8s.list("middlewares") == []


def test_operator_traefik_ingress_from_cr(k8s, tmp_path):
    k8s.put("h2os", "default", _cr("h2o-otr", nodes=1, ingress={"enabled": True, "className": "traefik"}))
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    mw = k8s.get("middlewares", "default", "h2o-otr-stripprefix")
    assert mw and mw["spec"]["stripPrefix"]["prefixes"] == ["/h2o-otr"]
    ing = k8s.get("ingresses", "default", "h2o-otr-ingress")
    assert ing["spec"]["rules"][0]["http"]["paths"][0]["pathType"] == "Prefix"
    cr = k8s.get("h2os", "default", "h2o-otr")
    cr["spec"]["ingress"]["enabled"] = False
    k8s.put("h2os", "default", cr, "MODIFIED")
    subprocess.run([OPERATOR, "--kubeconfig", k8s.cfg, "--once"], check=True, capture_output=True, timeout=60)
    assert k8s.get("middlewares", "default", "h2o-otr-stripprefix") is None
    assert k8s.get("ingresses", "default", "h2o-otr-ingress") is None


# ---- RBAC-enforcing apiserver (deploy/operator.yaml's ClusterRole) -------------------
_OPERATOR_YAML = os.path.join(ROOT, "deploy", "operator.yaml")
_TRAEFIK_CLASS = {"apiVersion": "networking.k8s.io/v1", "kind": "IngressClass",
                  "metadata": {"name": "traefik",
                               "annotations": {"ingressclass.kubernetes.io/is-default-class": "true"}},
                  "spec": {"controller": "traefik.io/ingress-controller"}}


@pytest.fixture()
def k3s_rbac(tmp_path):
    """A K3s-like cluster: Traefik CRDs served, Traefik the default IngressClass,
    and every request authorised against the operator's shipped ClusterRole."""
    from tests.fake_k8s import cluster_role_rules

    srv = FakeK8s(token="s3cr3t", rbac_rules=cluster_role_rules(_OPERATOR_YAML)).start()
    srv.put("ingressclasses", "", copy_obj(_TRAEFIK_CLASS))
    srv.cfg = srv.kubeconfig(str(tmp_path / "kubeconfig"), namespace="default")
    yield srv
    srv.stop()


def copy_obj(o):
    return json.loads(json.dumps(o))


def _op_once(srv):
    return subprocess.run([OPERATOR, "--kubeconfig", srv.cfg, "--once"], capture_output=True, text=True, timeout=60)


def test_fake_apiserver_enforces_rbac(tmp_path):
    """The enforcement itself: outside the rules a request is 403 (before
    routing, so even an unserved group), inside them it is served."""
    from tests.fake_k8s import cluster_role_rules

    rules = [r for r in cluster_role_rules(_OPERATOR_YAML) if "middlewares" not in r["resources"]]
    srv = FakeK8s(rbac_rules=rules, served_groups={"apps", "networking.k8s.io", "h2o.ai"}).start()
    try:
        import urllib.error
        import urllib.request

        def code(path, method="GET"):
            try:
                return urllib.request.urlopen(urllib.request.Request(srv.url + path, method=method)).status
            except urllib.error.HTTPError as e:
                return e.code

        assert code("/apis/traefik.io/v1alpha1/namespaces/default/middlewares/x") == 403
        assert code("/api/v1/namespaces/default/secrets/x") == 403
        assert code("/api/v1/namespaces/default/services/x") == 404      # allowed, absent
        assert code("/apis/networking.k8s.io/v1/ingressclasses") == 200
        assert code("/apis/apps/v1/namespaces/default/statefulsets/x", "PUT") == 403   # no "update"
        assert ("get", "traefik.io", "middlewares") in srv.forbidden
    finally:
        srv.stop()


def test_operator_under_rbac_ingress_modes(k3s_rbac):
    """Round-5 regression: with the Traefik CRDs present, every CR ended
    phase Failed because the operator GET the middlewares its role did not
    grant.  Under the shipped ClusterRole a CR with ingress disabled, an
    nginx-class and a traefik-class CR all reach Ready; only the traefik CR
    touches middlewares, and its middleware is owned by the CR (garbage-
    collected with it)."""
    srv = k3s_rbac
    srv.put("h2os", "default", _cr("h2o-off", nodes=1))
    srv.put("h2os", "default", _cr("h2o-ngx", nodes=1, ingress={"enabled": True, "className": "nginx"}))
    srv.put("h2os", "default", _cr("h2o-trf", nodes=1, ingress={"enabled": True, "className": "traefik"}))
    for _ in range(2):
        r = _op_once(srv)
        assert r.returncode == 0, r.stderr
    assert srv.forbidden == [], srv.forbidden
    for n in ("h2o-off", "h2o-ngx", "h2o-trf"):
        st = srv.get("h2os", "default", n)["status"]
        assert st["phase"] == "Ready", (n, st)
    mw_paths = [p for m, p in srv.requests if "/middlewares" in p]
    assert mw_paths and all("h2o-trf" in p or p.endswith("/middlewares") for p in mw_paths), mw_paths
    ngx = srv.get("ingresses", "default", "h2o-ngx-ingress")
    assert ngx["spec"]["ingressClassName"] == "nginx"
    assert ngx["spec"]["rules"][0]["http"]["paths"][0]["path"] == "/h2o-ngx(/|$)(.*)"
    mw = srv.get("middlewares", "default", "h2o-trf-stripprefix")
    cr = srv.get("h2os", "default", "h2o-trf")
    assert mw["metadata"]["ownerReferences"][0]["uid"] == cr["metadata"]["uid"]
    assert cr["status"]["ingressMiddleware"] == "h2o-trf-stripprefix"
    # ingress switched off: the recorded middleware goes, the status forgets it
    cr["spec"]["ingress"]["enabled"] = False
    srv.put("h2os", "default", cr, "MODIFIED")
    assert _op_once(srv).returncode == 0
    assert srv.get("middlewares", "default", "h2o-trf-stripprefix") is None
    st = srv.get("h2os", "default", "h2o-trf")["status"]
    assert st["phase"] == "Ready" and "ingressMiddleware" not in st
    # back on, then the CR deleted: the fake's GC removes the owned middleware
    cr = srv.get("h2os", "default", "h2o-trf")
    cr["spec"]["ingress"]["enabled"] = True
    srv.put("h2os", "default", cr, "MODIFIED")
    assert _op_once(srv).returncode == 0
    assert srv.get("middlewares", "default", "h2o-trf-stripprefix") is not None
    srv.delete("h2os", "default", "h2o-trf")
    assert srv.get("middlewares", "default", "h2o-trf-stripprefix") is None
    assert srv.forbidden == [], srv.forbidden


def test_operator_default_ingress_class_is_traefik(k3s_rbac):
    """A CR that names no className follows the cluster's default IngressClass
    (K3s: Traefik) - Prefix route + StripPrefix middleware, no class named."""
    srv = k3s_rbac
    srv.put("h2os", "default", _cr("h2o-dft", nodes=1, ingress={"enabled": True}))
    assert _op_once(srv).returncode == 0
    ing = srv.get("ingresses", "default", "h2o-dft-ingress")
    path = ing["spec"]["rules"][0]["http"]["paths"][0]
    assert path["path"] == "/h2o-dft" and path["pathType"] == "Prefix"
    assert "ingressClassName" not in ing["spec"]
    ann = {k: v for k, v in ing["metadata"]["annotations"].items() if not k.startswith("h2o.ai/")}
    assert ann == {"traefik.ingress.kubernetes.io/router.middlewares": "default-h2o-dft-stripprefix@kubernetescrd"}
    assert srv.get("middlewares", "default", "h2o-dft-stripprefix") is not None
    assert srv.get("h2os", "default", "h2o-dft")["status"]["phase"] == "Ready"
    assert srv.forbidden == []


def test_operator_rbac_without_middleware_rule_fails_only_traefik(tmp_path):
    """Negative control: a role without the middleware rule fails exactly the
    Traefik CR (403 in its status message), not the others."""
    from tests.fake_k8s import cluster_role_rules

    rules = [r for r in cluster_role_rules(_OPERATOR_YAML) if "middlewares" not in r["resources"]]
    srv = FakeK8s(rbac_rules=rules).start()
    try:
        srv.cfg = srv.kubeconfig(str(tmp_path / "kubeconfig"), namespace="default")
        srv.put("h2os", "default", _cr("h2o-a", nodes=1))
        srv.put("h2os", "default", _cr("h2o-t", nodes=1, ingress={"enabled": True, "className": "traefik"}))
        assert _op_once(srv).returncode == 0
        assert _op_once(srv).returncode == 0
        assert srv.get("h2os", "default", "h2o-a")["status"]["phase"] == "Ready"
        st = srv.get("h2os", "default", "h2o-t")["status"]
        assert st["phase"] == "Failed" and "forbidden" in st["message"].lower(), st
    finally:
        srv.stop()


def test_h2ok_ingress_follows_default_ingress_class(k3s_rbac, tmp_path):
    """`h2ok ingress` with no --ingress_class on a cluster whose default class
    is Traefik (K3s, the reference CI: rust.yml:18-20) emits the Prefix +
    StripPrefix pair; undeploy removes both."""
    srv = k3s_rbac
    r = run(["deploy", "--cluster_size", "1", "--kubeconfig", srv.cfg, "-c", "h2o-k3s"], tmp_path)
    assert r.returncode == 0, r.stderr
    desc = str(tmp_path / "h2o-k3s.h2ok")
    r = run(["ingress", "-f", desc], tmp_path)
    assert r.returncode == 0, r.stderr
    ing = srv.get("ingresses", "default", "h2o-k3s-ingress")
    path = ing["spec"]["rules"][0]["http"]["paths"][0]
    assert path["path"] == "/h2o-k3s" and path["pathType"] == "Prefix"
    assert "ingressClassName" not in ing["spec"]
    mw = srv.get("middlewares", "default", "h2o-k3s-stripprefix")
    assert mw["spec"] == {"stripPrefix": {"prefixes": ["/h2o-k3s"]}}
    d = json.load(open(desc))
    assert "ingress_class" not in d["specification"] and len(d["middlewares"]) == 1
    r = run(["undeploy", "-f", desc], tmp_path)
    assert r.returncode == 0, r.stderr
    assert srv.list("middlewares") == [] and srv.list("ingresses") == []
    # no default class (or classes unreadable): the nginx-style regex route, as before
    srv.delete("ingressclasses", "", "traefik")
    run(["deploy", "--cluster_size", "1", "--kubeconfig", srv.cfg, "-c", "h2o-nod"], tmp_path)
    assert run(["ingress", "-f", str(tmp_path / "h2o-nod.h2ok")], tmp_path).returncode == 0
    ing = srv.get("ingresses", "default", "h2o-nod-ingress")
    assert ing["spec"]["rules"][0]["http"]["paths"][0]["path"] == "/h2o-nod(/|$)(.*)"
