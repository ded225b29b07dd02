"""kubeadm phases, configuration and upgrade policy without a cluster (cmd/kubeadm/app/cmd/phases/
*_test.go, app/phases/upgrade/policy_test.go, app/cmd/config_test.go)."""
from __future__ import annotations

import os
import re
import subprocess
import sys

import yaml

from amdkube import GIT_VERSION
from amdkube.kubeadm.phases import _with_extra, apiserver_sans, dns_ip, master_config, merge_config
from amdkube.kubeadm.upgrade import enforce_policy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kubeadm(*args):
    r = subprocess.run([sys.executable, "-m", "amdkube", "kubeadm", *args], cwd=ROOT, capture_output=True, text=True,
                       timeout=120, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _san(crt):
    return subprocess.run(["openssl", "x509", "-in", crt, "-noout", "-ext", "subjectAltName"], capture_output=True,
                          text=True, check=True).stdout


def _subject(crt):
    return subprocess.run(["openssl", "x509", "-in", crt, "-noout", "-subject", "-issuer"], capture_output=True,
                          text=True, check=True).stdout


def test_phases_one_by_one(tmp_path):
    base = str(tmp_path / "k")
    cfg = tmp_path / "cluster.yaml"
    cfg.write_text(yaml.safe_dump({"apiVersion": "kubeadm.k8s.io/v1alpha1", "kind": "MasterConfiguration",
                                   "api": {"advertiseAddress": "10.1.2.3", "bindPort": 7443},
                                   "networking": {"serviceSubnet": "10.100.0.0/16", "podSubnet": "10.244.0.0/16"},
                                   "apiServerCertSANs": ["gpu-master.example", "192.168.7.7"],
                                   "apiServerExtraArgs": {"max-requests-inflight": "800"},
                                   "schedulerExtraArgs": {"kube-api-qps": "300"},
                                   "featureGates": {"GPUTopologyScheduling": True}}))
    common = ["--base-dir", base, "--config", str(cfg), "--node-name", "mi355x-0"]
    out = _kubeadm("alpha", "phase", "certs", "all", *common)
    assert "front-proxy-ca" in out and "front-proxy-client" in out
    pki = os.path.join(base, "pki")
    sans = _san(f"{pki}/apiserver.crt")
    for want in ("IP Address:10.1.2.3", "IP Address:10.100.0.1", "DNS:gpu-master.example", "IP Address:192.168.7.7",
                 "DNS:kubernetes.default.svc.cluster.local", "DNS:mi355x-0"):
        assert want in sans, (want, sans)
    assert "CN = front-proxy-client" in _subject(f"{pki}/front-proxy-client.crt")
    assert "issuer=CN = front-proxy-ca" in _subject(f"{pki}/front-proxy-client.crt")
    # re-running keeps what exists
    assert "nothing (all present)" in _kubeadm("alpha", "phase", "certs", "all", *common)
    _kubeadm("alpha", "phase", "kubeconfig", "all", *common)
    kc = yaml.safe_load(open(os.path.join(base, "kubelet.conf")))
    assert kc["clusters"][0]["cluster"]["server"] == "https://10.1.2.3:7443"
    assert kc["users"][0]["name"] == "system:node:mi355x-0"
    user = yaml.safe_load(_kubeadm("alpha", "phase", "kubeconfig", "user", "--client-name", "alice", "--client-org", "ml",
                                   *common))
    assert user["users"][0]["name"] == "alice"
    _kubeadm("alpha", "phase", "controlplane", "all", *common)
    api = yaml.safe_load(open(os.path.join(base, "manifests", "kube-apiserver.yaml")))
    args = api["spec"]["containers"][0]["args"]
    val = lambda f: args[args.index(f) + 1]  # noqa: E731
    assert val("--max-requests-inflight") == "800" and val("--port") == "7443"
    assert val("--requestheader-client-ca-file").endswith("front-proxy-ca.crt")
    assert val("--proxy-client-cert-file").endswith("front-proxy-client.crt")
    assert "ResourceV2" in val("--admission-control")
    assert api["metadata"]["annotations"]["amdkube.io/kubernetes-version"] == GIT_VERSION
    sched = yaml.safe_load(open(os.path.join(base, "manifests", "kube-scheduler.yaml")))["spec"]["containers"][0]["args"]
    assert sched[sched.index("--kube-api-qps") + 1] == "300"
    assert sched[sched.index("--feature-gates") + 1] == "GPUTopologyScheduling=true"
    cm = yaml.safe_load(open(os.path.join(base, "manifests", "kube-controller-manager.yaml")))["spec"]["containers"][0]["args"]
    assert cm[cm.index("--cluster-cidr") + 1] == "10.244.0.0/16" and "--feature-gates" not in cm
    assert "embedded" in _kubeadm("alpha", "phase", "etcd", "local", *common)
    assert os.path.isdir(os.path.join(base, "data"))


def test_config_defaults_merge_and_helpers(tmp_path):
    out = yaml.safe_load(_kubeadm("config", "print-default", "--base-dir", str(tmp_path)))
    assert out["kind"] == "MasterConfiguration" and out["kubernetesVersion"] == GIT_VERSION
    assert out["networking"] == {"serviceSubnet": "10.96.0.0/12", "podSubnet": "", "dnsDomain": "cluster.local"}
    assert out["tokenTTL"] == "24h0m0s"
    base = {"api": {"advertiseAddress": "a", "bindPort": 1}, "nodeName": "n"}
    assert merge_config(base, {"api": {"bindPort": 2}, "nodeName": "m"}) == {"api": {"advertiseAddress": "a", "bindPort": 2},
                                                                            "nodeName": "m"}
    assert _with_extra(["--a", "1", "--b", "2"], {"b": "3", "c": "4"}) == ["--a", "1", "--b", "3", "--c", "4"]
    import argparse
    mc = master_config(argparse.Namespace(base_dir=str(tmp_path), service_cidr="10.100.0.0/16", node_name="x",
                                          apiserver_cert_extra_sans="1.2.3.4,host.example", config=None))
    assert dns_ip(mc) == "10.100.0.10"
    assert "IP:1.2.3.4" in apiserver_sans(mc) and "DNS:host.example" in apiserver_sans(mc)
    assert re.fullmatch(r"[a-z0-9]{6}\.[a-z0-9]{16}\n", _kubeadm("token", "generate"))
    assert _kubeadm("version", "-o", "short").strip() == GIT_VERSION
    assert GIT_VERSION in _kubeadm("version")


def test_upgrade_version_policy():
    ok = lambda c, t, k="v1.10.5": enforce_policy(c, t, k) == ([], [])  # noqa: E731
    assert ok("v1.9.6", "v1.9.8") and ok("v1.9.6", "v1.10.2")
    sk, mand = enforce_policy("v1.9.6", "v1.11.0", "v1.11.0")
    assert mand and "one minor release at a time" in mand[0]
    sk, mand = enforce_policy("v1.9.6", "v1.9.2", "v1.9.6")
    assert not mand and "lower than the cluster version" in sk[0]        # a patch downgrade needs --force
    sk, mand = enforce_policy("v1.9.6", "v1.8.9", "v1.9.6")
    assert any("lower than the minor release" in e for e in mand)
    sk, mand = enforce_policy("v1.9.6", "v1.9.9", "v1.9.7")
    assert not mand and "higher than the kubeadm version" in sk[0]
    sk, mand = enforce_policy("v1.9.6", "v1.10.1", "v1.9.7")
    assert any("newer minor release than kubeadm" in e for e in mand)
    assert enforce_policy("v1.9.6", "v2.0.0", "v2.0.0")[1]
