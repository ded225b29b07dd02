"""kubeadm init → join → schedule → token → reset, every component a real process (reference
cmd/kubeadm/app/cmd/{init,join,reset,token}.go; test/e2e_kubeadm). TLS everywhere: the
apiserver serves the kubeadm-generated certificate and authenticates components by client
certificate; the worker joins through token discovery + TLS bootstrap (CSR auto-approved and
signed by the cluster CA)."""
from __future__ import annotations

import asyncio
import base64
import os
import re
import socket
import subprocess
import sys

import pytest

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.kubeadm import ca_cert_hash, new_token

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _kubeadm(*args, timeout=180):
    return subprocess.run([sys.executable, "-m", "amdkube", "kubeadm", *args], cwd=ROOT, capture_output=True, text=True,
                          timeout=timeout, env=dict(os.environ, PYTHONPATH=ROOT))


def test_token_format_and_ca_pin(tmp_path):
    t = new_token()
    assert re.fullmatch(r"[a-z0-9]{6}\.[a-z0-9]{16}", t)
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(tmp_path / "k"), "-out",
                    str(tmp_path / "c"), "-days", "1", "-subj", "/CN=x"], check=True, capture_output=True)
    h = ca_cert_hash(open(tmp_path / "c", "rb").read())
    assert h.startswith("sha256:") and len(h) == 7 + 64


@pytest.mark.slow
def test_kubeadm_init_join_reset(tmp_path):
    master, worker = str(tmp_path / "master"), str(tmp_path / "worker")
    port = _free_port()
    try:
        r = _kubeadm("init", "--base-dir", master, "--apiserver-bind-port", str(port), "--node-name", "master-0",
                     "--start-kubelet", "--kubelet-port", "0", "--pod-network-cidr", "10.244.0.0/16", "--service-cidr",
                     "10.96.0.0/12", "--timeout", "90")
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        assert "initialized successfully" in r.stdout
        join = re.search(r"kubeadm join (\S+) --token (\S+) --discovery-token-ca-cert-hash (\S+)", r.stdout)
        assert join, r.stdout
        server, token, h = join.groups()
        # a wrong CA pin is refused
        bad = _kubeadm("join", server, "--token", token, "--discovery-token-ca-cert-hash", "sha256:" + "0" * 64,
                       "--base-dir", str(tmp_path / "bad"), "--node-name", "bad", "--timeout", "20")
        assert bad.returncode != 0 and "does not match" in bad.stderr
        r = _kubeadm("join", server, "--token", token, "--discovery-token-ca-cert-hash", h, "--base-dir", worker,
                     "--node-name", "worker-1", "--start-kubelet", "--kubelet-port", "0")
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        asyncio.run(_check_cluster(os.path.join(master, "admin.conf")))
        admin = os.path.join(master, "admin.conf")
        r = _kubeadm("token", "list", "--kubeconfig", admin)
        assert token.split(".")[0] in r.stdout, r.stdout + r.stderr
        r = _kubeadm("token", "create", "--kubeconfig", admin, "--print-join-command")
        assert re.search(r"kubeadm join \S+ --token [a-z0-9]{6}\.[a-z0-9]{16} --discovery-token-ca-cert-hash " + re.escape(h),
                         r.stdout), r.stdout + r.stderr
        # the stored configuration, the upgrade plan and an upgrade that changes one component
        r = _kubeadm("config", "view", "--kubeconfig", admin)
        assert "kind: MasterConfiguration" in r.stdout and "nodeName: master-0" in r.stdout and "token:" not in r.stdout
        r = _kubeadm("upgrade", "plan", "--kubeconfig", admin)
        assert r.returncode == 0 and "kube-scheduler" in r.stdout and "up-to-date" in r.stdout, r.stdout + r.stderr
        r = _kubeadm("upgrade", "apply", "v1.8.0", "--kubeconfig", admin, "--base-dir", master, "-y")
        assert r.returncode == 1 and "lower than the minor release" in r.stderr
        newcfg = tmp_path / "upgrade.yaml"
        newcfg.write_text("apiVersion: kubeadm.k8s.io/v1alpha1\nkind: MasterConfiguration\n"
                          "schedulerExtraArgs: {kube-api-qps: '400'}\n")
        r = _kubeadm("upgrade", "apply", "--kubeconfig", admin, "--base-dir", master, "--config", str(newcfg), "-y",
                     "--timeout", "90")
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        assert "kube-apiserver is unchanged" in r.stdout and "Component kube-scheduler upgraded successfully" in r.stdout
        asyncio.run(_check_upgraded(admin))
    finally:
        for d in (worker, master):
            _kubeadm("reset", "--base-dir", d, "--drain-seconds", "1.5")


async def _check_upgraded(admin_conf):
    c = Client.from_kubeconfig(admin_conf)
    try:
        p = await c.get("pods", "kube-scheduler-master-0", "kube-system")
        args = p["spec"]["containers"][0]["args"]
        assert args[args.index("--kube-api-qps") + 1] == "400", args
        cm = await c.get("configmaps", "kubeadm-config", "kube-system")
        assert "kube-api-qps" in cm["data"]["MasterConfiguration"]
        ds = {m.name_of(d) for d in (await c.list("deployments.apps", "kube-system"))[0]}
        assert "kube-dns" in ds
    finally:
        await c.close()


async def _check_cluster(admin_conf):
    c = Client.from_kubeconfig(admin_conf)
    try:
        assert c.server.startswith("https://")

        async def ready(name):
            n = await c.get_or_none("nodes", name)
            conds = {x["type"]: x["status"] for x in ((n or {}).get("status") or {}).get("conditions") or []}
            return n if conds.get("Ready") == "True" else None
        end = asyncio.get_running_loop().time() + 60
        nodes = {}
        while asyncio.get_running_loop().time() < end and len(nodes) < 2:
            for name in ("master-0", "worker-1"):
                n = await ready(name)
                if n:
                    nodes[name] = n
            await asyncio.sleep(0.3)
        assert set(nodes) == {"master-0", "worker-1"}
        assert "node-role.kubernetes.io/master" in m.labels_of(nodes["master-0"])
        assert any(t["effect"] == "NoSchedule" for t in nodes["master-0"]["spec"].get("taints") or [])
        # control plane runs as static pods with mirror pods
        pods, _ = await c.list("pods", "kube-system")
        names = {m.name_of(p) for p in pods}
        assert {"kube-apiserver-master-0", "kube-controller-manager-master-0", "kube-scheduler-master-0"} <= names
        # a workload lands on the worker (the master is tainted) and runs
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "hello"},
                        "spec": {"containers": [{"name": "c", "image": "amdkube/pause:3.1"}]}}, "default")
        end = asyncio.get_running_loop().time() + 60
        p = None
        while asyncio.get_running_loop().time() < end:
            p = await c.get("pods", "hello", "default")
            if (p.get("status") or {}).get("phase") == "Running":
                break
            await asyncio.sleep(0.3)
        assert p["spec"]["nodeName"] == "worker-1" and p["status"]["phase"] == "Running", p.get("status")
        # the worker's kubelet identity is a node identity (NodeRestriction): it cannot touch the master
        csrs, _ = await c.list("certificatesigningrequests")
        assert any(x["spec"]["username"].startswith("system:bootstrap:") and x["status"].get("certificate") for x in csrs)
    finally:
        await c.close()


def test_kubeadm_local_etcd_static_pod(tmp_path):
    """etcd.dataDir in the MasterConfiguration: kubeadm writes an `amdkube etcd` static Pod
    (app/phases/etcd/local.go), the apiserver stores through --etcd-servers, the objects land
    in etcd's data directory, and reset removes that directory (reset.go resetEtcd)."""
    base, etcd_dir = str(tmp_path / "master"), str(tmp_path / "etcd-data")
    port, eport = _free_port(), _free_port()
    cfg = tmp_path / "cfg.yaml"
    cfg.write_text("apiVersion: kubeadm.k8s.io/v1alpha1\nkind: MasterConfiguration\n"
                   f"etcd:\n  dataDir: {etcd_dir}\n  extraArgs:\n    listen-client-urls: http://127.0.0.1:{eport}\n")
    try:
        r = _kubeadm("init", "--base-dir", base, "--config", str(cfg), "--apiserver-bind-port", str(port),
                     "--node-name", "master-0", "--start-kubelet", "--kubelet-port", "0", "--skip-addons", "--timeout", "90")
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        assert "Wrote Static Pod manifest for a local etcd instance" in r.stdout
        import yaml
        api = yaml.safe_load(open(os.path.join(base, "manifests", "kube-apiserver.yaml")))["spec"]["containers"][0]["args"]
        assert api[api.index("--etcd-servers") + 1] == f"http://127.0.0.1:{eport}" and "--data-dir" not in api

        async def check():
            c = Client.from_kubeconfig(os.path.join(base, "admin.conf"))
            try:
                await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "in-etcd"}, "data": {"k": "v"}},
                               "default")
                end = asyncio.get_running_loop().time() + 60
                while True:           # the mirror pods of the static pods appear
                    pods = {m.name_of(p) for p in (await c.list("pods", "kube-system"))[0]}
                    if "etcd-master-0" in pods or asyncio.get_running_loop().time() > end:
                        return pods
                    await asyncio.sleep(0.3)
            finally:
                await c.close()
        pods = asyncio.run(check())
        assert {"etcd-master-0", "kube-apiserver-master-0"} <= pods
        assert b"in-etcd" in open(os.path.join(etcd_dir, "wal.log"), "rb").read()
    finally:
        r = _kubeadm("reset", "--base-dir", base, "--drain-seconds", "1.5")
    assert r.returncode == 0 and etcd_dir in r.stdout and not os.path.exists(etcd_dir)


def test_kubeadm_store_modes():
    """embedded (default) / local etcd static Pod / external etcd with client TLS."""
    from amdkube.kubeadm import phases as ph
    base = {"api": {"advertiseAddress": "127.0.0.1", "bindPort": 6443}, "kubernetesVersion": "v1.9.0",
            "networking": {"serviceSubnet": "10.96.0.0/12", "podSubnet": ""}}
    p = ph.paths("/etc/kubernetes")

    def api_args(mc):
        return ph.control_plane_manifests(mc, p)["kube-apiserver"]["spec"]["containers"][0]["args"]
    a = api_args(base)
    assert ph.etcd_mode(base) == "embedded" and a[a.index("--data-dir") + 1] == p["data_dir"] and "--etcd-servers" not in a
    ext = dict(base, etcd={"endpoints": ["https://10.0.0.1:2379", "https://10.0.0.2:2379"], "caFile": "/pki/etcd-ca.crt",
                           "certFile": "/pki/c.crt", "keyFile": "/pki/c.key"})
    a = api_args(ext)
    assert ph.etcd_mode(ext) == "external" and "--data-dir" not in a
    assert a[a.index("--etcd-servers") + 1] == "https://10.0.0.1:2379,https://10.0.0.2:2379"
    assert [a[a.index(f) + 1] for f in ("--etcd-cafile", "--etcd-certfile", "--etcd-keyfile")] == \
        ["/pki/etcd-ca.crt", "/pki/c.crt", "/pki/c.key"]
    loc = dict(base, etcd={"dataDir": "/var/lib/etcd", "extraArgs": {"snapshot-count": "10000"}})
    a = api_args(loc)
    assert ph.etcd_mode(loc) == "local" and a[a.index("--etcd-servers") + 1] == "http://127.0.0.1:2379"
    e = ph.etcd_manifest(loc)["spec"]["containers"][0]["args"]
    assert e[:2] == ["-m", "amdkube"] and e[2] == "etcd" and e[e.index("--data-dir") + 1] == "/var/lib/etcd"
    assert e[e.index("--snapshot-count") + 1] == "10000"


def test_kubeadm_self_hosting(tmp_path):
    """--feature-gates SelfHosting=true,StoreCertsInSecrets=true: the static control plane
    becomes DaemonSets self-hosted-kube-{apiserver,controller-manager,scheduler}
    (selfhosting.go) that read their certificates and kubeconfigs from kube-system Secrets
    (selfhosting_volumes.go); the static manifests and their mirror pods go, the self-hosted
    apiserver takes over the embedded store's data directory, and the cluster keeps its
    objects and keeps working."""
    base = str(tmp_path / "master")
    port = _free_port()
    try:
        r = _kubeadm("init", "--base-dir", base, "--apiserver-bind-port", str(port), "--node-name", "master-0",
                     "--start-kubelet", "--kubelet-port", "0", "--skip-addons", "--feature-gates", "SelfHosting=true,StoreCertsInSecrets=true",
                     "--timeout", "120", timeout=300)
        assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-3000:]
        for comp in ("kube-apiserver", "kube-controller-manager", "kube-scheduler"):
            assert f"self-hosted {comp} ready" in r.stdout, r.stdout[-3000:]
            assert not os.path.exists(os.path.join(base, "manifests", f"{comp}.yaml"))

        async def check():
            c = Client.from_kubeconfig(os.path.join(base, "admin.conf"))
            try:
                pods = {m.name_of(p): p for p in (await c.list("pods", "kube-system"))[0]}
                assert not {"kube-apiserver-master-0", "kube-controller-manager-master-0", "kube-scheduler-master-0"} & set(pods)
                for comp in ("kube-apiserver", "kube-controller-manager", "kube-scheduler"):
                    ds = await c.get("daemonsets.apps", f"self-hosted-{comp}", "kube-system")
                    spec = ds["spec"]["template"]["spec"]
                    assert spec["nodeSelector"] == {"node-role.kubernetes.io/master": ""} and spec["dnsPolicy"] == "ClusterFirstWithHostNet"
                    vols = {v["name"]: v for v in spec.get("volumes") or []}
                    args = spec["containers"][0]["args"]
                    if comp != "kube-scheduler":
                        assert [x["secret"]["name"] for x in vols["k8s-certs"]["projected"]["sources"]][:1] == ["ca"]
                    if comp != "kube-apiserver":
                        conf = "scheduler.conf" if comp == "kube-scheduler" else "controller-manager.conf"
                        assert vols["kubeconfig"]["secret"]["secretName"] == conf
                        assert args[args.index("--kubeconfig") + 1] == os.path.join(base, "kubeconfig", conf)
                    mine = [p for p in pods.values() if m.labels_of(p).get("k8s-app") == f"self-hosted-{comp}"]
                    assert len(mine) == 1 and mine[0]["status"]["phase"] == "Running"
                # objects written before the hand-off are still there; the scheduler and the
                # controller-manager of the self-hosted plane still act
                assert await c.get_or_none("configmaps", "kubeadm-config", "kube-system") is not None
                tls = await c.get("secrets", "apiserver", "kube-system")
                assert tls["type"] == "kubernetes.io/tls" and set(tls["data"]) == {"tls.crt", "tls.key"}
                assert base64.b64decode(tls["data"]["tls.crt"]) == open(os.path.join(base, "pki", "apiserver.crt"), "rb").read()
                await c.create({"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": "after", "namespace": "kube-system"},
                                "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "after"}},
                                         "template": {"metadata": {"labels": {"app": "after"}},
                                                      "spec": {"tolerations": [{"key": "node-role.kubernetes.io/master", "effect": "NoSchedule"}],
                                                               "containers": [{"name": "c", "image": "amdkube/pause:3.1"}]}}}},
                               "kube-system")
                end = asyncio.get_running_loop().time() + 60
                while asyncio.get_running_loop().time() < end:
                    ps, _ = await c.list("pods", "kube-system", label_selector="app=after")
                    if ps and ps[0]["spec"].get("nodeName") == "master-0" and ps[0]["status"].get("phase") == "Running":
                        return
                    await asyncio.sleep(0.3)
                raise AssertionError("a pod created after self-hosting was not scheduled and started")
            finally:
                await c.close()
        asyncio.run(check())
        # an upgrade of a self-hosted component rolls its DaemonSet (no static manifest comes back)
        newcfg = tmp_path / "upgrade.yaml"
        newcfg.write_text("apiVersion: kubeadm.k8s.io/v1alpha1\nkind: MasterConfiguration\n"
                          "schedulerExtraArgs: {kube-api-qps: '300'}\n")
        admin = os.path.join(base, "admin.conf")
        r = _kubeadm("upgrade", "apply", "--kubeconfig", admin, "--base-dir", base, "--config", str(newcfg), "-y",
                     "--timeout", "90", timeout=200)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        assert "Component kube-scheduler upgraded successfully (DaemonSet self-hosted-kube-scheduler)" in r.stdout, r.stdout
        assert "[upgrade/selfhosted] kube-apiserver is unchanged" in r.stdout, r.stdout
        assert not os.path.exists(os.path.join(base, "manifests", "kube-scheduler.yaml"))

        async def rolled():
            c = Client.from_kubeconfig(admin)
            try:
                pods, _ = await c.list("pods", "kube-system", label_selector="k8s-app=self-hosted-kube-scheduler")
                args = pods[0]["spec"]["containers"][0]["args"]
                assert len(pods) == 1 and args[args.index("--kube-api-qps") + 1] == "300", args
                assert args[args.index("--kubeconfig") + 1] == os.path.join(base, "kubeconfig", "scheduler.conf")
            finally:
                await c.close()
        asyncio.run(rolled())
    finally:
        _kubeadm("reset", "--base-dir", base, "--drain-seconds", "1.5")


def test_self_hosting_secret_volumes_and_rootfs_paths(tmp_path, monkeypatch):
    """The StoreCertsInSecrets mutators (podspec_mutation.go setSelfHostedVolumesFor*) and how
    a process container resolves a command-line path inside its volumes."""
    from amdkube.__main__ import rootfs_paths
    from amdkube.kubeadm import selfhosting as sh
    pki = tmp_path / "pki"
    pki.mkdir()
    for f in ("ca.crt", "ca.key", "apiserver.crt", "apiserver.key", "sa.key"):
        (pki / f).write_text(f)
    spec = lambda args: {"containers": [{"name": "c", "args": list(args)}]}    # noqa: E731
    plain = sh.build_daemonset("kube-scheduler", spec(["--kubeconfig", "/k/scheduler.conf"]))
    assert "volumes" not in plain["spec"]["template"]["spec"]
    api = sh.build_daemonset("kube-apiserver", spec(["--data-dir", "/d"]), (str(pki), "/k"))["spec"]["template"]["spec"]
    srcs = api["volumes"][0]["projected"]["sources"]
    assert [x["secret"]["name"] for x in srcs] == ["ca", "apiserver", "sa"]      # front-proxy files absent
    assert api["containers"][0]["volumeMounts"] == [{"name": "k8s-certs", "mountPath": str(pki), "readOnly": True}]
    assert api["containers"][0]["args"][-2:] == ["--data-dir-lock-wait", sh.LOCK_WAIT]
    cm = sh.build_daemonset("kube-controller-manager", spec(["--kubeconfig", "/k/controller-manager.conf"]),
                            (str(pki), "/k"))["spec"]["template"]["spec"]
    assert [x["secret"]["name"] for x in cm["volumes"][0]["projected"]["sources"]] == ["ca", "sa"]
    assert cm["volumes"][1] == {"name": "kubeconfig", "secret": {"secretName": "controller-manager.conf"}}
    assert cm["containers"][0]["args"] == ["--kubeconfig", "/k/kubeconfig/controller-manager.conf"]
    again = sh.set_secret_volumes("kube-controller-manager", cm, str(pki), "/k")     # idempotent
    assert len(again["volumes"]) == 2 and len(again["containers"][0]["volumeMounts"]) == 2
    # $AMDKUBE_ROOTFS: a path that exists in the container's view wins over the host's
    root = tmp_path / "root"
    (root / "k" / "kubeconfig").mkdir(parents=True)
    (root / "k" / "kubeconfig" / "x.conf").write_text("")
    monkeypatch.setenv("AMDKUBE_ROOTFS", str(root))
    assert rootfs_paths(["--kubeconfig", "/k/kubeconfig/x.conf", "--a=/k/kubeconfig/x.conf", "/nope", "rel"]) == \
        ["--kubeconfig", f"{root}/k/kubeconfig/x.conf", f"--a={root}/k/kubeconfig/x.conf", "/nope", "rel"]
    monkeypatch.delenv("AMDKUBE_ROOTFS")
    assert rootfs_paths(["/k/kubeconfig/x.conf"]) == ["/k/kubeconfig/x.conf"]


def test_kubeadm_feature_gate_dependencies():
    """features.ResolveFeatureGateDependencies and the HighAvailability apiserver flag."""
    from amdkube.kubeadm import phases as ph
    assert ph.resolve_gate_dependencies({"StoreCertsInSecrets": True}) == {"StoreCertsInSecrets": True, "SelfHosting": True}
    assert ph.resolve_gate_dependencies({"HighAvailability": True}) == \
        {"HighAvailability": True, "SelfHosting": True, "StoreCertsInSecrets": True}
    assert ph.resolve_gate_dependencies({"CoreDNS": True}) == {"CoreDNS": True}
    mc = {"api": {"advertiseAddress": "127.0.0.1", "bindPort": 6443}, "kubernetesVersion": "v1.9.0",
          "networking": {"serviceSubnet": "10.96.0.0/12", "dnsDomain": "cluster.local"}, "featureGates": {"HighAvailability": True}}
    p = {"pki": "/nonexistent/pki", "kubeconfig_dir": "/k", "data_dir": "/d"}
    args = ph.control_plane_manifests(mc, p)["kube-apiserver"]["spec"]["containers"][0]["args"]
    assert args[args.index("--endpoint-reconciler-type") + 1] == "lease"
    mc["featureGates"] = {}
    assert "--endpoint-reconciler-type" not in ph.control_plane_manifests(mc, p)["kube-apiserver"]["spec"]["containers"][0]["args"]
