"""kubectl: three-way apply (+ prune, *-last-applied), set env/resources/selector/
serviceaccount/subject, create secret docker-registry|tls / service * / pdb, rolling-update,
convert, api-versions, completion, plugin, cluster-info dump (pkg/kubectl/cmd/*_test.go)."""
import asyncio
import base64
import io
import json
import subprocess
import os
import contextlib

import yaml

from amdkube.api import meta as m
from amdkube.kubectl.more import three_way, _SAME
from amdkube.localcluster import LocalCluster
from tests.conftest import run
from tests.test_rollout import kubectl


def test_three_way_patch():
    pod = {"apiVersion": "v1", "kind": "Pod"}
    orig = {**pod, "metadata": {"labels": {"a": "1", "b": "2"}}, "spec": {"containers": [{"name": "x", "image": "i1"},
                                                                                        {"name": "y", "image": "i2"}]}}
    cur = {**pod, "metadata": {"labels": {"a": "1", "b": "2", "c": "live"}}, "spec": {"containers": [
        {"name": "x", "image": "i1", "imagePullPolicy": "Always"}, {"name": "y", "image": "i2"}]}}
    mod = {**pod, "metadata": {"labels": {"a": "1"}}, "spec": {"containers": [{"name": "x", "image": "i9"}]}}
    p = three_way(orig, mod, cur)
    assert p == {"metadata": {"labels": {"b": None}},
                 "spec": {"$setElementOrder/containers": [{"name": "x"}],
                          "containers": [{"name": "x", "image": "i9"}, {"name": "y", "$patch": "delete"}]}}
    assert three_way(orig, orig, orig) is _SAME


def _write(tmp_path, name, docs):
    p = tmp_path / name
    p.write_text(yaml.safe_dump_all(docs))
    return str(p)


def test_kubectl_apply_set_create_convert_and_friends(tmp_path, capsys):
    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "app", "namespace": "default", "labels": {"tier": "x"}},
                  "data": {"a": "1", "b": "2"}}
            extra = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "old", "namespace": "default", "labels": {"tier": "x"}},
                     "data": {"z": "1"}}
            f1 = _write(tmp_path, "v1.yaml", [cm, extra])
            await kubectl(c, "apply", "-f", f1)
            await c.patch("configmaps", "app", {"data": {"live": "kept"}}, "default")     # someone else's field
            cm2 = json.loads(json.dumps(cm))
            del cm2["data"]["b"]
            cm2["data"]["a"] = "9"
            f2 = _write(tmp_path, "v2.yaml", [cm2])
            await kubectl(c, "apply", "-f", f2, "--prune", "-l", "tier=x")
            got = await c.get("configmaps", "app", "default")
            assert got["data"] == {"a": "9", "live": "kept"}                           # b deleted, live kept
            assert await c.get_or_none("configmaps", "old", "default") is None           # pruned
            capsys.readouterr()
            await kubectl(c, "apply", "view-last-applied", "configmap/app")
            assert yaml.safe_load(capsys.readouterr().out)["data"] == {"a": "9"}
            # set *
            dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web", "namespace": "default"},
                   "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "web"}}, "template": {
                       "metadata": {"labels": {"app": "web"}}, "spec": {"containers": [{"name": "c", "image": "busybox"}]}}}}
            await c.create(dep)
            await kubectl(c, "set", "env", "deployment/web", "FOO=bar", "X=1")
            await kubectl(c, "set", "env", "deployment/web", "X-")
            await kubectl(c, "set", "resources", "deployment/web", "--limits", "cpu=200m,memory=64Mi")
            await kubectl(c, "set", "serviceaccount", "deployment/web", "builder")
            d = await c.get("deployments.apps", "web", "default")
            ct = d["spec"]["template"]["spec"]["containers"][0]
            assert ct["env"] == [{"name": "FOO", "value": "bar"}] and ct["resources"]["limits"]["cpu"] == "200m"
            assert d["spec"]["template"]["spec"]["serviceAccountName"] == "builder"
            await kubectl(c, "create", "rolebinding", "rb", "--clusterrole", "view", "--user", "alice")
            await kubectl(c, "set", "subject", "rolebinding/rb", "--group", "devs", "--serviceaccount", "default:builder")
            rb = await c.get("rolebindings.rbac.authorization.k8s.io", "rb", "default")
            assert [s["name"] for s in rb["subjects"]] == ["alice", "devs", "builder"]
            # create generators
            await kubectl(c, "create", "secret", "docker-registry", "regcred", "--docker-username", "u",
                          "--docker-password", "p", "--docker-server", "r.example.com")
            sec = await c.get("secrets", "regcred", "default")
            cfg = json.loads(base64.b64decode(sec["data"][".dockerconfigjson"]))
            assert sec["type"] == "kubernetes.io/dockerconfigjson" and cfg["auths"]["r.example.com"]["username"] == "u"
            subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-subj", "/CN=t", "-days", "1", "-keyout",
                            str(tmp_path / "t.key"), "-out", str(tmp_path / "t.crt")], check=True, capture_output=True)   # the pair must load
            await kubectl(c, "create", "secret", "tls", "tls1", "--cert", str(tmp_path / "t.crt"), "--key", str(tmp_path / "t.key"))
            assert (await c.get("secrets", "tls1", "default"))["type"] == "kubernetes.io/tls"
            await kubectl(c, "create", "service", "nodeport", "np", "--tcp", "80:8080")
            svc = await c.get("services", "np", "default")
            assert svc["spec"]["type"] == "NodePort" and svc["spec"]["ports"][0]["targetPort"] == 8080
            await kubectl(c, "create", "service", "externalname", "ext", "--external-name", "db.example.com")
            assert (await c.get("services", "ext", "default"))["spec"]["externalName"] == "db.example.com"
            await kubectl(c, "create", "pdb", "budget", "--selector", "app=web", "--min-available", "1")
            assert (await c.get("poddisruptionbudgets.policy", "budget", "default"))["spec"]["minAvailable"] == 1
            # convert, api-versions, completion
            f3 = _write(tmp_path, "dep.yaml", [dict(dep, apiVersion="extensions/v1beta1")])
            capsys.readouterr()
            await kubectl(c, "convert", "-f", f3, "--output-version", "apps/v1beta2")
            assert yaml.safe_load(capsys.readouterr().out)["apiVersion"] == "apps/v1beta2"
            await kubectl(c, "api-versions")
            out = capsys.readouterr().out.split()
            assert "v1" in out and "extensions/v1beta1" in out and "apps/v1beta2" in out
            await kubectl(c, "completion", "bash")
            assert "complete -F" in capsys.readouterr().out
            # cluster-info dump
            await kubectl(c, "cluster-info", "dump", "--output-directory", str(tmp_path / "dump"))
            assert os.path.exists(tmp_path / "dump" / "default" / "services.json")
    run(go(), 60)


def test_kubectl_plugin(tmp_path, capsys, monkeypatch):
    pd = tmp_path / "plugins" / "hello"
    pd.mkdir(parents=True)
    (pd / "plugin.yaml").write_text(yaml.safe_dump({"name": "hello", "shortDesc": "says hello",
                                                    "command": "echo hello-$KUBECTL_PLUGINS_CURRENT_NAMESPACE > out.txt"}))
    monkeypatch.setenv("KUBECTL_PLUGINS_PATH", str(tmp_path / "plugins"))

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            await kubectl(lc.client, "plugin")
            assert "says hello" in capsys.readouterr().out
            await kubectl(lc.client, "plugin", "hello", "-n", "prod")
            assert (pd / "out.txt").read_text().strip() == "hello-prod"
    run(go(), 30)


def test_kubectl_rolling_update():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            rc = {"apiVersion": "v1", "kind": "ReplicationController", "metadata": {"name": "frontend", "namespace": "default"},
                  "spec": {"replicas": 2, "selector": {"app": "fe"}, "template": {"metadata": {"labels": {"app": "fe"}}, "spec": {
                      "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}}}
            await c.create(rc)
            for _ in range(100):
                if ((await c.get("replicationcontrollers", "frontend", "default")).get("status") or {}).get("readyReplicas") == 2:
                    break
                await asyncio.sleep(0.1)
            await kubectl(c, "rolling-update", "frontend", "--image", "python:3", "--timeout", "30")
            for _ in range(100):   # the renamed-away controller goes once the GC released its orphan finalizer
                rcs, _ = await c.list("replicationcontrollers", "default")
                if [m.name_of(x) for x in rcs] == ["frontend"]:
                    break
                await asyncio.sleep(0.1)
            assert [m.name_of(x) for x in rcs] == ["frontend"]
            assert rcs[0]["spec"]["template"]["spec"]["containers"][0]["image"] == "python:3"
    run(go(), 90)


def test_apply_two_port_service_and_strategic_patch_of_ports(tmp_path, capsys):
    """Round-3 review repro: `kubectl apply` of a 2-port Service with one changed targetPort
    kept only a duplicated port, and a strategic PATCH of spec.ports failed in the server.
    ServiceSpec.ports merges by `port` (core/v1/types.go:3372)."""
    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client

            def svc(tp):
                return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web", "namespace": "default"},
                        "spec": {"selector": {"app": "web"}, "ports": [
                            {"name": "http", "port": 80, "targetPort": tp},
                            {"name": "https", "port": 443, "targetPort": 8443}]}}
            await kubectl(c, "apply", "-f", _write(tmp_path, "s1.yaml", [svc(8080)]))
            await kubectl(c, "apply", "-f", _write(tmp_path, "s2.yaml", [svc(8081)]))
            live = await c.get("services", "web", "default")
            ports = {p["name"]: (p["port"], p["targetPort"]) for p in live["spec"]["ports"]}
            assert ports == {"http": (80, 8081), "https": (443, 8443)}
            assert len(live["spec"]["ports"]) == 2
            # a strategic PATCH of one port by its merge key
            out = await c.patch("services", "web", {"spec": {"ports": [{"port": 443, "targetPort": 9443}]}}, "default",
                                patch_type="application/strategic-merge-patch+json")
            assert [(p["port"], p["targetPort"]) for p in out["spec"]["ports"]] == [(80, 8081), (443, 9443)]
            # a port dropped from the manifest is removed, the other kept
            one = svc(8081)
            one["spec"]["ports"] = one["spec"]["ports"][:1]
            await kubectl(c, "apply", "-f", _write(tmp_path, "s3.yaml", [one]))
            live = await c.get("services", "web", "default")
            assert [p["port"] for p in live["spec"]["ports"]] == [80]
    run(go())


def test_auth_reconcile_rbac(tmp_path, capsys):
    """kubectl auth reconcile (pkg/kubectl/cmd/auth/reconcile.go, pkg/registry/rbac/reconciliation):
    idempotent on the bootstrap roles, missing rules/subjects are added (never removed), a
    changed roleRef re-creates the binding, autoupdate=false protects an object."""
    from amdkube.api import rbac

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False,
                                api_kw={"authorization_mode": "RBAC"}) as lc:
            c = lc.client
            boot = [r for r in (await c.list("clusterroles.rbac.authorization.k8s.io"))[0]
                    if m.name_of(r).startswith("system:")][:10]
            assert boot, "no bootstrap cluster roles"
            rvs = {m.name_of(r): r["metadata"]["resourceVersion"] for r in boot}
            docs = [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                     "metadata": {"name": m.name_of(r), "labels": r["metadata"].get("labels") or {},
                                  "annotations": r["metadata"].get("annotations") or {}},
                     "rules": r.get("rules") or []} for r in boot]
            f = _write(tmp_path, "boot.yaml", docs)
            await kubectl(c, "auth", "reconcile", "-f", f)
            await kubectl(c, "auth", "reconcile", "-f", f)
            for r in (await c.list("clusterroles.rbac.authorization.k8s.io"))[0]:
                if m.name_of(r) in rvs:
                    assert r["metadata"]["resourceVersion"] == rvs[m.name_of(r)], m.name_of(r)   # untouched
            # a role missing a rule gains it; an extra live rule stays (union)
            role = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                    "metadata": {"name": "gpu-reader", "namespace": "team", "labels": {"tier": "gpu"}},
                    "rules": [{"apiGroups": [""], "resources": ["pods", "pods/log"], "verbs": ["get", "list"]}]}
            rb = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                  "metadata": {"name": "readers", "namespace": "team"},
                  "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": "gpu-reader"},
                  "subjects": [{"kind": "User", "name": "alice", "apiGroup": "rbac.authorization.k8s.io"}]}
            await kubectl(c, "auth", "reconcile", "-f", _write(tmp_path, "r1.yaml", [role, rb]))   # creates (and the namespace)
            live = await c.get("roles.rbac.authorization.k8s.io", "gpu-reader", "team")
            live["rules"].append({"apiGroups": ["apps"], "resources": ["deployments"], "verbs": ["get"]})
            await c.update(live)
            role["rules"].append({"apiGroups": [""], "resources": ["services"], "verbs": ["watch"]})
            rb["subjects"].append({"kind": "User", "name": "bob", "apiGroup": "rbac.authorization.k8s.io"})
            await kubectl(c, "auth", "reconcile", "-f", _write(tmp_path, "r2.yaml", [role, rb]))
            live = await c.get("roles.rbac.authorization.k8s.io", "gpu-reader", "team")
            ok, missing = rbac.covers(live["rules"], role["rules"])
            assert ok, missing
            assert any("deployments" in (r.get("resources") or []) for r in live["rules"])
            assert live["metadata"]["labels"] == {"tier": "gpu"}
            b = await c.get("rolebindings.rbac.authorization.k8s.io", "readers", "team")
            assert {s["name"] for s in b["subjects"]} == {"alice", "bob"}
            # a changed roleRef re-creates the binding (new uid)
            old_uid = m.uid_of(b)
            rb["roleRef"]["name"] = "other"
            await kubectl(c, "auth", "reconcile", "-f", _write(tmp_path, "r3.yaml", [rb]))
            b = await c.get("rolebindings.rbac.authorization.k8s.io", "readers", "team")
            assert b["roleRef"]["name"] == "other" and m.uid_of(b) != old_uid
            # protected: left alone
            live = await c.get("roles.rbac.authorization.k8s.io", "gpu-reader", "team")
            live["metadata"].setdefault("annotations", {})[rbac.AUTOUPDATE] = "false"
            live = await c.update(live)
            role["rules"].append({"apiGroups": [""], "resources": ["secrets"], "verbs": ["get"]})
            await kubectl(c, "auth", "reconcile", "-f", _write(tmp_path, "r4.yaml", [role]))
            again = await c.get("roles.rbac.authorization.k8s.io", "gpu-reader", "team")
            assert again["metadata"]["resourceVersion"] == live["metadata"]["resourceVersion"]
    run(go())
    assert "reconciled" in capsys.readouterr().out


def test_rbac_rule_coverage():
    from amdkube.api.rbac import covers
    owner = [{"apiGroups": [""], "resources": ["pods", "*/status"], "verbs": ["get", "list"]},
             {"nonResourceURLs": ["/healthz", "/api/*"], "verbs": ["get"]},
             {"apiGroups": ["apps"], "resources": ["deployments"], "verbs": ["*"], "resourceNames": ["web"]}]
    assert covers(owner, [{"apiGroups": [""], "resources": ["pods", "nodes/status"], "verbs": ["get"]}])[0]
    assert covers(owner, [{"nonResourceURLs": ["/api/v1"], "verbs": ["get"]}])[0]
    ok, miss = covers(owner, [{"apiGroups": ["apps"], "resources": ["deployments"], "verbs": ["update"]}])
    assert not ok and miss == [{"apiGroups": ["apps"], "resources": ["deployments"], "verbs": ["update"]}]
    assert covers(owner, [{"apiGroups": ["apps"], "resources": ["deployments"], "verbs": ["update"], "resourceNames": ["web"]}])[0]
