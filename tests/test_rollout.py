"""Deployment rollouts and the kubectl commands around them.

Reference: pkg/controller/deployment/rolling_test.go (surge / unavailability bounds),
recreate_test.go, rollback_test.go, sync_test.go (pause, history cleanup),
util/deployment_util_test.go (ResolveFenceposts); pkg/kubectl/cmd/rollout, expose_test.go,
taint_test.go, autoscale_test.go, auth/cani_test.go; registry scale subresource tests.
"""
import asyncio
import os
import time

import yaml

from amdkube.api import meta as m
from amdkube.controllers.deployment import resolve_fenceposts as _fenceposts
from amdkube.kubectl.extra import cmd_config_sync
from amdkube.kubectl.taint import parse_taints
from amdkube.kubectl.main import COMMANDS, parser
from amdkube.localcluster import LocalCluster
from tests.test_controllers import until


def _deploy(name, replicas=3, image="busybox", strategy=None, **spec):
    s = {"replicas": replicas, "selector": {"matchLabels": {"app": name}},
         "template": {"metadata": {"labels": {"app": name}},
                      "spec": {"containers": [{"name": "c", "image": image, "command": ["sleep", "60"]}]}}}
    if strategy:
        s["strategy"] = strategy
    s.update(spec)
    return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "namespace": "default"}, "spec": s}


async def kubectl(c, *argv):
    a = parser().parse_args(list(argv))
    if a.command is None:
        a.command = []
    return await COMMANDS[a.cmd](c, a)


def resolve_fenceposts(d):
    ru = ((d.get("spec") or {}).get("strategy") or {}).get("rollingUpdate") or {}
    return _fenceposts(ru.get("maxSurge", "25%"), ru.get("maxUnavailable", "25%"), d["spec"]["replicas"])


def test_fenceposts():
    d = lambda r, s, u: {"spec": {"replicas": r, "strategy": {"rollingUpdate": {"maxSurge": s, "maxUnavailable": u}}}}
    assert resolve_fenceposts(d(10, "25%", "25%")) == (3, 2)
    assert resolve_fenceposts(d(1, "25%", "25%")) == (1, 0)
    assert resolve_fenceposts(d(5, 0, 0)) == (0, 1)
    assert resolve_fenceposts({"spec": {"replicas": 4}}) == (1, 1)
    assert parse_taints(["gpu=mi355x:NoSchedule"]) == ([{"key": "gpu", "value": "mi355x", "effect": "NoSchedule"}], [])
    assert parse_taints(["gpu:NoSchedule-"]) == ([], [{"key": "gpu", "effect": "NoSchedule"}])


def test_rolling_update_bounds_history_undo_pause():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create(_deploy("web", 3, strategy={"type": "RollingUpdate",
                                                       "rollingUpdate": {"maxSurge": 1, "maxUnavailable": 0}}))

            async def rolled(rev):
                d = await c.get("deployments.apps", "web", "default")
                st = d.get("status") or {}
                ok = (st.get("updatedReplicas") == 3 and st.get("availableReplicas") == 3 and st.get("replicas") == 3
                      and d["metadata"].get("annotations", {}).get("deployment.kubernetes.io/revision") == str(rev))
                return ok and d
            d = await until(lambda: rolled(1), 30)
            assert {x["type"]: x["reason"] for x in d["status"]["conditions"]} == {
                "Available": "MinimumReplicasAvailable", "Progressing": "NewReplicaSetAvailable"}
            # roll to a new image and sample the pod count while it progresses
            seen = []
            stop = asyncio.Event()

            async def sample():
                while not stop.is_set():
                    pods, _ = await c.list("pods", "default", label_selector="app=web")
                    live = [p for p in pods if not p["metadata"].get("deletionTimestamp")
                            and p.get("status", {}).get("phase") not in ("Succeeded", "Failed")]
                    seen.append(len(live))
                    await asyncio.sleep(0.01)
            t = asyncio.create_task(sample())
            await kubectl(c, "set", "image", "deployment/web", "c=busybox:latest", "--record")
            await until(lambda: rolled(2), 40)
            stop.set()
            await t
            assert max(seen) <= 4, seen          # replicas + maxSurge
            out = await kubectl(c, "rollout", "status", "deployment/web", "--timeout", "5")
            assert out == 0
            rss, _ = await c.list("replicasets.apps", "default", label_selector="app=web")
            assert sorted(int(r["metadata"]["annotations"]["deployment.kubernetes.io/revision"]) for r in rss) == [1, 2]
            assert any(r["metadata"]["annotations"].get("kubernetes.io/change-cause", "").startswith("kubectl set image")
                       for r in rss)
            # undo → the revision-1 template comes back as revision 3 (same ReplicaSet re-adopted)
            await kubectl(c, "rollout", "undo", "deployment/web")
            d = await until(lambda: rolled(3), 40)
            assert d["spec"]["template"]["spec"]["containers"][0]["image"] == "busybox"
            rss, _ = await c.list("replicasets.apps", "default", label_selector="app=web")
            assert len(rss) == 2
            # pause: template edits create no ReplicaSet until resume
            await kubectl(c, "rollout", "pause", "deployment/web")
            await c.patch("deployments.apps", "web", {"spec": {"template": {"spec": {"containers": [
                {"name": "c", "image": "python:3", "command": ["sleep", "60"]}]}}}}, "default")
            await asyncio.sleep(0.5)
            assert len((await c.list("replicasets.apps", "default", label_selector="app=web"))[0]) == 2
            d = await c.get("deployments.apps", "web", "default")
            assert any(x["reason"] == "DeploymentPaused" for x in d["status"]["conditions"])
            await kubectl(c, "rollout", "resume", "deployment/web")
            await until(lambda: rolled(4), 40)
            # the rollback subresource (extensions/v1beta1 DeploymentRollback) → revision 5 = revision 3's template
            await c.request("POST", "/apis/apps/v1/namespaces/default/deployments/web/rollback",
                            body={"kind": "DeploymentRollback", "name": "web", "rollbackTo": {"revision": 3}})
            d = await until(lambda: rolled(5), 40)
            assert d["spec"]["template"]["spec"]["containers"][0]["image"] == "busybox" and "rollbackTo" not in d["spec"]
            # scale subresource
            sc = await c.request("GET", "/apis/apps/v1/namespaces/default/deployments/web/scale")
            assert sc["kind"] == "Scale" and sc["spec"]["replicas"] == 3 and sc["status"]["selector"] == "app=web"
            sc["spec"]["replicas"] = 1
            out = await c.request("PUT", "/apis/apps/v1/namespaces/default/deployments/web/scale", body=sc)
            assert out["spec"]["replicas"] == 1
            try:
                await c.request("PUT", "/apis/apps/v1/namespaces/default/deployments/web/scale", body=sc)   # stale RV
                raise AssertionError("stale resourceVersion must conflict")
            except m.StatusError as e:
                assert e.code == 409

            async def one():
                pods, _ = await c.list("pods", "default", label_selector="app=web")
                return len([p for p in pods if not p["metadata"].get("deletionTimestamp")]) == 1
            await until(one, 30)
    from tests.conftest import run
    run(go(), 150)


def test_recreate_and_history_limit():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create(_deploy("rc", 2, strategy={"type": "Recreate"}, revisionHistoryLimit=1))

            async def avail(n, image):
                d = await c.get("deployments.apps", "rc", "default")
                st = d.get("status") or {}
                return (st.get("availableReplicas") == n and st.get("updatedReplicas") == n and st.get("replicas") == n
                        and d["spec"]["template"]["spec"]["containers"][0]["image"] == image)
            await until(lambda: avail(2, "busybox"), 30)
            mixed = []
            stop = asyncio.Event()

            async def sample():
                while not stop.is_set():
                    pods, _ = await c.list("pods", "default", label_selector="app=rc")
                    imgs = {p["spec"]["containers"][0]["image"] for p in pods if p.get("status", {}).get("phase") == "Running"
                            and not p["metadata"].get("deletionTimestamp")}
                    mixed.append(len(imgs) > 1)
                    await asyncio.sleep(0.01)
            t = asyncio.create_task(sample())
            for img in ("busybox:latest", "python:3"):
                await kubectl(c, "set", "image", "deploy/rc", f"c={img}")
                await until(lambda: avail(2, img), 40)
            stop.set()
            await t
            assert not any(mixed)   # never old and new pods running together

            async def pruned():
                rss, _ = await c.list("replicasets.apps", "default", label_selector="app=rc")
                return len(rss) == 2   # current + revisionHistoryLimit=1
            await until(pruned, 20)
    from tests.conftest import run
    run(go(), 120)


def test_kubectl_generators_expose_autoscale_taint_auth_certs_explain(tmp_path, capsys):
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, api_kw={"authorization_mode": "Node,RBAC"}) as lc:
            c = lc.client
            await kubectl(c, "create", "namespace", "team-a")
            await kubectl(c, "create", "configmap", "cfg", "--from-literal", "a=1", "--from-literal", "b=2", "-n", "team-a")
            assert (await c.get("configmaps", "cfg", "team-a"))["data"] == {"a": "1", "b": "2"}
            await kubectl(c, "create", "secret", "generic", "s", "--from-literal", "k=v", "-n", "team-a")
            assert (await c.get("secrets", "s", "team-a"))["data"] == {"k": "dg=="}
            await kubectl(c, "create", "serviceaccount", "bot", "-n", "team-a")
            await kubectl(c, "create", "deployment", "api", "--image", "busybox", "--replicas", "2", "-n", "team-a")
            await kubectl(c, "create", "clusterrole", "reader", "--verb", "get", "--verb", "list", "--resource", "pods")
            await kubectl(c, "create", "clusterrolebinding", "r", "--clusterrole", "reader", "--user", "alice")
            await kubectl(c, "create", "quota", "q", "--hard", "pods=10,amd.com/gpu=4", "-n", "team-a")
            assert (await c.get("resourcequotas", "q", "team-a"))["spec"]["hard"] == {"pods": "10", "amd.com/gpu": "4"}
            await kubectl(c, "expose", "deployment", "api", "--port", "80", "--target-port", "8080", "-n", "team-a")
            svc = await c.get("services", "api", "team-a")
            assert svc["spec"]["selector"] == {"app": "api"} and svc["spec"]["ports"][0]["targetPort"] == 8080
            assert svc["spec"]["clusterIP"]
            await kubectl(c, "autoscale", "deployment", "api", "--min", "1", "--max", "5", "--cpu-percent", "70", "-n", "team-a")
            hpa = await c.get("horizontalpodautoscalers.autoscaling", "api", "team-a")
            assert hpa["spec"]["scaleTargetRef"]["kind"] == "Deployment" and hpa["spec"]["maxReplicas"] == 5
            node = lc.node_name
            await kubectl(c, "taint", "nodes", node, "gpu=mi355x:NoSchedule")
            assert (await c.get("nodes", node))["spec"]["taints"] == [{"key": "gpu", "value": "mi355x", "effect": "NoSchedule"}]
            await kubectl(c, "taint", "nodes", node, "gpu:NoSchedule-")
            assert not (await c.get("nodes", node))["spec"].get("taints")
            assert await kubectl(c, "auth", "can-i", "list", "pods", "--as", "alice") == 0
            assert await kubectl(c, "auth", "can-i", "delete", "pods", "--as", "alice") == 1
            assert await kubectl(c, "auth", "can-i", "delete", "nodes") == 0    # the loopback client is a master
            csr = {"apiVersion": "certificates.k8s.io/v1beta1", "kind": "CertificateSigningRequest", "metadata": {"name": "x"},
                   "spec": {"request": "", "usages": ["client auth"]}}
            await c.create(csr)
            await kubectl(c, "certificate", "approve", "x")
            got = await c.get("certificatesigningrequests.certificates.k8s.io", "x")
            assert [x["type"] for x in got["status"]["conditions"]] == ["Approved"]
            await kubectl(c, "explain", "deployments")
    from tests.conftest import run
    run(go(), 90)
    out = capsys.readouterr().out
    assert "KIND:     Deployment" in out and 'service "api" exposed' in out
    # kubeconfig editing works offline
    kc = tmp_path / "config"
    kc.write_text(yaml.safe_dump({"apiVersion": "v1", "kind": "Config", "current-context": "a",
                                  "contexts": [{"name": "a", "context": {"cluster": "c", "user": "u"}},
                                               {"name": "b", "context": {"cluster": "c", "user": "v"}}],
                                  "users": [{"name": "u", "user": {"token": "secret"}}]}))
    base = ["--kubeconfig", str(kc), "config"]
    assert cmd_config_sync(parser().parse_args(base + ["use-context", "b"])) == 0
    assert yaml.safe_load(kc.read_text())["current-context"] == "b"
    cmd_config_sync(parser().parse_args(base + ["view"]))
    assert "secret" not in capsys.readouterr().out
    os.environ.pop("KUBECONFIG", None)
    time.sleep(0)
