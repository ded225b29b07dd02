"""Controller-manager: ReplicaSet / Deployment / DaemonSet / Job / Namespace / GC / node
lifecycle / pod GC on an in-process cluster (hollow nodes provide extra nodes)."""
import asyncio
import time

from amdkube.api import meta as m
from amdkube.controllers.lifecycle import NodeLifecycleController
from amdkube.hollow.hollow_node import HollowNode
from amdkube.localcluster import LocalCluster
from tests.conftest import run


async def until(pred, timeout=20.0, step=0.05):
    end = time.time() + timeout
    last = None
    while time.time() < end:
        last = await pred()
        if last:
            return last
        await asyncio.sleep(step)
    raise AssertionError(f"condition not met: {last!r}")


def tpl(labels, cmd=("sleep", "60"), gpus=0):
    c = {"name": "c", "image": "busybox", "command": list(cmd)}
    if gpus:
        c["resources"] = {"limits": {"amd.com/gpu": str(gpus)}}
    return {"metadata": {"labels": labels}, "spec": {"containers": [c]}}


def test_replicaset_deployment_and_gc():
    async def go():
        async with LocalCluster(gpus="fake", n_gpus=4, relist_period=0.2) as lc:
            c = lc.client
            await lc.wait_gpus(4)
            await c.create({"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": "rs", "namespace": "default"},
                            "spec": {"replicas": 3, "selector": {"matchLabels": {"app": "rs"}}, "template": tpl({"app": "rs"}, gpus=1)}})

            async def rs_ready():
                rs = await c.get("replicasets.apps", "rs", "default")
                return (rs.get("status") or {}).get("readyReplicas") == 3 and rs
            await until(rs_ready, 30)
            pods, _ = await c.list("pods", "default", label_selector="app=rs")
            ids = [d for p in pods for d in p["spec"]["extendedResources"][0]["assigned"]]
            assert len(set(ids)) == 3
            await c.patch("replicasets.apps", "rs", {"spec": {"replicas": 1}}, "default")

            async def scaled():
                pods, _ = await c.list("pods", "default", label_selector="app=rs")
                return len([p for p in pods if not p["metadata"].get("deletionTimestamp")]) == 1
            await until(scaled, 30)
            # cascading delete via the garbage collector
            await c.delete("replicasets.apps", "rs", "default")

            async def gone():
                pods, _ = await c.list("pods", "default", label_selector="app=rs")
                return not pods
            await until(gone, 30)
            # deployment: new template → new ReplicaSet, old scaled to zero
            await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d", "namespace": "default"},
                            "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "d"}}, "template": tpl({"app": "d"})}})

            async def d_ready():
                d = await c.get("deployments.apps", "d", "default")
                return (d.get("status") or {}).get("readyReplicas") == 2
            await until(d_ready, 30)
            await c.patch("deployments.apps", "d", {"spec": {"template": {"metadata": {"labels": {"app": "d", "v": "2"}}}}}, "default",
                          patch_type="application/strategic-merge-patch+json")

            async def rolled():
                rss, _ = await c.list("replicasets.apps", "default")
                mine = [r for r in rss if (m.controller_ref(r) or {}).get("name") == "d"]
                return len(mine) == 2 and sorted(int(r["spec"]["replicas"]) for r in mine) == [0, 2]
            await until(rolled, 30)
    run(go(), 150)


def test_job_and_daemonset_on_hollow_nodes():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            hollow = [await HollowNode(lc.api.url, f"hollow-{i}", gpus=8, run_seconds=0.3).start() for i in range(2)]
            try:
                await c.create({"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "j", "namespace": "default"},
                                "spec": {"completions": 4, "parallelism": 2,
                                         "template": {"spec": {"restartPolicy": "Never", "containers": [
                                             {"name": "c", "image": "busybox", "command": ["true"], "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}})

                async def done():
                    j = await c.get("jobs.batch", "j", "default")
                    return any(x["type"] == "Complete" for x in (j.get("status") or {}).get("conditions") or []) and j
                j = await until(done, 40)
                assert j["status"]["succeeded"] >= 4
                await c.create({"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "ds", "namespace": "kube-system"},
                                "spec": {"selector": {"matchLabels": {"app": "ds"}}, "template": tpl({"app": "ds"})}})

                async def ds_ok():
                    pods, _ = await c.list("pods", "kube-system", label_selector="app=ds")
                    return sorted(p["spec"]["nodeName"] for p in pods) == sorted([lc.node_name, "hollow-0", "hollow-1"])
                await until(ds_ok, 30)
            finally:
                for h in hollow:
                    await h.stop()
    run(go(), 150)


def test_namespace_deletion_and_node_lifecycle():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
            await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x", "namespace": "team"}, "data": {}})
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "team"},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}})
            await c.delete("namespaces", "team")

            async def ns_gone():
                return await c.get_or_none("namespaces", "team") is None
            await until(ns_gone, 40)
            # node lifecycle: a node whose heartbeat stops goes Unknown, is tainted, pods evicted
            await c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "ghost"},
                            "status": {"capacity": {"cpu": "4", "memory": "4Gi", "pods": "10"},
                                       "conditions": [{"type": "Ready", "status": "True", "lastHeartbeatTime": "2000-01-01T00:00:00Z"}]}})
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "stuck", "namespace": "default"},
                            "spec": {"nodeName": "ghost", "containers": [{"name": "c", "image": "busybox"}],
                                     "tolerations": [{"key": "node.kubernetes.io/unreachable", "operator": "Exists",
                                                      "effect": "NoExecute", "tolerationSeconds": 0}]}})
            nlc = NodeLifecycleController(lc.controllers, grace=1.0, eviction_timeout=0.0)
            nlc.setup()
            await until(lambda: _has(lc, "ghost"), 10)
            await nlc.monitor_once()
            node = await c.get("nodes", "ghost")
            assert any(x["type"] == "Ready" and x["status"] == "Unknown" for x in node["status"]["conditions"])
            assert any(t["key"] == "node.kubernetes.io/unreachable" for t in node["spec"]["taints"])
            await asyncio.sleep(0.3)
            await nlc.monitor_once()
            p = await c.get_or_none("pods", "stuck", "default")
            assert p is None or p["metadata"].get("deletionTimestamp")
    run(go(), 120)


async def _has(lc, name):
    return any(m.name_of(n) == name for n in lc.controllers.nodes.list())
