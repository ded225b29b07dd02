"""In-process apiserver over real HTTP (the reference's integration tier runs the master
in-process over httptest: test/integration/framework/master_utils.go:174).

Covers: CRUD + watch, ResourceV2 rewrite (a gap in the reference's tests),
pods/binding writing `assigned` atomically with nodeName, and the binding validation
fixes (§7.6 #1/#10: unknown, unhealthy and double-assigned device IDs are rejected).
"""
import asyncio

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import APIServer
from amdkube.client import Client, Informer
from tests.conftest import run


def gpu_node(name="n1", n=8, unhealthy=()):
    devs = {f"GPU-{i}": {"id": f"GPU-{i}", "health": "Unhealthy" if i in unhealthy else "Healthy",
                         "attributes": {"amd.com/gpu-type": "MI355X", "amd.com/gpu-memory": "294896",
                                        "amd.com/numa-node": str(i // 4)}} for i in range(n)}
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name},
            "status": {"capacity": {"cpu": "64", "memory": "1Ti", "pods": "110", "amd.com/gpu": str(n)},
                       "extendedResources": {"amd.com/gpu": {"resources": devs}},
                       "conditions": [{"type": "Ready", "status": "True"}]}}


def legacy_gpu_pod(name, n=1):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {"containers": [{"name": "c", "image": "rocm/vector-add",
                                     "resources": {"limits": {"amd.com/gpu": str(n)}}}]}}


async def _server(**kw):
    srv = APIServer(**kw)
    await srv.start()
    return srv, Client(srv.url)


def test_crud_watch_and_discovery():
    async def go():
        srv, c = await _server()
        try:
            assert "v1" in (await c.request("GET", "/api"))["versions"]
            rl = await c.request("GET", "/api/v1")
            assert any(r["name"] == "pods/binding" for r in rl["resources"])
            ns = await c.get("namespaces", "default")
            assert ns["status"]["phase"] == "Active"
            pod = await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "a", "labels": {"app": "x"}},
                                  "spec": {"containers": [{"name": "c", "image": "nginx"}]}})
            assert pod["status"]["phase"] == "Pending" and pod["spec"]["restartPolicy"] == "Always"
            items, rv = await c.list("pods", "default", label_selector="app=x")
            assert len(items) == 1
            events = []

            async def watcher():
                async for t, o in c.watch("pods", "default", rv):
                    events.append((t, o["metadata"]["name"]))
                    if len(events) == 2:
                        return
            wt = asyncio.create_task(watcher())
            await asyncio.sleep(0.1)
            await c.patch("pods", "a", {"metadata": {"labels": {"k": "v"}}}, "default")
            await c.delete("pods", "a", "default")
            await asyncio.wait_for(wt, 5)
            assert events == [("MODIFIED", "a"), ("DELETED", "a")]
            with pytest.raises(m.StatusError) as ei:
                await c.get("pods", "a", "default")
            assert ei.value.code == 404
            with pytest.raises(m.StatusError) as ei:
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "b", "namespace": "nope"},
                                "spec": {"containers": [{"name": "c", "image": "nginx"}]}})
            assert ei.value.code == 404  # NamespaceLifecycle
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_resourcev2_rewrite_and_binding():
    async def go():
        srv, c = await _server()
        try:
            await c.create(gpu_node(unhealthy=(7,)))
            p = await c.create(legacy_gpu_pod("g", 2))
            c0 = p["spec"]["containers"][0]
            assert "amd.com/gpu" not in (c0.get("resources") or {}).get("limits", {})
            [pres] = p["spec"]["extendedResources"]
            assert c0["extendedResourceRequests"] == [pres["name"]]
            assert pres["resources"]["limits"] == {"amd.com/gpu": "2"} == pres["resources"]["requests"]
            assert any(t["key"] == "amd.com/gpu" for t in p["spec"]["tolerations"])  # ExtendedResourceToleration
            r = pres["name"]
            # wrong count
            with pytest.raises(m.StatusError) as ei:
                await c.bind("default", "g", "n1", {r: {"resources": ["GPU-0"]}})
            assert ei.value.code == 422
            # unknown device
            with pytest.raises(m.StatusError):
                await c.bind("default", "g", "n1", {r: {"resources": ["GPU-0", "GPU-99"]}})
            # unhealthy device
            with pytest.raises(m.StatusError) as ei:
                await c.bind("default", "g", "n1", {r: {"resources": ["GPU-0", "GPU-7"]}})
            assert ei.value.code == 409
            await c.bind("default", "g", "n1", {r: {"resources": ["GPU-0", "GPU-1"]}})
            p = await c.get("pods", "g", "default")
            assert p["spec"]["nodeName"] == "n1"
            assert p["spec"]["extendedResources"][0]["assigned"] == ["GPU-0", "GPU-1"]
            assert any(x["type"] == "PodScheduled" and x["status"] == "True" for x in p["status"]["conditions"])
            # second bind conflicts; another pod can't take GPU-1
            with pytest.raises(m.StatusError) as ei:
                await c.bind("default", "g", "n1", {r: {"resources": ["GPU-2", "GPU-3"]}})
            assert ei.value.code == 409
            p2 = await c.create(legacy_gpu_pod("h", 1))
            r2 = p2["spec"]["extendedResources"][0]["name"]
            with pytest.raises(m.StatusError) as ei:
                await c.bind("default", "h", "n1", {r2: {"resources": ["GPU-1"]}})
            assert ei.value.code == 409 and "already assigned" in ei.value.message
            # after the first pod terminates its devices are free again
            p["status"]["phase"] = "Succeeded"
            await c.update_status(p)
            await c.bind("default", "h", "n1", {r2: {"resources": ["GPU-1"]}})
            # user updates can't rewrite assigned/nodeName
            p2 = await c.get("pods", "h", "default")
            p2["spec"]["extendedResources"][0]["assigned"] = ["GPU-5"]
            p2 = await c.update(p2)
            assert p2["spec"]["extendedResources"][0]["assigned"] == ["GPU-1"]
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_graceful_pod_delete_and_informer():
    async def go():
        srv, c = await _server()
        try:
            await c.create(gpu_node())
            inf = Informer(c, "pods", field_selector="spec.nodeName=n1").start()
            seen = []
            inf.add_handler(on_add=lambda o: seen.append(("add", m.name_of(o))),
                            on_update=lambda o, n: seen.append(("upd", m.name_of(n))),
                            on_delete=lambda o: seen.append(("del", m.name_of(o))))
            await inf.wait_synced(5)
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "x"},
                            "spec": {"containers": [{"name": "c", "image": "nginx"}]}})
            await c.bind("default", "x", "n1")
            for _ in range(50):
                if ("add", "x") in seen:
                    break
                await asyncio.sleep(0.02)
            assert ("add", "x") in seen  # entered the field selector via binding
            obj = await c.delete("pods", "x", "default")
            assert obj["metadata"].get("deletionTimestamp")  # graceful: bound + running
            await c.delete("pods", "x", "default", grace=0)
            for _ in range(50):
                if ("del", "x") in seen:
                    break
                await asyncio.sleep(0.02)
            assert ("del", "x") in seen
            await inf.stop()
        finally:
            await c.close()
            await srv.stop()
    run(go())


def test_namespace_lifecycle_and_generate_name():
    async def go():
        srv, c = await _server()
        try:
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
            o = await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"generateName": "cm-", "namespace": "team"},
                                "data": {"a": "b"}})
            assert o["metadata"]["name"].startswith("cm-")
            ns = await c.delete("namespaces", "team")
            assert ns["status"]["phase"] == "Terminating"
            with pytest.raises(m.StatusError) as ei:
                await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x", "namespace": "team"}})
            assert ei.value.code == 403
            with pytest.raises(m.StatusError) as ei:
                await c.delete("namespaces", "kube-system")
            assert ei.value.code == 403
        finally:
            await c.close()
            await srv.stop()
    run(go())
