"""apiserver semantics beyond CRUD (reference generic registry/handlers behaviour):

  * optimistic concurrency: PUT with a stale resourceVersion -> 409 Conflict
    (staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go:263 GuaranteedUpdate)
  * watch from a compacted revision -> 410 Gone ("too old resource version", etcd3/store.go:661)
  * list chunking with limit/continue and label/field selectors
  * merge, strategic-merge (containers merged by name) and JSON patch
  * pods/eviction subresource
  * token authentication (401) and AlwaysDeny authorization (403)
  * /metrics exposes apiserver_request_count
"""
import pytest

from amdkube.api import meta as m
from amdkube.apiserver import APIServer
from amdkube.client import Client
from tests.conftest import run


def cm(name, labels=None, data=None):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": "default", "labels": labels or {}},
            "data": data or {}}


def pod(name, node=None, labels=None):
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "labels": labels or {}},
         "spec": {"containers": [{"name": "a", "image": "busybox", "env": [{"name": "X", "value": "1"}]},
                                 {"name": "b", "image": "busybox"}]}}
    if node:
        p["spec"]["nodeName"] = node
    return p


async def _srv(**kw):
    s = await APIServer(**kw).start()
    return s, Client(s.url)


def test_conflict_on_stale_update():
    async def go():
        s, c = await _srv()
        try:
            o = await c.create(cm("x", data={"k": "1"}))
            o2 = dict(o, data={"k": "2"})
            await c.update(o2)
            with pytest.raises(m.StatusError) as ei:
                await c.update(dict(o, data={"k": "3"}))  # still carries the first resourceVersion
            assert ei.value.code == 409
            assert (await c.get("configmaps", "x", "default"))["data"] == {"k": "2"}
        finally:
            await c.close()
            await s.stop()
    run(go())


def test_watch_from_compacted_revision_is_gone():
    async def go():
        s, c = await _srv()
        try:
            first = await c.create(cm("a"))
            for i in range(5):
                await c.create(cm(f"b{i}"))
            s.store.compact(s.store.rev)
            with pytest.raises(m.StatusError) as ei:
                async for _ in c.watch("configmaps", "default", resource_version=first["metadata"]["resourceVersion"]):
                    break
            assert ei.value.code == 410
            # a current revision still works
            _, rv = await c.list("configmaps", "default")
            await c.create(cm("late"))
            async for typ, obj in c.watch("configmaps", "default", resource_version=rv):
                assert (typ, obj["metadata"]["name"]) == ("ADDED", "late")
                break
        finally:
            await c.close()
            await s.stop()
    run(go())


def test_list_chunking_and_selectors():
    async def go():
        s, c = await _srv()
        try:
            for i in range(7):
                await c.create(cm(f"c{i}", labels={"tier": "gpu" if i % 2 else "cpu"}))
            names, cont = [], None
            while True:
                params = {"limit": "3"}
                if cont:
                    params["continue"] = cont
                r = await c.request("GET", "/api/v1/namespaces/default/configmaps", params=params)
                names += [o["metadata"]["name"] for o in r["items"]]
                cont = r["metadata"].get("continue")
                assert len(r["items"]) <= 3
                if not cont:
                    break
            assert names == [f"c{i}" for i in range(7)]
            items, _ = await c.list("configmaps", "default", label_selector="tier=gpu")
            assert sorted(o["metadata"]["name"] for o in items) == ["c1", "c3", "c5"]
            items, _ = await c.list("configmaps", "default", label_selector="tier in (cpu),tier!=gpu")
            assert len(items) == 4
            await c.create(pod("p-on", node="n1"))
            await c.create(pod("p-off"))
            items, _ = await c.list("pods", "default", field_selector="spec.nodeName=n1")
            assert [o["metadata"]["name"] for o in items] == ["p-on"]
            items, _ = await c.list("pods", "default", field_selector="spec.nodeName=")
            assert [o["metadata"]["name"] for o in items] == ["p-off"]
        finally:
            await c.close()
            await s.stop()
    run(go())


def test_patch_flavours():
    async def go():
        s, c = await _srv()
        try:
            await c.create(pod("pp", labels={"a": "1"}))
            o = await c.patch("pods", "pp", {"metadata": {"labels": {"b": "2", "a": None}}}, "default")
            assert o["metadata"]["labels"] == {"b": "2"}
            # strategic merge: the containers list merges by name instead of being replaced
            o = await c.patch("pods", "pp", {"spec": {"containers": [{"name": "b", "image": "nginx"}]}}, "default",
                              patch_type="application/strategic-merge-patch+json")
            imgs = {x["name"]: x["image"] for x in o["spec"]["containers"]}
            assert imgs == {"a": "busybox", "b": "nginx"}
            o = await c.patch("pods", "pp", [{"op": "add", "path": "/metadata/annotations", "value": {"z": "9"}},
                                             {"op": "replace", "path": "/metadata/labels/b", "value": "3"}], "default",
                              patch_type="application/json-patch+json")
            assert o["metadata"]["annotations"] == {"z": "9"} and o["metadata"]["labels"] == {"b": "3"}
            with pytest.raises(m.StatusError) as ei:  # spec.containers[].name is immutable on a pod
                await c.patch("pods", "pp", [{"op": "replace", "path": "/spec/containers/0/name", "value": "q"}], "default",
                              patch_type="application/json-patch+json")
            assert ei.value.code == 422
        finally:
            await c.close()
            await s.stop()
    run(go())


def test_eviction_subresource():
    async def go():
        s, c = await _srv()
        try:
            await c.create(pod("ev"))
            await c.evict("default", "ev")
            assert await c.get_or_none("pods", "ev", "default") is None
        finally:
            await c.close()
            await s.stop()
    run(go())


def test_token_auth_and_authorization():
    async def go():
        s, c = await _srv(token_auth={"s3cret": {"name": "admin", "groups": ["system:masters"]}}, anonymous_auth=False)
        try:
            with pytest.raises(m.StatusError) as ei:
                await c.list("pods", "default")
            assert ei.value.code == 401
            ok = Client(s.url, token="s3cret")
            assert (await ok.list("pods", "default"))[0] == []
            bad = Client(s.url, token="nope")
            with pytest.raises(m.StatusError) as ei:
                await bad.list("pods", "default")
            assert ei.value.code == 401
            await ok.close()
            await bad.close()
        finally:
            await c.close()
            await s.stop()
        s, c = await _srv(authorization_mode="AlwaysDeny")
        try:
            with pytest.raises(m.StatusError) as ei:
                await c.create(cm("denied"))
            assert ei.value.code == 403
        finally:
            await c.close()
            await s.stop()
    run(go())


def test_metrics_endpoint():
    async def go():
        s, c = await _srv()
        try:
            await c.create(cm("mx"))
            await c.get("configmaps", "mx", "default")
            txt = await c.request("GET", "/metrics", raw=True)
            txt = txt.decode() if isinstance(txt, (bytes, bytearray)) else str(txt)
            assert "apiserver_request_count" in txt and 'resource="configmaps"' in txt
        finally:
            await c.close()
            await s.stop()
    run(go())
