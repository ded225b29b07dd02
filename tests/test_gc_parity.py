"""Garbage collector held to pkg/controller/garbagecollector/garbagecollector_test.go, plus the
behaviour its integration tests (test/integration/garbagecollector) pin, through a real apiserver:

* TestGarbageCollectorConstruction (:59) — monitors follow the resource set, before and after Run;
* TestAttemptToDeleteItem (:233) — the exact requests for an object whose owner is gone;
* TestProcessEvent (:338) — the graph invariants after every event of the four scenarios;
* TestAbsentUIDCache (:477) — the LRU absent-owner cache saves the second GET;
* TestDeleteOwnerRefPatch (:575), TestUnblockOwnerReference (:609) — through our strategic merge;
* TestOrphanDependentsFailure (:661); TestGetDeletableResources (:697); TestGarbageCollectorSync
  (:789) — a discovery error does not stop the resync loop.
TestDependentsRace (Go's race detector) and TestGCListWatcher (dynamic-client query encoding)
have no counterpart: the graph has one writer on one event loop, and the monitors are ordinary
informers.

End to end: foreground deletion keeps a Deployment (and its ReplicaSet) until the pods are gone;
orphaning strips the ownerReference; a dangling reference is patched out while a solid owner
remains; a custom resource owned by a ConfigMap is collected after discovery picks up its CRD;
3,000 owned pods cost no periodic work and one event per change.
"""
import asyncio
import types

import pytest

from amdkube.api import meta as m
from amdkube.api import strategicpatch as smp
from amdkube.client import Client
from amdkube.controllers import ControllerManager, Options
from amdkube.controllers.garbagecollector import (ADD, DELETE, UPDATE, GarbageCollector, GraphBuilder, Node,
                                                  ObjectReference, UIDCache, deletable_resources,
                                                  delete_owner_ref_patch, patch_to_unblock_owner_references)
from amdkube.client.workqueue import RateLimitingQueue
from tests.conftest import run


class FakeAPI:
    """fakeActionHandler: records (method, path); unknown paths answer 200 {"kind": "List"}."""
    path = Client.path

    def __init__(self, responses=None):
        self.responses = responses or {}
        self.actions = []

    async def request(self, method, path, params=None, body=None, content_type="application/json", raw=False,
                      timeout=None):
        self.actions.append(f"{method}={path}")
        code, content = self.responses.get(method + path, (200, {"kind": "List"}))
        if code == 404:
            raise m.not_found("x", path.rsplit("/", 1)[-1])
        if code == 409:
            raise m.conflict(path.split("/")[-2], path.rsplit("/", 1)[-1], "the object has been modified")
        if code >= 400:
            raise m.StatusError(code, "Error", "error")
        return content


def get_pod(name, owners):
    return {"kind": "Pod", "apiVersion": "v1",
            "metadata": {"name": name, "namespace": "ns1", "uid": "", "ownerReferences": owners}}


def rc_ref(name, uid):
    return {"kind": "ReplicationController", "name": name, "uid": uid, "apiVersion": "v1"}


def pod_node(pod):
    md = pod["metadata"]
    return Node(ObjectReference(pod["apiVersion"], pod["kind"], md["name"], md["uid"], md["namespace"]))


def setup_gc(api, **kw):
    return GarbageCollector(types.SimpleNamespace(client=api, factory=None), **kw)


def test_attempt_to_delete_item():
    pod = get_pod("ToBeDeletedPod", [rc_ref("owner1", "123")])
    api = FakeAPI({"GET/api/v1/namespaces/ns1/replicationcontrollers/owner1": (404, None),
                   "GET/api/v1/namespaces/ns1/pods/ToBeDeletedPod": (200, pod)})
    gc = setup_gc(api)
    run(gc.attempt_to_delete_item(pod_node(pod)))
    assert set(api.actions) == {"GET=/api/v1/namespaces/ns1/replicationcontrollers/owner1",
                                "DELETE=/api/v1/namespaces/ns1/pods/ToBeDeletedPod",
                                "GET=/api/v1/namespaces/ns1/pods/ToBeDeletedPod"}


def verify_graph_invariants(name, uid_to_node):
    for my_uid, n in uid_to_node.items():
        for dep in n.dependents:
            assert any(o.get("uid") == my_uid for o in dep.owners), \
                f"{name}: {n.identity} has {dep.identity} as a dependent, not in its owners"
        for owner in n.owners:
            on = uid_to_node.get(owner["uid"])
            if on is not None:
                assert n in on.dependents, f"{name}: {n.identity} has owner {on.identity} not listing it"


def create_event(typ, uid, owners):
    return (typ, {"metadata": {"uid": uid, "ownerReferences": [{"uid": o} for o in owners]}}, None, ("v1", "Pod"))


PROCESS_SCENARIOS = {
    "test1": [create_event(ADD, "1", []), create_event(ADD, "2", ["1"]), create_event(ADD, "3", ["1", "2"])],
    "test2": [create_event(ADD, "1", []), create_event(ADD, "2", ["1"]), create_event(ADD, "3", ["1", "2"]),
              create_event(ADD, "4", ["2"]), create_event(DELETE, "2", ["doesn't matter"])],
    "test3": [create_event(ADD, "1", []), create_event(ADD, "2", ["1"]), create_event(ADD, "3", ["1", "2"]),
              create_event(ADD, "4", ["3"]), create_event(UPDATE, "2", ["4"])],
    "reverse test2": [create_event(ADD, "4", ["2"]), create_event(ADD, "3", ["1", "2"]), create_event(ADD, "2", ["1"]),
                      create_event(ADD, "1", []), create_event(DELETE, "2", ["doesn't matter"])],
}


@pytest.mark.parametrize("name", list(PROCESS_SCENARIOS))
def test_process_event(name):
    gb = GraphBuilder(RateLimitingQueue(), RateLimitingQueue(), UIDCache(2))
    for ev in PROCESS_SCENARIOS[name]:
        gb.enqueue(ev)
        verify_graph_invariants(name, gb.uid_to_node)


def test_process_event_virtual_owner_and_delete_fanout():
    """Owners seen before they exist become virtual nodes queued for verification; deleting an
    owner queues its dependents and records it absent."""
    gb = GraphBuilder(RateLimitingQueue(), RateLimitingQueue(), UIDCache(10))
    gb.enqueue(create_event(ADD, "c", ["p"]))
    assert gb.uid_to_node["p"].virtual and gb.uid_to_node["p"] in gb.attempt_to_delete._dirty
    gb.enqueue(create_event(ADD, "p", []))
    assert not gb.uid_to_node["p"].virtual
    gb.enqueue(create_event(DELETE, "p", []))
    assert "p" not in gb.uid_to_node and gb.absent_owner_cache.has("p")
    assert gb.uid_to_node["c"] in gb.attempt_to_delete._dirty


def test_absent_uid_cache():
    pods = {n: get_pod(n, [rc_ref(rc, u)]) for n, rc, u in
            (("rc1Pod1", "rc1", "1"), ("rc1Pod2", "rc1", "1"), ("rc2Pod1", "rc2", "2"), ("rc3Pod1", "rc3", "3"))}
    resp = {f"GET/api/v1/namespaces/ns1/pods/{n}": (200, p) for n, p in pods.items()}
    resp.update({f"GET/api/v1/namespaces/ns1/replicationcontrollers/rc{i}": (404, None) for i in (1, 2, 3)})
    api = FakeAPI(resp)
    gc = setup_gc(api, absent_cache_size=2)

    async def go():
        for n in ("rc1Pod1", "rc2Pod1", "rc1Pod2", "rc3Pod1"):
            await gc.attempt_to_delete_item(pod_node(pods[n]))
    run(go())
    assert gc.absent_owner_cache.has("1") and not gc.absent_owner_cache.has("2") and gc.absent_owner_cache.has("3")
    assert api.actions.count("GET=/api/v1/namespaces/ns1/replicationcontrollers/rc1") == 1


def _pod_meta(refs):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"uid": "100", "ownerReferences": refs}}


def test_delete_owner_ref_patch():
    original = _pod_meta([{"uid": "1"}, {"uid": "2"}, {"uid": "3"}])
    got = smp.apply(original, delete_owner_ref_patch("100", "2", "3"), smp.schema_for("v1", "Pod"))
    assert got["metadata"] == {"uid": "100", "ownerReferences": [{"uid": "1"}]}


def test_unblock_owner_reference():
    refs = [{"uid": "1", "blockOwnerDeletion": True}, {"uid": "2", "blockOwnerDeletion": False}, {"uid": "3"}]
    original = _pod_meta(refs)
    n = Node(ObjectReference(uid="100"), owners=refs)
    got = smp.apply(original, patch_to_unblock_owner_references(n), smp.schema_for("v1", "Pod"))
    assert got["metadata"]["ownerReferences"] == [{"uid": "1", "blockOwnerDeletion": False},
                                                  {"uid": "2", "blockOwnerDeletion": False}, {"uid": "3"}]


def test_orphan_dependents_failure():
    api = FakeAPI({"PATCH/api/v1/namespaces/ns1/pods/pod": (409, None)})
    gc = setup_gc(api)
    deps = [Node(ObjectReference("v1", "Pod", "pod", "", "ns1"))]
    with pytest.raises(RuntimeError) as ei:
        run(gc.orphan_dependents(ObjectReference(), deps))
    assert "orphaning" in str(ei.value) and 'pods "pod"' in str(ei.value) and "cannot be fulfilled" in str(ei.value)


POD_RES = {"name": "pods", "namespaced": True, "kind": "Pod", "verbs": ["delete", "list", "watch"]}
SVC_RES = {"name": "services", "namespaced": True, "kind": "Service"}
DELETABLE_CASES = {
    "no error": ([{"groupVersion": "apps/v1", "resources": [POD_RES, SVC_RES]},
                  {"groupVersion": "foo//whatever", "resources": [dict(POD_RES, name="bars", kind="Bar")]},
                  {"groupVersion": "acme/v1", "resources": [{"name": "widgets", "namespaced": True, "kind": "Widget",
                                                             "verbs": ["delete"]}]}],
                 {("apps", "v1", "pods")}),
    "nonspecific failure, includes usable results": ([{"groupVersion": "apps/v1", "resources": [POD_RES, SVC_RES]}],
                                                     {("apps", "v1", "pods")}),
    "partial discovery failure, includes usable results": (
        [{"groupVersion": "apps/v1", "resources": [POD_RES, SVC_RES]}], {("apps", "v1", "pods")}),
    "discovery failure, no results": (None, set()),
}


@pytest.mark.parametrize("name", list(DELETABLE_CASES))
def test_get_deletable_resources(name):
    lists, expected = DELETABLE_CASES[name]
    assert set(deletable_resources(lists)) == expected


def test_get_deletable_resources_through_discovery_with_a_failing_group():
    api = FakeAPI({"GET/api": (200, {"versions": ["v1"]}),
                   "GET/api/v1": (200, {"groupVersion": "v1", "resources": [POD_RES, dict(POD_RES, name="pods/log")]}),
                   "GET/apis": (200, {"groups": [{"preferredVersion": {"groupVersion": "foo/v1"}},
                                                 {"preferredVersion": {"groupVersion": "apps/v1"}}]}),
                   "GET/apis/foo/v1": (500, None),
                   "GET/apis/apps/v1": (200, {"groupVersion": "apps/v1", "resources": [
                       dict(POD_RES, name="deployments", kind="Deployment")]})})
    gc = setup_gc(api)
    assert set(run(gc.get_deletable_resources())) == {("", "v1", "pods"), ("apps", "v1", "deployments")}


def test_garbage_collector_construction_and_monitor_resync():
    pods = {("", "v1", "pods"): POD_RES}
    two = {**pods, ("tpr.io", "v1", "unknown"): {"name": "unknown", "namespaced": True,
                                                 "verbs": ["delete", "list", "watch"]}}

    async def go():
        gc = setup_gc(FakeAPI())
        errs = gc.graph.sync_monitors(two)        # no kind known for the custom resource yet
        assert len(gc.graph.monitors) == 1 and errs
        two[("tpr.io", "v1", "unknown")]["kind"] = "Unknown"
        assert gc.graph.sync_monitors(two) == [] and len(gc.graph.monitors) == 2
        gc.graph.sync_monitors(pods)
        assert len(gc.graph.monitors) == 1
        # after Run: monitors are started and stopped as the set changes
        gc.graph.running = True
        gc.graph.sync_monitors(two)
        gc.graph.start_monitors()
        assert len(gc.graph.monitors) == 2 and all(mon.informer._task is not None for mon in gc.graph.monitors.values())
        gone = gc.graph.monitors[("tpr.io", "v1", "unknown")]
        gc.graph.sync_monitors(pods)
        assert len(gc.graph.monitors) == 1 and gone.handler not in gone.informer.handlers
        await gc.graph.stop()
        from amdkube.api.scheme import SCHEME
        SCHEME.by_kind.pop(("tpr.io/v1", "Unknown"), None)
        SCHEME.by_plural.pop(("tpr.io", "unknown"), None)
        SCHEME.by_gvr.pop(("tpr.io", "v1", "unknown"), None)
    run(go())


def test_garbage_collector_sync_survives_discovery_errors():
    """TestGarbageCollectorSync: discovery failing (no resources) is skipped, and the loop keeps
    polling discovery; when it recovers nothing is blocked."""
    state = {"fail": False}

    class Disco(FakeAPI):
        async def request(self, method, path, **kw):
            if state["fail"]:
                raise OSError("Error calling discoveryClient.ServerPreferredResources()")
            if path == "/api":
                return {"versions": ["v1"]}
            if path == "/api/v1":
                return {"groupVersion": "v1", "resources": [POD_RES]}
            if path == "/apis":
                return {"groups": []}
            return {"kind": "PodList", "items": [], "metadata": {"resourceVersion": "1"}}

    async def go():
        gc = setup_gc(Disco(), sync_period=0.01)
        gc.graph.running = True
        assert await gc._sync_once() is True
        task = asyncio.ensure_future(gc._sync_loop())
        await asyncio.sleep(0.1)
        before = gc.discovery_calls
        state["fail"] = True
        await asyncio.sleep(0.1)
        assert gc.discovery_calls > before and len(gc.graph.monitors) == 1
        state["fail"] = False
        mid = gc.discovery_calls
        await asyncio.sleep(0.1)
        assert gc.discovery_calls > mid
        task.cancel()
        await gc.graph.stop()
    run(go())


# ----------------------------------------------------------------------------- end to end
async def _cluster(period=0.2):
    from amdkube.apiserver import APIServer
    api = await APIServer().start()
    c = Client(api.url)
    cm = await ControllerManager(Client(api.url), ["garbagecollector", "replicaset", "deployment"],
                                 options=Options(extra={"gc_discovery_period": period})).start()
    return api, c, cm


async def _stop(api, c, cm):
    await cm.stop()
    await cm.client.close()
    await c.close()
    await api.stop()


async def _until(pred, timeout=15.0, what=""):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        v = await pred()
        if v:
            return v
        await asyncio.sleep(0.05)
    raise AssertionError(f"timed out waiting for {what}")


def _deploy(name, replicas=3):
    return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "namespace": "default"},
            "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": {"app": name}},
                                  "spec": {"containers": [{"name": "c", "image": "busybox"}]}}}}


async def _pods(c, app):
    items, _ = await c.list("pods", "default", label_selector=f"app={app}")
    return items


def test_foreground_delete_keeps_the_deployment_until_its_pods_are_gone():
    async def go():
        api, c, cm = await _cluster()
        try:
            await c.create(_deploy("web"))
            pods = await _until(lambda: _pods_n(c, "web", 3), what="3 pods")
            for p in pods:          # bound to a node without a kubelet: their deletion is graceful
                await c.bind("default", m.name_of(p), "node-x")
            await c.delete("deployments", "web", "default", propagation="Foreground")
            await _until(lambda: _all_terminating(c, "web"), what="pods marked for deletion")
            await asyncio.sleep(1.0)
            d = await c.get("deployments", "web", "default")
            assert d["metadata"].get("deletionTimestamp") and "foregroundDeletion" in d["metadata"]["finalizers"]
            rss, _ = await c.list("replicasets", "default")
            assert len(rss) == 1 and rss[0]["metadata"].get("deletionTimestamp")
            assert "foregroundDeletion" in rss[0]["metadata"]["finalizers"]
            for p in await _pods(c, "web"):      # the kubelet's final delete
                await c.delete("pods", m.name_of(p), "default", grace=0)
            await _until(lambda: _gone(c, "deployments", "web"), what="deployment deleted")
            assert (await c.list("replicasets", "default"))[0] == []
        finally:
            await _stop(api, c, cm)
    run(go(), 60)


async def _pods_n(c, app, n):
    ps = await _pods(c, app)
    return ps if len(ps) == n else None


async def _all_terminating(c, app):
    ps = await _pods(c, app)
    return ps and all(p["metadata"].get("deletionTimestamp") for p in ps)


async def _gone(c, res, name):
    return await c.get_or_none(res, name, "default") is None


def _cm(name):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": "default"}}


def _ref(o, block=None):
    r = {"apiVersion": o["apiVersion"], "kind": o["kind"], "name": m.name_of(o), "uid": m.uid_of(o)}
    if block is not None:
        r["blockOwnerDeletion"] = block
    return r


def _owned_pod(name, *owners):
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": "default", "ownerReferences": list(owners)},
            "spec": {"containers": [{"name": "c", "image": "busybox"}]}}


def test_orphan_and_dangling_references():
    async def go():
        api, c, cm = await _cluster()
        try:
            a, b, o = [await c.create(_cm(n)) for n in ("a", "b", "o")]
            await c.create(_owned_pod("two-owners", _ref(a), _ref(b)))
            await c.create(_owned_pod("orphan-me", _ref(o)))
            await asyncio.sleep(0.3)
            # b goes: the pod keeps its solid owner and loses the dangling reference
            await c.delete("configmaps", "b", "default")
            p = await _until(lambda: _refs_are(c, "two-owners", [m.uid_of(a)]), what="dangling ref removed")
            assert p["metadata"].get("deletionTimestamp") is None
            # o is deleted orphaning its dependents: the pod stays, without the reference
            await c.delete("configmaps", "o", "default", propagation="Orphan")
            await _until(lambda: _gone(c, "configmaps", "o"), what="orphaning owner deleted")
            p = await c.get("pods", "orphan-me", "default")
            assert not p["metadata"].get("ownerReferences") and not p["metadata"].get("deletionTimestamp")
            # a goes with background propagation: its last dependent is collected
            await c.delete("configmaps", "a", "default")
            await _until(lambda: _gone(c, "pods", "two-owners"), what="dependent collected")
        finally:
            await _stop(api, c, cm)
    run(go(), 60)


async def _refs_are(c, name, uids):
    p = await c.get("pods", name, "default")
    return p if [r["uid"] for r in p["metadata"].get("ownerReferences") or []] == uids else None


CRD = {"apiVersion": "apiextensions.k8s.io/v1beta1", "kind": "CustomResourceDefinition",
       "metadata": {"name": "gcwidgets.gc.amd.com"},
       "spec": {"group": "gc.amd.com", "version": "v1", "scope": "Namespaced",
                "names": {"plural": "gcwidgets", "kind": "GCWidget"}}}


def test_custom_resource_owned_by_a_configmap_is_collected():
    async def go():
        api, c, cm = await _cluster(period=0.1)
        try:
            await c.create(CRD)
            await _until(lambda: _discovered(c), what="CRD served")
            owner = await c.create(_cm("cr-owner"))
            w = {"apiVersion": "gc.amd.com/v1", "kind": "GCWidget",
                 "metadata": {"name": "w1", "namespace": "default", "ownerReferences": [_ref(owner)]}, "spec": {}}
            await c.create(w)
            gc = cm.get("garbagecollector")
            await _until(lambda: _has_uid(gc, owner), what="GC monitors the CR")
            await c.delete("configmaps", "cr-owner", "default")
            await _until(lambda: _gone(c, "gcwidgets.gc.amd.com", "w1"), what="CR collected")
        finally:
            await _stop(api, c, cm)
    run(go(), 60)


async def _discovered(c):
    await c.discover()
    try:
        await c.list("gcwidgets.gc.amd.com", "default")
        return True
    except (KeyError, m.StatusError):
        return False


async def _has_uid(gc, owner):
    n = gc.graph.uid_to_node.get(m.uid_of(owner))
    return n is not None and n.dependents


def test_custom_resource_dependent_patch_falls_back_to_json_patch():
    """A CR with a dangling and a solid owner: no strategic schema, so the JSON patch path."""
    async def go():
        api, c, cm = await _cluster(period=0.1)
        try:
            await c.create(CRD)
            await _until(lambda: _discovered(c), what="CRD served")
            keep, drop = await c.create(_cm("keep")), await c.create(_cm("drop"))
            w = {"apiVersion": "gc.amd.com/v1", "kind": "GCWidget",
                 "metadata": {"name": "w2", "namespace": "default", "ownerReferences": [_ref(keep), _ref(drop)]}}
            await c.create(w)
            gc = cm.get("garbagecollector")
            await _until(lambda: _has_uid(gc, keep), what="GC monitors the CR")
            await c.delete("configmaps", "drop", "default")

            async def patched():
                o = await c.get("gcwidgets.gc.amd.com", "w2", "default")
                return [r["uid"] for r in o["metadata"]["ownerReferences"]] == [m.uid_of(keep)]
            await _until(patched, what="dangling ref patched out of the CR")
        finally:
            await _stop(api, c, cm)
    run(go(), 60)


def test_three_thousand_owned_pods_cost_work_per_event_only():
    async def go():
        api, c, cm = await _cluster()
        try:
            owner = await c.create(_cm("many"))
            other = await c.create(_cm("one"))

            async def mk(i):
                await c.create(_owned_pod(f"p{i:04d}", _ref(owner)))
            for s in range(0, 3000, 200):
                await asyncio.gather(*(mk(i) for i in range(s, s + 200)))
            await c.create(_owned_pod("single", _ref(other)))
            gc = cm.get("garbagecollector")
            await _until(lambda: _dependents_n(gc, owner, 3000), what="graph has 3000 dependents")
            await asyncio.sleep(0.3)
            ev0, it0 = gc.graph.events_processed, gc.items_processed
            await asyncio.sleep(2.5)       # longer than the old 2 s rescan period: nothing happens
            assert (gc.graph.events_processed, gc.items_processed) == (ev0, it0)
            p = await c.get("pods", "p0007", "default")
            p["metadata"].setdefault("labels", {})["touched"] = "yes"
            await c.update(p)
            await _until(lambda: _ge(gc.graph.events_processed, ev0 + 1), what="update event")
            await asyncio.sleep(0.2)
            assert gc.graph.events_processed == ev0 + 1 and gc.items_processed == it0
            # an owner with one dependent: a handful of graph events and items, not thousands
            await c.delete("configmaps", "one", "default")
            await _until(lambda: _gone(c, "pods", "single"), what="single dependent collected")
            await asyncio.sleep(0.2)
            assert gc.graph.events_processed - ev0 <= 6 and gc.items_processed - it0 <= 4
        finally:
            await _stop(api, c, cm)
    run(go(), 120)


async def _dependents_n(gc, owner, n):
    node = gc.graph.uid_to_node.get(m.uid_of(owner))
    return node is not None and len(node.dependents) == n


async def _ge(a, b):
    return a >= b
