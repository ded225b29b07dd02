"""Pod GC and TTL controllers held to the reference's tests.

* pkg/controller/podgc/gc_controller_test.go — TestGCTerminated :58, TestGCOrphaned :153,
  TestGCUnscheduledTerminating :225 (every case; the deletePod hook records names, the node list
  comes from the client as the reference's fresh List does).
* pkg/controller/ttl/ttl_controller_test.go — TestPatchNode :33, TestUpdateNodeIfNeeded :93,
  TestDesiredTTL :155 (every case).
"""
from __future__ import annotations

import pytest

from amdkube.controllers.lifecycle import PodGCController
from amdkube.controllers.policy import TTL_ANNOTATION, TTLController
from tests.conftest import run
from tests.test_replicaset_parity import FakeInformer


class Client:
    def __init__(self, nodes=()):
        self.nodes = list(nodes)
        self.patches = []

    async def list(self, resource, ns="", **kw):
        assert resource == "nodes"
        return self.nodes, "1"

    async def patch(self, resource, name, patch, ns="", sub="", patch_type=""):
        self.patches.append((name, patch))


class Mgr:
    def __init__(self, nodes=()):
        self.client = Client(nodes)
        self.pods = FakeInformer()
        self.nodes = FakeInformer()


def gc_controller(threshold, nodes=()):
    mgr = Mgr(nodes)
    gcc = PodGCController(mgr, threshold=threshold)
    gcc.setup()
    deleted = []

    async def delete_pod(ns, name):
        deleted.append(name)
    gcc.delete_pod = delete_pod
    return gcc, deleted


def add_pods(gcc, pods):
    for i, (name, phase, *rest) in enumerate(pods):
        deletion, node = (rest + [None, "node"])[:2] if rest else (None, "node")
        md = {"name": name, "creationTimestamp": f"1970-01-01T{i + 1:02d}:00:00Z"}
        if deletion:
            md["deletionTimestamp"] = deletion
        gcc.pods.add({"metadata": md, "status": {"phase": phase}, "spec": {"nodeName": node} if node else {}})


@pytest.mark.parametrize("pods,threshold,deleted", [
    ([("a", "Failed"), ("b", "Succeeded")], 0, set()),                          # 0 disables terminated GC
    ([("a", "Failed"), ("b", "Succeeded"), ("c", "Failed")], 1, {"a", "b"}),
    ([("a", "Running"), ("b", "Succeeded"), ("c", "Failed")], 1, {"b"}),
    ([("a", "Failed"), ("b", "Succeeded")], 1, {"a"}),
    ([("a", "Failed"), ("b", "Succeeded")], 5, set()),
])
def test_gc_terminated(pods, threshold, deleted):
    gcc, got = gc_controller(threshold, nodes=[{"metadata": {"name": "node"}}])
    add_pods(gcc, pods)
    run(gcc.gc())
    assert set(got) == deleted and len(got) == len(deleted)


@pytest.mark.parametrize("pods,threshold,deleted", [
    ([("a", "Failed"), ("b", "Succeeded")], 0, {"a", "b"}),
    ([("a", "Running")], 1, {"a"}),
])
def test_gc_orphaned(pods, threshold, deleted):
    gcc, got = gc_controller(threshold)                                          # no nodes at all
    add_pods(gcc, pods)
    run(gcc.gc_orphaned(gcc.pods.list()))
    assert set(got) == deleted and len(got) == len(deleted)


@pytest.mark.parametrize("pods,deleted", [
    ([("a", "Failed", "1970-01-01T00:00:00Z", ""), ("b", "Succeeded", "1970-01-01T00:00:00Z", ""),
      ("c", "Running", "1970-01-01T00:00:00Z", "")], {"a", "b", "c"}),
    ([("a", "Failed", None, ""), ("b", "Succeeded", None, "node"), ("c", "Running", "1970-01-01T00:00:00Z", "node")], set()),
], ids=["Unscheduled pod in any phase must be deleted", "Scheduled pod in any phase must not be deleted"])
def test_gc_unscheduled_terminating(pods, deleted):
    gcc, got = gc_controller(-1)
    add_pods(gcc, pods)
    run(gcc.gc_unscheduled_terminating(gcc.pods.list()))
    assert set(got) == deleted and len(got) == len(deleted)


def test_terminated_order_is_creation_then_name():
    gcc, got = gc_controller(1, nodes=[{"metadata": {"name": "node"}}])
    for name in ("b", "a", "c"):
        gcc.pods.add({"metadata": {"name": name, "creationTimestamp": "1970-01-01T01:00:00Z"},
                      "status": {"phase": "Failed"}, "spec": {"nodeName": "node"}})
    run(gcc.gc_terminated(gcc.pods.list()))
    assert sorted(got) == ["a", "b"]


# ------------------------------------------------------------------ TTL
def _node(ann=None, name=""):
    md = {"name": name} if name else {}
    if ann is not None:
        md["annotations"] = ann
    return {"metadata": md}


@pytest.mark.parametrize("node,ttl,patch", [
    (_node(), 0, {"metadata": {"annotations": {TTL_ANNOTATION: "0"}}}),
    (_node(), 10, {"metadata": {"annotations": {TTL_ANNOTATION: "10"}}}),
    (_node(name="name"), 10, {"metadata": {"annotations": {TTL_ANNOTATION: "10"}}}),
    (_node({}), 10, {"metadata": {"annotations": {TTL_ANNOTATION: "10"}}}),
    (_node({TTL_ANNOTATION: "0"}), 10, {"metadata": {"annotations": {TTL_ANNOTATION: "10"}}}),
    (_node({TTL_ANNOTATION: "0", "a": "b"}), 10, {"metadata": {"annotations": {TTL_ANNOTATION: "10"}}}),
    (_node({TTL_ANNOTATION: "10", "a": "b"}), 10, {}),
])
def test_patch_node(node, ttl, patch):
    assert TTLController.ttl_patch(node, ttl) == patch


@pytest.mark.parametrize("ann,desired,patch", [
    (None, 0, {"metadata": {"annotations": {TTL_ANNOTATION: "0"}}}),
    (None, 15, {"metadata": {"annotations": {TTL_ANNOTATION: "15"}}}),
    (None, 30, {"metadata": {"annotations": {TTL_ANNOTATION: "30"}}}),
    ({TTL_ANNOTATION: "0"}, 60, {"metadata": {"annotations": {TTL_ANNOTATION: "60"}}}),
    ({TTL_ANNOTATION: "60"}, 60, None),
    ({TTL_ANNOTATION: "60"}, 30, {"metadata": {"annotations": {TTL_ANNOTATION: "30"}}}),
])
def test_update_node_if_needed(ann, desired, patch):
    mgr = Mgr()
    c = TTLController(mgr)
    c.setup()
    mgr.nodes.items["name"] = _node(ann, "name")          # nodes are cluster-scoped: keyed by name
    c.desired_ttl = desired
    run(c.update_node_if_needed("name"))
    assert mgr.client.patches == ([] if patch is None else [("name", patch)])


@pytest.mark.parametrize("add,delete,count,desired,step,expected", [
    (True, False, 0, 0, 0, 0), (True, False, 99, 0, 0, 0), (True, False, 100, 0, 0, 15),
    (False, True, 101, 15, 1, 15), (False, True, 91, 15, 1, 15), (True, False, 91, 15, 1, 15),
    (False, True, 90, 15, 1, 0),
])
def test_desired_ttl(add, delete, count, desired, step, expected):
    c = TTLController(Mgr())
    c.setup()
    c.node_count, c.desired_ttl, c.boundary_step = count, desired, step
    if add:
        c.add_node(_node())
    if delete:
        c.delete_node(_node())
    assert c.desired_ttl == expected
