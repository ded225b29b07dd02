"""PodDisruptionBudget controller held to pkg/controller/disruption/disruption_test.go.

Every test is transcribed (TestNoSelector :347 … TestUpdateDisruptedPods :715) against
controllers.policy.DisruptionController with fake informers and a status updater that records
the last written status per budget (the reference's pdbStates + getUpdater). The owners live in
the informers the reference's finders read (ReplicaSets, Deployments, RCs, StatefulSets), matched
by UID.
"""
from __future__ import annotations

import datetime
import time
import uuid

from amdkube.api import meta as m
from amdkube.controllers.policy import DisruptionController
from tests.conftest import run
from tests.test_replicaset_parity import FakeFactory, FakeInformer


class States:
    """pdbStates: the status each budget was last written with."""

    def __init__(self):
        self.pdbs: dict[str, dict] = {}

    async def update(self, obj, sub=""):
        assert sub == "status"
        self.pdbs[m.key_of(obj)] = obj
        return obj

    def status(self, key) -> dict:
        return self.pdbs[key]["status"]

    def verify(self, key, allowed, healthy, desired, expected, disrupted=None):
        st = self.status(key)
        got = (st["disruptionsAllowed"], st["currentHealthy"], st["desiredHealthy"], st["expectedPods"],
               st.get("disruptedPods") or {}, st["observedGeneration"])
        assert got == (allowed, healthy, desired, expected, disrupted or {}, 0), got

    def verify_allowed(self, key, allowed):
        assert self.status(key)["disruptionsAllowed"] == allowed


class Mgr:
    def __init__(self):
        self.client = States()
        self.factory = FakeFactory()
        self.pods = FakeInformer()


def new_controller():
    mgr = Mgr()
    dc = DisruptionController(mgr)
    dc.setup()
    return dc, mgr.client


def sync(dc, key):
    """dc.sync, and the budget informer then sees what was written (the reference's stores are
    refreshed by the informer; the fake updater's write is what the next sync reads)."""
    run(dc.sync(key))
    written = dc.mgr.client.pdbs.get(key)
    if written is not None:
        dc.pdb_inf.add(written)


def foo_bar():
    return {"foo": "bar"}


def new_pdb(min_available=None, max_unavailable=None):
    spec = {"selector": {"matchLabels": foo_bar()}}
    if min_available is not None:
        spec["minAvailable"] = min_available
    if max_unavailable is not None:
        spec["maxUnavailable"] = max_unavailable
    pdb = {"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget",
           "metadata": {"uid": str(uuid.uuid4()), "name": "foobar", "namespace": "default", "resourceVersion": "18"},
           "spec": spec}
    return pdb, "default/foobar"


def new_pod(name, ready=True):
    return {"metadata": {"uid": str(uuid.uuid4()), "annotations": {}, "name": name, "namespace": "default",
                         "resourceVersion": "18", "labels": foo_bar()},
            "spec": {}, "status": {"conditions": [{"type": "Ready", "status": "True"}] if ready else []}}


def owner(kind, size, selector=None):
    return {"kind": kind, "metadata": {"uid": str(uuid.uuid4()), "name": "foobar", "namespace": "default",
                                       "resourceVersion": "18", "labels": foo_bar()},
            "spec": {"replicas": size, "selector": selector or ({"matchLabels": foo_bar()} if kind != "ReplicationController"
                                                               else foo_bar())}}


def set_owner(pod, o):
    pod["metadata"].setdefault("ownerReferences", []).append(
        {"uid": m.uid_of(o), "kind": o["kind"], "name": m.name_of(o), "controller": True,
         "apiVersion": "v1" if o["kind"] == "ReplicationController" else "apps/v1"})


def unready(pod):
    pod["status"]["conditions"] = []


def test_no_selector():
    dc, ps = new_controller()
    pdb, key = new_pdb(min_available=3)
    pdb["spec"]["selector"] = {}
    dc.pdb_inf.add(pdb)
    sync(dc, key)
    ps.verify(key, 0, 0, 3, 0)
    dc.pod_inf.add(new_pod("yo-yo-yo"))
    sync(dc, key)
    ps.verify(key, 0, 0, 3, 0)


def test_unavailable():
    dc, ps = new_controller()
    pdb, key = new_pdb(min_available=3)
    dc.pdb_inf.add(pdb)
    sync(dc, key)
    pods = []
    for i in range(4):
        ps.verify(key, 0, i, 3, i)
        p = new_pod(f"yo-yo-yo {i}")
        pods.append(p)
        dc.pod_inf.add(p)
        sync(dc, key)
    ps.verify(key, 1, 4, 3, 4)
    unready(pods[0])
    sync(dc, key)
    ps.verify(key, 0, 3, 3, 4)


def test_integer_max_unavailable():
    dc, ps = new_controller()
    pdb, key = new_pdb(max_unavailable=1)
    dc.pdb_inf.add(pdb)
    sync(dc, key)
    ps.verify_allowed(key, 0)                      # no pods: no disruption
    dc.pod_inf.add(new_pod("naked"))
    sync(dc, key)
    ps.verify_allowed(key, 0)


def test_integer_max_unavailable_with_scaling():
    dc, ps = new_controller()
    pdb, key = new_pdb(max_unavailable=2)
    dc.pdb_inf.add(pdb)
    rs = owner("ReplicaSet", 7)
    dc.rs_inf.add(rs)
    pod = new_pod("pod")
    set_owner(pod, rs)
    dc.pod_inf.add(pod)
    sync(dc, key)
    ps.verify(key, 0, 1, 5, 7)
    rs["spec"]["replicas"] = 5
    sync(dc, key)
    ps.verify(key, 0, 1, 3, 5)


def test_naked_pod():
    dc, ps = new_controller()
    pdb, key = new_pdb(min_available="28%")
    dc.pdb_inf.add(pdb)
    sync(dc, key)
    ps.verify_allowed(key, 0)
    dc.pod_inf.add(new_pod("naked"))
    sync(dc, key)
    ps.verify_allowed(key, 0)


def test_replica_set():
    dc, ps = new_controller()
    pdb, key = new_pdb(min_available="20%")
    dc.pdb_inf.add(pdb)
    rs = owner("ReplicaSet", 10)
    dc.rs_inf.add(rs)
    pod = new_pod("pod")
    set_owner(pod, rs)
    dc.pod_inf.add(pod)
    sync(dc, key)
    ps.verify(key, 0, 1, 2, 10)


def test_multiple_controllers():
    dc, ps = new_controller()
    pdb, key = new_pdb(min_available="1%")
    dc.pdb_inf.add(pdb)
    pods = [new_pod(f"pod {i}") for i in range(2)]
    for p in pods:
        dc.pod_inf.add(p)
    sync(dc, key)
    ps.verify_allowed(key, 0)                       # no controllers yet
    rc = owner("ReplicationController", 1)
    rc["metadata"]["name"] = "rc 1"
    for p in pods:
        set_owner(p, rc)
    dc.rc_inf.add(rc)
    sync(dc, key)
    ps.verify_allowed(key, 1)                       # one RC, 200% > 1% healthy


def _controller_pods_test(kind, store_attr):
    labels = {"foo": "bar", "baz": "quux"}
    dc, ps = new_controller()
    pdb, key = new_pdb(min_available="34%")         # 34% of 3 rounds up to 2
    dc.pdb_inf.add(pdb)
    o = owner(kind, 3, selector=labels if kind == "ReplicationController" else {"matchLabels": labels})
    getattr(dc, store_attr).add(o)
    sync(dc, key)
    ps.verify(key, 0, 0, 0, 0)                      # no pods yet: the controller is not known
    for i in range(3):
        p = new_pod(f"foobar {i}")
        set_owner(p, o)
        p["metadata"]["labels"] = dict(labels)
        dc.pod_inf.add(p)
        sync(dc, key)
        if i < 2:
            ps.verify(key, 0, i + 1, 2, 3)
        else:
            ps.verify(key, 1, 3, 2, 3)
    return dc, ps, key


def test_replication_controller():
    dc, ps, key = _controller_pods_test("ReplicationController", "rc_inf")
    dc.pod_inf.add(new_pod("rogue"))                # matches the budget, no controller: fail safe
    sync(dc, key)
    ps.verify_allowed(key, 0)
    assert ps.status(key)["currentHealthy"] == 3    # the rest of the status stands


def test_stateful_set_controller():
    _controller_pods_test("StatefulSet", "ss_inf")


def test_two_controllers():
    rc_labels = {"foo": "bar", "baz": "quux"}
    d_labels = {"foo": "bar", "baz": "quuux"}
    dc, ps = new_controller()
    collection, minimum_one, minimum_two = 11, 4, 7
    pdb, key = new_pdb(min_available="28%")
    dc.pdb_inf.add(pdb)
    rc = owner("ReplicationController", collection, selector=rc_labels)
    dc.rc_inf.add(rc)
    sync(dc, key)
    ps.verify(key, 0, 0, 0, 0)
    pods = []
    unavailable = collection - minimum_one - 1
    for i in range(1, collection + 1):
        p = new_pod(f"quux {i}")
        set_owner(p, rc)
        pods.append(p)
        p["metadata"]["labels"] = dict(rc_labels)
        if i <= unavailable:
            unready(p)
        dc.pod_inf.add(p)
        sync(dc, key)
        if i <= unavailable:
            ps.verify(key, 0, 0, minimum_one, collection)
        elif i - unavailable <= minimum_one:
            ps.verify(key, 0, i - unavailable, minimum_one, collection)
        else:
            ps.verify(key, 1, i - unavailable, minimum_one, collection)
    d = owner("Deployment", collection, selector={"matchLabels": d_labels})
    dc.d_inf.add(d)
    sync(dc, key)
    ps.verify(key, 1, minimum_one + 1, minimum_one, collection)
    rs = owner("ReplicaSet", collection, selector={"matchLabels": d_labels})
    rs["metadata"]["labels"] = dict(d_labels)
    dc.rs_inf.add(rs)
    sync(dc, key)
    ps.verify(key, 1, minimum_one + 1, minimum_one, collection)
    unavailable = 2 * collection - (minimum_two + 2) - unavailable
    for i in range(1, collection + 1):
        p = new_pod(f"quuux {i}")
        set_owner(p, rs)
        pods.append(p)
        p["metadata"]["labels"] = dict(d_labels)
        if i <= unavailable:
            unready(p)
        dc.pod_inf.add(p)
        sync(dc, key)
        if i <= unavailable:
            ps.verify(key, 0, minimum_one + 1, minimum_two, 2 * collection)
        elif i - unavailable <= minimum_two - (minimum_one + 1):
            ps.verify(key, 0, (minimum_one + 1) + (i - unavailable), minimum_two, 2 * collection)
        else:
            ps.verify(key, i - unavailable - (minimum_two - (minimum_one + 1)), (minimum_one + 1) + (i - unavailable),
                      minimum_two, 2 * collection)
    ps.verify(key, 2, 2 + minimum_two, minimum_two, 2 * collection)
    unready(pods[collection - 1])
    sync(dc, key)
    ps.verify(key, 1, 1 + minimum_two, minimum_two, 2 * collection)
    unready(pods[collection - 2])
    sync(dc, key)
    ps.verify(key, 0, minimum_two, minimum_two, 2 * collection)
    pods[collection - 1]["status"]["conditions"] = [{"type": "Ready", "status": "True"}]
    sync(dc, key)
    ps.verify(key, 1, 1 + minimum_two, minimum_two, 2 * collection)


def test_pdb_not_exist():
    dc, ps = new_controller()
    pdb, _ = new_pdb(min_available="67%")
    dc.pdb_inf.add(pdb)
    sync(dc, "notExist")
    assert ps.pdbs == {}


def _ts(t: float) -> str:
    return datetime.datetime.fromtimestamp(int(t), datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def test_update_disrupted_pods():
    dc, ps = new_controller()
    pdb, key = new_pdb(min_available=1)
    now = time.time()
    pdb["status"] = {"disruptedPods": {"p1": _ts(now),            # removed: pod deletion started
                                       "p2": _ts(now - 300),      # removed: expired
                                       "p3": _ts(now),            # remains: pod untouched
                                       "notthere": _ts(now)}}     # removed: pod deleted
    dc.pdb_inf.add(pdb)
    p1 = new_pod("p1")
    p1["metadata"]["deletionTimestamp"] = _ts(now)
    for p in (p1, new_pod("p2"), new_pod("p3")):
        dc.pod_inf.add(p)
    sync(dc, key)
    ps.verify(key, 0, 1, 1, 3, {"p3": _ts(now)})


def test_recheck_is_scheduled_for_the_first_eviction_deadline():
    dc, ps = new_controller()
    pdb, key = new_pdb(min_available=1)
    now = time.time()
    pdb["status"] = {"disruptedPods": {"p3": _ts(now - 60)}}
    dc.pdb_inf.add(pdb)
    dc.pod_inf.add(new_pod("p3"))
    delays = []
    dc.queue.add_after = lambda item, delay: delays.append((item, delay))
    sync(dc, key)
    assert len(delays) == 1 and delays[0][0] == key and 55 < delays[0][1] <= 61
