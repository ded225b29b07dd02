"""ReplicaSet controller and the shared controller machinery, held to the reference's tests.

Transcribed, cited by line:
* pkg/controller/controller_utils_test.go — TestControllerExpectations :164, TestUIDExpectations
  :228, TestActivePodFiltering :317, TestSortingActivePods :344, TestActiveReplicaSetsFiltering
  :419; controller_ref_manager_test.go TestClaimPods :60.
* pkg/controller/replicaset/replica_set_utils_test.go — TestCalculateStatus :30,
  TestCalculateStatusConditions :150.
* pkg/controller/replicaset/replica_set_test.go — TestSyncReplicaSetDoesNothing :210,
  TestSyncReplicaSetCreateFailures :265, TestSyncReplicaSetDormancy :290, TestPodControllerLookup
  :358, TestUpdatePods :523, TestControllerUpdateRequeue :648,
  TestControllerUpdateStatusWithFailure :681, TestControllerBurstReplicas :727-879,
  TestRSSyncExpectations :888, TestDeleteControllerAndExpectations :915, TestOverlappingRSs :969,
  TestDeletionTimestamp :1012, TestDoNotPatchPodWithOtherControlRef :1118, TestPatchPodFails
  :1139, TestDoNotAdoptOrCreateIfBeingDeleted(Race) :1169-1248, TestSlowStartBatch :1376,
  TestGetPodsToDelete :1446.
The reference's fakes (FakePodControl, the fake clientset's reactors, informer indexers, a fake
clock) are re-expressed below; the controller under test is amdkube's.
"""
from __future__ import annotations

import asyncio
import itertools
import json
import random
import uuid

import pytest

from amdkube.api import meta as m
from amdkube.api.labels import selector_from_label_selector
from amdkube.controllers import controller_utils as CU
from amdkube.controllers.replicaset import ReplicaSetController, calculate_status, get_pods_to_delete
from tests.conftest import run

NOW = 1_700_000_000.0


# ------------------------------------------------------------------ fakes
class FakeInformer:
    def __init__(self):
        self.items: dict[str, dict] = {}

    def add(self, o):
        self.items[m.key_of(o)] = o

    def delete(self, o):
        self.items.pop(m.key_of(o), None)

    def get(self, key):
        return self.items.get(key)

    def list(self):
        return list(self.items.values())

    def add_handler(self, **kw):
        pass


class FakeFactory:
    def __init__(self):
        self.infs: dict[str, FakeInformer] = {}

    def informer(self, name):
        return self.infs.setdefault(name, FakeInformer())


class FakeClient:
    """fake.Clientset: an object tracker plus prepended reactors."""

    def __init__(self, *objs):
        self.objs = {m.key_of(o): json.loads(json.dumps(o)) for o in objs}
        self.actions: list[tuple] = []
        self.reactors: list = []          # fn(verb, resource, sub, obj) -> (handled, result | Exception)

    def _react(self, verb, resource, sub, obj):
        self.actions.append((verb, resource, sub, obj))
        for r in self.reactors:
            handled, res = r(verb, resource, sub, obj)
            if handled:
                if isinstance(res, BaseException):
                    raise res
                return res, True
        return None, False

    async def get(self, resource, name, ns=""):
        res, handled = self._react("get", resource, "", name)
        if handled:
            return res
        o = self.objs.get(f"{ns}/{name}" if ns else name)
        if o is None:
            raise m.StatusError(404, "NotFound", "not found")
        return json.loads(json.dumps(o))

    async def update(self, obj, sub=""):
        res, handled = self._react("update", "replicasets", sub, obj)
        if handled:
            return res
        self.objs[m.key_of(obj)] = json.loads(json.dumps(obj))
        return obj


class FakeMgr:
    def __init__(self, client):
        self.client = client
        self.factory = FakeFactory()
        self.pods = FakeInformer()
        self.recorder = None


class FakePodControl:
    """controller.FakePodControl: records templates / deletions / patches; CreateLimit and Err."""

    def __init__(self):
        self.clear()
        self.create_limit = 0
        self.err = None

    def clear(self):
        self.templates, self.delete_pod_names, self.patches = [], [], []
        self.create_call_count = 0

    async def create_pods_with_controller_ref(self, ns, template, owner, ref):
        self.create_call_count += 1
        if self.create_limit and self.create_call_count > self.create_limit:
            raise RuntimeError(f"Not creating pod, limit {self.create_limit} already reached")
        self.templates.append(template)
        if self.err:
            raise self.err

    async def delete_pod(self, ns, name, owner):
        self.delete_pod_names.append(name)
        if self.err:
            raise self.err

    async def patch_pod(self, ns, name, patch):
        self.patches.append(patch)
        if self.err:
            raise self.err


def new_replica_set(replicas, selector):
    """replica_set_test.go:91 newReplicaSet."""
    return {"apiVersion": "apps/v1", "kind": "ReplicaSet",
            "metadata": {"uid": str(uuid.uuid4()), "name": "foobar", "namespace": "default", "resourceVersion": "18"},
            "spec": {"replicas": replicas, "selector": {"matchLabels": dict(selector)},
                     "template": {"metadata": {"labels": {"name": "foo", "type": "production"}},
                                  "spec": {"containers": [{"image": "foo/bar"}], "restartPolicy": "Always",
                                           "dnsPolicy": "Default", "nodeSelector": {"baz": "blah"}}}},
            "status": {}}


def owner_ref(rs):
    return {"uid": m.uid_of(rs), "apiVersion": "v1beta1", "kind": "ReplicaSet", "name": m.name_of(rs), "controller": True}


def new_pod(name, rs, phase, last_transition=None, properly_owned=True):
    """replica_set_test.go:132 newPod (a Running pod is Ready)."""
    conds = []
    if phase == "Running":
        c = {"type": "Ready", "status": "True"}
        if last_transition is not None:
            c["lastTransitionTime"] = last_transition
        conds.append(c)
    return {"metadata": {"name": name, "namespace": m.namespace_of(rs), "labels": dict(rs["spec"]["selector"]["matchLabels"]),
                         "ownerReferences": [owner_ref(rs)] if properly_owned else [],
                         "resourceVersion": "1", "uid": str(uuid.uuid4())},
            "spec": {}, "status": {"phase": phase, "conditions": conds}}


def new_pod_list(store, count, phase, labels, rs, name):
    out = []
    for i in range(count):
        p = new_pod(f"{name}{i}", rs, phase, None, False)
        p["metadata"]["labels"] = dict(labels)
        p["metadata"]["ownerReferences"] = [owner_ref(rs)]
        if store is not None:
            store.add(p)
        out.append(p)
    return out


def manager(*objs, burst=500):
    client = FakeClient(*objs)
    mgr = FakeMgr(client)
    pc = FakePodControl()
    rsc = ReplicaSetController(mgr, pod_control=pc, clock=lambda: NOW)
    rsc.burst = burst
    rsc.setup()
    return rsc, pc, client


def validate(pc, creates, deletes, patches):
    assert (len(pc.templates), len(pc.delete_pod_names), len(pc.patches)) == (creates, deletes, patches)


def queued(rsc) -> set:
    out = set()
    while len(rsc.queue):
        k = rsc.queue.get_nowait()
        rsc.queue.done(k)
        out.add(k)
    return out


# ------------------------------------------------------------------ controller_utils_test.go
def test_controller_expectations():
    clock = [0.0]
    e = CU.ControllerExpectations(clock=lambda: clock[0], ttl=30.0)
    e.set_expectations("default/rc", 10, 30)
    for _ in range(11):
        e.creation_observed("default/rc")
    assert not e.satisfied_expectations("default/rc")
    for _ in range(31):
        e.deletion_observed("default/rc")
    assert e.get_expectations("default/rc") == (-1, -1) and e.satisfied_expectations("default/rc")
    e.set_expectations("default/rc", 1, 2)
    assert e.get_expectations("default/rc") == (1, 2)
    clock[0] += 31
    assert e.satisfied_expectations("default/rc")


def test_uid_expectations():
    e = CU.UIDTrackingControllerExpectations()
    rc_pods = {f"default/rc-{i}": [f"default/pod{j}-rc-{i}" for j in range(5)] for i in range(4)}
    for k, pods in rc_pods.items():
        e.expect_deletions(k, pods)
    keys = list(rc_pods)
    random.shuffle(keys)
    for k in keys:
        assert not e.satisfied_expectations(k)
        for p in rc_pods[k]:
            e.deletion_observed(k, p)
        assert e.satisfied_expectations(k)
        e.delete_expectations(k)
        assert e.get_uids(k) is None


def test_active_pod_filtering():
    rs = new_replica_set(0, {"foo": "bar"})
    pods = new_pod_list(None, 5, "Running", {"foo": "bar"}, rs, "pod")
    pods[0]["status"]["phase"], pods[1]["status"]["phase"] = "Succeeded", "Failed"
    assert {m.name_of(p) for p in CU.filter_active_pods(pods)} == {"pod2", "pod3", "pod4"}


def test_sorting_active_pods():
    rs = new_replica_set(0, {"foo": "bar"})
    pods = new_pod_list(None, 9, "Running", {"foo": "bar"}, rs, "pod")
    for p in pods:
        p["status"]["conditions"] = []
        p["spec"]["nodeName"] = "foo"
    now, then = m.format_time(NOW), m.format_time(NOW - 31 * 86400)
    pods[0]["spec"]["nodeName"], pods[0]["status"]["phase"] = "", "Pending"
    pods[1]["spec"]["nodeName"], pods[1]["status"]["phase"] = "bar", "Pending"
    pods[2]["status"]["phase"] = "Unknown"
    for i, t, restarts in ((4, None, [3, 0]), (5, now, [3, 0]), (6, then, [3, 0]), (7, then, [2, 1]), (8, then, [2, 1])):
        c = {"type": "Ready", "status": "True"}
        if t:
            c["lastTransitionTime"] = t
        pods[i]["status"]["conditions"] = [c]
        pods[i]["status"]["containerStatuses"] = [{"restartCount": r} for r in restarts]
    pods[7]["metadata"]["creationTimestamp"] = now
    pods[8]["metadata"]["creationTimestamp"] = then
    want = [m.name_of(p) for p in pods]
    for _ in range(20):
        shuffled = random.sample(pods, len(pods))
        assert [m.name_of(p) for p in CU.sort_active_pods(shuffled)] == want


def test_active_replica_sets_filtering():
    rss = [dict(new_replica_set(0, {}), metadata={"name": "zero"}), None,
           dict(new_replica_set(1, {}), metadata={"name": "foo"}), dict(new_replica_set(2, {}), metadata={"name": "bar"})]
    assert {m.name_of(r) for r in CU.filter_active_replica_sets(rss)} == {"foo", "bar"}


PROD = {"key": "production"}
TEST = {"key": "test"}


def _claim_pod(name, labels, owner=None, deleting=False):
    p = {"metadata": {"name": name, "namespace": "default", "uid": name, "labels": dict(labels),
                      "ownerReferences": [{"uid": m.uid_of(owner), "controller": True, "kind": "ReplicationController"}]
                      if owner else []}}
    if deleting:
        p["metadata"]["deletionTimestamp"] = m.format_time(NOW)
    return p


@pytest.mark.parametrize("case", ["correct-label", "deleting-controller", "deleting-controller-keeps-owned", "other-owner",
                                  "release", "orphan-being-deleted"])
def test_claim_pods(case):
    """TestClaimPods (controller_ref_manager_test.go:60-160)."""
    ctl = {"metadata": {"uid": "123", "name": "c"}}
    other = {"metadata": {"uid": "AAAAA"}}
    released, adopted = [], []
    if case == "correct-label":
        pods, want = [_claim_pod("pod1", PROD), _claim_pod("pod2", TEST)], ["pod1"]
    elif case == "deleting-controller":
        ctl["metadata"]["deletionTimestamp"] = m.format_time(NOW)
        pods, want = [_claim_pod("pod1", PROD), _claim_pod("pod2", PROD)], []
    elif case == "deleting-controller-keeps-owned":
        ctl["metadata"]["deletionTimestamp"] = m.format_time(NOW)
        pods, want = [_claim_pod("pod1", PROD, ctl), _claim_pod("pod2", PROD)], ["pod1"]
    elif case == "other-owner":
        pods, want = [_claim_pod("pod1", PROD, ctl), _claim_pod("pod2", PROD, other)], ["pod1"]
    elif case == "release":
        pods, want = [_claim_pod("pod1", PROD, ctl), _claim_pod("pod2", TEST, ctl)], ["pod1"]
    else:
        pods, want = [_claim_pod("pod1", PROD, ctl, True), _claim_pod("pod2", PROD, None, True)], ["pod1"]

    async def adopt(p):
        adopted.append(m.name_of(p))

    async def release(p):
        released.append(m.name_of(p))

    async def ok():
        return ctl
    sel = selector_from_label_selector({"matchLabels": PROD})
    got = run(CU.ControllerRefManager(ctl, sel, adopt, release, ok).claim(pods))
    assert [m.name_of(p) for p in got] == want
    assert released == (["pod2"] if case == "release" else [])


# ------------------------------------------------------------------ replica_set_utils_test.go
def test_calculate_status():
    nfl = new_replica_set(1, {"name": "foo"})
    fl = new_replica_set(2, {"name": "foo", "type": "production"})
    long = new_replica_set(1, {"name": "foo", "type": "production"})
    long["spec"]["minReadySeconds"] = 3600
    cases = [(fl, [new_pod("pod1", fl, "Running")], (1, 1, 1, 1)),
             (nfl, [new_pod("pod1", nfl, "Running")], (1, 0, 1, 1)),
             (fl, [new_pod("pod1", fl, "Running"), new_pod("pod2", fl, "Running")], (2, 2, 2, 2)),
             (nfl, [new_pod("pod1", nfl, "Running"), new_pod("pod2", nfl, "Running")], (2, 0, 2, 2)),
             (nfl, [new_pod("pod1", nfl, "Running"), new_pod("pod2", fl, "Running")], (2, 1, 2, 2)),
             (fl, [new_pod("pod1", fl, "Pending")], (1, 1, 0, 0)),
             (long, [new_pod("pod1", long, "Running")], (1, 1, 1, 0))]
    for rs, pods, want in cases:
        st = calculate_status(rs, pods, None, NOW)
        assert (st["replicas"], st["fullyLabeledReplicas"], st["readyReplicas"], st["availableReplicas"]) == want
        assert not st.get("conditions")


def test_calculate_status_conditions():
    rs = new_replica_set(2, {"name": "foo"})
    failing = new_replica_set(10, {"name": "foo"})
    failing["status"]["conditions"] = [{"type": "ReplicaFailure", "status": "True"}]
    err = RuntimeError("fake manageReplicasErr")

    def conds(r, pods, e):
        return [{k: c[k] for k in ("type", "status", "reason", "message") if k in c}
                for c in calculate_status(r, pods, e, NOW).get("conditions") or []]
    assert conds(rs, [new_pod("pod1", rs, "Running")], err) == [
        {"type": "ReplicaFailure", "status": "True", "reason": "FailedCreate", "message": "fake manageReplicasErr"}]
    assert conds(rs, [new_pod(f"pod{i}", rs, "Running") for i in range(3)], err) == [
        {"type": "ReplicaFailure", "status": "True", "reason": "FailedDelete", "message": "fake manageReplicasErr"}]
    assert conds(failing, [new_pod("pod1", failing, "Running")], None) == []
    assert conds(failing, [new_pod("pod1", failing, "Running")], err) == [{"type": "ReplicaFailure", "status": "True"}]
    assert conds(rs, [new_pod("pod1", rs, "Running")], None) == []


# ------------------------------------------------------------------ replica_set_test.go
def test_sync_replica_set_does_nothing():
    rs = new_replica_set(2, {"foo": "bar"})
    rsc, pc, _ = manager()
    rsc.rs_inf.add(rs)
    new_pod_list(rsc.pod_inf, 2, "Running", {"foo": "bar"}, rs, "pod")
    run(rsc.sync(m.key_of(rs)))
    validate(pc, 0, 0, 0)


def test_sync_replica_set_create_failures():
    rs = new_replica_set(100, {"foo": "bar"})
    rsc, pc, _ = manager(rs)
    pc.create_limit = 10
    rsc.rs_inf.add(rs)
    with pytest.raises(RuntimeError):
        run(rsc.sync(m.key_of(rs)))
    validate(pc, 10, 0, 0)
    limit, p = 0, 0
    while limit <= pc.create_limit:
        limit += 1 << p
        p += 1
    assert pc.create_call_count <= limit


def test_sync_replica_set_dormancy():
    rs = new_replica_set(2, {"foo": "bar"})
    rsc, pc, client = manager(rs)
    rsc.rs_inf.add(rs)
    new_pod_list(rsc.pod_inf, 1, "Running", {"foo": "bar"}, rs, "pod")
    rs["status"].update({"replicas": 1, "readyReplicas": 1, "availableReplicas": 1})
    run(rsc.sync(m.key_of(rs)))
    validate(pc, 1, 0, 0)
    rs["status"].update({"replicas": 0, "readyReplicas": 0, "availableReplicas": 0})   # expectations hold creates back
    pc.clear()
    run(rsc.sync(m.key_of(rs)))
    validate(pc, 0, 0, 0)
    rsc.expectations.creation_observed(m.key_of(rs))          # lowered: the next sync creates, and fails
    rs["status"].update({"replicas": 1, "readyReplicas": 1, "availableReplicas": 1})
    pc.clear()
    pc.err = RuntimeError("Fake Error")
    with pytest.raises(RuntimeError):
        run(rsc.sync(m.key_of(rs)))
    validate(pc, 1, 0, 0)
    pc.clear()                                                 # the failed create lowered the expectations
    pc.err = None
    run(rsc.sync(m.key_of(rs)))
    validate(pc, 1, 0, 0)


def test_pod_controller_lookup():
    rsc, _, _ = manager()
    cases = [([{"metadata": {"name": "basic", "namespace": ""}, "spec": {}}],
              {"metadata": {"name": "foo1", "namespace": ""}}, ""),
             ([{"metadata": {"name": "foo", "namespace": ""}, "spec": {"selector": {"matchLabels": {"foo": "bar"}}}}],
              {"metadata": {"name": "foo2", "namespace": "ns", "labels": {"foo": "bar"}}}, ""),
             ([{"metadata": {"name": "bar", "namespace": "ns"}, "spec": {"selector": {"matchLabels": {"foo": "bar"}}}}],
              {"metadata": {"name": "foo3", "namespace": "ns", "labels": {"foo": "bar"}}}, "bar")]
    for rss, pod, want in cases:
        for r in rss:
            rsc.rs_inf.add(r)
        got = rsc.pod_owners(pod)
        assert [m.name_of(r) for r in got] == ([want] if want else [])


def test_update_pods():
    async def go():
        rsc, _, _ = manager()
        rs1 = new_replica_set(1, {"foo": "bar"})
        rs2 = json.loads(json.dumps(rs1))
        rs2["spec"]["selector"] = {"matchLabels": {"bar": "foo"}}
        rs2["metadata"].update(name="barfoo", uid=str(uuid.uuid4()))
        rsc.rs_inf.add(rs1)
        rsc.rs_inf.add(rs2)
        ref1, ref2 = (dict(owner_ref(r), apiVersion="v1") for r in (rs1, rs2))

        def pair(labels1, refs1, labels2, refs2):
            p1 = new_pod_list(rsc.pod_inf, 1, "Running", {"foo": "bar"}, rs1, "pod")[0]
            p1["metadata"].update(resourceVersion="1", labels=labels1, ownerReferences=refs1)
            p2 = json.loads(json.dumps(p1))
            p2["metadata"].update(resourceVersion="2", labels=labels2, ownerReferences=refs2)
            return p1, p2
        for (l1, r1, l2, r2), want in (
                (({"foo": "bar"}, [ref1], {"bar": "foo"}, [ref1]), {m.key_of(rs1)}),
                (({"bar": "foo"}, [ref2], {"bar": "foo"}, []), {m.key_of(rs2)}),
                (({"bar": "foo"}, [ref1], {"bar": "foo"}, []), {m.key_of(rs1), m.key_of(rs2)}),
                (({"foo": "bar"}, [ref2], {"bar": "foo"}, [ref2]), {m.key_of(rs2)})):
            rsc.update_pod(*pair(l1, r1, l2, r2))
            assert queued(rsc) == want
    run(go())


def test_controller_update_requeue():
    async def go():
        rs = new_replica_set(1, {"foo": "bar"})
        rsc, pc, client = manager(rs)
        client.reactors.append(lambda verb, res, sub, obj: (True, RuntimeError("failed to update status"))
                               if verb == "update" and sub == "status" else (False, None))
        rsc.rs_inf.add(rs)
        rs["status"] = {"replicas": 2}
        new_pod_list(rsc.pod_inf, 1, "Running", {"foo": "bar"}, rs, "pod")
        await rsc.start()
        rsc.enqueue(rs)
        for _ in range(50):
            await asyncio.sleep(0.01)
            if rsc.queue.num_requeues(m.key_of(rs)):
                break
        await rsc.stop()
        assert rsc.queue.num_requeues(m.key_of(rs)) >= 1     # requeued with rate limiting
    run(go())


def test_controller_update_status_with_failure():
    rs = new_replica_set(1, {"foo": "bar"})
    rsc, _, client = manager()
    client.reactors.append(lambda verb, res, sub, obj: (True, rs) if verb == "get" else (False, None))
    client.reactors.append(lambda verb, res, sub, obj: (True, m.StatusError(500, "InternalError", "Fake error")))
    with pytest.raises(m.StatusError):
        run(rsc.update_status(rs, {"replicas": 10}))
    gets = [a for a in client.actions if a[0] == "get"]
    updates = [a for a in client.actions if a[0] == "update"]
    assert len(gets) == 1 and len(updates) == 2 and all(a[3]["status"]["replicas"] == 10 for a in updates)


def _burst(burst, num):
    rs = new_replica_set(num, {"foo": "bar"})
    rsc, pc, _ = manager(rs, burst=burst)
    rsc.rs_inf.add(rs)
    key = m.key_of(rs)
    pods = new_pod_list(None, num, "Pending", {"foo": "bar"}, rs, "pod")
    for replicas in (num, 0):
        rs["spec"]["replicas"] = replicas
        rsc.rs_inf.add(rs)
        for _ in range(0, num, burst):
            run(rsc.sync(key))
            active = len(rsc.pod_inf.list())
            if replicas:
                expected = min(replicas - active, burst)
                validate(pc, expected, 0, 0)
                for p in pods[:expected - 1]:
                    rsc.pod_inf.add(p)
                    rsc.add_pod(p)
                assert rsc.expectations.get_expectations(key)[0] == 1
            else:
                expected = min(active - replicas, burst)
                validate(pc, 0, expected, 0)
                dels = sorted(rsc.expectations.get_uids(key))
                victims = [{"metadata": {"name": k.split("/")[1], "namespace": k.split("/")[0],
                                         "labels": {"foo": "bar"}, "ownerReferences": [owner_ref(rs)]}} for k in dels]
                for v in victims[:-1]:
                    rsc.pod_inf.delete(v)
                    rsc.delete_pod(v)
                assert rsc.expectations.get_expectations(key)[1] == 1
            pc.clear()
            run(rsc.sync(key))
            validate(pc, 0, 0, 0)                   # expectations still outstanding
            if replicas:
                rsc.pod_inf.add(pods[expected - 1])
                rsc.add_pod(pods[expected - 1])
            else:
                (last,) = rsc.expectations.get_uids(key)
                lp = {"metadata": {"name": last.split("/")[1], "namespace": "default", "labels": {"foo": "bar"},
                                   "ownerReferences": [owner_ref(rs)]}}
                rsc.pod_inf.delete(lp)
                rsc.delete_pod(lp)
            pods = pods[expected:]
        assert len(rsc.pod_inf.list()) == replicas
        pods = new_pod_list(None, replicas, "Running", {"foo": "bar"}, rs, "pod")


@pytest.mark.parametrize("burst,num", [(5, 30), (5, 12), (3, 2)])
def test_controller_burst_replicas(burst, num):
    _burst(burst, num)


def test_rs_sync_expectations():
    """A pod that lands between the expectations check and the pod list is counted."""
    rs = new_replica_set(2, {"foo": "bar"})
    rsc, pc, _ = manager(burst=2)
    rsc.rs_inf.add(rs)
    pods = new_pod_list(None, 2, "Pending", {"foo": "bar"}, rs, "pod")
    rsc.pod_inf.add(pods[0])

    class Exp(CU.UIDTrackingControllerExpectations):
        def satisfied_expectations(self, key):
            rsc.pod_inf.add(pods[1])
            return True
    rsc.expectations = Exp()
    run(rsc.sync(m.key_of(rs)))
    validate(pc, 0, 0, 0)


def test_delete_controller_and_expectations():
    rs = new_replica_set(1, {"foo": "bar"})
    rsc, pc, _ = manager(rs, burst=10)
    rsc.rs_inf.add(rs)
    key = m.key_of(rs)
    run(rsc.sync(key))
    validate(pc, 1, 0, 0)
    pc.clear()
    assert rsc.expectations.get_expectations(key) is not None
    rsc.rs_inf.delete(rs)
    run(rsc.sync(key))
    assert rsc.expectations.get_expectations(key) is None
    rsc.pod_inf.items.clear()
    run(rsc.sync(key))
    validate(pc, 0, 0, 0)


def test_overlapping_rss():
    async def go():
        rsc, _, _ = manager(burst=10)
        rss = []
        for j in range(1, 10):
            r = new_replica_set(1, {"foo": "bar"})
            r["metadata"].update(name=f"rs{j}", creationTimestamp="2014-11-30T00:00:00Z")
            rss.append(r)
        for r in random.sample(rss, len(rss)):
            rsc.rs_inf.add(r)
        rs = rss[3]
        pod = new_pod_list(None, 1, "Pending", {"foo": "bar"}, rs, "pod")[0]
        pod["metadata"]["ownerReferences"] = [dict(owner_ref(rs), apiVersion="v1")]
        rsc.add_pod(pod)
        assert queued(rsc) == {m.key_of(rs)}
    run(go())


def test_deletion_timestamp():
    async def go():
        rsc, _, _ = manager(burst=10)
        rs = new_replica_set(1, {"foo": "bar"})
        rsc.rs_inf.add(rs)
        key = m.key_of(rs)
        pod = new_pod_list(None, 1, "Pending", {"foo": "bar"}, rs, "pod")[0]
        pod["metadata"].update(deletionTimestamp=m.format_time(NOW), resourceVersion="1")
        rsc.expectations.expect_deletions(key, [CU.pod_key(pod)])
        rsc.add_pod(pod)                                     # a pod added with a deletion timestamp
        assert queued(rsc) == {key} and rsc.expectations.satisfied_expectations(key)
        old = new_pod_list(None, 1, "Pending", {"foo": "bar"}, rs, "pod")[0]
        old["metadata"]["resourceVersion"] = "2"
        rsc.expectations.expect_deletions(key, [CU.pod_key(pod)])
        rsc.update_pod(old, pod)                             # an update that sets it
        assert queued(rsc) == {key} and rsc.expectations.satisfied_expectations(key)
        second = {"metadata": {"namespace": "default", "name": "secondPod", "labels": {"foo": "bar"},
                               "ownerReferences": [dict(owner_ref(rs), apiVersion="v1")]}}
        rsc.expectations.expect_deletions(key, [CU.pod_key(second)])
        old["metadata"].update(deletionTimestamp=m.format_time(NOW), resourceVersion="2")
        rsc.update_pod(old, pod)                             # an unrelated deletion does not count
        assert not rsc.expectations.satisfied_expectations(key)
        rsc.delete_pod(pod)
        assert not rsc.expectations.satisfied_expectations(key)
        rsc.delete_pod(second)
        assert key in queued(rsc) and rsc.expectations.satisfied_expectations(key)
    run(go())


def test_do_not_patch_pod_with_other_control_ref():
    rs = new_replica_set(2, {"foo": "bar"})
    rsc, pc, _ = manager(rs)
    rsc.rs_inf.add(rs)
    pod = new_pod("pod", rs, "Running")
    pod["metadata"]["ownerReferences"] = [{"uid": str(uuid.uuid4()), "apiVersion": "v1beta1", "kind": "ReplicaSet",
                                           "name": "AnotherRS", "controller": True}]
    rsc.pod_inf.add(pod)
    run(rsc.sync(m.key_of(rs)))
    validate(pc, 2, 0, 0)


def test_patch_pod_fails():
    rs = new_replica_set(2, {"foo": "bar"})
    rsc, pc, _ = manager(rs)
    rsc.rs_inf.add(rs)
    rsc.pod_inf.add(new_pod("pod1", rs, "Running", properly_owned=False))
    rsc.pod_inf.add(new_pod("pod2", rs, "Running", properly_owned=False))
    pc.err = RuntimeError("Fake Error")
    with pytest.raises(RuntimeError, match="Fake Error"):
        run(rsc.sync(m.key_of(rs)))
    validate(pc, 0, 0, 2)


def test_do_not_adopt_or_create_if_being_deleted():
    rs = new_replica_set(2, {"foo": "bar"})
    rs["metadata"]["deletionTimestamp"] = m.format_time(NOW)
    rsc, pc, _ = manager(rs)
    rsc.rs_inf.add(rs)
    rsc.pod_inf.add(new_pod("pod1", rs, "Running", properly_owned=False))
    run(rsc.sync(m.key_of(rs)))
    validate(pc, 0, 0, 0)


def test_do_not_adopt_or_create_if_being_deleted_race():
    """The cached ReplicaSet is live, the fresh read says it is being deleted: no adoption."""
    rs = new_replica_set(2, {"foo": "bar"})
    rs["metadata"]["deletionTimestamp"] = m.format_time(NOW)
    rsc, pc, _ = manager(rs)
    live = json.loads(json.dumps(rs))
    live["metadata"].pop("deletionTimestamp")
    rsc.rs_inf.add(live)
    rsc.pod_inf.add(new_pod("pod1", rs, "Running", properly_owned=False))
    with pytest.raises(Exception):
        run(rsc.sync(m.key_of(rs)))
    validate(pc, 0, 0, 0)


@pytest.mark.parametrize("limit,successes,err,calls", [(0, 0, True, 1), (10, 10, False, 10), (5, 5, True, 7)])
def test_slow_start_batch(limit, successes, err, calls):
    counter = itertools.count(1)
    seen = []

    async def fn():
        n = next(counter)
        seen.append(n)
        if n > limit:
            raise RuntimeError("fake error")
    ok, e = run(CU.slow_start_batch(10, 1, fn))
    assert ok == successes and (e is not None) == err and len(seen) == calls


def test_get_pods_to_delete():
    rs = new_replica_set(1, {"name": "foo"})
    unscheduled_pending = new_pod("unscheduled-pending-pod", rs, "Pending")
    scheduled_pending = new_pod("scheduled-pending-pod", rs, "Pending")
    scheduled_pending["spec"]["nodeName"] = "fake-node"
    not_ready = new_pod("scheduled-running-not-ready-pod", rs, "Running")
    not_ready["spec"]["nodeName"] = "fake-node"
    not_ready["status"]["conditions"] = [{"type": "Ready", "status": "False"}]
    ready = new_pod("scheduled-running-ready-pod", rs, "Running")
    ready["spec"]["nodeName"] = "fake-node"
    ready["status"]["conditions"] = [{"type": "Ready", "status": "True"}]
    cases = [([], 0, []), ([not_ready, ready], 2, [not_ready, ready]), ([ready, not_ready], 1, [not_ready]),
             ([ready, not_ready, scheduled_pending, unscheduled_pending], 4, [ready, not_ready, scheduled_pending, unscheduled_pending]),
             ([scheduled_pending, unscheduled_pending], 1, [unscheduled_pending]),
             ([ready, not_ready, not_ready], 2, [not_ready, not_ready]),
             ([scheduled_pending, not_ready], 1, [scheduled_pending]),
             ([ready, not_ready, scheduled_pending, unscheduled_pending], 3, [unscheduled_pending, scheduled_pending, not_ready])]
    for pods, diff, want in cases:
        assert [m.name_of(p) for p in get_pods_to_delete(pods, diff)] == [m.name_of(p) for p in want]


# ------------------------------------------------------------------ in a LocalCluster
def test_orphans_are_adopted_and_relabelled_pods_released():
    """ClaimPods over the real apiserver: an orphan pod matching the selector gets the
    ReplicaSet as its controller (and counts toward replicas); a pod relabelled out of the
    selector loses the reference and a replacement is created."""
    from amdkube.localcluster import LocalCluster

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "orphan", "labels": {"app": "a"}},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}},
                           "default")
            rs = await c.create({"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": "a"},
                                 "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "a"}},
                                          "template": {"metadata": {"labels": {"app": "a"}}, "spec": {"containers": [
                                              {"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}}}, "default")
            for _ in range(200):
                o = await c.get("pods", "orphan", "default")
                pods = [p for p in (await c.list("pods", "default"))[0] if not p["metadata"].get("deletionTimestamp")]
                if (m.controller_ref(o) or {}).get("uid") == m.uid_of(rs) and len(pods) == 2:
                    break
                await asyncio.sleep(0.05)
            assert (m.controller_ref(o) or {}).get("uid") == m.uid_of(rs), o["metadata"].get("ownerReferences")
            assert len(pods) == 2          # the orphan counts: one pod created, not two
            await c.patch("pods", "orphan", {"metadata": {"labels": {"app": "other"}}}, "default")
            for _ in range(200):
                o = await c.get("pods", "orphan", "default")
                owned = [p for p in (await c.list("pods", "default"))[0]
                         if (m.controller_ref(p) or {}).get("uid") == m.uid_of(rs) and not p["metadata"].get("deletionTimestamp")]
                if m.controller_ref(o) is None and len(owned) == 2:
                    break
                await asyncio.sleep(0.05)
            assert m.controller_ref(o) is None and len(owned) == 2
    run(go(), 60)
