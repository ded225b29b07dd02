"""StatefulSet controller and ControllerRevision history held to the reference's tests.

Transcribed, cited by line (pkg/controller/statefulset/):
* stateful_set_utils_test.go — TestGetParentNameAndOrdinal :37, TestIsMemberOf :53,
  TestIdentityMatches :66, TestStorageMatches :88, TestUpdateIdentity :121, TestUpdateStorage
  :142, TestIsRunningAndReady :182, TestAscendingOrdinal :199, TestOverlappingStatefulSets :212,
  TestNewPodControllerRef :233, TestCreateApplyRevision :257.
* stateful_set_control_test.go — TestStatefulSetControl :73 (CreatesPods, ScalesUp, ScalesDown,
  ReplacesPods, RecreatesFailedPod, CreatePodFailure, UpdatePodFailure, UpdateSetStatusFailure,
  PodRecreateDeleteFailure, each Monotonic and Burst), ScaleDownDeleteError :407,
  _getSetRevisions :439, RollingUpdate :564, OnDeleteUpdate :737, RollingUpdateWithPartition
  :1003, LimitsHistory :1159, Rollback :1230; the fakes and the scale-up / scale-down / update
  drivers with their invariants (:1487-2090) re-expressed.
* stateful_pod_control_test.go — all 13 tests (:38-432).
* stateful_set_status_updater_test.go — all 5 tests.
* stateful_set_test.go — Creates / Deletes / RespectsTermination / BlocksScaling /
  DeletionTimestamp(Race) :37-235, the pod-event handler tests :236-495 (the tombstone case does
  not arise: amdkube informers deliver the last known object on delete), GetPodsForStatefulSet
  Adopt / Release :496-572.
pkg/controller/history/controller_history_test.go's behaviours (hash, equality, create with
collisions, renumber) are covered through getSetRevisions and the history unit tests below.
"""
from __future__ import annotations

import json
import random

import pytest

from amdkube.api import meta as m
from amdkube.api.labels import selector_from_label_selector
from amdkube.controllers import history as H
from amdkube.controllers import statefulset as S
from tests.conftest import run
from tests.test_replicaset_parity import FakeFactory, FakeInformer

RNG = random.Random(1234)


def _clone(o):
    return json.loads(json.dumps(o))


# ------------------------------------------------------------------ fixtures (stateful_set_utils_test.go:291-375)
def new_pvc(name):
    return {"metadata": {"name": name}, "spec": {"resources": {"requests": {"storage": "1"}}}}


def new_statefulset_with_volumes(replicas, name, pet_mounts, pod_mounts):
    mounts = pet_mounts + pod_mounts
    return {"apiVersion": "apps/v1beta1", "kind": "StatefulSet",
            "metadata": {"name": name, "namespace": "default", "uid": "test"},
            "spec": {"selector": {"matchLabels": {"foo": "bar"}}, "replicas": replicas,
                     "template": {"metadata": {"labels": {"foo": "bar"}},
                                  "spec": {"containers": [{"name": "nginx", "image": "nginx", "volumeMounts": mounts}],
                                           "volumes": [{"name": mt["name"], "hostPath": {"path": f"/tmp/{mt['name']}"}}
                                                       for mt in pod_mounts]}},
                     "volumeClaimTemplates": [new_pvc(mt["name"]) for mt in pet_mounts],
                     "serviceName": "governingsvc", "updateStrategy": {"type": "RollingUpdate"},
                     "revisionHistoryLimit": 2},
            "status": {}}


def new_statefulset(replicas):
    return new_statefulset_with_volumes(replicas, "foo", [{"name": "datadir", "mountPath": "/tmp/zookeeper"}],
                                        [{"name": "home", "mountPath": "/home"}])


def burst(s):
    s["spec"]["podManagementPolicy"] = "Parallel"
    return s


def set_ready(pod):
    conds = [c for c in pod.setdefault("status", {}).get("conditions") or [] if c.get("type") != "Ready"]
    pod["status"]["conditions"] = conds + [{"type": "Ready", "status": "True"}]


def fake_resource_version(o):
    md = o.setdefault("metadata", {})
    md["resourceVersion"] = str(int(md.get("resourceVersion") or 0) + 1)


# ------------------------------------------------------------------ stateful_set_utils_test.go
def test_get_parent_name_and_ordinal():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 1)
    assert S.parent_name_and_ordinal(pod) == ("foo", 1)
    pod["metadata"]["name"] = "1-bar"
    assert S.parent_name_and_ordinal(pod) == ("", -1)


def test_is_member_of():
    s, s2 = new_statefulset(3), new_statefulset(3)
    s2["metadata"]["name"] = "foo2"
    pod = S.new_statefulset_pod(s, 1)
    assert S.is_member_of(s, pod) and not S.is_member_of(s2, pod)


def test_identity_matches():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 1)
    assert S.identity_matches(s, pod)
    pod["metadata"]["name"] = "foo"
    assert not S.identity_matches(s, pod)
    pod = S.new_statefulset_pod(s, 1)
    pod["metadata"]["namespace"] = ""
    assert not S.identity_matches(s, pod)
    pod = S.new_statefulset_pod(s, 1)
    del pod["metadata"]["labels"][S.POD_NAME_LABEL]
    assert not S.identity_matches(s, pod)


def test_storage_matches():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 1)
    assert S.storage_matches(s, pod)
    pod["spec"]["volumes"] = None
    assert not S.storage_matches(s, pod)
    pod = S.new_statefulset_pod(s, 1)
    for v in pod["spec"]["volumes"]:
        v.pop("persistentVolumeClaim", None)
    assert not S.storage_matches(s, pod)
    pod = S.new_statefulset_pod(s, 1)
    for v in pod["spec"]["volumes"]:
        if v.get("persistentVolumeClaim"):
            v["persistentVolumeClaim"]["claimName"] = "foo"
    assert not S.storage_matches(s, pod)
    pod = S.new_statefulset_pod(s, 1)
    pod["metadata"]["name"] = "bar"
    assert not S.storage_matches(s, pod)


def test_update_identity():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 1)
    assert S.identity_matches(s, pod)
    pod["metadata"]["namespace"] = ""
    assert not S.identity_matches(s, pod)
    S.update_identity(s, pod)
    assert S.identity_matches(s, pod)
    del pod["metadata"]["labels"][S.POD_NAME_LABEL]
    S.update_identity(s, pod)
    assert S.identity_matches(s, pod)


def test_update_storage():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 1)
    assert S.storage_matches(s, pod)
    pod["spec"]["volumes"] = None
    assert not S.storage_matches(s, pod)
    S.update_storage(s, pod)
    assert S.storage_matches(s, pod)
    pod = S.new_statefulset_pod(s, 1)
    for v in pod["spec"]["volumes"]:
        v.pop("persistentVolumeClaim", None)
    assert not S.storage_matches(s, pod)
    S.update_storage(s, pod)
    assert S.storage_matches(s, pod)
    pod = S.new_statefulset_pod(s, 1)
    for v in pod["spec"]["volumes"]:
        if v.get("persistentVolumeClaim"):
            v["persistentVolumeClaim"]["claimName"] = "foo"
    assert not S.storage_matches(s, pod)
    S.update_storage(s, pod)
    assert S.storage_matches(s, pod)


def test_is_running_and_ready():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 1)
    assert not S.is_running_and_ready(pod)
    pod.setdefault("status", {})["phase"] = "Running"
    assert not S.is_running_and_ready(pod)
    set_ready(pod)
    assert S.is_running_and_ready(pod)


def test_ascending_ordinal():
    s = new_statefulset(10)
    perm = list(range(10))
    RNG.shuffle(perm)
    pods = S.sort_ascending_ordinal([S.new_statefulset_pod(s, v) for v in perm])
    assert [S.ordinal_of(p) for p in pods] == list(range(10))


def test_overlapping_statefulsets():
    perm = list(range(10))
    RNG.shuffle(perm)
    sets = []
    for v in perm:
        s = new_statefulset(10)
        s["metadata"]["creationTimestamp"] = m.format_time(1_600_000_000 + v)
        sets.append(s)
    sets.sort(key=S.overlapping_order)
    assert [S.overlapping_order(s) for s in sets] == sorted(S.overlapping_order(s) for s in sets)
    sets = []
    for v in perm:
        s = new_statefulset(10)
        s["metadata"]["name"] = str(v)
        sets.append(s)
    sets.sort(key=S.overlapping_order)
    assert [m.name_of(s) for s in sets] == [str(i) for i in range(10)]


def test_new_pod_controller_ref():
    s = new_statefulset(1)
    ref = m.controller_ref(S.new_statefulset_pod(s, 0))
    assert ref is not None
    assert (ref["apiVersion"], ref["kind"], ref["name"], ref["uid"], ref["controller"]) == \
        ("apps/v1", "StatefulSet", "foo", "test", True)


def test_create_apply_revision():
    s = new_statefulset(1)
    s["status"]["collisionCount"] = 0
    revision = S.new_revision(s, 1, 0)
    s["spec"]["template"]["spec"]["containers"][0]["name"] = "foo"
    s["metadata"].setdefault("annotations", {})["foo"] = "bar"
    restored = S.apply_revision(s, revision)
    restored_revision = S.new_revision(restored, 2, restored["status"].get("collisionCount"))
    assert H.equal_revision(revision, restored_revision)
    assert restored_revision["metadata"]["annotations"]["foo"] == "bar"


# ------------------------------------------------------------------ history
def test_history_hash_name_and_equality():
    s = new_statefulset(1)
    r1, r2 = S.new_revision(s, 1, 0), S.new_revision(s, 7, 0)
    assert m.name_of(r1) == m.name_of(r2) and H.equal_revision(r1, r2)        # revision number is not hashed
    r3 = S.new_revision(s, 1, 1)
    assert m.name_of(r3) != m.name_of(r1)                                     # the collision count is
    assert H.equal_revision(r1, r3) is False                                  # differing hash labels
    r3["metadata"]["labels"].pop(H.HASH_LABEL)
    assert H.equal_revision(r1, r3)                                           # same data, label gone
    assert r1["metadata"]["name"].startswith("foo-") and r1["metadata"]["labels"]["foo"] == "bar"
    assert H.revision_name("x" * 300, 5).startswith("x" * 223 + "-")
    assert H.fnv32(b"") == 0x811C9DC5 and H.fnv32(b"a") == 0x050C5D7E         # FNV-1 (32-bit) vectors


# ------------------------------------------------------------------ fakes (stateful_set_control_test.go:1487-1728)
class Tracker:
    def __init__(self):
        self.requests, self.err, self.after = 0, None, 0

    def error_ready(self):
        return self.err is not None and self.requests >= self.after

    def reset(self):
        self.err, self.after = None, 0


def internal_error():
    return m.StatusError(500, "InternalError", "Internal error occurred: API server failed")


def is_internal_error(e):
    return isinstance(e, m.StatusError) and e.reason == "InternalError"


class FakeHistory:
    """history.NewFakeHistory over a revision indexer."""

    def __init__(self, indexer):
        self.indexer = indexer

    def list(self, parent, selector):
        out = []
        for r in self.indexer.list():
            if m.namespace_of(r) != m.namespace_of(parent) or not selector.matches(m.labels_of(r)):
                continue
            ref = m.controller_ref(r)
            if ref is None or ref.get("uid") == m.uid_of(parent):
                out.append(r)
        return out

    async def create(self, parent, rev, collision):
        clone = _clone(rev)
        clone["metadata"]["namespace"] = m.namespace_of(parent)
        while True:
            clone["metadata"]["name"] = H.revision_name(m.name_of(parent), H.hash_revision(rev, collision[0]))
            if self.indexer.get(m.key_of(clone)) is not None:
                collision[0] += 1
                continue
            self.indexer.add(_clone(clone))
            return clone

    async def delete(self, rev):
        if self.indexer.get(m.key_of(rev)) is None:
            raise m.StatusError(404, "NotFound", "not found")
        self.indexer.delete(rev)

    async def update(self, rev, new_revision):
        clone = _clone(rev)
        clone["revision"] = new_revision
        self.indexer.add(clone)
        return clone

    async def adopt(self, parent, api_version, kind, rev):
        if m.controller_ref(rev) is not None:
            raise ValueError("attempt to adopt revision owned by another controller")
        clone = _clone(rev)
        clone["metadata"].setdefault("ownerReferences", []).append(m.new_controller_ref(parent, api_version, kind))
        self.indexer.add(clone)
        return clone


class FakePodControl:
    def __init__(self, pods, sets):
        self.pods, self.sets, self.claims = pods, sets, FakeInformer()
        self.create_tracker, self.update_tracker, self.delete_tracker = Tracker(), Tracker(), Tracker()

    def _selected(self, s):
        sel = selector_from_label_selector(s["spec"]["selector"])
        return [p for p in self.pods.list() if m.namespace_of(p) == m.namespace_of(s) and sel.matches(m.labels_of(p))]

    def list_pods(self, s):
        return [_clone(p) for p in self._selected(s)]

    def _mutate(self, s, ordinal, fn):
        pods = S.sort_ascending_ordinal(self.list_pods(s))
        if not 0 <= ordinal < len(pods):
            raise IndexError(f"ordinal {ordinal} out of range [0,{len(pods)})")
        pod = pods[ordinal]
        fn(pod)
        fake_resource_version(pod)
        self.pods.add(pod)
        return self.list_pods(s)

    def set_pod_pending(self, s, o):
        return self._mutate(s, o, lambda p: p.setdefault("status", {}).__setitem__("phase", "Pending"))

    def set_pod_running(self, s, o):
        return self._mutate(s, o, lambda p: p.setdefault("status", {}).__setitem__("phase", "Running"))

    def set_pod_ready(self, s, o):
        return self._mutate(s, o, set_ready)

    def add_terminating_pod(self, s, o):
        pod = S.new_statefulset_pod(s, o)
        pod["status"] = {"phase": "Running"}
        pod["metadata"]["deletionTimestamp"] = m.format_time(1_700_000_000)
        set_ready(pod)
        fake_resource_version(pod)
        self.pods.add(pod)
        return self.list_pods(s)

    def set_pod_terminated(self, s, o):
        pod = S.new_statefulset_pod(s, o)
        pod["metadata"]["deletionTimestamp"] = m.format_time(1_700_000_000)
        fake_resource_version(pod)
        self.pods.add(pod)
        return self.list_pods(s)

    @staticmethod
    def _gate(tracker):
        tracker.requests += 1
        if tracker.requests - 1 >= tracker.after and tracker.err is not None:
            err = tracker.err
            tracker.reset()
            raise err

    async def create(self, s, pod):
        self._gate(self.create_tracker)
        for c in S.get_pvcs(s, pod).values():
            self.claims.add(c)
        self.pods.add(_clone(pod))

    async def update(self, s, pod):
        self._gate(self.update_tracker)
        if not S.identity_matches(s, pod):
            S.update_identity(s, pod)
        if not S.storage_matches(s, pod):
            S.update_storage(s, pod)
            for c in S.get_pvcs(s, pod).values():
                self.claims.add(c)
        self.pods.add(_clone(pod))

    async def delete(self, s, pod):
        self._gate(self.delete_tracker)
        if self.pods.get(m.key_of(pod)) is not None:
            self.pods.delete(pod)


class FakeStatusUpdater:
    def __init__(self, sets):
        self.sets, self.tracker = sets, Tracker()

    async def update_status(self, s, status):
        FakePodControl._gate(self.tracker)
        s = _clone(s)
        s["status"] = dict(status)
        self.sets.add(s)
        return s


def setup_controller(*sets):
    pods, set_idx, revs = FakeInformer(), FakeInformer(), FakeInformer()
    for s in sets:
        set_idx.add(_clone(s))
    spc = FakePodControl(pods, set_idx)
    ssu = FakeStatusUpdater(set_idx)
    ssc = S.StatefulSetControl(spc, ssu, FakeHistory(revs))
    return spc, ssu, ssc


def get_set(spc, s):
    return _clone(spc.sets.get(m.key_of(s)))


# ------------------------------------------------------------------ invariants
def _claims_exist(s, spc, pod):
    for c in S.get_pvcs(s, pod).values():
        if spc.claims.get(m.key_of(c)) is None:
            raise AssertionError(f"claim {m.name_of(c)} for Pod {m.name_of(pod)} was not created")


def assert_monotonic_invariants(s, spc):
    pods = S.sort_ascending_ordinal(spc.list_pods(s))
    for o, p in enumerate(pods):
        if o > 0 and S.is_running_and_ready(p) and not S.is_running_and_ready(pods[o - 1]):
            raise AssertionError(f"Successor {m.name_of(p)} is Running and Ready while {m.name_of(pods[o - 1])} is not")
        if S.ordinal_of(p) != o:
            raise AssertionError(f"pods {m.name_of(p)} deployed in the wrong order {o}")
        if not S.storage_matches(s, p):
            raise AssertionError(f"pods {m.name_of(p)} does not match the storage specification")
        _claims_exist(s, spc, p)
        if not S.identity_matches(s, p):
            raise AssertionError(f"pods {m.name_of(p)} does not match the identity specification")


def assert_burst_invariants(s, spc):
    for p in S.sort_ascending_ordinal(spc.list_pods(s)):
        if not S.storage_matches(s, p):
            raise AssertionError(f"pods {m.name_of(p)} does not match the storage specification")
        _claims_exist(s, spc, p)
        if not S.identity_matches(s, p):
            raise AssertionError(f"pods {m.name_of(p)} does not match the identity specification")


def assert_update_invariants(s, spc):
    pods = S.sort_ascending_ordinal(spc.list_pods(s))
    assert_burst_invariants(s, spc)
    st = s["spec"].get("updateStrategy") or {}
    if st.get("type") == "OnDelete":
        return
    status = s.get("status") or {}
    for i in range(min(int(status.get("currentReplicas") or 0), len(pods))):
        if S.get_pod_revision(pods[i]) != status.get("currentRevision"):
            raise AssertionError(f"pod {m.name_of(pods[i])} want current revision {status.get('currentRevision')}")
    i = len(pods) - 1
    for _ in range(int(status.get("updatedReplicas") or 0)):
        if S.get_pod_revision(pods[i]) != status.get("updateRevision"):
            raise AssertionError(f"pod {m.name_of(pods[i])} want update revision {status.get('updateRevision')}")
        i -= 1


# ------------------------------------------------------------------ drivers (stateful_set_control_test.go:1842-2083)
async def _advance_one(s, spc, pods):
    """Give the first phaseless pod a phase, else move a random pod forward one step."""
    pods = S.sort_ascending_ordinal(pods)
    for o, p in enumerate(pods):
        if not (p.get("status") or {}).get("phase"):
            pods = spc.set_pod_pending(s, o)
            break
    if pods:
        o = RNG.randrange(len(pods))
        phase = (S.sort_ascending_ordinal(pods)[o].get("status") or {}).get("phase")
        if phase == "Pending":
            pods = spc.set_pod_running(s, o)
        elif phase == "Running":
            pods = spc.set_pod_ready(s, o)
        else:
            return None
    return pods


async def scale_up(s, ssc, spc, invariants, max_iter=2000):
    for _ in range(max_iter):
        if int((s.get("status") or {}).get("readyReplicas") or 0) >= int(s["spec"]["replicas"]):
            break
        pods = await _advance_one(s, spc, spc.list_pods(s))
        if pods is None:
            continue
        await ssc.update(s, pods)
        s = get_set(spc, s) | {"spec": s["spec"]}
        invariants(s, spc)
    else:
        raise AssertionError("scale up did not converge")
    invariants(s, spc)
    return s


async def scale_down(s, ssc, spc, invariants, max_iter=200):
    for _ in range(max_iter):
        if int((s.get("status") or {}).get("replicas") or 0) <= int(s["spec"]["replicas"]):
            break
        pods = S.sort_ascending_ordinal(spc.list_pods(s))
        ordinal = len(pods) - 1
        if ordinal >= 0:
            await ssc.update(s, pods)
            s = get_set(spc, s) | {"spec": s["spec"]}
            pods = spc.add_terminating_pod(s, ordinal)
            await ssc.update(s, pods)
            s = get_set(spc, s) | {"spec": s["spec"]}
            pods = S.sort_ascending_ordinal(spc.list_pods(s))
            if pods:
                spc.pods.delete(pods[-1])
        await ssc.update(s, pods)
        s = get_set(spc, s) | {"spec": s["spec"]}
        invariants(s, spc)
    else:
        raise AssertionError("scale down did not converge")
    invariants(s, spc)
    return s


def update_complete(s, pods) -> bool:
    pods = S.sort_ascending_ordinal(pods)
    st, status = s["spec"].get("updateStrategy") or {}, s.get("status") or {}
    if len(pods) != int(s["spec"]["replicas"]) or int(status.get("readyReplicas") or 0) != int(s["spec"]["replicas"]):
        return False
    if st.get("type") == "OnDelete":
        return True
    ru = st.get("rollingUpdate")
    if ru is None or int(ru.get("partition") or 0) <= 0:
        if int(status.get("currentReplicas") or 0) < int(s["spec"]["replicas"]):
            return False
        return all(S.get_pod_revision(p) == status.get("currentRevision") for p in pods)
    partition = int(ru["partition"])
    if len(pods) < partition:
        return False
    return all(S.get_pod_revision(p) == status.get("updateRevision") for p in pods[partition:])


async def update_control(s, ssc, spc, invariants, max_iter=3000):
    await ssc.update(s, spc.list_pods(s))
    s = get_set(spc, s) | {"spec": s["spec"]}
    pods = spc.list_pods(s)
    for _ in range(max_iter):
        if update_complete(s, pods):
            break
        pods = await _advance_one(s, spc, spc.list_pods(s))
        if pods is None:
            pods = spc.list_pods(s)
            continue
        await ssc.update(s, pods)
        s = get_set(spc, s) | {"spec": s["spec"]}
        invariants(s, spc)
        pods = spc.list_pods(s)
    else:
        raise AssertionError("update did not converge")
    invariants(s, spc)
    return s


# ------------------------------------------------------------------ TestStatefulSetControl
async def creates_pods(s, invariants):
    spc, _, ssc = setup_controller(s)
    await scale_up(s, ssc, spc, invariants)
    assert get_set(spc, s)["status"]["replicas"] == 3


async def scales_up(s, invariants):
    spc, _, ssc = setup_controller(s)
    s = await scale_up(s, ssc, spc, invariants)
    s["spec"]["replicas"] = 4
    await scale_up(s, ssc, spc, invariants)
    assert get_set(spc, s)["status"]["replicas"] == 4


async def scales_down(s, invariants):
    spc, _, ssc = setup_controller(s)
    s = await scale_up(s, ssc, spc, invariants)
    s["spec"]["replicas"] = 0
    s = await scale_down(s, ssc, spc, invariants)
    assert s["status"]["replicas"] == 0


async def replaces_pods(s, invariants):
    spc, _, ssc = setup_controller(s)
    await scale_up(s, ssc, spc, invariants)
    s = get_set(spc, s)
    assert s["status"]["replicas"] == 5
    pods = S.sort_ascending_ordinal(spc.list_pods(s))
    for i in (0, 2, 4):
        spc.pods.delete(pods[i])
    for i in range(0, 5, 2):
        await ssc.update(s, spc.list_pods(s))
        s = get_set(spc, s)
        pods = spc.set_pod_running(s, i)
        await ssc.update(s, pods)
        s = get_set(spc, s)
        spc.set_pod_ready(s, i)
    await ssc.update(s, spc.list_pods(s))
    assert get_set(spc, s)["status"]["replicas"] == 5


async def recreates_failed_pod(s, invariants):
    spc, _, ssc = setup_controller()
    await ssc.update(s, spc.list_pods(s))
    invariants(s, spc)
    pods = spc.list_pods(s)
    pods[0]["status"] = {"phase": "Failed"}
    spc.pods.add(_clone(pods[0]))
    await ssc.update(s, pods)
    invariants(s, spc)
    pods = spc.list_pods(s)
    assert not S.is_created(pods[0]), "StatefulSet did not recreate failed Pod"


async def create_pod_failure(s, invariants):
    spc, _, ssc = setup_controller(s)
    spc.create_tracker.err, spc.create_tracker.after = internal_error(), 2
    with pytest.raises(m.StatusError) as ei:
        await scale_up(s, ssc, spc, invariants)
    assert is_internal_error(ei.value)
    await scale_up(s, ssc, spc, invariants)
    assert get_set(spc, s)["status"]["replicas"] == 3


async def update_pod_failure(s, invariants):
    spc, _, ssc = setup_controller(s)
    spc.update_tracker.err, spc.update_tracker.after = internal_error(), 0
    await scale_up(s, ssc, spc, invariants)
    s = get_set(spc, s)
    assert s["status"]["replicas"] == 3
    pods = S.sort_ascending_ordinal([_clone(p) for p in spc.pods.list()])
    assert len(pods) == 3
    spc.pods.delete(pods[0])
    pods[0]["metadata"]["name"] = "goo-0"
    spc.pods.add(pods[0])
    with pytest.raises(m.StatusError) as ei:
        await ssc.update(s, pods)
    assert is_internal_error(ei.value)


async def update_set_status_failure(s, invariants):
    spc, ssu, ssc = setup_controller(s)
    ssu.tracker.err, ssu.tracker.after = internal_error(), 2
    with pytest.raises(m.StatusError) as ei:
        await scale_up(s, ssc, spc, invariants)
    assert is_internal_error(ei.value)
    await scale_up(s, ssc, spc, invariants)
    assert get_set(spc, s)["status"]["replicas"] == 3


async def pod_recreate_delete_failure(s, invariants):
    spc, _, ssc = setup_controller(s)
    await ssc.update(s, spc.list_pods(s))
    invariants(s, spc)
    pods = spc.list_pods(s)
    pods[0]["status"] = {"phase": "Failed"}
    spc.pods.add(_clone(pods[0]))
    spc.delete_tracker.err, spc.delete_tracker.after = internal_error(), 0
    with pytest.raises(m.StatusError) as ei:
        await ssc.update(s, pods)
    assert is_internal_error(ei.value)
    invariants(s, spc)
    await ssc.update(s, pods)
    invariants(s, spc)
    pods = spc.list_pods(s)
    assert not S.is_created(pods[0]), "StatefulSet did not recreate failed Pod"


CONTROL_CASES = [(creates_pods, 3), (scales_up, 3), (scales_down, 3), (replaces_pods, 5),
                 (recreates_failed_pod, 3), (create_pod_failure, 3), (update_pod_failure, 3),
                 (update_set_status_failure, 3), (pod_recreate_delete_failure, 3)]


@pytest.mark.parametrize("fn,size", CONTROL_CASES, ids=[f.__name__ for f, _ in CONTROL_CASES])
@pytest.mark.parametrize("mode", ["Monotonic", "Burst"])
def test_statefulset_control(fn, size, mode):
    s = new_statefulset(size)
    if mode == "Burst":
        run(fn(burst(s), assert_burst_invariants))
    else:
        run(fn(s, assert_monotonic_invariants))


def test_statefulset_control_scale_down_delete_error():
    async def go():
        s = new_statefulset(3)
        spc, _, ssc = setup_controller(s)
        await scale_up(s, ssc, spc, assert_monotonic_invariants)
        s = get_set(spc, s)
        s["spec"]["replicas"] = 0
        spc.delete_tracker.err, spc.delete_tracker.after = internal_error(), 2
        with pytest.raises(m.StatusError):
            await scale_down(s, ssc, spc, assert_monotonic_invariants)
        await scale_down(s, ssc, spc, assert_monotonic_invariants)
        assert get_set(spc, s)["status"]["replicas"] == 0
    run(go())


def test_statefulset_control_get_set_revisions():
    s = new_statefulset(3)
    s["status"]["collisionCount"] = 0
    rev0 = S.new_revision(s, 1, 0)
    s1 = _clone(s)
    s1["spec"]["template"]["spec"]["containers"][0]["image"] = "foo"
    s1["status"]["currentRevision"] = m.name_of(rev0)
    rev1 = S.new_revision(s1, 2, 0)
    s2 = _clone(s1)
    s2["spec"]["template"]["metadata"]["labels"]["new"] = "label"
    rev2 = S.new_revision(s2, 3, 0)

    def renumbered(r, n):
        r = _clone(r)
        r["revision"] = n
        return r
    cases = [("creates initial revision", [], s, 1, rev0, rev0),
             ("creates revision on update", [rev0], s1, 2, rev0, rev1),
             ("must not recreate a new revision of same set", [rev0, rev1], s1, 2, rev0, rev1),
             ("must rollback to a previous revision", [rev0, rev1, rev2], s1, 3, rev0, renumbered(rev1, 4))]

    async def go(existing, st, count, want_current, want_update):
        st = _clone(st)
        st["status"]["collisionCount"] = 0
        _, _, ssc = setup_controller()
        for r in existing:
            await ssc.history.create(st, r, [0])
        revisions = ssc.list_revisions(st)
        current, update, _ = await ssc.get_revisions(st, revisions)
        assert len(ssc.list_revisions(st)) == count
        assert H.equal_revision(current, want_current) and H.equal_revision(update, want_update)
        assert H.revision_of(current) == H.revision_of(want_current)
        assert H.revision_of(update) == H.revision_of(want_update)
    for name, existing, st, count, cur, upd in cases:
        run(go(existing, st, count, cur, upd))


ORIGINAL_IMAGE = "nginx"


def _images(pods):
    return [p["spec"]["containers"][0]["image"] for p in S.sort_ascending_ordinal(pods)]


def _image(s, image="foo", replicas=None):
    s["spec"]["template"]["spec"]["containers"][0]["image"] = image
    if replicas is not None:
        s["spec"]["replicas"] = replicas
    return s


UPDATE_CASES = [("monotonic image update", False, 3, None), ("monotonic image update and scale up", False, 3, 5),
                ("monotonic image update and scale down", False, 5, 3), ("burst image update", True, 3, None),
                ("burst image update and scale up", True, 3, 5), ("burst image update and scale down", True, 5, 3)]


@pytest.mark.parametrize("name,is_burst,initial,replicas", UPDATE_CASES, ids=[c[0] for c in UPDATE_CASES])
def test_statefulset_control_rolling_update(name, is_burst, initial, replicas):
    async def go():
        s = new_statefulset(initial)
        inv = assert_monotonic_invariants
        if is_burst:
            s, inv = burst(s), assert_burst_invariants
        spc, _, ssc = setup_controller(s)
        await scale_up(s, ssc, spc, inv)
        s = _image(get_set(spc, s), replicas=replicas)
        await update_control(s, ssc, spc, assert_update_invariants)
        assert all(i == "foo" for i in _images(spc.list_pods(s)))
    run(go())


@pytest.mark.parametrize("name,is_burst,initial,replicas", UPDATE_CASES, ids=[c[0] for c in UPDATE_CASES])
def test_statefulset_control_on_delete_update(name, is_burst, initial, replicas):
    async def go():
        s = new_statefulset(initial)
        s["spec"]["updateStrategy"] = {"type": "OnDelete"}
        inv = assert_monotonic_invariants
        if is_burst:
            s, inv = burst(s), assert_burst_invariants
        spc, _, ssc = setup_controller(s)
        await scale_up(s, ssc, spc, inv)
        s = _image(get_set(spc, s), replicas=replicas)
        s = await update_control(s, ssc, spc, assert_update_invariants)
        images = _images(spc.list_pods(s))
        want = [ORIGINAL_IMAGE if i < initial else "foo" for i in range(len(images))]
        assert images == want                                   # OnDelete: existing pods keep their template
        n = s["spec"]["replicas"]
        s["spec"]["replicas"] = 0
        s = await scale_down(s, ssc, spc, inv)
        s = get_set(spc, s) | {"spec": dict(s["spec"], replicas=n)}
        await scale_up(s, ssc, spc, inv)
        assert all(i == "foo" for i in _images(spc.list_pods(s)))   # recreated pods take the update
    run(go())


PARTITION_CASES = [("monotonic image update", False, None), ("monotonic image update and scale up", False, 5),
                   ("burst image update", True, None), ("burst image update and scale up", True, 5)]


@pytest.mark.parametrize("name,is_burst,replicas", PARTITION_CASES, ids=[c[0] for c in PARTITION_CASES])
def test_statefulset_control_rolling_update_with_partition(name, is_burst, replicas):
    async def go():
        s = new_statefulset(3)
        s["spec"]["updateStrategy"] = {"type": "RollingUpdate", "rollingUpdate": {"partition": 2}}
        inv = assert_monotonic_invariants
        if is_burst:
            s, inv = burst(s), assert_burst_invariants
        spc, _, ssc = setup_controller(s)
        await scale_up(s, ssc, spc, inv)
        s = _image(get_set(spc, s), replicas=replicas)
        await update_control(s, ssc, spc, assert_update_invariants)
        images = _images(spc.list_pods(s))
        assert images == [ORIGINAL_IMAGE if i < 2 else "foo" for i in range(len(images))]
    run(go())


@pytest.mark.parametrize("is_burst", [False, True], ids=["monotonic update", "burst update"])
def test_statefulset_control_limits_history(is_burst):
    async def go():
        s = new_statefulset(3)
        inv = assert_monotonic_invariants
        if is_burst:
            s, inv = burst(s), assert_burst_invariants
        spc, _, ssc = setup_controller(s)
        await scale_up(s, ssc, spc, inv)
        s = get_set(spc, s)
        for i in range(10):
            s = _image(s, f"foo-{i}")
            await update_control(s, ssc, spc, assert_update_invariants)
            s = get_set(spc, s) | {"spec": s["spec"]}
            await ssc.update(s, spc.list_pods(s))
            assert len(ssc.list_revisions(s)) <= s["spec"]["revisionHistoryLimit"] + 2
    run(go())


@pytest.mark.parametrize("name,is_burst,initial,replicas", UPDATE_CASES, ids=[c[0] for c in UPDATE_CASES])
def test_statefulset_control_rollback(name, is_burst, initial, replicas):
    async def go():
        s = new_statefulset(initial)
        inv = assert_monotonic_invariants
        if is_burst:
            s, inv = burst(s), assert_burst_invariants
        spc, _, ssc = setup_controller(s)
        await scale_up(s, ssc, spc, inv)
        s = _image(get_set(spc, s), replicas=replicas)
        s = await update_control(s, ssc, spc, assert_update_invariants)
        assert all(i == "foo" for i in _images(spc.list_pods(s)))
        revisions = H.sort_revisions(ssc.list_revisions(s))
        s = S.apply_revision(s, revisions[0])
        await update_control(s, ssc, spc, assert_update_invariants)
        assert all(i == ORIGINAL_IMAGE for i in _images(spc.list_pods(s)))
    run(go())


# ------------------------------------------------------------------ stateful_pod_control_test.go
class Recorder:
    def __init__(self):
        self.events = []

    def event(self, obj, etype, reason, msg):
        self.events.append(f"{etype} {reason} {msg}")


class ReactorClient:
    """fake.Clientset with reactors: fn(verb, resource, obj) -> (handled, result, error)."""

    def __init__(self):
        self.reactors, self.calls = [], []

    def on(self, verb, resource, fn, prepend=False):
        entry = (verb, resource, fn)
        if prepend:
            self.reactors.insert(0, entry)
        else:
            self.reactors.append(entry)

    def _react(self, verb, resource, obj):
        self.calls.append((verb, resource))
        for v, r, fn in self.reactors:
            if v in (verb, "*") and r in (resource, "*"):
                handled, res, err = fn(obj)
                if handled:
                    if err is not None:
                        raise err
                    return res
        return obj

    @staticmethod
    def _res(obj):
        return {"Pod": "pods", "PersistentVolumeClaim": "persistentvolumeclaims",
                "StatefulSet": "statefulsets"}.get(obj.get("kind"), "pods")

    async def create(self, obj, ns=""):
        return self._react("create", self._res(obj), obj)

    async def update(self, obj, sub=""):
        return self._react("update", self._res(obj), obj)

    async def delete(self, resource, name, ns=""):
        return self._react("delete", resource, name)


class ErrLister:
    def get(self, key):
        raise RuntimeError("API server down")


def _pod_control(client=None, pvcs=None, pods=None):
    rec = Recorder()
    return S.RealStatefulPodControl(client or ReactorClient(), pvcs if pvcs is not None else FakeInformer(),
                                    pods if pods is not None else FakeInformer(), rec), rec


def _ok(obj):
    return True, obj, None


def _fail(obj):
    return True, None, internal_error()


def test_pod_control_creates_pods():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    client = ReactorClient()
    client.on("create", "persistentvolumeclaims", _ok)
    client.on("create", "pods", _ok)
    control, rec = _pod_control(client)
    run(control.create(s, pod))
    assert len(rec.events) == 2 and all(e.startswith("Normal") for e in rec.events)


def test_pod_control_create_pod_exists():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    pvcs = FakeInformer()
    for c in S.get_pvcs(s, pod).values():
        pvcs.add(c)
    client = ReactorClient()
    client.on("create", "persistentvolumeclaims", _ok)
    client.on("create", "pods", lambda o: (True, pod, m.StatusError(409, "AlreadyExists", "exists")))
    control, rec = _pod_control(client, pvcs)
    with pytest.raises(m.StatusError) as ei:
        run(control.create(s, pod))
    assert m.is_already_exists(ei.value) and rec.events == []


def test_pod_control_create_pod_pvc_create_failure():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    client = ReactorClient()
    client.on("create", "persistentvolumeclaims", _fail)
    client.on("create", "pods", _ok)
    control, rec = _pod_control(client)
    with pytest.raises(Exception):
        run(control.create(s, pod))
    assert len(rec.events) == 2 and all(e.startswith("Warning") for e in rec.events)


def test_pod_control_create_pod_pvc_get_failure():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    client = ReactorClient()
    client.on("create", "persistentvolumeclaims", _fail)
    client.on("create", "pods", _ok)
    control, rec = _pod_control(client, ErrLister())
    with pytest.raises(Exception):
        run(control.create(s, pod))
    assert len(rec.events) == 2 and all(e.startswith("Warning") for e in rec.events)


def test_pod_control_create_pod_failed():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    client = ReactorClient()
    client.on("create", "persistentvolumeclaims", _ok)
    client.on("create", "pods", _fail)
    control, rec = _pod_control(client)
    with pytest.raises(m.StatusError):
        run(control.create(s, pod))
    assert len(rec.events) == 2 and rec.events[0].startswith("Normal") and rec.events[1].startswith("Warning")


def test_pod_control_no_op_update():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    client = ReactorClient()
    client.on("*", "*", lambda o: pytest.fail("no-op update should not make any client invocation"))
    control, rec = _pod_control(client)
    run(control.update(s, pod))
    assert rec.events == [] and client.calls == []


def test_pod_control_updates_identity():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    updated = []
    client = ReactorClient()
    client.on("update", "pods", lambda o: (updated.append(_clone(o)), (True, o, None))[1], prepend=True)
    control, rec = _pod_control(client)
    pod["metadata"]["name"] = "goo-0"
    run(control.update(s, pod))
    assert len(rec.events) == 1 and rec.events[0].startswith("Normal")
    assert S.identity_matches(s, updated[0])


def test_pod_control_update_identity_failure():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    pods = FakeInformer()
    goo = S.new_statefulset_pod(s, 0)
    goo["metadata"]["name"] = "goo-0"
    pods.add(goo)
    client = ReactorClient()

    def fail(o):
        pod["metadata"]["name"] = "goo-0"
        return True, None, internal_error()
    client.on("update", "pods", fail)
    control, rec = _pod_control(client, pods=pods)
    pod["metadata"]["name"] = "goo-0"
    with pytest.raises(m.StatusError):
        run(control.update(s, pod))
    assert len(rec.events) == 1 and rec.events[0].startswith("Warning")
    assert not S.identity_matches(s, pod)


def _without_claim_volumes(s, pod):
    pvcs = S.get_pvcs(s, pod)
    pod["spec"]["volumes"] = [v for v in pod["spec"]["volumes"] if v["name"] not in pvcs]


def test_pod_control_updates_pod_storage():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    _without_claim_volumes(s, pod)
    updated = []
    client = ReactorClient()
    client.on("update", "pods", _ok)
    client.on("create", "persistentvolumeclaims", _ok)
    client.on("update", "pods", lambda o: (updated.append(_clone(o)), (True, o, None))[1], prepend=True)
    control, rec = _pod_control(client)
    run(control.update(s, pod))
    assert len(rec.events) == 2 and all(e.startswith("Normal") for e in rec.events)
    assert S.storage_matches(s, updated[0])


def test_pod_control_update_pod_storage_failure():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    _without_claim_volumes(s, pod)
    client = ReactorClient()
    client.on("update", "pods", _ok)
    client.on("create", "persistentvolumeclaims", _fail)
    control, rec = _pod_control(client)
    with pytest.raises(Exception):
        run(control.update(s, pod))
    assert len(rec.events) == 2 and all(e.startswith("Warning") for e in rec.events)


def test_pod_control_update_pod_conflict_success():
    s = new_statefulset(3)
    pod = S.new_statefulset_pod(s, 0)
    pods = FakeInformer()
    goo = S.new_statefulset_pod(s, 0)
    goo["metadata"]["name"] = "goo-0"
    pods.add(goo)
    conflict = []
    client = ReactorClient()

    def update(o):
        if not conflict:
            conflict.append(1)
            return True, o, m.StatusError(409, "Conflict", "conflict")
        return True, o, None
    client.on("update", "pods", update)
    control, rec = _pod_control(client, pods=pods)
    pod["metadata"]["name"] = "goo-0"
    run(control.update(s, pod))
    assert len(rec.events) == 1 and rec.events[0].startswith("Normal")
    assert S.identity_matches(s, pod)


def test_pod_control_deletes_stateful_pod():
    s = new_statefulset(3)
    client = ReactorClient()
    client.on("delete", "pods", lambda o: (True, None, None))
    control, rec = _pod_control(client)
    run(control.delete(s, S.new_statefulset_pod(s, 0)))
    assert len(rec.events) == 1 and rec.events[0].startswith("Normal")


def test_pod_control_delete_failure():
    s = new_statefulset(3)
    client = ReactorClient()
    client.on("delete", "pods", _fail)
    control, rec = _pod_control(client)
    with pytest.raises(m.StatusError):
        run(control.delete(s, S.new_statefulset_pod(s, 0)))
    assert len(rec.events) == 1 and rec.events[0].startswith("Warning")


# ------------------------------------------------------------------ stateful_set_status_updater_test.go
def _status():
    return {"observedGeneration": 1, "replicas": 2}


def test_status_updater_updates_set_status():
    s = new_statefulset(3)
    client = ReactorClient()
    client.on("update", "statefulsets", _ok)
    out = run(S.RealStatusUpdater(client, FakeInformer()).update_status(s, _status()))
    assert out["status"]["replicas"] == 2


def test_status_updater_updates_observed_generation():
    s = new_statefulset(3)
    seen = []
    client = ReactorClient()
    client.on("update", "statefulsets", lambda o: (seen.append(o["status"].get("observedGeneration")), (True, o, None))[1])
    run(S.RealStatusUpdater(client, FakeInformer()).update_status(s, {"observedGeneration": 3, "replicas": 2}))
    assert seen == [3]


def test_status_updater_update_replicas_failure():
    s = new_statefulset(3)
    sets = FakeInformer()
    sets.add(s)
    client = ReactorClient()
    client.on("update", "statefulsets", _fail)
    with pytest.raises(m.StatusError):
        run(S.RealStatusUpdater(client, sets).update_status(s, _status()))


def test_status_updater_update_replicas_conflict():
    s = new_statefulset(3)
    sets = FakeInformer()
    sets.add(s)
    conflict = []
    client = ReactorClient()

    def update(o):
        if not conflict:
            conflict.append(1)
            return True, o, m.StatusError(409, "Conflict", "Object already exists")
        return True, o, None
    client.on("update", "statefulsets", update)
    out = run(S.RealStatusUpdater(client, sets).update_status(s, _status()))
    assert out["status"]["replicas"] == 2


def test_status_updater_update_replicas_conflict_failure():
    s = new_statefulset(3)
    sets = FakeInformer()
    sets.add(s)
    client = ReactorClient()
    client.on("update", "statefulsets", lambda o: (True, o, m.StatusError(409, "Conflict", "Object already exists")))
    with pytest.raises(m.StatusError):
        run(S.RealStatusUpdater(client, sets).update_status(s, _status()))


# ------------------------------------------------------------------ stateful_set_test.go
class Mgr:
    def __init__(self, client):
        self.client = client
        self.factory = FakeFactory()
        self.pods = FakeInformer()
        self.recorder = None


class GetClient:
    """The bare client the controller re-checks sets with, and patches pods through."""

    def __init__(self, *objs):
        self.objs = {m.key_of(o): _clone(o) for o in objs}
        self.patches = []

    async def get(self, resource, name, ns=""):
        o = self.objs.get(f"{ns}/{name}")
        if o is None:
            raise m.StatusError(404, "NotFound", "not found")
        return _clone(o)

    async def patch(self, resource, name, patch, ns="", patch_type=None):
        self.patches.append((resource, name, patch))
        return {}


def new_fake_controller(*objs):
    mgr = Mgr(GetClient(*objs))
    ssc = S.StatefulSetController(mgr)
    ssc.setup()
    spc = FakePodControl(ssc.pod_inf, ssc.set_inf)
    ssc.control = S.StatefulSetControl(spc, FakeStatusUpdater(ssc.set_inf), FakeHistory(ssc.rev_inf))
    return ssc, spc


async def fake_worker(ssc):
    k = ssc.queue.get_nowait()
    if k is not None:
        await ssc.sync(k)
        ssc.queue.done(k)


def _at(pods, o):
    return S.sort_ascending_ordinal(pods)[o] if 0 <= o < len(pods) else None


async def scale_up_controller(s, ssc, spc):
    spc.sets.add(_clone(s))
    ssc.enqueue(s)
    await fake_worker(ssc)
    for _ in range(100):
        if int((s.get("status") or {}).get("readyReplicas") or 0) >= int(s["spec"]["replicas"]):
            break
        pods = spc.list_pods(s)
        o = len(pods) - 1
        pods = spc.set_pod_pending(s, o)
        ssc.add_pod(_at(pods, o))
        await fake_worker(ssc)
        prev = _at(pods, o)
        pods = spc.set_pod_running(s, o)
        ssc.update_pod(prev, _at(pods, o))
        await fake_worker(ssc)
        prev = _at(pods, o)
        pods = spc.set_pod_ready(s, o)
        ssc.update_pod(prev, _at(pods, o))
        await fake_worker(ssc)
        assert_monotonic_invariants(s, spc)
        s = get_set(spc, s)
    assert_monotonic_invariants(s, spc)
    return s


async def scale_down_controller(s, ssc, spc):
    pods = spc.list_pods(s)
    o = len(pods) - 1
    prev = _at(pods, o)
    fake_resource_version(s)
    spc.sets.add(_clone(s))
    ssc.enqueue(s)
    await fake_worker(ssc)
    pods = spc.add_terminating_pod(s, o)
    pod = _at(pods, o)
    ssc.update_pod(prev, pod)
    await fake_worker(ssc)
    await spc.delete(s, pod)
    ssc.delete_pod(pod)
    await fake_worker(ssc)
    for _ in range(100):
        if int((s.get("status") or {}).get("replicas") or 0) <= int(s["spec"]["replicas"]):
            break
        pods = spc.list_pods(s)
        o = len(pods)
        pods = spc.add_terminating_pod(s, o)
        pod = _at(pods, o)
        ssc.update_pod(prev, pod)
        await fake_worker(ssc)
        await spc.delete(s, pod)
        ssc.delete_pod(pod)
        await fake_worker(ssc)
        s = get_set(spc, s)
    assert_monotonic_invariants(s, spc)
    return s


def test_controller_creates():
    async def go():
        s = new_statefulset(3)
        ssc, spc = new_fake_controller(s)
        s = await scale_up_controller(s, ssc, spc)
        assert get_set(spc, s)["status"]["replicas"] == 3
    run(go())


def test_controller_deletes():
    async def go():
        s = new_statefulset(3)
        ssc, spc = new_fake_controller(s)
        s = await scale_up_controller(s, ssc, spc)
        assert s["status"]["replicas"] == 3
        s["spec"]["replicas"] = 0
        s = await scale_down_controller(s, ssc, spc)
        assert get_set(spc, s)["status"]["replicas"] == 0
    run(go())


def test_controller_respects_termination():
    async def go():
        s = new_statefulset(3)
        ssc, spc = new_fake_controller(s)
        s = await scale_up_controller(s, ssc, spc)
        assert s["status"]["replicas"] == 3
        spc.add_terminating_pod(s, 3)
        pods = spc.add_terminating_pod(s, 4)
        await ssc.control.update(s, pods)
        pods = S.sort_ascending_ordinal(spc.list_pods(s))
        assert len(pods) == 5, "StatefulSet does not respect termination"
        await spc.delete(s, pods[3])
        await spc.delete(s, pods[4])
        s["spec"]["replicas"] = 0
        s = await scale_down_controller(s, ssc, spc)
        assert get_set(spc, s)["status"]["replicas"] == 0
    run(go())


def test_controller_blocks_scaling():
    async def go():
        s = new_statefulset(3)
        ssc, spc = new_fake_controller(s)
        s = await scale_up_controller(s, ssc, spc)
        s["spec"]["replicas"] = 5
        fake_resource_version(s)
        spc.sets.add(_clone(s))
        spc.set_pod_terminated(s, 0)
        ssc.enqueue(s)
        await fake_worker(ssc)
        pods = S.sort_ascending_ordinal(spc.list_pods(s))
        assert len(pods) == 3, "StatefulSet does not block scaling"
        await spc.delete(s, pods[0])
        ssc.enqueue(s)
        await fake_worker(ssc)
        assert len(spc.list_pods(s)) == 3, "StatefulSet does not resume when terminated Pod is removed"
    run(go())


def test_controller_deletion_timestamp():
    async def go():
        s = new_statefulset(3)
        s["metadata"]["deletionTimestamp"] = m.format_time(1_700_000_000)
        ssc, spc = new_fake_controller(s)
        spc.sets.add(_clone(s))
        ssc.enqueue(s)
        await fake_worker(ssc)
        assert spc.list_pods(s) == []
    run(go())


def test_controller_deletion_timestamp_race():
    async def go():
        s = new_statefulset(3)
        s["metadata"]["deletionTimestamp"] = m.format_time(1_700_000_000)    # the bare client: deleted
        ssc, spc = new_fake_controller(s)
        s2 = _clone(s)
        del s2["metadata"]["deletionTimestamp"]                              # the cache: not deleted
        spc.sets.add(s2)
        pod = S.new_statefulset_pod(s, 1)
        pod["metadata"]["ownerReferences"] = []                              # a matching orphan
        spc.pods.add(pod)
        ssc.enqueue(s)
        with pytest.raises(Exception):
            await fake_worker(ssc)
        assert len(spc.list_pods(s)) == 1
    run(go())


def _queued(ssc):
    out = []
    while len(ssc.queue):
        k = ssc.queue.get_nowait()
        ssc.queue.done(k)
        out.append(k)
    return out


def _named(name):
    s = new_statefulset(3)
    s["metadata"]["name"] = name
    return s


def test_controller_add_pod():
    ssc, spc = new_fake_controller()
    s1, s2 = new_statefulset(3), _named("foo2")
    spc.sets.add(s1)
    spc.sets.add(s2)
    ssc.add_pod(S.new_statefulset_pod(s1, 0))
    assert _queued(ssc) == ["default/foo"]
    ssc.add_pod(S.new_statefulset_pod(s2, 0))
    assert _queued(ssc) == ["default/foo2"]


def test_controller_add_pod_orphan():
    ssc, spc = new_fake_controller()
    s1, s2, s3 = new_statefulset(3), _named("foo2"), _named("foo3")
    s3["spec"]["selector"]["matchLabels"] = {"foo3": "bar"}
    for s in (s1, s2, s3):
        spc.sets.add(s)
    pod = S.new_statefulset_pod(s1, 0)
    pod["metadata"]["ownerReferences"] = []
    ssc.add_pod(pod)
    assert len(ssc.queue) == 2


def test_controller_add_pod_no_set():
    ssc, _ = new_fake_controller()
    ssc.add_pod(S.new_statefulset_pod(new_statefulset(3), 0))
    assert len(ssc.queue) == 0


def test_controller_update_pod():
    ssc, spc = new_fake_controller()
    s1, s2 = new_statefulset(3), _named("foo2")
    spc.sets.add(s1)
    spc.sets.add(s2)
    for s in (s1, s2):
        pod = S.new_statefulset_pod(s, 0)
        prev = _clone(pod)
        fake_resource_version(pod)
        ssc.update_pod(prev, pod)
        assert _queued(ssc) == [m.key_of(s)]


def test_controller_update_pod_with_no_set():
    ssc, _ = new_fake_controller()
    pod = S.new_statefulset_pod(new_statefulset(3), 0)
    prev = _clone(pod)
    fake_resource_version(pod)
    ssc.update_pod(prev, pod)
    assert len(ssc.queue) == 0


def test_controller_update_pod_with_same_version():
    ssc, spc = new_fake_controller()
    s = new_statefulset(3)
    spc.sets.add(s)
    pod = S.new_statefulset_pod(s, 0)
    ssc.update_pod(pod, pod)
    assert len(ssc.queue) == 0


def test_controller_update_pod_orphan_with_new_labels():
    ssc, spc = new_fake_controller()
    s, s2 = new_statefulset(3), _named("foo2")
    spc.sets.add(s)
    spc.sets.add(s2)
    pod = S.new_statefulset_pod(s, 0)
    pod["metadata"]["ownerReferences"] = []
    clone = _clone(pod)
    clone["metadata"]["labels"] = {"foo2": "bar2"}
    fake_resource_version(clone)
    ssc.update_pod(clone, pod)
    assert len(ssc.queue) == 2


def test_controller_update_pod_change_controller_ref():
    ssc, spc = new_fake_controller()
    s, s2 = new_statefulset(3), _named("foo2")
    spc.sets.add(s)
    spc.sets.add(s2)
    pod, pod2 = S.new_statefulset_pod(s, 0), S.new_statefulset_pod(s2, 0)
    clone = _clone(pod)
    clone["metadata"]["ownerReferences"] = pod2["metadata"]["ownerReferences"]
    fake_resource_version(clone)
    ssc.update_pod(clone, pod)
    assert len(ssc.queue) == 2


def test_controller_update_pod_release():
    ssc, spc = new_fake_controller()
    s, s2 = new_statefulset(3), _named("foo2")
    spc.sets.add(s)
    spc.sets.add(s2)
    pod = S.new_statefulset_pod(s, 0)
    clone = _clone(pod)
    clone["metadata"]["ownerReferences"] = []
    fake_resource_version(clone)
    ssc.update_pod(pod, clone)
    assert len(ssc.queue) == 2


def test_controller_delete_pod():
    ssc, spc = new_fake_controller()
    s1, s2 = new_statefulset(3), _named("foo2")
    spc.sets.add(s1)
    spc.sets.add(s2)
    ssc.delete_pod(S.new_statefulset_pod(s1, 0))
    assert _queued(ssc) == ["default/foo"]
    ssc.delete_pod(S.new_statefulset_pod(s2, 0))
    assert _queued(ssc) == ["default/foo2"]


def test_controller_delete_pod_orphan():
    ssc, spc = new_fake_controller()
    s1, s2 = new_statefulset(3), _named("foo2")
    spc.sets.add(s1)
    spc.sets.add(s2)
    pod = S.new_statefulset_pod(s1, 0)
    pod["metadata"]["ownerReferences"] = []
    ssc.delete_pod(pod)
    assert len(ssc.queue) == 0


def test_controller_get_statefulsets_for_pod():
    ssc, spc = new_fake_controller()
    s1, s2 = new_statefulset(3), _named("foo2")
    spc.sets.add(s1)
    spc.sets.add(s2)
    assert len(ssc.sets_for_pod(S.new_statefulset_pod(s1, 0))) == 2


def test_get_pods_for_statefulset_adopt():
    s = new_statefulset(5)
    ssc, spc = new_fake_controller(s)
    pod1 = S.new_statefulset_pod(s, 1)
    pod2 = S.new_statefulset_pod(s, 2)
    pod2["metadata"]["ownerReferences"] = []                    # an orphan with matching labels and name
    pod3 = S.new_statefulset_pod(s, 3)
    pod3["metadata"]["ownerReferences"] = []
    pod3["metadata"]["labels"] = None                           # wrong labels
    pod4 = S.new_statefulset_pod(s, 4)
    pod4["metadata"]["ownerReferences"] = []
    pod4["metadata"]["name"] = "x" + pod4["metadata"]["name"]   # wrong name
    for p in (pod1, pod2, pod3, pod4):
        spc.pods.add(p)
    sel = selector_from_label_selector(s["spec"]["selector"])
    got = {m.name_of(p) for p in run(ssc.pods_for_set(s, sel))}
    assert got == {m.name_of(pod1), m.name_of(pod2)}


def test_get_pods_for_statefulset_release():
    s = new_statefulset(3)
    ssc, spc = new_fake_controller(s)
    pod1 = S.new_statefulset_pod(s, 1)
    pod2 = S.new_statefulset_pod(s, 2)
    pod2["metadata"]["name"] = "x" + pod2["metadata"]["name"]   # owned, wrong name
    pod3 = S.new_statefulset_pod(s, 3)
    pod3["metadata"]["labels"] = None                           # owned, wrong labels
    for p in (pod1, pod2, pod3):
        spc.pods.add(p)
    sel = selector_from_label_selector(s["spec"]["selector"])
    got = {m.name_of(p) for p in run(ssc.pods_for_set(s, sel))}
    assert got == {m.name_of(pod1)}
    released = [name for _, name, patch in ssc.client.patches if patch["metadata"]["ownerReferences"][0].get("$patch")]
    assert sorted(released) == sorted([m.name_of(pod2), m.name_of(pod3)])
