"""Deployment controller held to the reference's tests.

Transcribed, cited by line (pkg/controller/deployment/):
* sync_test.go — TestScale :39 (18 cases, same harness: replicas annotations from the old
  deployment, then the update actions give the sizes), TestDeploymentController_cleanupDeployment
  :339.
* rolling_test.go — reconcileNewReplicaSet :29, reconcileOldReplicaSets :119,
  cleanupUnhealthyReplicas :216, scaleDownOldReplicaSetsForRollingUpdate :280.
* recreate_test.go — TestScaleDownOldReplicaSets :33, TestOldPodsRunning :85.
* progress_test.go — TestRequeueStuckDeployment :68, TestSyncRolloutStatus :176.
* deployment_controller_test.go — TestSyncDeploymentCreatesReplicaSet :276, ...DontDoAnything
  DuringDeletion :292, ...DeletionRace :305, TestDontSyncDeploymentsWithEmptyPodSelector :331,
  TestReentrantRollback :344, the four TestPodDeletion* :375-515, TestGetReplicaSetsForDeployment
  (AdoptRelease) :516-603, TestGetPodMapForReplicaSets :604, TestAdd/Update/DeleteReplicaSet*
  :670-975.
* util/deployment_util_test.go — TestEqualIgnoreHash :335, TestFindNewReplicaSet :416,
  TestFindOldReplicaSets :469, TestGetReplicaCountForReplicaSets :564, TestResolveFenceposts :606,
  TestNewRSNewReplicas :667, TestGet/Set/RemoveCondition :755-884, TestDeploymentComplete :885,
  TestDeploymentProgressing :962, TestDeploymentTimedOut :1057, TestMaxUnavailable :1131,
  TestAnnotationUtils :1211; util/hash_test.go TestPodTemplateSpecHash :107.
TestGetNewRS / TestGetOldRSs (:184, :242) exercise client-listing helpers amdkube does not have
(the controller lists from its informer); FindNew/FindOld cover the same selection logic.

Go aliasing the tests rely on is spelled out: newDeployment shares one map between the selector
and the template labels, newReplicaSet shares the deployment's selector, generateRS shares the
RS labels with its template labels.
"""
from __future__ import annotations

import asyncio
import copy
import json
import uuid

import pytest

from amdkube.api import meta as m
from amdkube.controllers import deployment as D
from amdkube.controllers.deployment import DeploymentController
from tests.conftest import run
from tests.test_replicaset_parity import FakeFactory, FakeInformer


def ts(*a) -> str:
    import datetime as _dt
    return _dt.datetime(*a, tzinfo=_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


NEW_TS = ts(2016, 5, 20, 2, 0, 0)
OLD_TS = ts(2016, 5, 20, 1, 0, 0)
OLDER_TS = ts(2016, 5, 20, 0, 0, 0)


# ------------------------------------------------------------------ fixtures (deployment_controller_test.go:56-146)
def rs(name, replicas, selector=None, timestamp=None):
    md = {"name": name, "namespace": "default"}
    if timestamp:
        md["creationTimestamp"] = timestamp
    return {"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": md,
            "spec": {"replicas": replicas, "selector": {"matchLabels": selector}, "template": {}}, "status": {}}


def new_rs_with_status(name, spec_replicas, status_replicas, selector=None):
    r = rs(name, spec_replicas, selector)
    r["status"] = {"replicas": status_replicas}
    return r


def new_deployment(name, replicas, history=None, max_surge=None, max_unavailable=None, selector=None):
    labels = selector                      # one map: selector and template labels (Go aliasing)
    d = {"apiVersion": "apps/v1", "kind": "Deployment",
         "metadata": {"uid": str(uuid.uuid4()), "name": name, "namespace": "default", "annotations": {}},
         "spec": {"strategy": {"type": "RollingUpdate",
                               "rollingUpdate": {"maxUnavailable": 0 if max_unavailable is None else max_unavailable,
                                                 "maxSurge": 0 if max_surge is None else max_surge}},
                  "replicas": replicas, "selector": {"matchLabels": labels},
                  "template": {"metadata": {"labels": labels}, "spec": {"containers": [{"image": "foo/bar"}]}}},
         "status": {}}
    if history is not None:
        d["spec"]["revisionHistoryLimit"] = history
    return d


def new_replica_set(d, name, replicas):
    return {"apiVersion": "apps/v1", "kind": "ReplicaSet",
            "metadata": {"name": name, "uid": str(uuid.uuid4()), "namespace": "default",
                         "labels": d["spec"]["selector"]["matchLabels"],
                         "ownerReferences": [m.new_controller_ref(d, "apps/v1", "Deployment")]},
            "spec": {"selector": d["spec"]["selector"], "replicas": replicas,
                     "template": copy.copy(d["spec"]["template"])},
            "status": {}}


def generate_pod_from_rs(r):
    return {"metadata": {"name": m.name_of(r) + "-pod", "namespace": m.namespace_of(r),
                         "labels": r["spec"]["selector"]["matchLabels"],
                         "ownerReferences": [{"uid": m.uid_of(r), "apiVersion": "v1beta1", "kind": "ReplicaSet",
                                              "name": m.name_of(r), "controller": True}]},
            "spec": (r["spec"].get("template") or {}).get("spec") or {}, "status": {}}


def _clone(o):
    return json.loads(json.dumps(o))


class Client:
    """fake.Clientset: tracked objects, recorded (verb, resource, subresource, object) actions."""

    def __init__(self, *objs):
        self.objs = {(self._res(o), m.key_of(o)): _clone(o) for o in objs}
        self.actions: list[tuple] = []

    @staticmethod
    def _res(o):
        return {"Deployment": "deployments", "ReplicaSet": "replicasets"}.get(o.get("kind"), "pods")

    async def get(self, resource, name, ns=""):
        self.actions.append(("get", resource, "", name))
        o = self.objs.get((resource, f"{ns}/{name}" if ns else name))
        if o is None:
            raise m.StatusError(404, "NotFound", f"{resource} {name} not found")
        return _clone(o)

    async def update(self, obj, sub=""):
        self.actions.append(("update", self._res(obj), sub, _clone(obj)))
        self.objs[(self._res(obj), m.key_of(obj))] = _clone(obj)
        return _clone(obj)

    async def create(self, obj, ns=""):
        self.actions.append(("create", self._res(obj), "", _clone(obj)))
        key = (self._res(obj), m.key_of(obj))
        if key in self.objs:
            raise m.StatusError(409, "AlreadyExists", "exists")
        self.objs[key] = _clone(obj)
        return _clone(obj)

    async def delete(self, resource, name, ns=""):
        self.actions.append(("delete", resource, "", name))
        self.objs.pop((resource, f"{ns}/{name}"), None)

    async def patch(self, resource, name, patch, ns="", patch_type=None):
        self.actions.append(("patch", resource, "", patch))
        return _clone(self.objs.get((resource, f"{ns}/{name}")) or {})

    def verbs(self):
        return [(a[0], a[1], a[2]) for a in self.actions]


class Mgr:
    def __init__(self, client):
        self.client = client
        self.factory = FakeFactory()
        self.pods = FakeInformer()
        self.recorder = None


def controller(objects=(), d_lister=(), rs_lister=(), pod_lister=(), clock=None):
    client = Client(*objects)
    mgr = Mgr(client)
    dc = DeploymentController(mgr, **({"clock": clock} if clock else {}))
    dc.setup()
    for d in d_lister:
        dc.d_inf.add(d)
    for r in rs_lister:
        dc.rs_inf.add(r)
    for p in pod_lister:
        dc.pod_inf.add(p)
    return dc, client


def queue_len(dc):
    return len(dc.queue)


# ------------------------------------------------------------------ sync_test.go TestScale
def _updated_template(replicas):
    d = new_deployment("foo", replicas, None, None, None, {"foo": "bar"})
    d["spec"]["template"]["metadata"]["labels"]["another"] = "label"
    return d


def _broken_new():
    r = rs("foo-v2", 2, None, NEW_TS)
    r["status"]["availableReplicas"] = 0
    return r


SCALE_CASES = [
    # name, deployment, oldDeployment, newRS, oldRSs, expectedNew, expectedOld, wasntUpdated, desiredAnnotations
    ("normal scaling event: 10 -> 12", lambda: new_deployment("foo", 12), lambda: new_deployment("foo", 10),
     lambda: rs("foo-v1", 10, None, NEW_TS), lambda: [], 12, [], set(), {}),
    ("normal scaling event: 10 -> 5", lambda: new_deployment("foo", 5), lambda: new_deployment("foo", 10),
     lambda: rs("foo-v1", 10, None, NEW_TS), lambda: [], 5, [], set(), {}),
    ("proportional scaling: 5 -> 10", lambda: new_deployment("foo", 10), lambda: new_deployment("foo", 5),
     lambda: rs("foo-v2", 2, None, NEW_TS), lambda: [rs("foo-v1", 3, None, OLD_TS)], 4, [6], set(), {}),
    ("proportional scaling: 5 -> 3", lambda: new_deployment("foo", 3), lambda: new_deployment("foo", 5),
     lambda: rs("foo-v2", 2, None, NEW_TS), lambda: [rs("foo-v1", 3, None, OLD_TS)], 1, [2], set(), {}),
    ("proportional scaling: 9 -> 4", lambda: new_deployment("foo", 4), lambda: new_deployment("foo", 9),
     lambda: rs("foo-v2", 8, None, NEW_TS), lambda: [rs("foo-v1", 1, None, OLD_TS)], 4, [0], set(), {}),
    ("proportional scaling: 7 -> 10", lambda: new_deployment("foo", 10), lambda: new_deployment("foo", 7),
     lambda: rs("foo-v3", 2, None, NEW_TS),
     lambda: [rs("foo-v2", 3, None, OLD_TS), rs("foo-v1", 2, None, OLDER_TS)], 3, [4, 3], set(), {}),
    ("proportional scaling: 13 -> 8", lambda: new_deployment("foo", 8), lambda: new_deployment("foo", 13),
     lambda: rs("foo-v3", 2, None, NEW_TS),
     lambda: [rs("foo-v2", 8, None, OLD_TS), rs("foo-v1", 3, None, OLDER_TS)], 1, [5, 2], set(), {}),
    ("leftover distribution: 3 -> 4", lambda: new_deployment("foo", 4), lambda: new_deployment("foo", 3),
     lambda: rs("foo-v3", 1, None, NEW_TS),
     lambda: [rs("foo-v2", 1, None, OLD_TS), rs("foo-v1", 1, None, OLDER_TS)], 2, [1, 1], set(), {}),
    ("leftover distribution: 3 -> 2", lambda: new_deployment("foo", 2), lambda: new_deployment("foo", 3),
     lambda: rs("foo-v3", 1, None, NEW_TS),
     lambda: [rs("foo-v2", 1, None, OLD_TS), rs("foo-v1", 1, None, OLDER_TS)], 1, [1, 0], set(), {}),
    ("proportional scaling (no new rs): 4 -> 5", lambda: new_deployment("foo", 5), lambda: new_deployment("foo", 4),
     lambda: None, lambda: [rs("foo-v2", 2, None, OLD_TS), rs("foo-v1", 2, None, OLDER_TS)], None, [3, 2], set(), {}),
    ("proportional scaling: 6 -> 0", lambda: new_deployment("foo", 0), lambda: new_deployment("foo", 6),
     lambda: rs("foo-v3", 3, None, NEW_TS),
     lambda: [rs("foo-v2", 2, None, OLD_TS), rs("foo-v1", 1, None, OLDER_TS)], 0, [0, 0], set(), {}),
    ("proportional scaling: 0 -> 6", lambda: new_deployment("foo", 6), lambda: new_deployment("foo", 6),
     lambda: rs("foo-v3", 0, None, NEW_TS),
     lambda: [rs("foo-v2", 0, None, OLD_TS), rs("foo-v1", 0, None, OLDER_TS)], 6, [0, 0], {"foo-v2", "foo-v1"}, {}),
    ("failed rs update", lambda: new_deployment("foo", 5), lambda: new_deployment("foo", 5),
     lambda: rs("foo-v3", 2, None, NEW_TS),
     lambda: [rs("foo-v2", 1, None, OLD_TS), rs("foo-v1", 1, None, OLDER_TS)], 2, [2, 1], {"foo-v3", "foo-v1"},
     {"foo-v2": 3}),
    ("deployment with surge pods", lambda: new_deployment("foo", 20, None, 2), lambda: new_deployment("foo", 10, None, 2),
     lambda: rs("foo-v2", 6, None, NEW_TS), lambda: [rs("foo-v1", 6, None, OLD_TS)], 11, [11], set(), {}),
    ("change both surge and size", lambda: new_deployment("foo", 50, None, 6), lambda: new_deployment("foo", 10, None, 3),
     lambda: rs("foo-v2", 5, None, NEW_TS), lambda: [rs("foo-v1", 8, None, OLD_TS)], 22, [34], set(), {}),
    ("change both size and template", lambda: _updated_template(14),
     lambda: new_deployment("foo", 10, None, None, None, {"foo": "bar"}),
     lambda: None, lambda: [rs("foo-v2", 7, None, NEW_TS), rs("foo-v1", 3, None, OLD_TS)], None, [10, 4], set(), {}),
    ("saturated but broken new replica set does not affect old pods",
     lambda: new_deployment("foo", 2, None, 1, 1), lambda: new_deployment("foo", 2, None, 1, 1),
     _broken_new, lambda: [rs("foo-v1", 1, None, OLD_TS)], 2, [1], set(), {}),
]


@pytest.mark.parametrize("case", SCALE_CASES, ids=[c[0] for c in SCALE_CASES])
def test_scale(case):
    _, mk_d, mk_old_d, mk_new, mk_olds, exp_new, exp_old, wasnt_updated, desired_ann = case
    d, old_d, new, olds = mk_d(), mk_old_d(), mk_new(), mk_olds()
    for r in ([new] if new is not None else []) + olds:
        desired = desired_ann.get(m.name_of(r), D.d_replicas(old_d))
        D.set_replicas_annotations(r, desired, desired + D.max_surge(old_d))
    dc, client = controller()
    run(dc.scale(d, new, olds))
    sizes = {}
    if new is not None:
        sizes[m.name_of(new)] = D.rs_replicas(new)
    for r in olds:
        sizes[m.name_of(r)] = D.rs_replicas(r)
    for verb, _, _, obj in client.actions:
        assert verb == "update"
        if m.name_of(obj) not in wasnt_updated:
            sizes[m.name_of(obj)] = D.rs_replicas(obj)
    if exp_new is not None and new is not None:
        assert sizes[m.name_of(new)] == exp_new
    assert len(exp_old) == len(olds)
    for r, want in zip(olds, exp_old):
        assert sizes[m.name_of(r)] == want, m.name_of(r)


CLEANUP_CASES = [
    ([("foo-1", 0, 0), ("foo-2", 0, 0), ("foo-3", 0, 0)], 1, 2),
    ([("foo-1", 0, 0), ("foo-2", 0, 1), ("foo-3", 1, 0), ("foo-4", 1, 1)], 0, 1),
    ([("foo-1", 0, 0), ("foo-2", 0, 0)], 0, 2),
    ([("foo-1", 1, 1), ("foo-2", 1, 1)], 0, 0),
    ("already-deleted", 0, 0),
]


@pytest.mark.parametrize("olds,limit,deletions", CLEANUP_CASES)
def test_cleanup_deployment(olds, limit, deletions):
    sel = {"foo": "bar"}
    if olds == "already-deleted":
        r = new_rs_with_status("foo-1", 0, 0, sel)
        r["metadata"]["deletionTimestamp"] = ts(2017, 1, 1, 0, 0, 0)
        rss = [r]
    else:
        rss = [new_rs_with_status(n, a, b, sel) for n, a, b in olds]
    dc, client = controller(rs_lister=rss)
    d = new_deployment("foo", 1, limit, None, None, {"foo": "bar"})
    run(dc.cleanup_deployment(rss, d))
    assert sum(1 for a in client.actions if a[0] == "delete") == deletions


# ------------------------------------------------------------------ rolling_test.go
@pytest.mark.parametrize("replicas,surge,old,new,scale,expected", [
    (10, 0, 10, 0, False, None),
    (10, 2, 10, 0, True, 2),
    (10, 2, 5, 0, True, 7),
    (10, 2, 10, 2, False, None),
    (10, 2, 2, 11, True, 10),
])
def test_reconcile_new_replica_set(replicas, surge, old, new, scale, expected):
    new_rs = rs("foo-v2", new)
    old_rs = rs("foo-v2", old)
    d = new_deployment("foo", replicas, None, surge, 0, {"foo": "bar"})
    dc, client = controller()
    scaled = run(dc.reconcile_new_rs([new_rs, old_rs], new_rs, d))
    if not scale:
        assert not scaled and not client.actions
        return
    assert scaled and len(client.actions) == 1
    assert D.rs_replicas(client.actions[0][3]) == expected


@pytest.mark.parametrize("replicas,unavailable,old,new,ready_old,ready_new,scale", [
    (10, 0, 10, 0, 10, 0, True),
    (10, 2, 10, 0, 10, 0, True),
    (10, 2, 10, 0, 8, 0, True),          # unhealthy old replicas cleaned up
    (10, 2, 10, 0, 9, 0, True),          # one unhealthy cleaned, one ready scaled down
    (10, 2, 8, 2, 8, 0, False),          # the new RS's unavailable pods block further scale-down
])
def test_reconcile_old_replica_sets(replicas, unavailable, old, new, ready_old, ready_new, scale):
    new_rs = rs("foo-new", new, {"foo": "new"})
    new_rs["status"]["availableReplicas"] = ready_new
    old_rs = rs("foo-old", old, {"foo": "old"})
    old_rs["status"]["availableReplicas"] = ready_old
    d = new_deployment("foo", replicas, None, 0, unavailable, {"foo": "new"})
    dc, client = controller()
    scaled = run(dc.reconcile_old_rss([old_rs, new_rs], [old_rs], new_rs, d))
    assert scaled == scale


@pytest.mark.parametrize("old,ready,max_cleanup,expected", [
    (10, 8, 1, 1), (10, 8, 3, 2), (10, 8, 0, 0), (10, 10, 3, 0),
])
def test_cleanup_unhealthy_replicas(old, ready, max_cleanup, expected):
    old_rs = rs("foo-v2", old)
    old_rs["status"]["availableReplicas"] = ready
    d = new_deployment("foo", 10, None, 2, 2)
    dc, _ = controller()
    _, count = run(dc.cleanup_unhealthy_replicas([old_rs], d, max_cleanup))
    assert count == expected


@pytest.mark.parametrize("replicas,unavailable,ready,old,scale,expected", [
    (10, 0, 10, 10, True, 9),
    (10, 2, 10, 10, True, 8),
    (10, 2, 8, 10, False, None),
    (10, 2, 10, 0, False, None),
    (10, 2, 1, 10, False, None),
])
def test_scale_down_old_replica_sets_for_rolling_update(replicas, unavailable, ready, old, scale, expected):
    old_rs = rs("foo-v2", old)
    old_rs["status"]["availableReplicas"] = ready
    d = new_deployment("foo", replicas, None, 0, unavailable, {"foo": "bar"})
    dc, client = controller()
    scaled = run(dc.scale_down_old_rss_for_rolling_update([old_rs], [old_rs], d))
    if not scale:
        assert scaled == 0
        return
    assert scaled != 0
    updates = [a for a in client.actions if a[0] == "update"]
    assert len(updates) == 1 and D.rs_replicas(updates[0][3]) == expected


# ------------------------------------------------------------------ recreate_test.go
def test_scale_down_old_replica_sets_for_recreate():
    d = new_deployment("foo", 3, None, None, None, {"foo": "bar"})
    olds = [new_replica_set(d, f"foo-{n}", size) for n, size in enumerate([3])]
    dc, _ = controller(objects=[dict(_clone(r), spec=dict(r["spec"], replicas=0)) for r in olds])
    run(dc.scale_down_old_rss_for_recreate(olds, d))
    assert all(D.rs_replicas(r) == 0 for r in olds)


def _rs_with_uid(uid):
    d = new_deployment("foo", 1, None, None, None, {"foo": "bar"})
    r = new_replica_set(d, f"foo-{uid}", 0)
    r["metadata"]["uid"] = uid
    return r


def _phases(*ps):
    return [{"status": {"phase": p}} for p in ps]


@pytest.mark.parametrize("name,olds,pod_map,expected", [
    ("no old RSs", [], {}, False),
    ("old RSs with running pods", [_rs_with_uid("some-uid"), _rs_with_uid("other-uid")],
     {"some-uid": [{}, {}], "other-uid": [{}, {}]}, True),
    ("old RSs without pods but with non-zero status replicas", [new_rs_with_status("rs-1", 0, 1)], {}, True),
    ("old RSs without pods or non-zero status replicas", [new_rs_with_status("rs-1", 0, 0)], {}, False),
    ("terminal pods only", [new_rs_with_status("rs-1", 0, 0)], {"uid-1": _phases("Failed", "Succeeded")}, False),
    ("unknown phase", [new_rs_with_status("rs-1", 0, 0)], {"uid-1": _phases("Unknown")}, True),
    ("pending pod", [new_rs_with_status("rs-1", 0, 0)], {"uid-1": _phases("Pending")}, True),
    ("running pod", [new_rs_with_status("rs-1", 0, 0)], {"uid-1": _phases("Running")}, True),
    ("terminal and pending", [new_rs_with_status("rs-1", 0, 0)],
     {"uid-1": _phases("Failed", "Succeeded"), "uid-2": [], "uid-3": _phases("Pending")}, True),
])
def test_old_pods_running(name, olds, pod_map, expected):
    assert D.old_pods_running(None, olds, pod_map) == expected


# ------------------------------------------------------------------ progress_test.go
def current_deployment(pds, replicas, status_replicas, updated, available, conditions):
    d = {"metadata": {"name": "progress-test"},
         "spec": {"replicas": replicas, "strategy": {"type": "Recreate"}},
         "status": {"replicas": status_replicas, "updatedReplicas": updated, "availableReplicas": available}}
    if pds is not None:
        d["spec"]["progressDeadlineSeconds"] = pds
    if conditions is not None:
        d["status"]["conditions"] = [dict(c) for c in conditions]
    return d


def deployment_status(replicas, updated, available):
    return {"replicas": replicas, "updatedReplicas": updated, "availableReplicas": available}


def new_rs_with_available(name, spec, status, available):
    r = rs(name, spec)
    r["status"] = {"replicas": status, "availableReplicas": available}
    return r


T0 = m.parse_time(ts(2017, 2, 15, 18, 49, 0))
FAILED = [{"type": "Progressing", "status": "False", "reason": D.TIMED_OUT}]
STUCK = [{"type": "Progressing", "status": "True", "lastUpdateTime": ts(2017, 2, 15, 18, 49, 0)}]


@pytest.mark.parametrize("name,d,status,now,expected", [
    ("no progressDeadlineSeconds specified", current_deployment(None, 4, 3, 3, 2, None),
     deployment_status(3, 3, 2), None, -1),
    ("no progressing condition found", current_deployment(60, 4, 3, 3, 2, None), deployment_status(3, 3, 2), None, -1),
    ("complete deployment does not need to be requeued", current_deployment(60, 3, 3, 3, 3, None),
     deployment_status(3, 3, 3), None, -1),
    ("already failed deployment does not need to be requeued", current_deployment(60, 3, 3, 3, 0, FAILED),
     deployment_status(3, 3, 0), None, -1),
    ("stuck deployment - 30s", current_deployment(60, 3, 3, 3, 1, STUCK), deployment_status(3, 3, 1), T0 + 30, 30),
    ("stuck deployment - 1s", current_deployment(60, 3, 3, 3, 1, STUCK), deployment_status(3, 3, 1), T0 + 59, 1),
    # the reference uses 1ns short of the second; a float epoch resolves ~0.2us, so 1ms here
    ("failed deployment - less than a second => now", current_deployment(60, 3, 3, 3, 1, STUCK),
     deployment_status(3, 3, 1), T0 + 59.001, 0),
    ("failed deployment - now", current_deployment(60, 3, 3, 3, 1, STUCK), deployment_status(3, 3, 1), T0 + 60, 0),
    ("failed deployment - 1s after deadline", current_deployment(60, 3, 3, 3, 1, STUCK),
     deployment_status(3, 3, 1), T0 + 61, 0),
    ("failed deployment - 60s after deadline", current_deployment(60, 3, 3, 3, 1, STUCK),
     deployment_status(3, 3, 1), T0 + 120, 0),
])
def test_requeue_stuck_deployment(name, d, status, now, expected):
    dc, _ = controller(clock=(lambda: now) if now is not None else None)

    async def go():
        got = dc.requeue_stuck_deployment(d, status)
        dc.queue.shutdown()
        return got
    got = run(go())
    assert got == pytest.approx(expected, abs=1e-6)


_TT = ts(2017, 2, 15, 18, 49, 0)
NEW_RS_AVAILABLE = {"type": "Progressing", "status": "True", "reason": D.NEW_RS_AVAILABLE,
                    "lastUpdateTime": _TT, "lastTransitionTime": _TT}
RS_UPDATED = {"type": "Progressing", "status": "True", "reason": D.RS_UPDATED, "lastUpdateTime": _TT,
              "lastTransitionTime": _TT}
TIMED_OUT = {"type": "Progressing", "status": "False", "reason": D.TIMED_OUT}

ROLLOUT_CASES = [
    ("General: remove Progressing condition without a progress deadline",
     current_deployment(None, 3, 2, 2, 2, [RS_UPDATED]), [new_rs_with_available("bar", 0, 1, 1)],
     new_rs_with_available("foo", 3, 2, 2), None, None, None),
    ("General: only one active ReplicaSet",
     current_deployment(60, 3, 3, 3, 3, [NEW_RS_AVAILABLE]), [new_rs_with_available("bar", 3, 3, 3)], None,
     "True", D.NEW_RS_AVAILABLE, _TT),
    ("DeploymentProgressing: keep lastTransitionTime when already Progressing=True",
     current_deployment(60, 3, 2, 2, 2, [RS_UPDATED]), [new_rs_with_available("bar", 0, 1, 1)],
     new_rs_with_available("foo", 3, 2, 2), "True", D.RS_UPDATED, _TT),
    ("DeploymentProgressing: update everything from Progressing=False",
     current_deployment(60, 3, 2, 2, 2, [TIMED_OUT]), [new_rs_with_available("bar", 0, 1, 1)],
     new_rs_with_available("foo", 3, 2, 2), "True", D.RS_UPDATED, None),
    ("DeploymentProgressing: create the condition",
     current_deployment(60, 3, 2, 2, 2, []), [new_rs_with_available("bar", 0, 1, 1)],
     new_rs_with_available("foo", 3, 2, 2), "True", D.RS_UPDATED, None),
    ("DeploymentComplete: keep lastTransitionTime when already Progressing=True",
     current_deployment(60, 3, 3, 3, 3, [RS_UPDATED]), [], new_rs_with_available("foo", 3, 3, 3),
     "True", D.NEW_RS_AVAILABLE, _TT),
    ("DeploymentComplete: update everything from Progressing=False",
     current_deployment(60, 3, 3, 3, 3, [TIMED_OUT]), [], new_rs_with_available("foo", 3, 3, 3),
     "True", D.NEW_RS_AVAILABLE, None),
    ("DeploymentComplete: create the condition",
     current_deployment(60, 3, 3, 3, 3, []), [], new_rs_with_available("foo", 3, 3, 3), "True", D.NEW_RS_AVAILABLE, None),
    ("DeploymentComplete: newRS=nil",
     current_deployment(60, 0, 3, 3, 3, [RS_UPDATED]), [new_rs_with_available("foo", 0, 0, 0)], None,
     "True", D.NEW_RS_AVAILABLE, None),
    ("DeploymentTimedOut: exceeds the deadline",
     current_deployment(60, 3, 2, 2, 2, [RS_UPDATED]), [], new_rs_with_available("foo", 3, 2, 2),
     "False", D.TIMED_OUT, None),
    ("DeploymentTimedOut: keep an existing timed-out condition",
     current_deployment(60, 3, 2, 2, 2, [TIMED_OUT]), [], new_rs_with_available("foo", 3, 2, 2),
     "False", D.TIMED_OUT, None),
]


@pytest.mark.parametrize("case", ROLLOUT_CASES, ids=[c[0] for c in ROLLOUT_CASES])
def test_sync_rollout_status(case):
    _, d, all_rss, new, cond_status, cond_reason, transition = case
    d, all_rss = _clone(d), _clone(all_rss)
    new = _clone(new) if new is not None else None
    if new is not None:
        all_rss.append(new)
    dc, _ = controller()

    async def go():
        await dc.sync_rollout_status(all_rss, new, d)
        dc.queue.shutdown()
    run(go())
    cond = D.get_condition(d.get("status"), "Progressing")
    if cond is None:
        assert d["spec"].get("progressDeadlineSeconds") is None and cond_status is None
        return
    assert (cond["status"], cond["reason"]) == (cond_status, cond_reason)
    if transition is not None:
        assert cond["lastTransitionTime"] == transition


# ------------------------------------------------------------------ deployment_controller_test.go
def test_sync_deployment_creates_replica_set():
    d = new_deployment("foo", 1, None, None, None, {"foo": "bar"})
    dc, client = controller(objects=[d], d_lister=[d])
    run(dc.sync(m.key_of(d)))
    assert client.verbs() == [("create", "replicasets", ""), ("update", "deployments", "status"),
                              ("update", "deployments", "status")]
    created = client.actions[0][3]
    assert D.rs_replicas(created) == 1 and created["metadata"]["annotations"][D.REVISION] == "1"


def test_sync_deployment_dont_do_anything_during_deletion():
    d = new_deployment("foo", 1, None, None, None, {"foo": "bar"})
    d["metadata"]["deletionTimestamp"] = ts(2017, 1, 1, 0, 0, 0)
    dc, client = controller(objects=[d], d_lister=[d])
    run(dc.sync(m.key_of(d)))
    assert client.verbs() == [("update", "deployments", "status")]


def test_sync_deployment_deletion_race():
    d = new_deployment("foo", 1, None, None, None, {"foo": "bar"})
    d2 = _clone(d)
    d2["metadata"]["deletionTimestamp"] = ts(2017, 1, 1, 0, 0, 0)   # the client knows it is deleted
    r = new_replica_set(d, "rs1", 1)
    r["metadata"]["ownerReferences"] = []                             # a matching orphan triggers the recheck
    dc, client = controller(objects=[d2, r], d_lister=[d], rs_lister=[r])
    with pytest.raises(Exception):
        run(dc.sync(m.key_of(d)))
    assert client.verbs() == [("get", "deployments", "")]


def test_dont_sync_deployments_with_empty_pod_selector():
    d = new_deployment("foo", 1, None, None, None, {"foo": "bar"})
    d["spec"]["selector"] = {}
    dc, client = controller(objects=[d], d_lister=[d])
    run(dc.sync(m.key_of(d)))
    assert client.actions == []


def test_reentrant_rollback():
    labels = {"foo": "bar"}
    d = new_deployment("foo", 1, None, None, None, labels)
    d["spec"]["rollbackTo"] = {"revision": 0}
    d["metadata"]["annotations"] = {D.REVISION: "2"}
    rs1 = new_replica_set(d, "deploymentrs-old", 0)
    rs1["metadata"]["annotations"] = {D.REVISION: "1"}
    rs1["spec"]["template"] = _clone(d["spec"]["template"])
    rs1["spec"]["template"]["spec"]["terminationGracePeriodSeconds"] = 1
    labels[D.HASH_LABEL] = "hash"          # the shared selector map: every object sees the hash label
    rs1["spec"]["template"]["metadata"]["labels"] = labels
    rs2 = new_replica_set(d, "deploymentrs-new", 1)
    rs2["metadata"]["annotations"] = {D.REVISION: "2"}
    dc, client = controller(objects=[d, rs1, rs2], d_lister=[d], rs_lister=[rs1, rs2])
    run(dc.sync(m.key_of(d)))
    assert client.verbs() == [("update", "deployments", "")]
    rolled = client.actions[0][3]
    assert rolled["spec"]["template"]["spec"]["terminationGracePeriodSeconds"] == 1
    assert "rollbackTo" not in rolled["spec"]


def _recreate(name="foo"):
    d = new_deployment(name, 1, None, None, None, {"foo": "bar"})
    d["spec"]["strategy"]["type"] = "Recreate"
    return d


def _capture_enqueue(dc):
    got = []
    dc.enqueue = lambda d: got.append(m.name_of(d))
    return got


def test_pod_deletion_enqueues_recreate_deployment():
    foo = _recreate()
    r = new_replica_set(foo, "foo-1", 1)
    dc, _ = controller(objects=[foo, r], d_lister=[foo], rs_lister=[r])
    got = _capture_enqueue(dc)
    dc.delete_pod(generate_pod_from_rs(r))
    assert "foo" in got


def test_pod_deletion_doesnt_enqueue_recreate_deployment():
    foo = _recreate()
    rs1, rs2 = new_replica_set(foo, "foo-1", 1), new_replica_set(foo, "foo-1", 1)
    pod1, pod2 = generate_pod_from_rs(rs1), generate_pod_from_rs(rs2)
    pod2["metadata"]["name"] = "foo-1-pod-b"
    dc, _ = controller(d_lister=[foo], pod_lister=[pod1, pod2])
    got = _capture_enqueue(dc)
    dc.delete_pod(pod1)
    assert got == []


def test_pod_deletion_partial_rs_ownership_enqueues_recreate_deployment():
    foo = _recreate()
    rs1, rs2 = new_replica_set(foo, "foo-1", 1), new_replica_set(foo, "foo-2", 2)
    rs2["metadata"]["ownerReferences"] = []
    dc, _ = controller(objects=[foo, rs1, rs2], d_lister=[foo], rs_lister=[rs1, rs2])
    got = _capture_enqueue(dc)
    dc.delete_pod(generate_pod_from_rs(rs1))
    assert "foo" in got


def test_pod_deletion_partial_rs_ownership_doesnt_enqueue_recreate_deployment():
    foo = _recreate()
    rs1, rs2 = new_replica_set(foo, "foo-1", 1), new_replica_set(foo, "foo-2", 2)
    rs2["metadata"]["ownerReferences"] = []
    pod = generate_pod_from_rs(rs1)
    dc, _ = controller(objects=[foo, rs1, rs2], d_lister=[foo], rs_lister=[rs1, rs2], pod_lister=[pod])
    got = _capture_enqueue(dc)
    dc.delete_pod(pod)
    assert got == []


def test_get_replica_sets_for_deployment():
    d1 = new_deployment("foo", 1, None, None, None, {"foo": "bar"})
    d2 = new_deployment("bar", 1, None, None, None, {"foo": "bar"})
    rs1, rs2 = new_replica_set(d1, "rs1", 1), new_replica_set(d2, "rs2", 1)
    dc, _ = controller(objects=[d1, d2, rs1, rs2], d_lister=[d1, d2], rs_lister=[rs1, rs2])
    assert [m.name_of(r) for r in run(dc.replica_sets_for(d1))] == ["rs1"]
    assert [m.name_of(r) for r in run(dc.replica_sets_for(d2))] == ["rs2"]


def test_get_replica_sets_for_deployment_adopt_release():
    d = new_deployment("foo", 1, None, None, None, {"foo": "bar"})
    adopt = new_replica_set(d, "rsAdopt", 1)
    adopt["metadata"]["ownerReferences"] = []
    release = new_replica_set(d, "rsRelease", 1)
    release["metadata"]["labels"] = {"foo": "notbar"}
    dc, client = controller(objects=[d, adopt, release], d_lister=[d], rs_lister=[adopt, release])
    assert [m.name_of(r) for r in run(dc.replica_sets_for(d))] == ["rsAdopt"]
    patches = [a[3] for a in client.actions if a[0] == "patch"]
    assert len(patches) == 2
    assert patches[0]["metadata"]["ownerReferences"][0]["uid"] == m.uid_of(d)
    assert patches[1]["metadata"]["ownerReferences"][0] == {"$patch": "delete", "uid": m.uid_of(d)}


def test_get_pod_map_for_replica_sets():
    d = new_deployment("foo", 1, None, None, None, {"foo": "bar"})
    rs1, rs2 = new_replica_set(d, "rs1", 1), new_replica_set(d, "rs2", 1)
    pod1, pod2 = generate_pod_from_rs(rs1), generate_pod_from_rs(rs2)
    pod3 = _clone(generate_pod_from_rs(rs1))
    pod3["metadata"]["name"] = "pod3"
    pod3["metadata"]["ownerReferences"] = []
    pod4 = _clone(generate_pod_from_rs(rs1))
    pod4["metadata"]["name"] = "pod4"
    pod4["status"]["phase"] = "Failed"
    dc, _ = controller(objects=[d, rs1, rs2], d_lister=[d], rs_lister=[rs1, rs2], pod_lister=[pod1, pod2, pod3, pod4])
    pod_map = dc.pod_map(d, [rs1, rs2])
    assert sum(len(v) for v in pod_map.values()) == 3 and len(pod_map) == 2
    assert sorted(m.name_of(p) for p in pod_map[m.uid_of(rs1)]) == ["pod4", "rs1-pod"]
    assert [m.name_of(p) for p in pod_map[m.uid_of(rs2)]] == ["rs2-pod"]


def _two_deployments():
    d1 = new_deployment("d1", 1, None, None, None, {"foo": "bar"})
    d2 = new_deployment("d2", 1, None, None, None, {"foo": "bar"})
    return d1, d2


def _bumped(o):
    o = _clone(o)
    o["metadata"]["resourceVersion"] = str(int(o["metadata"].get("resourceVersion") or 0) + 1)
    return o


def _pop(dc):
    k = dc.queue.get_nowait()
    dc.queue.done(k)
    return k


def test_add_replica_set():
    d1, d2 = _two_deployments()
    rs1, rs2 = new_replica_set(d1, "rs1", 1), new_replica_set(d2, "rs2", 1)
    dc, _ = controller(d_lister=[d1, d2])
    dc.add_rs(rs1)
    assert queue_len(dc) == 1 and _pop(dc) == m.key_of(d1)
    dc.add_rs(rs2)
    assert queue_len(dc) == 1 and _pop(dc) == m.key_of(d2)


def test_add_replica_set_orphan():
    d1, d2 = _two_deployments()
    d3 = new_deployment("d3", 1, None, None, None, {"foo": "notbar"})
    r = new_replica_set(d1, "rs1", 1)
    r["metadata"]["ownerReferences"] = []
    dc, _ = controller(d_lister=[d1, d2, d3])
    dc.add_rs(r)
    assert queue_len(dc) == 2


def test_update_replica_set():
    d1, d2 = _two_deployments()
    rs1, rs2 = new_replica_set(d1, "rs1", 1), new_replica_set(d2, "rs2", 1)
    dc, _ = controller(d_lister=[d1, d2], rs_lister=[rs1, rs2])
    dc.update_rs(rs1, _bumped(rs1))
    assert queue_len(dc) == 1 and _pop(dc) == m.key_of(d1)
    dc.update_rs(rs2, _bumped(rs2))
    assert queue_len(dc) == 1 and _pop(dc) == m.key_of(d2)


def test_update_replica_set_orphan_with_new_labels():
    d1, d2 = _two_deployments()
    r = new_replica_set(d1, "rs1", 1)
    r["metadata"]["ownerReferences"] = []
    prev = _clone(r)
    prev["metadata"]["labels"] = {"foo": "notbar"}
    dc, _ = controller(d_lister=[d1, d2], rs_lister=[r])
    dc.update_rs(prev, _bumped(r))
    assert queue_len(dc) == 2


def test_update_replica_set_change_controller_ref():
    d1, d2 = _two_deployments()
    r = new_replica_set(d1, "rs1", 1)
    prev = _clone(r)
    prev["metadata"]["ownerReferences"] = [m.new_controller_ref(d2, "apps/v1", "Deployment")]
    dc, _ = controller(d_lister=[d1, d2], rs_lister=[r])
    dc.update_rs(prev, _bumped(r))
    assert queue_len(dc) == 2


def test_update_replica_set_release():
    d1, d2 = _two_deployments()
    r = new_replica_set(d1, "rs1", 1)
    nxt = _bumped(r)
    nxt["metadata"]["ownerReferences"] = []
    dc, _ = controller(d_lister=[d1, d2], rs_lister=[r])
    dc.update_rs(r, nxt)
    assert queue_len(dc) == 2


def test_delete_replica_set():
    d1, d2 = _two_deployments()
    rs1, rs2 = new_replica_set(d1, "rs1", 1), new_replica_set(d2, "rs2", 1)
    dc, _ = controller(d_lister=[d1, d2], rs_lister=[rs1, rs2])
    dc.delete_rs(rs1)
    assert queue_len(dc) == 1 and _pop(dc) == m.key_of(d1)
    dc.delete_rs(rs2)
    assert queue_len(dc) == 1 and _pop(dc) == m.key_of(d2)


def test_delete_replica_set_orphan():
    d1, d2 = _two_deployments()
    r = new_replica_set(d1, "rs1", 1)
    r["metadata"]["ownerReferences"] = []
    dc, _ = controller(d_lister=[d1, d2], rs_lister=[r])
    dc.delete_rs(r)
    assert queue_len(dc) == 0


# ------------------------------------------------------------------ util/deployment_util_test.go
def generate_deployment(image):
    labels = {"name": image}
    return {"metadata": {"name": image, "annotations": {}},
            "spec": {"replicas": 1, "selector": {"matchLabels": labels},
                     "template": {"metadata": {"labels": labels},
                                  "spec": {"containers": [{"name": image, "image": image, "imagePullPolicy": "Always",
                                                           "terminationMessagePath": "/dev/termination-log"}],
                                           "dnsPolicy": "ClusterFirst", "terminationGracePeriodSeconds": 30,
                                           "restartPolicy": "Always", "securityContext": {}}}}}


def generate_rs(d):
    tpl = _clone(d["spec"]["template"])
    return {"metadata": {"uid": str(uuid.uuid4()), "name": "replicaset" + uuid.uuid4().hex[:5],
                         "labels": tpl["metadata"]["labels"],            # shared with the template (Go aliasing)
                         "ownerReferences": [{"apiVersion": "extensions/v1beta1", "kind": "Deployment",
                                              "name": m.name_of(d), "uid": m.uid_of(d), "controller": True}]},
            "spec": {"replicas": 0, "template": tpl, "selector": {"matchLabels": tpl["metadata"]["labels"]}},
            "status": {}}


def pod_template(name, node, annotations, labels):
    return {"metadata": {"name": name, "annotations": annotations, "labels": labels}, "spec": {"nodeName": node}}


H = D.HASH_LABEL


@pytest.mark.parametrize("name,former,latter,expected", [
    ("Same spec, same labels", pod_template("foo", "foo-node", {}, {H: "value-1", "something": "else"}),
     pod_template("foo", "foo-node", {}, {H: "value-1", "something": "else"}), True),
    ("Same spec, only pod-template-hash label value is different",
     pod_template("foo", "foo-node", {}, {H: "value-1", "something": "else"}),
     pod_template("foo", "foo-node", {}, {H: "value-2", "something": "else"}), True),
    ("Same spec, the former doesn't have pod-template-hash label",
     pod_template("foo", "foo-node", {}, {"something": "else"}),
     pod_template("foo", "foo-node", {}, {H: "value-2", "something": "else"}), True),
    ("Same spec, the label is different, and the pod-template-hash label value is the same",
     pod_template("foo", "foo-node", {}, {H: "value-1"}),
     pod_template("foo", "foo-node", {}, {H: "value-1", "something": "else"}), False),
    ("Different spec, same labels", pod_template("foo", "foo-node", {"former": "value"}, {H: "value-1", "something": "else"}),
     pod_template("foo", "foo-node", {"latter": "value"}, {H: "value-1", "something": "else"}), False),
    ("Different spec, different pod-template-hash label value",
     pod_template("foo-1", "foo-node", {}, {H: "value-1", "something": "else"}),
     pod_template("foo-2", "foo-node", {}, {H: "value-2", "something": "else"}), False),
    ("Different spec, the former doesn't have pod-template-hash label",
     pod_template("foo-1", "foo-node-1", {}, {"something": "else"}),
     pod_template("foo-2", "foo-node-2", {}, {H: "value-2", "something": "else"}), False),
    ("Different spec, different labels", pod_template("foo", "foo-node-1", {}, {"something": "else"}),
     pod_template("foo", "foo-node-2", {}, {"nothing": "else"}), False),
])
def test_equal_ignore_hash(name, former, latter, expected):
    for a, b in ((former, latter), (latter, former)):
        before = _clone([a, b])
        assert D.equal_ignore_hash(a, b) == expected
        assert [a, b] == before                       # the inputs' labels are left alone


def test_equal_ignore_hash_empty_equals_missing():
    """apiequality.Semantic treats nil and empty maps alike."""
    a = pod_template("foo", "n", {}, {"x": "y"})
    b = pod_template("foo", "n", None, {"x": "y"})
    assert D.equal_ignore_hash(a, b)


def _find_fixture():
    now = 1_700_000_000.0
    d = generate_deployment("nginx")
    new = generate_rs(d)
    new["spec"]["replicas"] = 1
    new["metadata"]["labels"][H] = "hash"
    new["metadata"]["creationTimestamp"] = m.format_time(now + 60)
    dup = generate_rs(d)
    dup["metadata"]["labels"][H] = "different-hash"
    dup["metadata"]["creationTimestamp"] = m.format_time(now)
    old_d = generate_deployment("nginx")
    old_d["spec"]["template"]["spec"]["containers"][0]["name"] = "nginx-old-1"
    old = generate_rs(old_d)
    old["metadata"]["creationTimestamp"] = m.format_time(now - 60)
    return d, new, dup, old


def test_find_new_replica_set():
    d, new, dup, old = _find_fixture()
    assert D.find_new_rs(d, [new, old]) is new
    assert D.find_new_rs(d, [new, old, dup]) is dup            # the oldest of the equal templates
    assert D.find_new_rs(d, [old]) is None


def test_find_old_replica_sets():
    d, new, dup, old = _find_fixture()
    names = lambda rss: sorted(m.name_of(r) for r in rss)     # noqa: E731
    req, all_old = D.find_old_rss(d, [new, old])
    assert names(all_old) == names([old]) and req == []
    req, all_old = D.find_old_rss(d, [old])
    assert names(all_old) == names([old]) and req == []
    req, all_old = D.find_old_rss(d, [old, new, dup])
    assert names(all_old) == names([old, new]) and names(req) == names([new])
    req, all_old = D.find_old_rss(d, [new])
    assert all_old == [] and req == []


def test_get_replica_count_for_replica_sets():
    rs1 = generate_rs(generate_deployment("foo"))
    rs1["spec"]["replicas"], rs1["status"]["replicas"] = 1, 2
    rs2 = generate_rs(generate_deployment("bar"))
    rs2["spec"]["replicas"], rs2["status"]["replicas"] = 2, 3
    assert (D.replica_count([rs1]), D.actual_replica_count([rs1])) == (1, 2)
    assert (D.replica_count([rs1, rs2]), D.actual_replica_count([rs1, rs2])) == (3, 5)


@pytest.mark.parametrize("surge,unavailable,desired,exp_surge,exp_unavailable,error", [
    ("0%", "0%", 0, 0, 1, False),
    ("39%", "39%", 10, 4, 3, False),
    ("oops", "39%", 10, 0, 0, True),
    ("55%", "urg", 10, 0, 0, True),
])
def test_resolve_fenceposts(surge, unavailable, desired, exp_surge, exp_unavailable, error):
    if error:
        with pytest.raises(ValueError):
            D.resolve_fenceposts(surge, unavailable, desired)
        return
    assert D.resolve_fenceposts(surge, unavailable, desired) == (exp_surge, exp_unavailable)


@pytest.mark.parametrize("name,strategy,dep_replicas,new_replicas,surge,expected", [
    ("can not scale up - to newRSReplicas", "RollingUpdate", 1, 5, 1, 5),
    ("scale up - to depReplicas", "RollingUpdate", 6, 2, 10, 6),
    ("recreate - to depReplicas", "Recreate", 3, 1, 1, 3),
])
def test_new_rs_new_replicas(name, strategy, dep_replicas, new_replicas, surge, expected):
    d = generate_deployment("nginx")
    new = generate_rs(d)
    rs5 = generate_rs(d)
    rs5["spec"]["replicas"] = 5
    d["spec"]["replicas"] = dep_replicas
    d["spec"]["strategy"] = {"type": strategy, "rollingUpdate": {"maxUnavailable": 1, "maxSurge": surge}}
    new["spec"]["replicas"] = new_replicas
    assert D.new_rs_new_replicas(d, [rs5], new) == expected


def cond_progressing():
    return {"type": "Progressing", "status": "False", "reason": "ForSomeReason"}


def cond_progressing2():
    return {"type": "Progressing", "status": "True", "reason": "BecauseItIs"}


def cond_available():
    return {"type": "Available", "status": "True", "reason": "AwesomeController"}


def example_status():
    return {"conditions": [cond_progressing(), cond_available()]}


def test_get_condition():
    assert D.get_condition(example_status(), "Available") is not None
    assert D.get_condition(example_status(), "ReplicaFailure") is None


@pytest.mark.parametrize("status,cond,expected", [
    ({}, cond_available(), {"conditions": [cond_available()]}),
    ({"conditions": [cond_progressing()]}, cond_available(), example_status()),
    ({"conditions": [cond_progressing()]}, cond_progressing2(), {"conditions": [cond_progressing2()]}),
])
def test_set_condition(status, cond, expected):
    D.set_condition(status, cond)
    assert status == expected


@pytest.mark.parametrize("status,kind,expected", [
    ({}, "Progressing", {}),
    ({"conditions": [cond_progressing()]}, "Progressing", {}),
    (example_status(), "ReplicaFailure", example_status()),
])
def test_remove_condition(status, kind, expected):
    D.remove_condition(status, kind)
    assert status == expected


def _complete_d(desired, current, updated, available, max_unavailable, max_surge):
    return {"spec": {"replicas": desired, "strategy": {"type": "RollingUpdate", "rollingUpdate": {
        "maxUnavailable": max_unavailable, "maxSurge": max_surge}}},
        "status": {"replicas": current, "updatedReplicas": updated, "availableReplicas": available}}


@pytest.mark.parametrize("d,expected", [
    (_complete_d(5, 5, 5, 4, 1, 0), False),
    (_complete_d(5, 5, 5, 3, 1, 0), False),
    (_complete_d(5, 5, 5, 5, 0, 0), True),
    (_complete_d(5, 5, 4, 5, 0, 0), False),
    (_complete_d(1, 2, 1, 1, 0, 1), False),
    (_complete_d(1, 1, 1, 0, 1, 1), False),
])
def test_deployment_complete(d, expected):
    assert D.deployment_complete(d, d["status"]) == expected


def _st(current, updated, ready, available):
    return {"replicas": current, "updatedReplicas": updated, "readyReplicas": ready, "availableReplicas": available}


@pytest.mark.parametrize("old,new,expected", [
    (_st(10, 4, 4, 4), _st(10, 6, 4, 4), True),
    (_st(10, 4, 4, 4), _st(10, 4, 4, 4), False),
    (_st(10, 4, 6, 6), _st(8, 4, 6, 6), True),
    (_st(10, 7, 3, 3), _st(10, 6, 3, 3), False),
    (_st(10, 4, 7, 7), _st(8, 8, 5, 5), True),
    (_st(10, 10, 9, 8), _st(10, 10, 10, 8), True),
    (_st(10, 10, 10, 9), _st(10, 10, 10, 10), True),
])
def test_deployment_progressing(old, new, expected):
    assert D.deployment_progressing({"status": old}, new) == expected


def _t(minute, sec):
    return m.parse_time(ts(2016, 1, 1, 0, minute, sec))


@pytest.mark.parametrize("pds,reason,frm,now,expected", [
    (None, "", _t(1, 9), _t(1, 20), False),
    (10, "", _t(1, 9), _t(1, 20), True),
    (10, "", _t(1, 11), _t(1, 20), False),
    (None, D.NEW_RS_AVAILABLE, None, None, False),
])
def test_deployment_timed_out(pds, reason, frm, now, expected):
    cond = {"type": "Progressing", "status": "True", "reason": reason}
    if frm is not None:
        cond["lastUpdateTime"] = m.format_time(frm)
    d = {"spec": {} if pds is None else {"progressDeadlineSeconds": pds}, "status": {"conditions": [cond]}}
    assert D.deployment_timed_out(d, d["status"], now or 0.0) == expected


def _mu_d(replicas, max_unavailable):
    return {"spec": {"replicas": replicas, "strategy": {"type": "RollingUpdate", "rollingUpdate": {
        "maxSurge": 1, "maxUnavailable": max_unavailable}}}}


@pytest.mark.parametrize("d,expected", [
    (_mu_d(10, 5), 5), (_mu_d(10, 10), 10), (_mu_d(5, 10), 5), (_mu_d(0, 10), 0),
    ({"spec": {"strategy": {"type": "Recreate"}}}, 0),
    (_mu_d(10, "50%"), 5), (_mu_d(10, "100%"), 10), (_mu_d(5, "100%"), 5),
])
def test_max_unavailable(d, expected):
    assert D.max_unavailable(d) == expected


def test_annotation_utils():
    d = generate_deployment("nginx")
    r = generate_rs(d)
    d["metadata"]["annotations"][D.REVISION] = "1"
    for i in range(20):
        nxt = str(i + 1)
        D.set_new_rs_annotations(d, r, nxt, True)
        assert r["metadata"]["annotations"][D.REVISION] == nxt
    assert D.set_replicas_annotations(r, 10, 11)
    assert r["metadata"]["annotations"][D.DESIRED] == "10"
    assert r["metadata"]["annotations"][D.MAX_REPLICAS] == "11"
    r["metadata"]["annotations"][D.DESIRED] = "1"
    r["status"]["availableReplicas"] = 1
    r["spec"]["replicas"] = 1
    assert D.is_saturated(d, r)


def test_pod_template_spec_hash_no_collisions():
    """util/hash_test.go:107 — 1000 templates differing in one field hash to 1000 values."""
    seen = {}
    for i in range(1000):
        spec = {"metadata": {"labels": {"app": "cats"}},
                "spec": {"containers": [{"name": "cats", "image": f"registry/cats:v{i}",
                                         "ports": [{"containerPort": 8080, "protocol": "TCP"}],
                                         "imagePullPolicy": "IfNotPresent"}],
                         "restartPolicy": "Always", "terminationGracePeriodSeconds": 30, "dnsPolicy": "ClusterFirst",
                         "securityContext": {}}}
        h = D.compute_hash(spec, None)
        assert h not in seen, f"collision between {seen.get(h)} and {i}"
        seen[h] = i
    assert D.compute_hash(spec, None) != D.compute_hash(spec, 1)
