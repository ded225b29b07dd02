"""StatefulSet controller (pkg/controller/statefulset/*.go).

Pods are `<set>-<ordinal>` with a stable identity (hostname, subdomain = spec.serviceName, the
statefulset.kubernetes.io/pod-name label) and stable storage (claim `<template>-<set>-<ordinal>`
per volumeClaimTemplate, created before the pod). One pass of `StatefulSetControl.update`
(stateful_set_control.go UpdateStatefulSet):
  1. history: the template is snapshot as a ControllerRevision (history.py); the update
     revision is the newest equal one (renumbered to the top if it is an older one — a
     rollback) or a new one; the current revision is status.currentRevision's, else the update;
  2. pods are split into replicas [0, spec.replicas) and condemned (higher ordinals); missing
     ordinals get a pod of the current revision below the partition (or below
     status.currentReplicas when RollingUpdate has no partition struct), else of the update
     revision (newVersionedStatefulSetPod);
  3. failed replicas are deleted and recreated; missing ones created; under OrderedReady
     (`monotonic`) the pass stops at the first create, the first terminating pod and the first
     pod not Running and Ready; identity/storage drift is repaired in place;
  4. condemned pods go highest ordinal first (monotonic: one per pass, and only while every
     replica is healthy — the first unhealthy pod itself may go);
  5. RollingUpdate: from the highest ordinal down to the partition, the first pod not at the
     update revision is deleted (it comes back at the update revision), waiting for unhealthy
     ones; OnDelete does nothing;
  6. status (replicas / ready / current / updated / revisions / collisionCount, with
     completeRollingUpdate) is written when it changed; revisions beyond
     revisionHistoryLimit that no pod, nor the current or update revision, uses are deleted.
The controller (stateful_set.go) claims pods that are members (`<set>-<n>`) and match the
selector, adopts orphan revisions, and enqueues sets from pod events by ControllerRef.
"""
from __future__ import annotations

import asyncio
import functools
import math
import re
import time

from ..api import meta as m
from ..api import strategicpatch
from ..api.helpers import is_pod_ready
from ..api.labels import selector_from_label_selector
from . import history as H
from .base import Controller, split_key
from .controller_utils import ControllerRefManager, adopt_patch, recheck_deletion, release_patch
from .replicaset import pod_from_template

POD_NAME_LABEL = "statefulset.kubernetes.io/pod-name"
REVISION_LABEL = "controller-revision-hash"
API_VERSION, KIND = "apps/v1", "StatefulSet"

_POD_RE = re.compile(r"(.*)-([0-9]+)$")


# ============================================================================ utils
def parent_name_and_ordinal(pod: dict) -> tuple[str, int]:
    mt = _POD_RE.match(m.name_of(pod) or "")
    if not mt:
        return "", -1
    o = int(mt.group(2))
    return mt.group(1), (o if o < 2 ** 31 else -1)


def parent_name(pod) -> str:
    return parent_name_and_ordinal(pod)[0]


def ordinal_of(pod) -> int:
    return parent_name_and_ordinal(pod)[1]


def pod_name(s: dict, ordinal: int) -> str:
    return f"{m.name_of(s)}-{ordinal}"


def pvc_name(s: dict, claim: dict, ordinal: int) -> str:
    return f"{m.name_of(claim)}-{m.name_of(s)}-{ordinal}"


def is_member_of(s, pod) -> bool:
    return parent_name(pod) == m.name_of(s)


def identity_matches(s, pod) -> bool:
    parent, o = parent_name_and_ordinal(pod)
    return o >= 0 and parent == m.name_of(s) and m.name_of(pod) == pod_name(s, o) and \
        m.namespace_of(pod) == m.namespace_of(s) and m.labels_of(pod).get(POD_NAME_LABEL) == m.name_of(pod)


def _spec(o) -> dict:
    return (o or {}).get("spec") or {}


def _status(o) -> dict:
    return (o or {}).get("status") or {}


def storage_matches(s, pod) -> bool:
    o = ordinal_of(pod)
    if o < 0:
        return False
    vols = {v.get("name"): v for v in _spec(pod).get("volumes") or []}
    for claim in _spec(s).get("volumeClaimTemplates") or []:
        v = vols.get(m.name_of(claim))
        if v is None or not v.get("persistentVolumeClaim") or \
                v["persistentVolumeClaim"].get("claimName") != pvc_name(s, claim, o):
            return False
    return True


def get_pvcs(s, pod) -> dict:
    """getPersistentVolumeClaims: template name -> the claim this pod uses."""
    o = ordinal_of(pod)
    out = {}
    for t in _spec(s).get("volumeClaimTemplates") or []:
        c = m.deepcopy(t)
        md = c.setdefault("metadata", {})
        md["name"] = pvc_name(s, t, o)
        md["namespace"] = m.namespace_of(s)
        md["labels"] = dict((_spec(s).get("selector") or {}).get("matchLabels") or {})
        c.setdefault("apiVersion", "v1")
        c.setdefault("kind", "PersistentVolumeClaim")
        out[m.name_of(t)] = c
    return out


def update_storage(s, pod):
    claims = get_pvcs(s, pod)
    vols = [{"name": name, "persistentVolumeClaim": {"claimName": m.name_of(c)}} for name, c in claims.items()]
    vols += [v for v in _spec(pod).get("volumes") or [] if v.get("name") not in claims]
    pod.setdefault("spec", {})["volumes"] = vols


def update_identity(s, pod):
    md = pod.setdefault("metadata", {})
    md["name"] = pod_name(s, ordinal_of(pod))
    md["namespace"] = m.namespace_of(s)
    if md.get("labels") is None:
        md["labels"] = {}
    md["labels"][POD_NAME_LABEL] = md["name"]


def init_identity(s, pod):
    update_identity(s, pod)
    spec = pod.setdefault("spec", {})
    spec["hostname"] = m.name_of(pod)
    if _spec(s).get("serviceName"):
        spec["subdomain"] = _spec(s)["serviceName"]
    else:
        spec.pop("subdomain", None)


def is_running_and_ready(pod) -> bool:
    return _status(pod).get("phase") == "Running" and is_pod_ready(pod)


def is_created(pod) -> bool:
    return bool(_status(pod).get("phase"))


def is_failed(pod) -> bool:
    return _status(pod).get("phase") == "Failed"


def is_terminating(pod) -> bool:
    return bool((pod.get("metadata") or {}).get("deletionTimestamp"))


def is_healthy(pod) -> bool:
    return is_running_and_ready(pod) and not is_terminating(pod)


def allows_burst(s) -> bool:
    return _spec(s).get("podManagementPolicy") == "Parallel"


def set_pod_revision(pod, rev: str):
    md = pod.setdefault("metadata", {})
    if md.get("labels") is None:
        md["labels"] = {}
    md["labels"][REVISION_LABEL] = rev


def get_pod_revision(pod) -> str:
    return m.labels_of(pod).get(REVISION_LABEL, "")


def controller_ref(s) -> dict:
    return m.new_controller_ref(s, API_VERSION, KIND)


def new_statefulset_pod(s, ordinal: int) -> dict:
    pod = pod_from_template(_spec(s).get("template") or {}, s, controller_ref(s))
    pod["metadata"]["name"] = pod_name(s, ordinal)
    init_identity(s, pod)
    update_storage(s, pod)
    return pod


def _strategy(s) -> dict:
    return _spec(s).get("updateStrategy") or {}


def new_versioned_pod(current_set, update_set, current_rev: str, update_rev: str, ordinal: int) -> dict:
    """newVersionedStatefulSetPod, the reference's operator precedence kept:
    (RollingUpdate && no rollingUpdate struct && ordinal < currentReplicas) ||
    (rollingUpdate struct && ordinal < partition)."""
    st = _strategy(current_set)
    ru = st.get("rollingUpdate")
    rolling = (st.get("type") or "RollingUpdate") == "RollingUpdate"
    if (rolling and ru is None and ordinal < int(_status(current_set).get("currentReplicas") or 0)) or \
            (ru is not None and ordinal < int(ru.get("partition") or 0)):
        pod = new_statefulset_pod(current_set, ordinal)
        set_pod_revision(pod, current_rev)
        return pod
    pod = new_statefulset_pod(update_set, ordinal)
    set_pod_revision(pod, update_rev)
    return pod


def get_patch(s) -> dict:
    """The revision data: the template, marked to replace the whole template when applied."""
    tpl = m.deepcopy(_spec(s).get("template") or {})
    tpl["$patch"] = "replace"
    return {"spec": {"template": tpl}}


def match(s, rev) -> bool:
    return H.raw(get_patch(s)) == H.raw(rev.get("data"))


def new_revision(s, revision: int, collision_count: int | None) -> dict:
    sel = (_spec(s).get("selector") or {}).get("matchLabels") or {}
    cr = H.new_controller_revision(s, API_VERSION, KIND, sel, get_patch(s), revision, collision_count)
    ann = cr["metadata"].setdefault("annotations", {})
    ann.update(m.annotations_of(s) or {})
    return cr


def apply_revision(s, rev) -> dict:
    """ApplyRevision: the set with the revision's template (a strategic merge of its data)."""
    return strategicpatch.apply(m.deepcopy(s), rev.get("data") or {}, strategicpatch.schema_for(API_VERSION, KIND))


def next_revision(revs: list) -> int:
    return H.revision_of(revs[-1]) + 1 if revs else 1


def inconsistent_status(s, status: dict) -> bool:
    cur = _status(s)
    if cur.get("observedGeneration") is None:
        return True
    if int(status.get("observedGeneration") or 0) > int(cur.get("observedGeneration") or 0):
        return True
    for k in ("replicas", "currentReplicas", "readyReplicas", "updatedReplicas"):
        if int(status.get(k) or 0) != int(cur.get(k) or 0):
            return True
    return status.get("currentRevision", "") != cur.get("currentRevision", "") or \
        status.get("updateRevision", "") != cur.get("updateRevision", "")


def complete_rolling_update(s, status: dict):
    if (_strategy(s).get("type") or "RollingUpdate") == "RollingUpdate" and \
            status["updatedReplicas"] == status["replicas"] and status["readyReplicas"] == status["replicas"]:
        status["currentReplicas"] = status["updatedReplicas"]
        status["currentRevision"] = status["updateRevision"]


def sort_ascending_ordinal(pods: list) -> list:
    pods.sort(key=ordinal_of)
    return pods


def overlapping_order(s):
    """overlappingStatefulSets: older first, the name breaking ties."""
    return (m.parse_time((s.get("metadata") or {}).get("creationTimestamp")) or 0.0, m.name_of(s))


# ============================================================================ pod control
class RealStatefulPodControl:
    """stateful_pod_control.go: claims before pods, identity/storage repair with conflict
    retries, Successful*/Failed* events."""

    def __init__(self, client, pvc_lister, pod_lister, recorder=None):
        self.client, self.pvcs, self.pods, self.recorder = client, pvc_lister, pod_lister, recorder

    def _pod_event(self, verb, s, pod, err):
        if self.recorder is None:
            return
        if err is None:
            self.recorder.event(s, "Normal", f"Successful{verb.title()}",
                                f"{verb} Pod {m.name_of(pod)} in StatefulSet {m.name_of(s)} successful")
        else:
            self.recorder.event(s, "Warning", f"Failed{verb.title()}",
                                f"{verb} Pod {m.name_of(pod)} in StatefulSet {m.name_of(s)} failed error: {err}")

    def _claim_event(self, verb, s, pod, claim, err):
        if self.recorder is None:
            return
        if err is None:
            self.recorder.event(s, "Normal", f"Successful{verb.title()}",
                                f"{verb} Claim {m.name_of(claim)} Pod {m.name_of(pod)} in StatefulSet {m.name_of(s)} success")
        else:
            self.recorder.event(s, "Warning", f"Failed{verb.title()}",
                                f"{verb} Claim {m.name_of(claim)} for Pod {m.name_of(pod)} in StatefulSet "
                                f"{m.name_of(s)} failed error: {err}")

    async def create_claims(self, s, pod):
        errs = []
        for claim in get_pvcs(s, pod).values():
            try:
                found = self.pvcs.get(m.key_of(claim))
            except Exception as e:                    # noqa: BLE001 — a lister failure
                errs.append(RuntimeError(f"Failed to retrieve PVC {m.name_of(claim)}: {e}"))
                self._claim_event("create", s, pod, claim, e)
                continue
            if found is not None:
                continue
            try:
                await self.client.create(claim, m.namespace_of(claim))
                self._claim_event("create", s, pod, claim, None)
            except m.StatusError as e:
                errs.append(RuntimeError(f"Failed to create PVC {m.name_of(claim)}: {e}"))
                if not m.is_already_exists(e):
                    self._claim_event("create", s, pod, claim, e)
        if errs:
            raise errs[0] if len(errs) == 1 else RuntimeError("[" + ", ".join(str(e) for e in errs) + "]")

    async def create(self, s, pod):
        try:
            await self.create_claims(s, pod)
        except Exception as e:
            self._pod_event("create", s, pod, e)
            raise
        try:
            await self.client.create(pod, m.namespace_of(s))
        except m.StatusError as e:
            if not m.is_already_exists(e):
                self._pod_event("create", s, pod, e)
            raise
        self._pod_event("create", s, pod, None)

    async def update(self, s, pod):
        attempted, err = False, None
        for _ in range(5):
            consistent = True
            if not identity_matches(s, pod):
                update_identity(s, pod)
                consistent = False
            if not storage_matches(s, pod):
                update_storage(s, pod)
                consistent = False
                try:
                    await self.create_claims(s, pod)
                except Exception as e:
                    self._pod_event("update", s, pod, e)
                    raise
            if consistent:
                err = None
                break
            attempted = True
            try:
                await self.client.update(dict(pod, apiVersion="v1", kind="Pod"))
                err = None
                break
            except m.StatusError as e:
                err = e
                cached = self.pods.get(f"{m.namespace_of(s)}/{m.name_of(pod)}")
                if cached is not None:
                    pod = m.deepcopy(cached)
                if not m.is_conflict(e):
                    break
        if attempted:
            self._pod_event("update", s, pod, err)
        if err is not None:
            raise err

    async def delete(self, s, pod):
        try:
            await self.client.delete("pods", m.name_of(pod), m.namespace_of(s))
        except Exception as e:
            self._pod_event("delete", s, pod, e)
            raise
        self._pod_event("delete", s, pod, None)


class RealStatusUpdater:
    """stateful_set_status_updater.go: UpdateStatus with conflict retries from the lister."""

    def __init__(self, client, set_lister):
        self.client, self.sets = client, set_lister

    async def update_status(self, s, status: dict):
        s = m.deepcopy(s)
        for _ in range(5):
            s["status"] = dict(status)
            try:
                return await self.client.update(dict(s, apiVersion=API_VERSION, kind=KIND), "status")
            except m.StatusError as e:
                cached = self.sets.get(m.key_of(s))
                if cached is not None:
                    s = m.deepcopy(cached)
                if not m.is_conflict(e):
                    raise
        raise m.StatusError(409, "Conflict", f"statefulset {m.key_of(s)}: too many conflicts")


# ============================================================================ set control
class StatefulSetControl:
    """defaultStatefulSetControl."""

    def __init__(self, pod_control, status_updater, history):
        self.pod_control, self.status_updater, self.history = pod_control, status_updater, history

    def list_revisions(self, s) -> list:
        return self.history.list(s, selector_from_label_selector(_spec(s).get("selector")))

    async def adopt_orphan_revisions(self, s, revisions: list):
        for i, r in enumerate(revisions):
            revisions[i] = await self.history.adopt(s, API_VERSION, KIND, r)

    async def update(self, s, pods: list):
        """UpdateStatefulSet."""
        revisions = H.sort_revisions(list(self.list_revisions(s)))
        current, update, collision = await self.get_revisions(s, revisions)
        status = await self.update_pods(s, current, update, collision, pods)
        await self.update_status(s, status)
        await self.truncate_history(s, pods, revisions, current, update)
        return status

    async def truncate_history(self, s, pods, revisions, current, update):
        live = {m.name_of(current), m.name_of(update)} | {get_pod_revision(p) for p in pods}
        hist = [r for r in revisions if m.name_of(r) not in live]
        limit = int(_spec(s).get("revisionHistoryLimit", 10))
        if len(hist) <= limit:
            return
        for r in hist[:len(hist) - limit]:
            await self.history.delete(r)

    async def get_revisions(self, s, revisions: list):
        """getStatefulSetRevisions -> (current, update, collisionCount)."""
        H.sort_revisions(revisions)
        collision = [int(_status(s).get("collisionCount") or 0)]
        update = new_revision(s, next_revision(revisions), collision[0])
        equal = H.find_equal_revisions(revisions, update)
        if equal and H.equal_revision(revisions[-1], equal[-1]):
            update = revisions[-1]                   # the newest revision already is this template
        elif equal:
            update = await self.history.update(equal[-1], H.revision_of(update))   # a rollback: renumber
        else:
            update = await self.history.create(s, update, collision)
        current = next((r for r in revisions if m.name_of(r) == _status(s).get("currentRevision")), None)
        return (current if current is not None else update), update, collision[0]

    async def update_pods(self, s, current_rev, update_rev, collision: int, pods: list) -> dict:
        """updateStatefulSet: one pass over the pods; returns the status to record."""
        current_set = apply_revision(s, current_rev)
        update_set = apply_revision(s, update_rev)
        cur_name, upd_name = m.name_of(current_rev), m.name_of(update_rev)
        status = {"observedGeneration": int((s.get("metadata") or {}).get("generation") or 0),
                  "replicas": 0, "readyReplicas": 0, "currentReplicas": 0, "updatedReplicas": 0,
                  "currentRevision": cur_name, "updateRevision": upd_name, "collisionCount": collision}
        replica_count = int(_spec(s).get("replicas", 1))

        def count(p, d):
            """A pod counts toward currentReplicas and/or updatedReplicas by its revision label.
            1.9 used else-if here, so a set whose current and update revisions are the same
            reported updatedReplicas 0; the later upstream fix counts both (docs/PARITY.md)."""
            if get_pod_revision(p) == cur_name:
                status["currentReplicas"] += d
            if get_pod_revision(p) == upd_name:
                status["updatedReplicas"] += d

        replicas: list = [None] * replica_count
        condemned = []
        for p in pods:
            status["replicas"] += 1
            if is_running_and_ready(p):
                status["readyReplicas"] += 1
            if is_created(p) and not is_terminating(p):
                count(p, 1)
            o = ordinal_of(p)
            if 0 <= o < replica_count:
                replicas[o] = p
            elif o >= replica_count:
                condemned.append(p)
        for o in range(replica_count):
            if replicas[o] is None:
                replicas[o] = new_versioned_pod(current_set, update_set, cur_name, upd_name, o)
        sort_ascending_ordinal(condemned)
        first_unhealthy, first_ord = None, math.inf
        for p in replicas + condemned:
            if not is_healthy(p) and ordinal_of(p) < first_ord:
                first_ord, first_unhealthy = ordinal_of(p), p
        if (s.get("metadata") or {}).get("deletionTimestamp"):
            return status
        monotonic = not allows_burst(s)

        for i in range(replica_count):
            if is_failed(replicas[i]):
                await self.pod_control.delete(s, replicas[i])
                count(replicas[i], -1)
                status["replicas"] -= 1
                replicas[i] = new_versioned_pod(current_set, update_set, cur_name, upd_name, i)
            if not is_created(replicas[i]):
                await self.pod_control.create(s, replicas[i])
                status["replicas"] += 1
                count(replicas[i], 1)
                if monotonic:
                    return status
                continue
            if is_terminating(replicas[i]) and monotonic:
                return status
            if not is_running_and_ready(replicas[i]) and monotonic:
                return status
            if identity_matches(s, replicas[i]) and storage_matches(s, replicas[i]):
                continue
            await self.pod_control.update(update_set, m.deepcopy(replicas[i]))
        for target in range(len(condemned) - 1, -1, -1):
            p = condemned[target]
            if is_terminating(p):
                if monotonic:
                    return status
                continue
            if not is_running_and_ready(p) and monotonic and p is not first_unhealthy:
                return status
            await self.pod_control.delete(s, p)
            count(p, -1)
            if monotonic:
                return status
        st = _strategy(s)
        if (st.get("type") or "RollingUpdate") == "OnDelete":
            return status
        update_min = int((st.get("rollingUpdate") or {}).get("partition") or 0) if st.get("rollingUpdate") else 0
        for target in range(len(replicas) - 1, update_min - 1, -1):
            p = replicas[target]
            if get_pod_revision(p) != upd_name and not is_terminating(p):
                status["currentReplicas"] -= 1
                await self.pod_control.delete(s, p)
                return status
            if not is_healthy(p):
                return status
        return status

    async def update_status(self, s, status: dict):
        complete_rolling_update(s, status)
        if not inconsistent_status(s, status):
            return
        await self.status_updater.update_status(m.deepcopy(s), status)


# ============================================================================ controller
class StatefulSetController(Controller):
    """stateful_set.go."""
    name = "statefulset"

    def __init__(self, mgr, control: StatefulSetControl | None = None):
        super().__init__(mgr)
        self.control = control

    def setup(self):
        f = self.mgr.factory
        self.set_inf = f.informer("statefulsets")
        self.pvc_inf = f.informer("persistentvolumeclaims")
        self.rev_inf = f.informer("controllerrevisions.apps")
        self.pod_inf = self.mgr.pods
        self.set_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.pod_inf.add_handler(on_add=self.add_pod, on_update=self.update_pod, on_delete=self.delete_pod)
        if self.control is None:
            rec = getattr(self.mgr, "recorder", None)
            self.control = StatefulSetControl(RealStatefulPodControl(self.client, self.pvc_inf, self.pod_inf, rec),
                                              RealStatusUpdater(self.client, self.set_inf),
                                              H.History(self.client, self.rev_inf))

    # ------------------------------------------------------------------ pod events
    def resolve(self, ns, ref):
        if ref.get("kind") != KIND:
            return None
        s = self.set_inf.get(f"{ns}/{ref.get('name')}")
        if s is None or m.uid_of(s) != ref.get("uid"):
            return None
        return s

    def sets_for_pod(self, pod) -> list:
        """GetPodStatefulSets: the namespace's sets whose selector matches the pod's labels."""
        out = []
        labels = m.labels_of(pod)
        if not labels:
            return out
        for s in self.set_inf.list():
            if m.namespace_of(s) != m.namespace_of(pod):
                continue
            try:
                sel = selector_from_label_selector(_spec(s).get("selector"))
            except Exception:
                continue
            if sel.empty() or not sel.matches(labels):
                continue
            out.append(s)
        return out

    def add_pod(self, pod):
        if (pod.get("metadata") or {}).get("deletionTimestamp"):
            self.delete_pod(pod)
            return
        ref = m.controller_ref(pod)
        if ref is not None:
            s = self.resolve(m.namespace_of(pod), ref)
            if s is not None:
                self.enqueue(s)
            return
        for s in self.sets_for_pod(pod):
            self.enqueue(s)

    def update_pod(self, old, cur):
        if (old.get("metadata") or {}).get("resourceVersion") == (cur.get("metadata") or {}).get("resourceVersion"):
            return
        label_changed = m.labels_of(old) != m.labels_of(cur)
        cur_ref, old_ref = m.controller_ref(cur), m.controller_ref(old)
        ref_changed = cur_ref != old_ref
        if ref_changed and old_ref is not None:
            s = self.resolve(m.namespace_of(old), old_ref)
            if s is not None:
                self.enqueue(s)
        if cur_ref is not None:
            s = self.resolve(m.namespace_of(cur), cur_ref)
            if s is not None:
                self.enqueue(s)
            return
        if label_changed or ref_changed:
            for s in self.sets_for_pod(cur):
                self.enqueue(s)

    def delete_pod(self, pod):
        ref = m.controller_ref(pod)
        if ref is None:
            return
        s = self.resolve(m.namespace_of(pod), ref)
        if s is not None:
            self.enqueue(s)

    # ------------------------------------------------------------------ sync
    def _fresh(self, s):
        client = self.client

        async def get():
            f = await client.get("statefulsets", m.name_of(s), m.namespace_of(s))
            if m.uid_of(f) != m.uid_of(s):
                raise RuntimeError(f"original StatefulSet {m.key_of(s)} is gone: got uid {m.uid_of(f)}, "
                                   f"wanted {m.uid_of(s)}")
            return f
        return get

    async def pods_for_set(self, s, selector) -> list:
        """getPodsForStatefulSet: claim the namespace's member pods matching the selector."""
        pods = [p for p in self.pod_inf.list() if m.namespace_of(p) == m.namespace_of(s)]
        client = self.client

        async def adopt(pod):
            await client.patch("pods", m.name_of(pod), adopt_patch(s, API_VERSION, KIND, pod), m.namespace_of(pod),
                               patch_type="application/strategic-merge-patch+json")

        async def release(pod):
            try:
                await client.patch("pods", m.name_of(pod), release_patch(s, pod), m.namespace_of(pod),
                                   patch_type="application/strategic-merge-patch+json")
            except m.StatusError as e:
                if not (m.is_not_found(e) or e.code == 422):
                    raise
        mgr = ControllerRefManager(s, selector, adopt, release, recheck_deletion(self._fresh(s)))
        return await mgr.claim(pods, filters=(lambda p: is_member_of(s, p),))

    async def adopt_orphan_revisions(self, s):
        revisions = self.control.list_revisions(s)
        if any(m.controller_ref(r) is None for r in revisions):
            await self._fresh(s)()
            await self.control.adopt_orphan_revisions(s, revisions)

    async def sync(self, key):
        s = self.set_inf.get(key)
        if s is None:
            return
        try:
            selector = selector_from_label_selector(_spec(s).get("selector"))
        except Exception:
            return
        await self.adopt_orphan_revisions(s)
        pods = await self.pods_for_set(s, selector)
        await self.control.update(m.deepcopy(s), pods)
