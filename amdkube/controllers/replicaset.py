"""ReplicaSet controller (pkg/controller/replicaset/replica_set.go, replica_set_utils.go); the
ReplicationController manager (pkg/controller/replication) is the same logic over a v1 map
selector (controllers/apps.py).

syncReplicaSet (:572-643):
  * expectations gate manageReplicas: after issuing creates/deletes the controller waits for
    its informer to observe them (ControllerExpectations / UID-tracked deletions);
  * the active pods of the namespace are claimed through the ControllerRef manager — matching
    orphans adopted, owned pods whose labels stopped matching released;
  * manageReplicas (:460-570): too few -> create (at most burstReplicas = 500) in slow-start
    batches 1, 2, 4, … (a failing batch skips the rest and lowers the expectations); too many
    -> delete the pods that sort first by controller.ActivePods;
  * the status (calculateStatus, replica_set_utils.go:85-128): replicas, fullyLabeledReplicas
    (pods carrying all the template's labels), ready, available (ready for minReadySeconds),
    a ReplicaFailure condition (FailedCreate / FailedDelete) while manageReplicas errs, written
    with up to one retry over a fresh read (updateReplicaSetStatus :36-83);
  * a ReplicaSet whose pods are ready but not yet available is requeued after minReadySeconds.
Pod events resolve the ControllerRef (creation / deletion observed, orphan pods enqueue every
ReplicaSet selecting them).
"""
from __future__ import annotations

import json
import time

from ..api import meta as m
from ..api.helpers import get_condition, is_pod_ready
from ..api.labels import selector_from_label_selector, selector_from_set
from .base import Controller, split_key
from .controller_utils import (SLOW_START_INITIAL_BATCH, ControllerRefManager, UIDTrackingControllerExpectations,
                               adopt_patch, filter_active_pods, is_pod_active, pod_key, recheck_deletion, release_patch,
                               slow_start_batch, sort_active_pods)

BURST_REPLICAS = 500
STATUS_UPDATE_RETRIES = 1


def is_pod_available(p: dict, min_ready_seconds: int, now: float) -> bool:
    """podutil.IsPodAvailable: ready for at least minReadySeconds."""
    if not is_pod_ready(p):
        return False
    if not min_ready_seconds:
        return True
    since = m.parse_time((get_condition(p, "Ready") or {}).get("lastTransitionTime"))
    return since is not None and since + min_ready_seconds < now          # Time.Before: strictly earlier


def pod_from_template(template: dict, owner: dict, controller_ref: dict | None) -> dict:
    """controller_utils.go GetPodFromTemplate: labels, annotations and finalizers of the
    template, generateName `<owner>-`, the controller reference, the template's spec."""
    tpl = json.loads(json.dumps(template or {}))
    md = tpl.get("metadata") or {}
    labels = dict(md.get("labels") or {})
    if not labels:
        raise ValueError("unable to create pods, no labels")
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"generateName": m.name_of(owner) + "-", "labels": labels,
                        "annotations": dict(md.get("annotations") or {})},
           "spec": tpl.get("spec") or {}}
    if md.get("finalizers"):
        pod["metadata"]["finalizers"] = list(md["finalizers"])
    if controller_ref is not None:
        pod["metadata"]["ownerReferences"] = [controller_ref]
    return pod


class RealPodControl:
    """controller.RealPodControl over the API client, recording SuccessfulCreate /
    FailedCreate / SuccessfulDelete / FailedDelete events on the owner."""

    def __init__(self, client, recorder=None):
        self.client, self.recorder = client, recorder

    def _event(self, obj, typ, reason, msg):
        if self.recorder is not None:
            self.recorder.event(obj, typ, reason, msg)

    async def create_pods_with_controller_ref(self, ns: str, template: dict, owner: dict, controller_ref: dict):
        pod = pod_from_template(template, owner, controller_ref)
        try:
            created = await self.client.create(pod, ns)
        except Exception as e:
            self._event(owner, "Warning", "FailedCreate", f"Error creating: {e}")
            raise
        self._event(owner, "Normal", "SuccessfulCreate", f"Created pod: {m.name_of(created)}")
        return created

    async def delete_pod(self, ns: str, name: str, owner: dict):
        try:
            await self.client.delete("pods", name, ns)
        except Exception as e:
            self._event(owner, "Warning", "FailedDelete", f"Error deleting: {e}")
            raise
        self._event(owner, "Normal", "SuccessfulDelete", f"Deleted pod: {name}")

    async def patch_pod(self, ns: str, name: str, patch: dict):
        return await self.client.patch("pods", name, patch, ns, patch_type="application/strategic-merge-patch+json")


def get_pods_to_delete(pods: list, diff: int) -> list:
    """getPodsToDelete: all of them, or the first `diff` in ActivePods order."""
    pods = list(pods)
    if diff < len(pods):
        sort_active_pods(pods)
    return pods[:diff]


def rs_condition(kind: str, status: str, reason: str, msg: str) -> dict:
    return {"type": kind, "status": status, "lastTransitionTime": m.now_rfc3339(), "reason": reason, "message": msg}


def set_condition(status: dict, cond: dict):
    conds = status.get("conditions") or []
    cur = next((c for c in conds if c.get("type") == cond["type"]), None)
    if cur is not None and cur.get("status") == cond["status"] and cur.get("reason") == cond["reason"]:
        return
    status["conditions"] = [c for c in conds if c.get("type") != cond["type"]] + [cond]


def remove_condition(status: dict, kind: str):
    conds = [c for c in status.get("conditions") or [] if c.get("type") != kind]
    if conds:
        status["conditions"] = conds
    else:
        status.pop("conditions", None)


def calculate_status(rs: dict, pods: list, manage_err: BaseException | None, now: float | None = None) -> dict:
    """calculateStatus (replica_set_utils.go:85-128)."""
    now = time.time() if now is None else now
    status = json.loads(json.dumps(rs.get("status") or {}))
    tpl_sel = selector_from_set(((rs.get("spec") or {}).get("template") or {}).get("metadata", {}).get("labels") or {})
    mrs = int((rs.get("spec") or {}).get("minReadySeconds") or 0)
    labeled = ready = available = 0
    for p in pods:
        if tpl_sel.matches(m.labels_of(p)):
            labeled += 1
        if is_pod_ready(p):
            ready += 1
            if is_pod_available(p, mrs, now):
                available += 1
    failure = next((c for c in status.get("conditions") or [] if c.get("type") == "ReplicaFailure"), None)
    if manage_err is not None and failure is None:
        diff = len(pods) - int((rs.get("spec") or {}).get("replicas", 1))
        reason = "FailedCreate" if diff < 0 else ("FailedDelete" if diff > 0 else "")
        set_condition(status, rs_condition("ReplicaFailure", "True", reason, str(manage_err)))
    elif manage_err is None and failure is not None:
        remove_condition(status, "ReplicaFailure")
    status.update({"replicas": len(pods), "fullyLabeledReplicas": labeled, "readyReplicas": ready,
                   "availableReplicas": available})
    return status


class ReplicaSetController(Controller):
    name = "replicaset"
    burst = BURST_REPLICAS
    owner_api, owner_kind, plural = "apps/v1", "ReplicaSet", "replicasets"
    workers = 5

    def __init__(self, mgr, pod_control=None, clock=time.time):
        super().__init__(mgr)
        self.clock = clock
        self.expectations = UIDTrackingControllerExpectations()
        self.pod_control = pod_control or RealPodControl(mgr.client, getattr(mgr, "recorder", None))

    # ------------------------------------------------------------------ informers
    def setup(self):
        self.rs_inf = self.mgr.factory.informer(self.plural)
        self.pod_inf = self.mgr.pods
        self.rs_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self._rs_deleted)
        self.pod_inf.add_handler(on_add=self.add_pod, on_update=self.update_pod, on_delete=self.delete_pod)

    def _rs_deleted(self, rs):
        self.expectations.delete_expectations(m.key_of(rs))
        self.enqueue(rs)

    def selector_of(self, rs):
        return selector_from_label_selector((rs.get("spec") or {}).get("selector"))

    def _resolve(self, ns: str, ref: dict):
        """resolveControllerRef: the ReplicaSet the reference names, if it is still that one."""
        if ref.get("kind") != self.owner_kind:
            return None
        rs = self.rs_inf.get(f"{ns}/{ref.get('name')}")
        if rs is None or m.uid_of(rs) != ref.get("uid"):
            return None
        return rs

    def pod_owners(self, pod) -> list:
        """getPodReplicaSets: every ReplicaSet of the namespace selecting this (orphan) pod."""
        ns, labels = m.namespace_of(pod), m.labels_of(pod)
        out = []
        for rs in self.rs_inf.list():
            if m.namespace_of(rs) != ns:
                continue
            try:
                sel = self.selector_of(rs)
            except Exception:
                continue
            if not sel.empty() and sel.matches(labels):
                out.append(rs)
        return out

    def add_pod(self, pod):
        if (pod.get("metadata") or {}).get("deletionTimestamp"):
            self.delete_pod(pod)
            return
        ref = m.controller_ref(pod)
        if ref is not None:
            rs = self._resolve(m.namespace_of(pod), ref)
            if rs is not None:
                self.expectations.creation_observed(m.key_of(rs))
                self.enqueue(rs)
            return
        for rs in self.pod_owners(pod):
            self.enqueue(rs)

    def update_pod(self, old, cur):
        if (old.get("metadata") or {}).get("resourceVersion") == (cur.get("metadata") or {}).get("resourceVersion"):
            return
        label_changed = m.labels_of(old) != m.labels_of(cur)
        if (cur.get("metadata") or {}).get("deletionTimestamp"):
            self.delete_pod(cur)
            if label_changed:
                self.delete_pod(old)
            return
        cur_ref, old_ref = m.controller_ref(cur), m.controller_ref(old)
        ref_changed = cur_ref != old_ref
        if ref_changed and old_ref is not None:
            rs = self._resolve(m.namespace_of(old), old_ref)
            if rs is not None:
                self.enqueue(rs)
        if cur_ref is not None:
            rs = self._resolve(m.namespace_of(cur), cur_ref)
            if rs is None:
                return
            self.enqueue(rs)
            mrs = int((rs.get("spec") or {}).get("minReadySeconds") or 0)
            if not is_pod_ready(old) and is_pod_ready(cur) and mrs > 0:
                self.queue.add_after(m.key_of(rs), mrs + 1.0)
            return
        if label_changed or ref_changed:
            for rs in self.pod_owners(cur):
                self.enqueue(rs)

    def delete_pod(self, pod):
        ref = m.controller_ref(pod)
        if ref is None:
            return
        rs = self._resolve(m.namespace_of(pod), ref)
        if rs is None:
            return
        key = m.key_of(rs)
        self.expectations.deletion_observed(key, pod_key(pod))
        self.enqueue(rs)

    # ------------------------------------------------------------------ sync
    async def claim_pods(self, rs, selector, pods):
        client = self.client

        async def fresh():
            f = await client.get(self.plural, m.name_of(rs), m.namespace_of(rs))
            if m.uid_of(f) != m.uid_of(rs):
                raise RuntimeError(f"original {self.owner_kind} {m.key_of(rs)} is gone: got uid {m.uid_of(f)}, "
                                   f"wanted {m.uid_of(rs)}")
            return f

        async def adopt(pod):
            await self.pod_control.patch_pod(m.namespace_of(pod), m.name_of(pod),
                                             adopt_patch(rs, self.owner_api, self.owner_kind, pod))

        async def release(pod):
            await self.pod_control.patch_pod(m.namespace_of(pod), m.name_of(pod), release_patch(rs, pod))
        return await ControllerRefManager(rs, selector, adopt, release, recheck_deletion(fresh)).claim(pods)

    def controller_ref(self, rs) -> dict:
        return m.new_controller_ref(rs, self.owner_api, self.owner_kind)

    async def manage_replicas(self, pods: list, rs: dict):
        """manageReplicas (replica_set.go:460-570)."""
        want = int((rs.get("spec") or {}).get("replicas", 1))
        diff = len(pods) - want
        key = m.key_of(rs)
        ns = m.namespace_of(rs)
        if diff < 0:
            n = min(-diff, self.burst)
            self.expectations.expect_creations(key, n)
            template = (rs.get("spec") or {}).get("template") or {}
            ref = self.controller_ref(rs)

            async def create():
                try:
                    await self.pod_control.create_pods_with_controller_ref(ns, template, rs, ref)
                except m.StatusError as e:
                    if e.code == 504:            # a timeout: the informer sees the pod when it lands
                        return
                    raise
            ok, err = await slow_start_batch(n, SLOW_START_INITIAL_BATCH, create)
            for _ in range(n - ok):
                self.expectations.creation_observed(key)
            if err is not None:
                raise err
        elif diff > 0:
            n = min(diff, self.burst)
            victims = get_pods_to_delete(pods, n)
            self.expectations.expect_deletions(key, [pod_key(p) for p in victims])
            errs = []
            for p in victims:
                try:
                    await self.pod_control.delete_pod(ns, m.name_of(p), rs)
                except Exception as e:
                    self.expectations.deletion_observed(key, pod_key(p))
                    errs.append(e)
            if errs:
                raise errs[0]

    async def update_status(self, rs: dict, status: dict) -> dict:
        """updateReplicaSetStatus (replica_set_utils.go:36-83)."""
        cur = rs.get("status") or {}
        gen = (rs.get("metadata") or {}).get("generation", 1)
        fields = ("replicas", "fullyLabeledReplicas", "readyReplicas", "availableReplicas")
        if all(int(cur.get(k) or 0) == int(status.get(k) or 0) for k in fields) and \
                gen == cur.get("observedGeneration") and (cur.get("conditions") or []) == (status.get("conditions") or []):
            return rs
        status["observedGeneration"] = gen
        obj = rs
        err = None
        for i in range(STATUS_UPDATE_RETRIES + 1):
            obj = {**obj, "status": status}
            try:
                return await self.client.update(dict(obj, apiVersion=obj.get("apiVersion") or self.owner_api,
                                                     kind=obj.get("kind") or self.owner_kind), "status")
            except m.StatusError as e:
                err = e
                if i >= STATUS_UPDATE_RETRIES:
                    break
                obj = await self.client.get(self.plural, m.name_of(rs), m.namespace_of(rs))
        raise err

    async def sync(self, key):
        ns, name = split_key(key)
        rs = self.rs_inf.get(key)
        if rs is None:
            self.expectations.delete_expectations(key)
            return
        needs_sync = self.expectations.satisfied_expectations(key)
        try:
            selector = self.selector_of(rs)
        except Exception:
            return
        pods = [p for p in self.pod_inf.list() if m.namespace_of(p) == ns and is_pod_active(p)]
        pods = await self.claim_pods(rs, selector, pods)
        manage_err = None
        if needs_sync and not (rs.get("metadata") or {}).get("deletionTimestamp"):
            try:
                await self.manage_replicas(pods, rs)
            except Exception as e:          # noqa: BLE001 — reported in the status, then raised
                manage_err = e
        rs = json.loads(json.dumps(rs))
        status = calculate_status(rs, filter_active_pods(pods), manage_err, self.clock())
        updated = await self.update_status(rs, status)
        st, spec = updated.get("status") or {}, updated.get("spec") or {}
        mrs = int(spec.get("minReadySeconds") or 0)
        want = int(spec.get("replicas", 1))
        if manage_err is None and mrs > 0 and int(st.get("readyReplicas") or 0) == want and \
                int(st.get("availableReplicas") or 0) != want:
            self.queue.add_after(key, float(mrs))
        if manage_err is not None:
            raise manage_err
