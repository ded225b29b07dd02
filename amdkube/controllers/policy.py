"""Disruption budgets, resource-quota usage, node TTL and ClusterRole aggregation.

Reference:
  * pkg/controller/disruption/disruption.go — for every PodDisruptionBudget (an empty selector
    selects no pods): expectedPods from the scale of the pods' controllers, each found by UID
    (ReplicaSet, Deployment through its ReplicaSet, ReplicationController, StatefulSet) for a
    percentage minAvailable or any maxUnavailable, else the matching pod count; desiredHealthy
    from minAvailable / maxUnavailable (rounded up); currentHealthy = ready matching pods not
    being deleted and not recently evicted (status.disruptedPods, kept 2 min, the budget
    rechecked when the first expires); disruptionsAllowed = currentHealthy - desiredHealthy,
    0 when negative or no pods are expected. A pod without a known controller makes the sync
    fail safe: the old status with disruptionsAllowed 0.
  * pkg/controller/resourcequota/resource_quota_controller.go over amdkube.quota (the
    pkg/quota/evaluator/core evaluators): status.used for pods (compute, requests.*, limits.*,
    scopes), services (nodeports, loadbalancers), PVCs (storage, per StorageClass) and object
    counts; status.hard mirrors spec.hard. Extended resources (amd.com/gpu) count from the
    device-granular spec.extendedResources too.
  * pkg/controller/ttl/ttl_controller.go — node annotation node.alpha.kubernetes.io/ttl from
    cluster size with hysteresis (0 s up to 100 nodes, 15 s from 90 to 500, 30 s 450-1000, 60 s
    900-2000, 300 s 1800-10000, then 600 s).
  * pkg/controller/clusterroleaggregation — a ClusterRole with aggregationRule gets the union
    of the rules of every ClusterRole its clusterRoleSelectors match.
"""
from __future__ import annotations

import math
import time

from ..api import meta as m
from ..api.helpers import is_pod_ready, is_pod_terminal
from ..api.labels import selector_from_label_selector
from .base import Controller, split_key

DISRUPTED_TIMEOUT = 120.0          # DeletionTimeout: an evicted pod not gone by then counts again


def _int_or_percent(v, total: int, round_up: bool = True) -> int:
    """intstr.GetValueFromIntOrPercent."""
    if isinstance(v, str) and v.endswith("%"):
        f = float(v[:-1]) * total / 100.0
        return int(math.ceil(f) if round_up else math.floor(f))
    return int(v)


class _NoController(Exception):
    pass


class DisruptionController(Controller):
    """pkg/controller/disruption/disruption.go."""
    name = "disruption"

    def setup(self):
        f = self.mgr.factory
        self.pdb_inf = f.informer("poddisruptionbudgets")
        self.pod_inf = self.mgr.pods
        self.rc_inf, self.rs_inf = f.informer("replicationcontrollers"), f.informer("replicasets")
        self.d_inf, self.ss_inf = f.informer("deployments"), f.informer("statefulsets")
        self.pdb_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=lambda o: None)
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)

    def _event(self, obj, etype, reason, msg):
        rec = getattr(self.mgr, "recorder", None)
        if rec is not None:
            rec.event(obj, etype, reason, msg)

    def _pod(self, pod):
        labels = m.labels_of(pod)
        for pdb in self.pdb_inf.list():
            if m.namespace_of(pdb) == m.namespace_of(pod) and self._selects(pdb, labels):
                self.enqueue(pdb)

    @staticmethod
    def _selects(pdb, labels) -> bool:
        """getPodsForPdb: an empty selector selects nothing."""
        sel = (pdb.get("spec") or {}).get("selector")
        return bool(sel) and bool(sel.get("matchLabels") or sel.get("matchExpressions")) and \
            selector_from_label_selector(sel).matches(labels)

    # ---------------------------------------------------------------- finders
    def _owner(self, inf, ns, ref):
        o = inf.get(f"{ns}/{ref.get('name')}")
        return o if o is not None and m.uid_of(o) == ref.get("uid") else None

    def _finders(self, ref, ns):
        """finders(): (uid, scale) of the pod's controller, if it is one of the supported kinds.
        A ReplicaSet owned by a Deployment is answered by the Deployment finder."""
        kind = ref.get("kind")
        if kind == "ReplicaSet":
            rs = self._owner(self.rs_inf, ns, ref)
            if rs is None:
                return None
            dref = m.controller_ref(rs)
            if dref is None:
                return m.uid_of(rs), int((rs.get("spec") or {}).get("replicas", 1))
            if dref.get("kind") == "Deployment":
                d = self._owner(self.d_inf, ns, dref)
                if d is not None:
                    return m.uid_of(d), int((d.get("spec") or {}).get("replicas", 1))
            return None
        for k, inf in (("ReplicationController", self.rc_inf), ("StatefulSet", self.ss_inf)):
            if kind == k:
                o = self._owner(inf, ns, ref)
                return (m.uid_of(o), int((o.get("spec") or {}).get("replicas", 1))) if o is not None else None
        return None

    def expected_scale(self, pdb, pods) -> int:
        """getExpectedScale: the sum of the scales of the pods' controllers, each counted once."""
        scale: dict[str, int] = {}
        for p in pods:
            ref = m.controller_ref(p)
            if ref is None:
                msg = f'found no controller ref for pod "{m.name_of(p)}"'
                self._event(pdb, "Warning", "NoControllerRef", msg)
                raise _NoController(msg)
            if ref.get("uid") in scale:
                continue
            found = self._finders(ref, m.namespace_of(p))
            if found is None:
                msg = f'found no controllers for pod "{m.name_of(p)}"'
                self._event(pdb, "Warning", "NoControllers", msg)
                raise _NoController(msg)
            scale[found[0]] = found[1]
        return sum(scale.values())

    def expected_pod_count(self, pdb, pods) -> tuple[int, int]:
        """getExpectedPodCount -> (expectedCount, desiredHealthy)."""
        spec = pdb.get("spec") or {}
        if spec.get("maxUnavailable") is not None:
            expected = self.expected_scale(pdb, pods)
            return expected, max(0, expected - _int_or_percent(spec["maxUnavailable"], expected))
        mina = spec.get("minAvailable")
        if mina is None:
            return 0, 0
        if isinstance(mina, str):
            expected = self.expected_scale(pdb, pods)
            return expected, _int_or_percent(mina, expected)
        return len(pods), int(mina)

    def disrupted_pod_map(self, pods, pdb, now: float) -> tuple[dict, float | None]:
        """buildDisruptedPodMap: evictions of pods still present and not yet being deleted, within
        the deletion timeout; and the earliest time one of them expires (to recheck then)."""
        old = (pdb.get("status") or {}).get("disruptedPods") or {}
        result, recheck = {}, None
        if not old:
            return result, recheck
        for p in pods:
            if (p.get("metadata") or {}).get("deletionTimestamp") or m.name_of(p) not in old:
                continue
            t = m.parse_time(old[m.name_of(p)]) or 0
            if t + DISRUPTED_TIMEOUT < now:
                self._event(p, "Warning", "NotDeleted",
                            f"Pod was expected by PDB {m.namespace_of(pdb)}/{m.name_of(pdb)} to be deleted but it wasn't")
                continue
            result[m.name_of(p)] = old[m.name_of(p)]
            recheck = t + DISRUPTED_TIMEOUT if recheck is None else min(recheck, t + DISRUPTED_TIMEOUT)
        return result, recheck

    @staticmethod
    def count_healthy(pods, disrupted: dict, now: float) -> int:
        """countHealthyPods: ready pods not being deleted and not expected to be deleted soon."""
        n = 0
        for p in pods:
            if (p.get("metadata") or {}).get("deletionTimestamp"):
                continue
            t = disrupted.get(m.name_of(p))
            if t is not None and (m.parse_time(t) or 0) + DISRUPTED_TIMEOUT > now:
                continue
            if is_pod_ready(p):
                n += 1
        return n

    async def _update(self, pdb, status: dict):
        body = dict(pdb, status=status)
        try:
            await self.client.update(body, sub="status")   # CAS on resourceVersion vs concurrent evictions
        except m.StatusError as e:
            if not m.is_conflict(e):
                raise
            self.enqueue(m.key_of(pdb))

    async def sync(self, key):
        pdb = self.pdb_inf.get(key)
        if pdb is None:
            return
        try:
            await self._try_sync(pdb)
        except _NoController:
            # failSafe: the budget's last status stands, but nothing may be disrupted
            await self._update(pdb, dict(pdb.get("status") or {}, disruptionsAllowed=0))

    async def _try_sync(self, pdb):
        ns = m.namespace_of(pdb)
        pods = [p for p in self.pod_inf.list() if m.namespace_of(p) == ns and self._selects(pdb, m.labels_of(p))]
        if not pods:
            self._event(pdb, "Normal", "NoPods", "No matching pods found")
        expected, desired = self.expected_pod_count(pdb, pods)
        now = time.time()
        disrupted, recheck = self.disrupted_pod_map(pods, pdb, now)
        healthy = self.count_healthy(pods, disrupted, now)
        allowed = healthy - desired
        if expected <= 0 or allowed <= 0:
            allowed = 0
        old = pdb.get("status") or {}
        st = {"currentHealthy": healthy, "desiredHealthy": desired, "expectedPods": expected, "disruptionsAllowed": allowed,
              "disruptedPods": disrupted, "observedGeneration": (pdb.get("metadata") or {}).get("generation", 0)}
        # a status never written (fields absent) is always written, as the reference's nil
        # DisruptedPods never DeepEquals the computed map
        if any(k not in old for k in st if k != "disruptedPods") or \
                {k: (old.get(k) or {}) if k == "disruptedPods" else old.get(k) for k in st} != st:
            await self._update(pdb, st)
        if recheck is not None:
            self.queue.add_after(m.key_of(pdb), max(0.0, recheck - now))


# ------------------------------------------------------------------------ quota usage
# object kinds whose count a quota can limit: (group, plural); the legacy names and count/<res>
COUNTED = {("", "services"), ("", "configmaps"), ("", "secrets"), ("", "persistentvolumeclaims"),
           ("", "replicationcontrollers"), ("", "resourcequotas"), ("apps", "deployments"), ("apps", "replicasets"),
           ("apps", "statefulsets"), ("apps", "daemonsets"), ("batch", "jobs"), ("batch", "cronjobs")}


class ResourceQuotaController(Controller):
    """pkg/controller/resourcequota/resource_quota_controller.go: status.hard := spec.hard and
    status.used := the namespace's usage under amdkube.quota's evaluators and the quota's scopes.
    A quota is re-synced when its spec.hard changes (never on a status-only update: those are the
    admission plugin's reservations, :118-130), when an object it counts changes, and every
    30 s (the full resync that settles reservations of objects that never got created)."""
    name = "resourcequota"
    resync = 30.0

    def setup(self):
        f = self.mgr.factory
        self.q_inf = f.informer("resourcequotas")
        self.pod_inf = self.mgr.pods
        self.count_infs = {gr: f.informer(gr[1]) for gr in COUNTED}
        self.q_inf.add_handler(on_add=self.enqueue, on_update=self._quota_update)
        self.pod_inf.add_handler(on_add=self._ns, on_update=self._pod_update, on_delete=self._ns)
        for inf in self.count_infs.values():
            inf.add_handler(on_add=self._ns, on_update=lambda o, n: self._ns(n), on_delete=self._ns)

    def _quota_update(self, old, new):
        if (old.get("spec") or {}) != (new.get("spec") or {}) or not (new.get("status") or {}).get("hard"):
            self.enqueue(new)

    def _pod_update(self, old, new):
        # replenishment: a pod that turns terminal (or starts deleting) frees its usage
        if is_pod_terminal(new) != is_pod_terminal(old) or \
                bool((new.get("metadata") or {}).get("deletionTimestamp")) != bool((old.get("metadata") or {}).get("deletionTimestamp")):
            self._ns(new)

    def _ns(self, obj):
        ns = m.namespace_of(obj)
        for q in self.q_inf.list():
            if m.namespace_of(q) == ns:
                self.enqueue(q)

    def _objects(self, ns):
        def lister(group, resource):
            inf = self.pod_inf if (group, resource) == ("", "pods") else self.count_infs.get((group, resource))
            return [o for o in inf.list() if m.namespace_of(o) == ns] if inf is not None else []
        return lister

    async def sync(self, key):
        from .. import quota as Q
        q = self.q_inf.get(key)
        if q is None:
            return
        ns, name = split_key(key)
        hard = (q.get("spec") or {}).get("hard") or {}
        used = Q.format_list(Q.calculate_usage(q, self._objects(ns)))
        st = {"hard": dict(hard), "used": used}
        if (q.get("status") or {}) != st:
            # UpdateStatus with the resourceVersion that was read (resource_quota_controller.go
            # :350-371): a reservation the admission plugin made since then is a conflict, and
            # the key is retried once the informer has the newer quota
            out = m.deepcopy(q)
            out["status"] = st
            await self.client.update_status(out)


# --------------------------------------------------------------------------- node TTL
TTL_ANNOTATION = "node.alpha.kubernetes.io/ttl"
# ttlBoundaries: overlapping (sizeMin, sizeMax, ttl) steps; the step moves up only when the node
# count passes sizeMax and down only when it falls under sizeMin (hysteresis)
TTL_BOUNDARIES = ((0, 100, 0), (90, 500, 15), (450, 1000, 30), (900, 2000, 60), (1800, 10000, 300),
                  (9000, 2**31 - 1, 600))


def ttl_for(nodes: int) -> int:
    """The TTL a cluster grown from empty to `nodes` nodes settles on."""
    for _lo, hi, ttl in TTL_BOUNDARIES:
        if nodes <= hi:
            return ttl
    return TTL_BOUNDARIES[-1][2]


class TTLController(Controller):
    """pkg/controller/ttl/ttl_controller.go: the node annotation node.alpha.kubernetes.io/ttl (how
    long kubelets may cache secrets / config maps) follows cluster size with hysteresis."""
    name = "ttl"
    workers = 1

    def __init__(self, mgr):
        super().__init__(mgr)
        self.node_count, self.boundary_step, self.desired_ttl = 0, 0, 0

    def setup(self):
        self.node_inf = self.mgr.nodes
        self.node_inf.add_handler(on_add=self.add_node, on_update=lambda o, n: self.enqueue(n), on_delete=self.delete_node)

    def add_node(self, node):
        self.node_count += 1
        if self.node_count > TTL_BOUNDARIES[self.boundary_step][1]:
            self.boundary_step += 1
            self.desired_ttl = TTL_BOUNDARIES[self.boundary_step][2]
            for n in self.node_inf.list():      # every node's annotation changes with the step
                self.enqueue(n)
        if m.name_of(node):
            self.enqueue(node)

    def delete_node(self, node):
        self.node_count -= 1
        if self.node_count < TTL_BOUNDARIES[self.boundary_step][0]:
            self.boundary_step -= 1
            self.desired_ttl = TTL_BOUNDARIES[self.boundary_step][2]
            for n in self.node_inf.list():
                self.enqueue(n)

    @staticmethod
    def ttl_patch(node, ttl: int) -> dict:
        """patchNodeWithAnnotation's strategic merge patch: empty when the value is already set."""
        if m.annotations_of(node).get(TTL_ANNOTATION) == str(ttl):
            return {}
        return {"metadata": {"annotations": {TTL_ANNOTATION: str(ttl)}}}

    async def update_node_if_needed(self, name: str):
        node = self.node_inf.get(name)
        if node is None:
            return
        if m.annotations_of(node).get(TTL_ANNOTATION) == str(self.desired_ttl):
            return
        await self.client.patch("nodes", name, self.ttl_patch(node, self.desired_ttl),
                                patch_type="application/strategic-merge-patch+json")

    async def sync(self, key):
        await self.update_node_if_needed(split_key(key)[1])


# ------------------------------------------------------------- ClusterRole aggregation
class ClusterRoleAggregationController(Controller):
    name = "clusterrole-aggregation"
    workers = 1

    def setup(self):
        self.cr_inf = self.mgr.factory.informer("clusterroles")
        self.cr_inf.add_handler(on_add=lambda o: self._all(), on_update=lambda o, n: self._all(), on_delete=lambda o: self._all())

    def _all(self):
        for cr in self.cr_inf.list():
            if cr.get("aggregationRule"):
                self.enqueue(cr)

    async def sync(self, key):
        _, name = split_key(key)
        cr = self.cr_inf.get(name)
        if cr is None or not cr.get("aggregationRule"):
            return
        sels = [selector_from_label_selector(s) for s in cr["aggregationRule"].get("clusterRoleSelectors") or []]
        rules = []
        for other in sorted(self.cr_inf.list(), key=m.name_of):
            if m.name_of(other) == name:
                continue
            if any(s.matches(m.labels_of(other)) for s in sels):
                for r in other.get("rules") or []:
                    if r not in rules:
                        rules.append(r)
        if (cr.get("rules") or []) != rules:
            await self.client.patch("clusterroles", name, {"rules": rules})
