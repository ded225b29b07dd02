"""Disruption budgets, resource-quota usage, node TTL and ClusterRole aggregation.

Reference:
  * pkg/controller/disruption/disruption.go — for every PodDisruptionBudget: expectedPods
    from the pods' controllers' scale (or the matching pod count), desiredHealthy from
    minAvailable / maxUnavailable (int or percent, rounded up), currentHealthy = ready
    matching pods not being deleted, disruptionsAllowed = max(currentHealthy -
    desiredHealthy, 0) minus pods evicted (status.disruptedPods) but not yet gone; entries
    older than 2 min expire.
  * pkg/controller/resourcequota/resource_quota_controller.go over amdkube.quota (the
    pkg/quota/evaluator/core evaluators): status.used for pods (compute, requests.*, limits.*,
    scopes), services (nodeports, loadbalancers), PVCs (storage, per StorageClass) and object
    counts; status.hard mirrors spec.hard. Extended resources (amd.com/gpu) count from the
    device-granular spec.extendedResources too.
  * pkg/controller/ttl/ttl_controller.go — node annotation node.alpha.kubernetes.io/ttl from
    cluster size (0 s up to 100 nodes, 15 ≤ 500, 30 ≤ 1000, 60 ≤ 2000, 300 ≤ 5000, else 600).
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

DISRUPTED_TIMEOUT = 120.0


def _int_or_percent(v, total: int, round_up: bool = True) -> int:
    if isinstance(v, str) and v.endswith("%"):
        f = float(v[:-1]) * total / 100.0
        return int(math.ceil(f) if round_up else math.floor(f))
    return int(v)


class DisruptionController(Controller):
    name = "disruption"

    def setup(self):
        f = self.mgr.factory
        self.pdb_inf = f.informer("poddisruptionbudgets")
        self.pod_inf = self.mgr.pods
        self.scale_infs = {k: f.informer(p) for k, p in (("ReplicaSet", "replicasets"), ("Deployment", "deployments"),
                                                          ("StatefulSet", "statefulsets"),
                                                          ("ReplicationController", "replicationcontrollers"))}
        self.pdb_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=lambda o: None)
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)

    def _pod(self, pod):
        labels = m.labels_of(pod)
        for pdb in self.pdb_inf.list():
            if m.namespace_of(pdb) == m.namespace_of(pod) and self._selects(pdb, labels):
                self.enqueue(pdb)

    @staticmethod
    def _selects(pdb, labels) -> bool:
        sel = (pdb.get("spec") or {}).get("selector")
        return bool(sel) and selector_from_label_selector(sel).matches(labels)

    def _expected(self, pods) -> int:
        """getExpectedScale: the sum of the controllers' replicas (a Deployment owns through its RS)."""
        seen, total = set(), 0
        for p in pods:
            ref = m.controller_ref(p)
            if not ref:
                return -1
            key = (ref.get("kind"), m.namespace_of(p), ref.get("name"))
            if key in seen:
                continue
            seen.add(key)
            inf = self.scale_infs.get(ref.get("kind"))
            owner = inf.get(f"{m.namespace_of(p)}/{ref.get('name')}") if inf else None
            if owner is None:
                return -1
            dref = m.controller_ref(owner) if ref.get("kind") == "ReplicaSet" else None
            if dref and dref.get("kind") == "Deployment":
                d = self.scale_infs["Deployment"].get(f"{m.namespace_of(p)}/{dref.get('name')}")
                if d is not None and ("Deployment", m.namespace_of(p), dref.get("name")) not in seen:
                    seen.add(("Deployment", m.namespace_of(p), dref.get("name")))
                    total += int((d.get("spec") or {}).get("replicas", 1))
                continue
            total += int((owner.get("spec") or {}).get("replicas", 1))
        return total

    async def sync(self, key):
        pdb = self.pdb_inf.get(key)
        if pdb is None:
            return
        ns, name = split_key(key)
        spec, old = pdb.get("spec") or {}, pdb.get("status") or {}
        pods = [p for p in self.pod_inf.list() if m.namespace_of(p) == ns and self._selects(pdb, m.labels_of(p))]
        healthy = sum(1 for p in pods if is_pod_ready(p) and not (p.get("metadata") or {}).get("deletionTimestamp")
                      and not is_pod_terminal(p))
        if "maxUnavailable" in spec:
            expected = self._expected(pods)
            if expected < 0:
                expected = len(pods)
            desired = max(0, expected - _int_or_percent(spec["maxUnavailable"], expected))
        else:
            mina = spec.get("minAvailable", 1)
            if isinstance(mina, str) and mina.endswith("%"):
                expected = self._expected(pods)
                if expected < 0:
                    expected = len(pods)
                desired = _int_or_percent(mina, expected)
            else:
                expected, desired = len(pods), int(mina)
        now = time.time()
        live = {m.name_of(p) for p in pods if not (p.get("metadata") or {}).get("deletionTimestamp")}
        disrupted = {k: v for k, v in (old.get("disruptedPods") or {}).items()
                     if k in live and now - (m.parse_time(v) or 0) < DISRUPTED_TIMEOUT}
        allowed = max(0, healthy - desired - len(disrupted))
        st = {"currentHealthy": healthy, "desiredHealthy": desired, "expectedPods": expected, "disruptionsAllowed": allowed,
              "disruptedPods": disrupted, "observedGeneration": (pdb.get("metadata") or {}).get("generation", 1)}
        if {k: old.get(k) for k in st} != st:
            body = dict(pdb, status=st)
            try:
                await self.client.update(body, sub="status")   # CAS on resourceVersion vs concurrent evictions
            except m.StatusError as e:
                if not m.is_conflict(e):
                    raise
                self.enqueue(key)


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
            await self.client.patch("resourcequotas", name, {"status": st}, ns, sub="status")


# --------------------------------------------------------------------------- node TTL
TTL_ANNOTATION = "node.alpha.kubernetes.io/ttl"
TTL_BOUNDARIES = ((100, 0), (500, 15), (1000, 30), (2000, 60), (5000, 300))


def ttl_for(nodes: int) -> int:
    for limit, ttl in TTL_BOUNDARIES:
        if nodes <= limit:
            return ttl
    return 600


class TTLController(Controller):
    name = "ttl"
    workers = 1

    def setup(self):
        self.node_inf = self.mgr.nodes
        self.node_inf.add_handler(on_add=lambda n: self._all(), on_update=lambda o, n: self.enqueue(n),
                                  on_delete=lambda n: self._all())

    def _all(self):
        for n in self.node_inf.list():
            self.enqueue(n)

    async def sync(self, key):
        _, name = split_key(key)
        node = self.node_inf.get(name)
        if node is None:
            return
        want = str(ttl_for(len(self.node_inf.list())))
        if m.annotations_of(node).get(TTL_ANNOTATION) != want:
            await self.client.patch("nodes", name, {"metadata": {"annotations": {TTL_ANNOTATION: want}}})


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
