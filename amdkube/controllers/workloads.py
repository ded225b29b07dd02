"""Workload controllers: ReplicaSet, Deployment, DaemonSet, Job.

Reference: pkg/controller/replicaset (manage replicas via controllerRef + expectations),
pkg/controller/deployment (ReplicaSets per pod-template-hash; Recreate / RollingUpdate),
pkg/controller/daemon (one pod per eligible node — how the AMD device plugin is rolled
out, deploy/amd-gpu-device-plugin.yaml). The Job controller is in controllers/job.py.
"""
from __future__ import annotations

import hashlib
import json
import math
import time

from ..api import meta as m
from ..api.helpers import find_untolerated_taint, get_condition, is_pod_ready, is_pod_terminal
from ..api.labels import node_requirements_as_selector
from .base import Controller, split_key


def _owned(pods, owner):
    uid = m.uid_of(owner)
    return [p for p in pods if (m.controller_ref(p) or {}).get("uid") == uid]


def _pod_from_template(owner, api_version, kind, extra_labels=None, node=None):
    tpl = json.loads(json.dumps((owner.get("spec") or {}).get("template") or {}))
    md = tpl.get("metadata") or {}
    labels = dict(md.get("labels") or {})
    labels.update(extra_labels or {})
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"generateName": m.name_of(owner) + "-", "namespace": m.namespace_of(owner), "labels": labels,
                        "annotations": dict(md.get("annotations") or {}),
                        "ownerReferences": [m.new_controller_ref(owner, api_version, kind)]},
           "spec": tpl.get("spec") or {}}
    if node:
        pod["spec"]["nodeName"] = node
    return pod


from .replicaset import ReplicaSetController  # noqa: E402,F401  (controllers/replicaset.py)


def template_hash(tpl) -> str:
    return hashlib.sha1(json.dumps(tpl, sort_keys=True).encode()).hexdigest()[:10]


REVISION_HASH_LABEL = "controller-revision-hash"          # DaemonSet and StatefulSet pods / ControllerRevisions
TEMPLATE_GEN_LABEL = "pod-template-generation"


def _int_or_percent(v, total: int, round_up: bool) -> int:
    if isinstance(v, str) and v.endswith("%"):
        f = float(v[:-1]) * total / 100.0
        return int(math.ceil(f) if round_up else math.floor(f))
    return int(v)


from .deployment import DeploymentController  # noqa: E402,F401  (controllers/deployment.py)


class DaemonSetController(Controller):
    """One pod per eligible node (pkg/controller/daemon/daemon_controller.go) with the update
    strategies of update.go:
      * every template is recorded as a ControllerRevision `<ds>-<hash>` labelled
        controller-revision-hash (constructHistory); its `revision` is one past the highest
        when the template is new or comes back (a rollback), and revisions beyond
        spec.revisionHistoryLimit (10) that no pod uses are removed (cleanupHistory);
      * pods carry controller-revision-hash and pod-template-generation;
      * RollingUpdate (the apps/v1 default): old pods that are not available go at once, then
        available old pods while fewer than maxUnavailable (int or % of desired, rounded up;
        default 1) are unavailable; a node whose pod went gets a pod of the new template on
        the next pass (rollingUpdate :44-80, getUnavailableNumbers);
      * OnDelete: old pods stay until deleted by hand.
    Status adds updatedNumberScheduled, numberAvailable and numberUnavailable."""
    name = "daemonset"
    HISTORY_LIMIT = 10

    def setup(self):
        f = self.mgr.factory
        self.ds_inf = f.informer("daemonsets")
        self.node_inf = self.mgr.nodes
        self.pod_inf = self.mgr.pods
        self.ds_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.node_inf.add_handler(on_add=lambda n: self._all(), on_update=lambda o, n: self._all(), on_delete=lambda n: self._all())
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)
        self._recorded: dict[str, str] = {}       # ds uid -> template hash already recorded as the newest revision

    def _all(self):
        for ds in self.ds_inf.list():
            self.enqueue(ds)

    def _pod(self, pod):
        ref = m.controller_ref(pod)
        if ref and ref.get("kind") == "DaemonSet":
            self.enqueue(f"{m.namespace_of(pod)}/{ref['name']}")

    @staticmethod
    def should_run(ds, node) -> bool:
        spec = ((ds.get("spec") or {}).get("template") or {}).get("spec") or {}
        labels = m.labels_of(node)
        for k, v in (spec.get("nodeSelector") or {}).items():
            if labels.get(k) != v:
                return False
        terms = ((((spec.get("affinity") or {}).get("nodeAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or {})
                 .get("nodeSelectorTerms") or [])
        if terms and not any(node_requirements_as_selector(t.get("matchExpressions")).matches(labels) for t in terms):
            return False
        return find_untolerated_taint((node.get("spec") or {}).get("taints"), spec.get("tolerations"),
                                      ("NoSchedule", "NoExecute")) is None

    async def _history(self, ds, live_hashes: set[str]) -> str:
        """Record the current template as the newest ControllerRevision; returns its hash."""
        tpl = (ds.get("spec") or {}).get("template") or {}
        h = template_hash(tpl)
        uid = m.uid_of(ds)
        if self._recorded.get(uid) == h:
            return h
        ns, name = m.namespace_of(ds), m.name_of(ds)
        revs = [r for r in (await self.client.list("controllerrevisions.apps", ns))[0] if (m.controller_ref(r) or {}).get("uid") == uid]
        top = max((int(r.get("revision", 0)) for r in revs), default=0)
        mine = next((r for r in revs if m.labels_of(r).get(REVISION_HASH_LABEL) == h), None)
        if mine is None:
            try:
                await self.client.create({"apiVersion": "apps/v1", "kind": "ControllerRevision",
                                          "metadata": {"name": f"{name}-{h}", "namespace": ns,
                                                       "labels": dict((tpl.get("metadata") or {}).get("labels") or {},
                                                                      **{REVISION_HASH_LABEL: h}),
                                                       "annotations": {k: v for k, v in (m.annotations_of(ds) or {}).items()
                                                                       if k == "kubernetes.io/change-cause"},
                                                       "ownerReferences": [m.new_controller_ref(ds, "apps/v1", "DaemonSet")]},
                                          "data": {"spec": {"template": tpl}}, "revision": top + 1}, ns)
            except m.StatusError as e:
                if not m.is_already_exists(e):
                    raise
        elif int(mine.get("revision", 0)) < top:          # a template that comes back (rollback) is newest again
            mine = dict(mine, apiVersion="apps/v1", kind="ControllerRevision", revision=top + 1)
            await self.client.update(mine)
        limit = int((ds.get("spec") or {}).get("revisionHistoryLimit", self.HISTORY_LIMIT))
        old = sorted((r for r in revs if m.labels_of(r).get(REVISION_HASH_LABEL) not in live_hashes | {h}),
                     key=lambda r: int(r.get("revision", 0)))
        for r in old[:max(0, len(old) - limit)]:
            try:
                await self.client.delete("controllerrevisions.apps", m.name_of(r), ns)
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise
        self._recorded[uid] = h
        return h

    @staticmethod
    def _available(p, mrs: int, now: float) -> tuple[bool, float | None]:
        if not is_pod_ready(p):
            return False, None
        since = m.parse_time((get_condition(p, "Ready") or {}).get("lastTransitionTime")) or 0.0
        if mrs == 0 or since + mrs <= now:
            return True, None
        return False, since + mrs - now

    async def sync(self, key):
        ds = self.ds_inf.get(key)
        if ds is None or (ds.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        spec = ds.get("spec") or {}
        all_pods = _owned(self.pod_inf.list(), ds)
        pods = [p for p in all_pods if not (p.get("metadata") or {}).get("deletionTimestamp")]
        h = await self._history(ds, {m.labels_of(p).get(REVISION_HASH_LABEL) for p in all_pods})
        gen = str((ds.get("metadata") or {}).get("generation", 1))
        by_node: dict[str, list] = {}
        for p in pods:
            by_node.setdefault((p.get("spec") or {}).get("nodeName", ""), []).append(p)
        mrs = int(spec.get("minReadySeconds", 0))
        now, wake = time.time(), None
        desired = current = ready = updated = available = misscheduled = 0
        old_avail, old_unavail = [], []
        for node in self.node_inf.list():
            nn = m.name_of(node)
            run = self.should_run(ds, node)
            have = [p for p in by_node.get(nn, []) if not is_pod_terminal(p)]
            if run:
                desired += 1
                if not have:
                    await self.client.create(_pod_from_template(ds, "apps/v1", "DaemonSet", node=nn,
                                                                extra_labels={REVISION_HASH_LABEL: h, TEMPLATE_GEN_LABEL: gen}), ns)
                else:
                    current += 1
                    p = have[0]
                    ready += int(is_pod_ready(p))
                    ok, w = self._available(p, mrs, now)
                    available += int(ok)
                    if w is not None:
                        wake = min(wake or 1e18, w)
                    if m.labels_of(p).get(REVISION_HASH_LABEL) == h:
                        updated += 1
                    else:
                        (old_avail if ok else old_unavail).append(p)
                    for extra in have[1:]:
                        await self.client.delete("pods", m.name_of(extra), ns)
            else:
                misscheduled += int(bool(have))
                for p in have:
                    await self.client.delete("pods", m.name_of(p), ns)
            for p in by_node.get(nn, []):
                if is_pod_terminal(p) and run:
                    await self.client.delete("pods", m.name_of(p), ns, grace=0)
        strategy = spec.get("updateStrategy") or {}
        if strategy.get("type", "RollingUpdate") == "RollingUpdate" and (old_avail or old_unavail):
            max_unavail = _int_or_percent((strategy.get("rollingUpdate") or {}).get("maxUnavailable", 1), desired, True)
            unavailable = desired - available
            victims = list(old_unavail)
            for p in old_avail:
                if unavailable >= max_unavail:
                    break
                victims.append(p)
                unavailable += 1
            for p in victims:
                try:
                    await self.client.delete("pods", m.name_of(p), ns)
                except m.StatusError as e:
                    if not m.is_not_found(e):
                        raise
        if wake is not None:
            self.queue.add_after(key, wake + 0.05)
        st = {"desiredNumberScheduled": desired, "currentNumberScheduled": current, "numberReady": ready,
              "numberMisscheduled": misscheduled, "updatedNumberScheduled": updated, "numberAvailable": available,
              "numberUnavailable": desired - available,
              "observedGeneration": (ds.get("metadata") or {}).get("generation", 1)}
        if {k: (ds.get("status") or {}).get(k) for k in st} != st:
            await self.client.patch("daemonsets", name, {"status": st}, ns, sub="status")


from .job import JobController  # noqa: E402,F401  (moved to controllers/job.py)
