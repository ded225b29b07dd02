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


REVISION = "deployment.kubernetes.io/revision"
DESIRED = "deployment.kubernetes.io/desired-replicas"
MAX_REPLICAS = "deployment.kubernetes.io/max-replicas"
HASH_LABEL = "pod-template-hash"
REVISION_HASH_LABEL = "controller-revision-hash"          # DaemonSet and StatefulSet pods / ControllerRevisions
TEMPLATE_GEN_LABEL = "pod-template-generation"


def _int_or_percent(v, total: int, round_up: bool) -> int:
    if isinstance(v, str) and v.endswith("%"):
        f = float(v[:-1]) * total / 100.0
        return int(math.ceil(f) if round_up else math.floor(f))
    return int(v)


def resolve_fenceposts(d: dict) -> tuple[int, int]:
    """(maxSurge, maxUnavailable) for a RollingUpdate deployment (deployment_util.go:959
    ResolveFenceposts): surge rounds up, unavailable rounds down, and both 0 means 1 unavailable."""
    spec = d.get("spec") or {}
    want = int(spec.get("replicas", 1))
    ru = (spec.get("strategy") or {}).get("rollingUpdate") or {}
    surge = _int_or_percent(ru.get("maxSurge", "25%"), want, True)
    unavail = _int_or_percent(ru.get("maxUnavailable", "25%"), want, False)
    if surge == 0 and unavail == 0:
        unavail = 1
    return surge, unavail


def _rev(rs) -> int:
    try:
        return int(((rs.get("metadata") or {}).get("annotations") or {}).get(REVISION, "0"))
    except ValueError:
        return 0


def _reps(rs) -> int:
    return int((rs.get("spec") or {}).get("replicas", 0))


def _st(rs, k) -> int:
    return int((rs.get("status") or {}).get(k, 0))


def _copyable(d: dict) -> dict:
    """Deployment annotations that follow it onto its ReplicaSets (deployment_util.go
    skipCopyAnnotation): everything but last-applied and the controller's own keys."""
    skip = {"kubectl.kubernetes.io/last-applied-configuration", REVISION, DESIRED, MAX_REPLICAS,
            "deployment.kubernetes.io/revision-history"}
    return {k: v for k, v in ((d.get("metadata") or {}).get("annotations") or {}).items() if k not in skip}


def _strip_hash(tpl: dict) -> dict:
    t = json.loads(json.dumps(tpl or {}))
    (t.get("metadata") or {}).get("labels", {}).pop(HASH_LABEL, None)
    return t


class DeploymentController(Controller):
    """pkg/controller/deployment: one ReplicaSet per template (pod-template-hash), revision
    annotations (max + 1 on every new or re-adopted template, deployment_util.go:50-60),
    RollingUpdate with maxSurge/maxUnavailable (rolling.go:31-235: scale the new RS up to
    replicas + surge, scale old RSs down while availability stays ≥ replicas − maxUnavailable,
    unhealthy old replicas first), Recreate (recreate.go: old to zero, wait for their pods,
    then new), paused deployments only scale (sync.go:40), spec.rollbackTo (rollback.go:31-117),
    revisionHistoryLimit cleanup, and the Available / Progressing conditions with
    progressDeadlineSeconds (progress.go)."""
    name = "deployment"

    def __init__(self, mgr, clock=time.time):
        super().__init__(mgr)
        self.clock = clock

    def setup(self):
        f = self.mgr.factory
        self.d_inf = f.informer("deployments")
        self.rs_inf = f.informer("replicasets")
        self.pod_inf = self.mgr.pods
        self.d_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.rs_inf.add_handler(on_add=self._rs, on_update=lambda o, n: self._rs(n), on_delete=self._rs)
        self.pod_inf.add_handler(on_delete=self._pod)

    def _rs(self, rs):
        ref = m.controller_ref(rs)
        if ref and ref.get("kind") == "Deployment":
            self.enqueue(f"{m.namespace_of(rs)}/{ref['name']}")

    def _pod(self, pod):   # Recreate waits for old pods to be gone
        ref = m.controller_ref(pod)
        if ref and ref.get("kind") == "ReplicaSet":
            rs = self.rs_inf.get(f"{m.namespace_of(pod)}/{ref['name']}")
            if rs is not None:
                self._rs(rs)

    def _event(self, d, etype, reason, msg):
        rec = getattr(self.mgr, "recorder", None)
        if rec is not None:
            rec.event(d, etype, reason, msg)

    async def _scale(self, d, rs, n: int):
        if _reps(rs) == n:
            return rs
        ann = {DESIRED: str(int((d.get("spec") or {}).get("replicas", 1))),
               MAX_REPLICAS: str(int((d.get("spec") or {}).get("replicas", 1)) + self._surge(d))}
        rs = await self.client.patch("replicasets", m.name_of(rs), {"metadata": {"annotations": ann}, "spec": {"replicas": n}},
                                     m.namespace_of(rs))
        self._event(d, "Normal", "ScalingReplicaSet",
                    f"Scaled {'up' if n > _reps(rs) else 'down'} replica set {m.name_of(rs)} to {n}")
        return rs

    @staticmethod
    def _surge(d) -> int:
        if ((d.get("spec") or {}).get("strategy") or {}).get("type") == "Recreate":
            return 0
        return resolve_fenceposts(d)[0]

    async def sync(self, key):
        d = self.d_inf.get(key)
        if d is None or (d.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        spec = d.get("spec") or {}
        rss = _owned(self.rs_inf.list(), d)
        if spec.get("rollbackTo") is not None:
            await self._rollback(d, rss)
            return
        want = int(spec.get("replicas", 1))
        h = template_hash(spec.get("template") or {})
        new = next((r for r in rss if m.labels_of(r).get(HASH_LABEL) == h), None)
        olds = sorted([r for r in rss if r is not new], key=lambda r: (r.get("metadata") or {}).get("creationTimestamp", ""))
        max_rev = max((_rev(r) for r in olds), default=0)
        recreate = (spec.get("strategy") or {}).get("type") == "Recreate"
        if spec.get("paused"):
            # a paused deployment only scales (proportionally is not needed with one active RS)
            if new is not None and _reps(new) != want and not any(_reps(r) for r in olds):
                await self._scale(d, new, want)
            await self._status(d, new, rss, paused=True)
            return
        if new is None:
            tpl = json.loads(json.dumps(spec.get("template") or {}))
            tpl.setdefault("metadata", {}).setdefault("labels", {})[HASH_LABEL] = h
            sel = json.loads(json.dumps(spec.get("selector") or {}))
            sel.setdefault("matchLabels", {})[HASH_LABEL] = h
            surge = self._surge(d)
            if recreate:
                start = 0
            else:
                start = max(0, min(want, want + surge - sum(_reps(r) for r in olds)))
            rs = {"apiVersion": "apps/v1", "kind": "ReplicaSet",
                  "metadata": {"name": f"{name}-{h}", "namespace": ns, "labels": {**(tpl["metadata"]["labels"])},
                               "annotations": {**_copyable(d), REVISION: str(max_rev + 1), DESIRED: str(want),
                                               MAX_REPLICAS: str(want + surge)},
                               "ownerReferences": [m.new_controller_ref(d, "apps/v1", "Deployment")]},
                  "spec": {"replicas": start, "selector": sel, "template": tpl,
                           "minReadySeconds": int(spec.get("minReadySeconds", 0))}}
            new = await self.client.create(rs, ns)
            self._event(d, "Normal", "ScalingReplicaSet", f"Scaled up replica set {m.name_of(new)} to {start}")
        elif _rev(new) <= max_rev:
            # an old template came back (rollback or a revert): it becomes the newest revision
            new = await self.client.patch("replicasets", m.name_of(new),
                                          {"metadata": {"annotations": {**_copyable(d), REVISION: str(max_rev + 1)}}}, ns)
        if (d.get("metadata") or {}).get("annotations", {}).get(REVISION) != str(_rev(new)):
            await self.client.patch("deployments", name, {"metadata": {"annotations": {REVISION: str(_rev(new))}}}, ns)
        if recreate:
            await self._recreate(d, new, olds, want)
        else:
            await self._rolling(d, new, olds, want)
        rss = _owned(self.rs_inf.list(), d)
        await self._status(d, new, rss)
        await self._cleanup(d, new, olds)

    async def _recreate(self, d, new, olds, want):
        active = [r for r in olds if _reps(r)]
        for r in active:
            await self._scale(d, r, 0)
        uids = {m.uid_of(r) for r in olds}
        running = [p for p in self.pod_inf.list() if (m.controller_ref(p) or {}).get("uid") in uids and not is_pod_terminal(p)]
        if active or running:
            return
        await self._scale(d, new, want)

    async def _rolling(self, d, new, olds, want):
        surge, unavail = resolve_fenceposts(d)
        all_rs = [new] + olds
        total = sum(_reps(r) for r in all_rs)
        # reconcileNewReplicaSet
        if _reps(new) > want:
            new = await self._scale(d, new, want)
        elif _reps(new) < want:
            n = min(want, _reps(new) + max(0, want + surge - total))
            if n != _reps(new):
                new = await self._scale(d, new, n)
        # reconcileOldReplicaSets
        total = sum(_reps(r) for r in [new] + olds)
        old_count = sum(_reps(r) for r in olds)
        if not old_count:
            return
        min_avail = want - unavail
        new_unavail = _reps(new) - _st(new, "availableReplicas")
        budget = total - min_avail - new_unavail
        if budget <= 0:
            return
        for r in olds:   # cleanupUnhealthyReplicas: oldest first
            if budget <= 0:
                break
            unhealthy = _reps(r) - _st(r, "availableReplicas")
            k = min(unhealthy, budget)
            if k > 0:
                await self._scale(d, r, _reps(r) - k)
                r.setdefault("spec", {})["replicas"] = _reps(r) - k
                budget -= k
        # scaleDownOldReplicaSetsForRollingUpdate: keep total availability ≥ min_avail
        avail = sum(_st(r, "availableReplicas") for r in [new] + olds)
        can = avail - min_avail
        for r in olds:
            if can <= 0:
                break
            k = min(_reps(r), can)
            if k > 0:
                await self._scale(d, r, _reps(r) - k)
                can -= k

    async def _rollback(self, d, rss):
        ns, name = m.namespace_of(d), m.name_of(d)
        to = int(((d.get("spec") or {}).get("rollbackTo") or {}).get("revision", 0))
        revs = sorted((_rev(r), r) for r in rss)
        if to == 0:
            to = revs[-2][0] if len(revs) >= 2 else 0   # LastRevision: the one before the current
        target = next((r for v, r in revs if v == to and to), None)
        patch = {"spec": {"rollbackTo": None}}
        if target is None:
            self._event(d, "Warning", "DeploymentRollbackRevisionNotFound", "Unable to find the revision to rollback to.")
        elif _strip_hash((target.get("spec") or {}).get("template")) == _strip_hash((d.get("spec") or {}).get("template")):
            self._event(d, "Warning", "DeploymentRollbackTemplateUnchanged",
                        f"The rollback revision contains the same template as current deployment {name!r}")
        else:
            patch["spec"]["template"] = _strip_hash((target.get("spec") or {}).get("template"))
            self._event(d, "Normal", "DeploymentRollback", f"Rolled back deployment {name!r} to revision {to}")
        await self.client.patch("deployments", name, patch, ns)

    async def _cleanup(self, d, new, olds):
        limit = (d.get("spec") or {}).get("revisionHistoryLimit", 10)
        dead = [r for r in olds if _reps(r) == 0 and _st(r, "replicas") == 0]
        dead.sort(key=_rev)
        for r in dead[:max(0, len(dead) - int(limit))]:
            try:
                await self.client.delete("replicasets", m.name_of(r), m.namespace_of(r))
            except m.StatusError:
                pass

    async def _status(self, d, new, rss, paused=False):
        ns, name = m.namespace_of(d), m.name_of(d)
        spec = d.get("spec") or {}
        want = int(spec.get("replicas", 1))
        unavail = resolve_fenceposts(d)[1] if (spec.get("strategy") or {}).get("type") != "Recreate" else 0
        avail = sum(_st(r, "availableReplicas") for r in rss)
        updated = _st(new, "replicas") if new is not None else 0
        total = sum(_st(r, "replicas") for r in rss)
        st = {"replicas": total, "updatedReplicas": updated,
              "readyReplicas": sum(_st(r, "readyReplicas") for r in rss), "availableReplicas": avail,
              "unavailableReplicas": max(0, total - avail) if total >= want else max(0, want - avail),
              "observedGeneration": (d.get("metadata") or {}).get("generation", 1)}
        now = m.format_time(self.clock())
        old = {c["type"]: c for c in (d.get("status") or {}).get("conditions") or []}

        def cond(typ, status, reason, msg):
            prev = old.get(typ)
            if prev and prev.get("status") == status and prev.get("reason") == reason:
                return prev
            return {"type": typ, "status": status, "reason": reason, "message": msg, "lastUpdateTime": now,
                    "lastTransitionTime": prev["lastTransitionTime"] if prev and prev.get("status") == status else now}

        conds = [cond("Available", "True" if avail >= want - unavail else "False",
                      "MinimumReplicasAvailable" if avail >= want - unavail else "MinimumReplicasUnavailable",
                      "Deployment has minimum availability." if avail >= want - unavail
                      else "Deployment does not have minimum availability.")]
        complete = new is not None and updated == want and avail >= want and total == want
        rs_name = m.name_of(new) if new is not None else ""
        if paused:
            conds.append(cond("Progressing", "Unknown", "DeploymentPaused", "Deployment is paused"))
        elif complete:
            conds.append(cond("Progressing", "True", "NewReplicaSetAvailable", f'ReplicaSet "{rs_name}" has successfully progressed.'))
        else:
            prev = old.get("Progressing")
            deadline = spec.get("progressDeadlineSeconds", 600)
            changed = {k: (d.get("status") or {}).get(k) for k in st} != st
            if prev and prev.get("reason") == "ProgressDeadlineExceeded":
                conds.append(prev)
            elif (deadline is not None and prev is not None and not changed and prev.get("status") == "True" and
                    self.clock() - (m.parse_time(prev.get("lastUpdateTime")) or self.clock()) > int(deadline)):
                conds.append(cond("Progressing", "False", "ProgressDeadlineExceeded",
                                  f'ReplicaSet "{rs_name}" has timed out progressing.'))
                self._event(d, "Warning", "ProgressDeadlineExceeded", f"Deployment {name!r} has timed out progressing.")
            else:
                c = {"type": "Progressing", "status": "True", "reason": "ReplicaSetUpdated",
                     "message": f'ReplicaSet "{rs_name}" is progressing.', "lastUpdateTime": now,
                     "lastTransitionTime": prev["lastTransitionTime"] if prev and prev.get("status") == "True" else now}
                if prev and prev.get("reason") == "ReplicaSetUpdated" and not changed:
                    c = prev   # no progress since the last sync: keep lastUpdateTime for the deadline
                conds.append(c)
                if deadline is not None:
                    self.queue.add_after(m.key_of(d), float(deadline) + 1.0)
        st["conditions"] = conds
        if {k: (d.get("status") or {}).get(k) for k in st} != st:
            await self.client.patch("deployments", name, {"status": st}, ns, sub="status")


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
