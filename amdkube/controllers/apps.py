"""ReplicationController, StatefulSet and CronJob controllers.

Reference:
  * pkg/controller/replication — the ReplicaSet logic over a v1 map selector.
  * pkg/controller/statefulset/stateful_set_control.go (1.9, apps/v1 defaults) — pods
    `<set>-<ordinal>` with hostname/subdomain from spec.serviceName; volumeClaimTemplates
    become PVCs `<claim>-<set>-<ordinal>` created before their pod; OrderedReady creates
    ordinal i only when 0..i-1 are Running and Ready and scales down from the highest
    ordinal, one pod at a time; Parallel does not wait; failed pods are replaced;
    RollingUpdate (default) replaces pods whose controller-revision-hash differs from the
    update revision from the highest ordinal down to spec.updateStrategy.rollingUpdate
    .partition, one at a time, once the set is ready; ControllerRevisions record templates.
  * pkg/controller/cronjob/{cronjob_controller.go, utils.go} — polled every 10 s;
    getRecentUnmetScheduleTimes since lastScheduleTime (or creation), >100 misses is an
    error; startingDeadlineSeconds drops too-late starts; concurrencyPolicy Allow / Forbid
    / Replace; suspend; job name `<cronjob>-<hash of the scheduled time>`
    (getTimeHash = unix minutes); status.active / lastScheduleTime; finished jobs beyond
    successfulJobsHistoryLimit (3) / failedJobsHistoryLimit (1) are deleted.
"""
from __future__ import annotations

import asyncio
import calendar
import json
import time

from ..api import meta as m
from ..api.helpers import is_pod_ready, is_pod_terminal
from ..api.labels import selector_from_set
from .base import Controller, split_key
from .workloads import ReplicaSetController, _owned, template_hash

REVISION_LABEL = "controller-revision-hash"
POD_NAME_LABEL = "statefulset.kubernetes.io/pod-name"


class ReplicationManager(ReplicaSetController):
    """pkg/controller/replication: the ReplicaSet controller over a v1 map selector."""
    name = "replicationcontroller"
    owner_api, owner_kind, plural = "v1", "ReplicationController", "replicationcontrollers"

    def selector_of(self, rc):
        return selector_from_set((rc.get("spec") or {}).get("selector") or {})


# ============================================================================ StatefulSet
def _running_ready(p) -> bool:
    return (p.get("status") or {}).get("phase") == "Running" and is_pod_ready(p)


class StatefulSetController(Controller):
    name = "statefulset"

    def setup(self):
        f = self.mgr.factory
        self.sts_inf = f.informer("statefulsets")
        self.pvc_inf = f.informer("persistentvolumeclaims")
        self.pod_inf = self.mgr.pods
        self.sts_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.pod_inf.add_handler(on_add=self._pod, on_update=lambda o, n: self._pod(n), on_delete=self._pod)

    def _pod(self, pod):
        ref = m.controller_ref(pod)
        if ref and ref.get("kind") == "StatefulSet":
            self.enqueue(f"{m.namespace_of(pod)}/{ref['name']}")

    @staticmethod
    def ordinal(set_name: str, pod: dict) -> int:
        n = m.name_of(pod)
        pre, _, o = n.rpartition("-")
        return int(o) if pre == set_name and o.isdigit() else -1

    def new_pod(self, sts, ordinal, revision):
        name = m.name_of(sts)
        tpl = json.loads(json.dumps((sts.get("spec") or {}).get("template") or {}))
        md = tpl.get("metadata") or {}
        pname = f"{name}-{ordinal}"
        labels = dict(md.get("labels") or {})
        labels.update({POD_NAME_LABEL: pname, REVISION_LABEL: revision})
        spec = tpl.get("spec") or {}
        spec["hostname"] = pname
        if (sts.get("spec") or {}).get("serviceName"):
            spec["subdomain"] = sts["spec"]["serviceName"]
        vols = [v for v in spec.get("volumes") or []]
        for ct in (sts.get("spec") or {}).get("volumeClaimTemplates") or []:
            cname = m.name_of(ct)
            vols = [v for v in vols if v.get("name") != cname]
            vols.append({"name": cname, "persistentVolumeClaim": {"claimName": f"{cname}-{pname}"}})
        if vols:
            spec["volumes"] = vols
        return {"apiVersion": "v1", "kind": "Pod",
                "metadata": {"name": pname, "namespace": m.namespace_of(sts), "labels": labels,
                             "annotations": dict(md.get("annotations") or {}),
                             "ownerReferences": [m.new_controller_ref(sts, "apps/v1", "StatefulSet")]},
                "spec": spec}

    async def _ensure_claims(self, sts, ordinal):
        ns, name = m.namespace_of(sts), m.name_of(sts)
        for ct in (sts.get("spec") or {}).get("volumeClaimTemplates") or []:
            cname = f"{m.name_of(ct)}-{name}-{ordinal}"
            if self.pvc_inf.get(f"{ns}/{cname}") is not None:
                continue
            labels = dict(((sts.get("spec") or {}).get("selector") or {}).get("matchLabels") or {})
            pvc = {"apiVersion": "v1", "kind": "PersistentVolumeClaim",
                   "metadata": {"name": cname, "namespace": ns, "labels": labels},
                   "spec": json.loads(json.dumps(ct.get("spec") or {}))}
            try:
                await self.client.create(pvc, ns)
            except m.StatusError as e:
                if not m.is_already_exists(e):
                    raise

    async def _revision(self, sts) -> str:
        """Record the template as the newest ControllerRevision (history.go) and return its hash:
        a new template gets one past the highest revision, a template that comes back (a
        rollback) has its old revision renumbered to the newest."""
        tpl = (sts.get("spec") or {}).get("template") or {}
        h = template_hash(tpl)
        uid = m.uid_of(sts)
        cache = self.__dict__.setdefault("_recorded", {})
        if cache.get(uid) == h:
            return h
        ns, name = m.namespace_of(sts), m.name_of(sts)
        revs = [r for r in (await self.client.list("controllerrevisions.apps", ns))[0] if (m.controller_ref(r) or {}).get("uid") == uid]
        top = max((int(r.get("revision", 0)) for r in revs), default=0)
        mine = next((r for r in revs if m.labels_of(r).get(REVISION_LABEL) == h), None)
        if mine is None:
            try:
                await self.client.create({"apiVersion": "apps/v1", "kind": "ControllerRevision",
                                          "metadata": {"name": f"{name}-{h}", "namespace": ns,
                                                       "labels": dict(m.labels_of(sts), **{REVISION_LABEL: h}),
                                                       "ownerReferences": [m.new_controller_ref(sts, "apps/v1", "StatefulSet")]},
                                          "data": {"spec": {"template": tpl}}, "revision": top + 1}, ns)
            except m.StatusError as e:
                if not m.is_already_exists(e):
                    raise
        elif int(mine.get("revision", 0)) < top:
            await self.client.update(dict(mine, apiVersion="apps/v1", kind="ControllerRevision", revision=top + 1))
        cache[uid] = h
        return h

    async def sync(self, key):
        sts = self.sts_inf.get(key)
        if sts is None or (sts.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        spec = sts.get("spec") or {}
        replicas = int(spec.get("replicas", 1))
        parallel = spec.get("podManagementPolicy") == "Parallel"
        revision = await self._revision(sts)
        pods = {}
        for p in _owned(self.pod_inf.list(), sts):
            o = self.ordinal(name, p)
            if o >= 0:
                pods[o] = p
        # 1. replace failed pods, create missing ones (in order unless Parallel)
        for o in range(replicas):
            p = pods.get(o)
            if p is not None and (p.get("status") or {}).get("phase") == "Failed" and \
                    not (p.get("metadata") or {}).get("deletionTimestamp"):
                await self.client.delete("pods", m.name_of(p), ns, grace=0)
                return
            if p is None:
                await self._ensure_claims(sts, o)
                await self.client.create(self.new_pod(sts, o, revision), ns)
                if not parallel:
                    return
                continue
            if not parallel and not _running_ready(p):
                break  # OrderedReady: wait for this ordinal before touching the next one
        # 2. scale down from the highest ordinal, one at a time
        extra = sorted((o for o in pods if o >= replicas), reverse=True)
        if extra:
            if not parallel and not all(_running_ready(pods[o]) for o in pods if o < replicas):
                await self._status(sts, pods, revision)
                return
            for o in (extra if parallel else extra[:1]):
                if not (pods[o].get("metadata") or {}).get("deletionTimestamp"):
                    await self.client.delete("pods", m.name_of(pods[o]), ns)
        # 3. rolling update, highest ordinal first, down to the partition
        us = spec.get("updateStrategy") or {}
        if us.get("type", "RollingUpdate") == "RollingUpdate" and not extra:
            partition = int(((us.get("rollingUpdate") or {}).get("partition")) or 0)
            live = [pods[o] for o in range(replicas) if o in pods]
            if len(live) == replicas and all(_running_ready(p) for p in live):
                for o in range(replicas - 1, partition - 1, -1):
                    if m.labels_of(pods[o]).get(REVISION_LABEL) != revision:
                        await self.client.delete("pods", m.name_of(pods[o]), ns)
                        break
        await self._status(sts, pods, revision)

    async def _status(self, sts, pods, revision):
        ns, name = m.namespace_of(sts), m.name_of(sts)
        live = [p for p in pods.values() if not is_pod_terminal(p)]
        updated = sum(1 for p in live if m.labels_of(p).get(REVISION_LABEL) == revision)
        st = {"replicas": len(live), "readyReplicas": sum(1 for p in live if _running_ready(p)),
              "currentReplicas": len(live), "updatedReplicas": updated, "updateRevision": f"{name}-{revision}",
              "currentRevision": f"{name}-{revision}" if updated == len(live) else (sts.get("status") or {}).get("currentRevision", ""),
              "observedGeneration": (sts.get("metadata") or {}).get("generation", 1)}
        if {k: (sts.get("status") or {}).get(k) for k in st} != st:
            await self.client.patch("statefulsets", name, {"status": st}, ns, sub="status")


# ============================================================================== cron
_NAMES = {"jan": 1, "feb": 2, "mar": 3, "apr": 4, "may": 5, "jun": 6, "jul": 7, "aug": 8, "sep": 9, "oct": 10,
          "nov": 11, "dec": 12, "sun": 0, "mon": 1, "tue": 2, "wed": 3, "thu": 4, "fri": 5, "sat": 6}
_MACROS = {"@yearly": "0 0 1 1 *", "@annually": "0 0 1 1 *", "@monthly": "0 0 1 * *", "@weekly": "0 0 * * 0",
           "@daily": "0 0 * * *", "@midnight": "0 0 * * *", "@hourly": "0 * * * *"}


class CronSchedule:
    """Standard 5-field cron (robfig/cron as used by the reference), evaluated in UTC."""

    def __init__(self, expr: str):
        expr = expr.strip()
        self.every = None
        if expr.startswith("@every "):
            self.every = _duration(expr[7:])
            if self.every < 1:
                raise ValueError(f"invalid duration in {expr!r}")
            return
        expr = _MACROS.get(expr, expr)
        f = expr.split()
        if len(f) != 5:
            raise ValueError(f"expected exactly 5 fields, found {len(f)}: {expr!r}")
        self.minute = self._field(f[0], 0, 59)
        self.hour = self._field(f[1], 0, 23)
        self.dom = self._field(f[2], 1, 31)
        self.month = self._field(f[3], 1, 12)
        self.dow = {d % 7 for d in self._field(f[4], 0, 7)}
        self.dom_star, self.dow_star = f[2] in ("*", "?"), f[4] in ("*", "?")

    @staticmethod
    def _field(s, lo, hi) -> set:
        out = set()
        for part in s.lower().split(","):
            rng, _, step = part.partition("/")
            step = int(step) if step else 1
            if step < 1:
                raise ValueError(f"invalid step in {s!r}")
            if rng in ("*", "?"):
                a, b = lo, hi
            else:
                x, _, y = rng.partition("-")
                a = _NAMES.get(x, None) if not x.isdigit() else int(x)
                if a is None:
                    raise ValueError(f"invalid value {x!r} in {s!r}")
                b = (_NAMES.get(y) if not y.isdigit() else int(y)) if y else (hi if step > 1 else a)
                if b is None:
                    raise ValueError(f"invalid value {y!r} in {s!r}")
            if not (lo <= a <= hi and lo <= b <= hi and a <= b):
                raise ValueError(f"value out of range [{lo}, {hi}] in {s!r}")
            out.update(range(a, b + 1, step))
        return out

    def _day_ok(self, y, mo, d) -> bool:
        dow = (calendar.weekday(y, mo, d) + 1) % 7
        if self.dom_star or self.dow_star:
            return (self.dom_star or d in self.dom) and (self.dow_star or dow in self.dow)
        return d in self.dom or dow in self.dow  # both restricted: either matches (cron semantics)

    def next_after(self, t: float) -> float:
        """First activation strictly after t (UTC seconds)."""
        if self.every is not None:
            return t + self.every
        tm = time.gmtime(int(t) // 60 * 60 + 60)
        y, mo, d, h, mi = tm.tm_year, tm.tm_mon, tm.tm_mday, tm.tm_hour, tm.tm_min
        for _ in range(366 * 5):
            if mo in self.month and self._day_ok(y, mo, d):
                for hh in range(h, 24):
                    if hh not in self.hour:
                        continue
                    for mm in range(mi if hh == h else 0, 60):
                        if mm in self.minute:
                            return calendar.timegm((y, mo, d, hh, mm, 0))
            # next day
            h = mi = 0
            d += 1
            if d > calendar.monthrange(y, mo)[1]:
                d, mo = 1, mo + 1
                if mo > 12:
                    mo, y = 1, y + 1
        raise ValueError("schedule never fires")


def _duration(s: str) -> float:
    total, num = 0.0, ""
    units = {"h": 3600, "m": 60, "s": 1, "ms": 0.001}
    i = 0
    while i < len(s):
        c = s[i]
        if c.isdigit() or c == ".":
            num += c
            i += 1
            continue
        u = "ms" if s[i:i + 2] == "ms" else c
        if u not in units or not num:
            raise ValueError(f"invalid duration {s!r}")
        total += float(num) * units[u]
        num = ""
        i += len(u)
    if num:
        raise ValueError(f"missing unit in duration {s!r}")
    return total


def unmet_schedule_times(sched: CronSchedule, earliest: float, now: float, limit: int = 100) -> list[float]:
    out = []
    t = sched.next_after(earliest)
    while t <= now:
        out.append(t)
        if len(out) > limit:
            raise RuntimeError("too many missed start times (> 100); check clock skew or set startingDeadlineSeconds")
        t = sched.next_after(t)
    return out


class CronJobController(Controller):
    name = "cronjob"
    workers = 1
    period = 10.0            # cronjob_controller.go: wait.Until(syncAll, 10s)

    def __init__(self, mgr, clock=time.time):
        super().__init__(mgr)
        self.clock = clock
        self._poll = None

    def setup(self):
        f = self.mgr.factory
        self.cj_inf = f.informer("cronjobs")
        self.job_inf = f.informer("jobs")
        self.cj_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))
        self.job_inf.add_handler(on_update=lambda o, n: self._job(n), on_delete=self._job)

    def _job(self, job):
        ref = m.controller_ref(job)
        if ref and ref.get("kind") == "CronJob":
            self.enqueue(f"{m.namespace_of(job)}/{ref['name']}")

    async def start(self):
        await super().start()
        self._poll = asyncio.create_task(self._poll_loop(), name="cronjob-poll")

    async def stop(self):
        if self._poll:
            self._poll.cancel()
        await super().stop()

    async def _poll_loop(self):
        while True:
            await asyncio.sleep(self.period)
            for cj in self.cj_inf.list():
                self.enqueue(cj)

    async def sync(self, key):
        cj = self.cj_inf.get(key)
        if cj is None or (cj.get("metadata") or {}).get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        spec, st = cj.get("spec") or {}, dict(cj.get("status") or {})
        jobs = [j for j in self.job_inf.list() if (m.controller_ref(j) or {}).get("uid") == m.uid_of(cj)]

        def finished(j):
            for c in (j.get("status") or {}).get("conditions") or []:
                if c.get("type") in ("Complete", "Failed") and c.get("status") == "True":
                    return c["type"]
            return None
        active = [j for j in jobs if not finished(j)]
        active_refs = [{"kind": "Job", "namespace": ns, "name": m.name_of(j), "uid": m.uid_of(j), "apiVersion": "batch/v1"}
                       for j in active]
        # history limits (cleanupFinishedJobs)
        for kind, limit in (("Complete", spec.get("successfulJobsHistoryLimit", 3)), ("Failed", spec.get("failedJobsHistoryLimit", 1))):
            done = sorted((j for j in jobs if finished(j) == kind), key=lambda j: (j.get("metadata") or {}).get("creationTimestamp", ""))
            for j in done[:max(0, len(done) - int(limit))]:
                await self.client.delete("jobs", m.name_of(j), ns, propagation="Background")
        changed = st.get("active", []) != active_refs
        st["active"] = active_refs
        if not spec.get("suspend"):
            now = self.clock()
            sched = CronSchedule(spec["schedule"])
            earliest = m.parse_time(st.get("lastScheduleTime")) or m.parse_time((cj.get("metadata") or {}).get("creationTimestamp")) or now
            deadline = spec.get("startingDeadlineSeconds")
            if deadline is not None:
                earliest = max(earliest, now - float(deadline))
            try:
                times = unmet_schedule_times(sched, earliest, now)
            except RuntimeError as e:
                self.mgr_event(cj, "Warning", "FailedNeedsStart", str(e))
                times = []
            if times:
                t = times[-1]
                policy = spec.get("concurrencyPolicy", "Allow")
                if policy == "Forbid" and active:
                    pass
                else:
                    if policy == "Replace":
                        for j in active:
                            await self.client.delete("jobs", m.name_of(j), ns, propagation="Background")
                        st["active"] = []
                    jt = (spec.get("jobTemplate") or {})
                    jname = f"{name}-{int(t // 60)}"
                    job = {"apiVersion": "batch/v1", "kind": "Job",
                           "metadata": {"name": jname, "namespace": ns,
                                        "labels": dict((jt.get("metadata") or {}).get("labels") or {}),
                                        "annotations": dict((jt.get("metadata") or {}).get("annotations") or {},
                                                            **{"cronjob.kubernetes.io/scheduled-time": m.format_time(t)}),
                                        "ownerReferences": [m.new_controller_ref(cj, "batch/v1beta1", "CronJob")]},
                           "spec": json.loads(json.dumps(jt.get("spec") or {}))}
                    try:
                        j = await self.client.create(job, ns)
                        st["active"] = st["active"] + [{"kind": "Job", "namespace": ns, "name": jname, "uid": m.uid_of(j),
                                                        "apiVersion": "batch/v1"}]
                    except m.StatusError as e:
                        if not m.is_already_exists(e):
                            raise
                st["lastScheduleTime"] = m.format_time(t)
                changed = True
        if changed:
            await self.client.patch("cronjobs", name, {"status": st}, ns, sub="status")

    def mgr_event(self, obj, typ, reason, msg):
        rec = getattr(self.mgr, "recorder", None)
        if rec is not None:
            rec.event(obj, typ, reason, msg)
