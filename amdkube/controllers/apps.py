"""ReplicationController, StatefulSet and CronJob controllers.

Reference:
  * pkg/controller/replication — the ReplicaSet logic over a v1 map selector.
  * pkg/controller/statefulset — controllers/statefulset.py (re-exported here).
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
from ..api.labels import selector_from_set
from .base import Controller, split_key
from .workloads import ReplicaSetController

REVISION_LABEL = "controller-revision-hash"
POD_NAME_LABEL = "statefulset.kubernetes.io/pod-name"


class ReplicationManager(ReplicaSetController):
    """pkg/controller/replication: the ReplicaSet controller over a v1 map selector."""
    name = "replicationcontroller"
    owner_api, owner_kind, plural = "v1", "ReplicationController", "replicationcontrollers"

    def selector_of(self, rc):
        return selector_from_set((rc.get("spec") or {}).get("selector") or {})


from .statefulset import StatefulSetController  # noqa: E402,F401  (controllers/statefulset.py)


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
