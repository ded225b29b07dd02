"""ReplicationController, StatefulSet and CronJob controllers.

Reference:
  * pkg/controller/replication — the ReplicaSet logic over a v1 map selector.
  * pkg/controller/statefulset — controllers/statefulset.py (re-exported here).
  * pkg/controller/cronjob/{cronjob_controller.go, utils.go} — polled every 10 s;
    syncOne reconciles status.active with the jobs seen (UnexpectedJob / SawCompletedJob /
    MissingJob), then starts the latest of getRecentUnmetScheduleTimes (since lastScheduleTime
    or creation, bounded by startingDeadlineSeconds; >100 misses is an error) unless suspended,
    past its deadline, or Forbid with an active job; Replace deletes active jobs the way the
    kubectl JobReaper does (scale to 0, delete pods, delete job); job names are
    `<cronjob>-<getTimeHash>` (Unix seconds in 1.9); cleanupFinishedJobs deletes the
    earliest-started finished jobs beyond the history limits (defaulted 3 / 1 by the API).
"""
from __future__ import annotations

import asyncio
import calendar
import functools
import json
import logging
import time

from ..api import meta as m
from ..api.labels import selector_from_set
from .base import Controller, split_key
from .replicaset import ReplicaSetController

log = logging.getLogger("amdkube.controllers.cronjob")

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


def get_finished_status(job: dict):
    """getFinishedStatus: (finished, "Complete" | "Failed" | "")."""
    for c in (job.get("status") or {}).get("conditions") or []:
        if c.get("type") in ("Complete", "Failed") and c.get("status") == "True":
            return True, c["type"]
    return False, ""


def is_job_finished(job: dict) -> bool:
    return get_finished_status(job)[0]


def in_active_list(sj: dict, uid: str) -> bool:
    return any(r.get("uid") == uid for r in (sj.get("status") or {}).get("active") or [])


def delete_from_active_list(sj: dict, uid: str):
    st = sj.setdefault("status", {})
    st["active"] = [r for r in st.get("active") or [] if r.get("uid") != uid]


def get_parent_uid_from_job(job: dict):
    """getParentUIDFromJob: the controlling CronJob's UID, if the job has one."""
    ref = m.controller_ref(job)
    if ref is None or ref.get("kind") != "CronJob":
        return "", False
    return ref.get("uid", ""), True


def group_jobs_by_parent(jobs: list) -> dict:
    out: dict[str, list] = {}
    for j in jobs:
        uid, ok = get_parent_uid_from_job(j)
        if ok:
            out.setdefault(uid, []).append(j)
    return out


def get_recent_unmet_schedule_times(sj: dict, now: float) -> list[float]:
    """getRecentUnmetScheduleTimes: every activation after max(lastScheduleTime or
    creationTimestamp, now - startingDeadlineSeconds) up to now; more than 100 is an error."""
    spec, st = sj.get("spec") or {}, sj.get("status") or {}
    try:
        sched = CronSchedule(spec.get("schedule", ""))
    except ValueError as e:
        raise ValueError(f"Unparseable schedule: {spec.get('schedule', '')} : {e}") from e
    earliest = m.parse_time(st.get("lastScheduleTime")) if st.get("lastScheduleTime") else \
        m.parse_time((sj.get("metadata") or {}).get("creationTimestamp")) or 0.0
    if spec.get("startingDeadlineSeconds") is not None:
        earliest = max(earliest, now - float(spec["startingDeadlineSeconds"]))
    if earliest > now:
        return []
    try:
        return unmet_schedule_times(sched, earliest, now)
    except RuntimeError:
        raise ValueError("Too many missed start time (> 100). Set or decrease .spec.startingDeadlineSeconds or check "
                         "clock skew.") from None


def get_time_hash(t: float) -> int:
    """getTimeHash: the scheduled time in Unix seconds (the job name's suffix)."""
    return int(t)


def get_job_from_template(sj: dict, scheduled: float) -> dict:
    """getJobFromTemplate: the template's labels and annotations, a deterministic name per
    scheduled time, and a controller reference to the CronJob."""
    jt = (sj.get("spec") or {}).get("jobTemplate") or {}
    md = jt.get("metadata") or {}
    job = {"apiVersion": "batch/v1", "kind": "Job",
           "metadata": {"name": f"{m.name_of(sj)}-{get_time_hash(scheduled)}",
                        "ownerReferences": [m.new_controller_ref(sj, "batch/v1beta1", "CronJob")]},
           "spec": json.loads(json.dumps(jt.get("spec") or {}))}
    if md.get("labels"):
        job["metadata"]["labels"] = dict(md["labels"])
    if md.get("annotations"):
        job["metadata"]["annotations"] = dict(md["annotations"])
    return job


def _job_ref(job: dict) -> dict:
    """ref.GetReference of a created job."""
    md = job.get("metadata") or {}
    ref = {"kind": "Job", "namespace": md.get("namespace", ""), "name": md.get("name", ""), "uid": md.get("uid", ""),
           "apiVersion": "batch/v1"}
    if md.get("resourceVersion"):
        ref["resourceVersion"] = md["resourceVersion"]
    return ref


def _by_job_start_time(a: dict, b: dict) -> int:
    """byJobStartTime.Less as a comparison: jobs with a start time first, earlier first, equal
    times by name; two without one compare equal (the stable sort keeps their order, as Go's
    insertion sort does for such short lists)."""
    ta, tb = (a.get("status") or {}).get("startTime"), (b.get("status") or {}).get("startTime")
    if ta is None or tb is None:
        return 0 if ta is None and tb is None else (-1 if tb is None else 1)
    fa, fb = m.parse_time(ta) or 0.0, m.parse_time(tb) or 0.0
    if fa == fb:
        return (m.name_of(a) > m.name_of(b)) - (m.name_of(a) < m.name_of(b))
    return -1 if fa < fb else 1


class RealJobControl:
    def __init__(self, client):
        self.client = client

    async def get_job(self, ns, name):
        return await self.client.get("jobs", name, ns)

    async def create_job(self, ns, job):
        return await self.client.create(job, ns)

    async def update_job(self, ns, job):
        return await self.client.update(job)

    async def delete_job(self, ns, name):
        await self.client.delete("jobs", name, ns)


class RealPodControl:
    def __init__(self, client):
        self.client = client

    async def list_pods(self, ns, selector: str):
        items, _ = await self.client.list("pods", ns, label_selector=selector or None)
        return items

    async def delete_pod(self, ns, name):
        await self.client.delete("pods", name, ns)


class RealSJControl:
    def __init__(self, client):
        self.client = client

    async def update_status(self, sj):
        return await self.client.update(sj, sub="status")


async def delete_job(sj, job, jc, pc, recorder, reason: str = "") -> bool:
    """deleteJob (the kubectl JobReaper's steps): scale to 0, delete its pods, delete it, drop it
    from the active list."""
    def event(etype, r, msg):
        if recorder is not None:
            recorder.event(sj, etype, r, msg)
    ns = m.namespace_of(job)
    if (job.get("spec") or {}).get("parallelism", 1) != 0:
        job = json.loads(json.dumps(job))
        job["spec"]["parallelism"] = 0
        try:
            job = await jc.update_job(ns, job)
        except Exception as e:
            event("Warning", "FailedUpdate", f"Update job: {e}")
            return False
    from ..api.labels import selector_from_label_selector
    sel = (job.get("spec") or {}).get("selector")
    try:
        pods = await pc.list_pods(ns, str(selector_from_label_selector(sel)) if sel else "")
    except Exception as e:
        event("Warning", "FailedList", f"List job-pods: {e}")
        return False
    errs = []
    for p in pods:
        try:
            await pc.delete_pod(m.namespace_of(p), m.name_of(p))
        except m.StatusError as e:
            if not m.is_not_found(e):
                errs.append(e)
    if errs:
        event("Warning", "FailedDelete", f"Deleted job-pods: {errs}")
        return False
    try:
        await jc.delete_job(ns, m.name_of(job))
    except Exception as e:
        event("Warning", "FailedDelete", f"Deleted job: {e}")
        return False
    delete_from_active_list(sj, m.uid_of(job))
    event("Normal", "SuccessfulDelete", f"Deleted job {m.name_of(job)}")
    return True


async def sync_one(sj, jobs, now, jc, sjc, pc, recorder):
    """syncOne: reconcile the active list with the jobs seen, write status, then start the most
    recent unmet scheduled run if the policy allows it."""
    def event(etype, reason, msg):
        if recorder is not None:
            recorder.event(sj, etype, reason, msg)
    children = set()
    for j in jobs:
        children.add(m.uid_of(j))
        found, finished = in_active_list(sj, m.uid_of(j)), is_job_finished(j)
        if not found and not finished:
            event("Warning", "UnexpectedJob", f"Saw a job that the controller did not create or forgot: {m.name_of(j)}")
        elif found and finished:
            delete_from_active_list(sj, m.uid_of(j))
            event("Normal", "SawCompletedJob", f"Saw completed job: {m.name_of(j)}")
    for ref in list((sj.get("status") or {}).get("active") or []):
        if ref.get("uid") not in children:
            event("Normal", "MissingJob", f"Active job went missing: {ref.get('name', '')}")
            delete_from_active_list(sj, ref.get("uid"))
    try:
        updated = await sjc.update_status(sj)
    except Exception as e:
        log.error("unable to update status for %s: %r", m.key_of(sj), e)
        return
    sj.clear()
    sj.update(updated)
    spec = sj.get("spec") or {}
    if (sj.get("metadata") or {}).get("deletionTimestamp") or spec.get("suspend"):
        return
    try:
        times = get_recent_unmet_schedule_times(sj, now)
    except ValueError as e:
        event("Warning", "FailedNeedsStart", f"Cannot determine if job needs to be started: {e}")
        return
    if not times:
        return
    scheduled = times[-1]
    if spec.get("startingDeadlineSeconds") is not None and scheduled + float(spec["startingDeadlineSeconds"]) < now:
        return                                          # missed the starting window
    active = (sj.get("status") or {}).get("active") or []
    if spec.get("concurrencyPolicy") == "Forbid" and active:
        return
    if spec.get("concurrencyPolicy") == "Replace":
        for ref in list(active):
            try:
                job = await jc.get_job(ref.get("namespace", ""), ref.get("name", ""))
            except Exception as e:
                event("Warning", "FailedGet", f"Get job: {e}")
                return
            if not await delete_job(sj, job, jc, pc, recorder):
                return
    req = get_job_from_template(sj, scheduled)
    try:
        resp = await jc.create_job(m.namespace_of(sj), req)
    except Exception as e:
        event("Warning", "FailedCreate", f"Error creating job: {e}")
        return
    event("Normal", "SuccessfulCreate", f"Created job {m.name_of(resp)}")
    st = sj.setdefault("status", {})
    st["active"] = list(st.get("active") or []) + [_job_ref(resp)]
    st["lastScheduleTime"] = m.format_time(scheduled)
    try:
        await sjc.update_status(sj)
    except Exception as e:
        log.info("unable to update status for %s: %r", m.key_of(sj), e)


async def remove_oldest_jobs(sj, jobs, jc, pc, max_jobs: int, recorder):
    n = len(jobs) - int(max_jobs)
    if n <= 0:
        return
    for j in sorted(jobs, key=functools.cmp_to_key(_by_job_start_time))[:n]:
        await delete_job(sj, j, jc, pc, recorder, "history limit reached")


async def cleanup_finished_jobs(sj, jobs, jc, sjc, pc, recorder):
    """cleanupFinishedJobs: beyond successfulJobsHistoryLimit / failedJobsHistoryLimit (when set),
    the earliest-started finished jobs are deleted; status is written after."""
    spec = sj.get("spec") or {}
    if spec.get("failedJobsHistoryLimit") is None and spec.get("successfulJobsHistoryLimit") is None:
        return
    ok, failed = [], []
    for j in jobs:
        fin, kind = get_finished_status(j)
        if fin and kind == "Complete":
            ok.append(j)
        elif fin and kind == "Failed":
            failed.append(j)
    if spec.get("successfulJobsHistoryLimit") is not None:
        await remove_oldest_jobs(sj, ok, jc, pc, spec["successfulJobsHistoryLimit"], recorder)
    if spec.get("failedJobsHistoryLimit") is not None:
        await remove_oldest_jobs(sj, failed, jc, pc, spec["failedJobsHistoryLimit"], recorder)
    try:
        await sjc.update_status(sj)
    except Exception as e:
        log.info("unable to update status for %s: %r", m.key_of(sj), e)


class CronJobController(Controller):
    """pkg/controller/cronjob/cronjob_controller.go: every 10 s each CronJob is synced with the
    jobs it controls (syncOne, then cleanupFinishedJobs)."""
    name = "cronjob"
    workers = 1
    period = 10.0            # cronjob_controller.go: wait.Until(syncAll, 10s)

    def __init__(self, mgr, clock=time.time):
        super().__init__(mgr)
        self.clock = clock
        self._poll = None
        self.jc, self.pc, self.sjc = RealJobControl(self.client), RealPodControl(self.client), RealSJControl(self.client)

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
        if cj is None:
            return
        sj = json.loads(json.dumps(cj))
        jobs = group_jobs_by_parent(self.job_inf.list()).get(m.uid_of(sj), [])
        rec = getattr(self.mgr, "recorder", None)
        await sync_one(sj, jobs, self.clock(), self.jc, self.sjc, self.pc, rec)
        await cleanup_finished_jobs(sj, jobs, self.jc, self.sjc, self.pc, rec)
