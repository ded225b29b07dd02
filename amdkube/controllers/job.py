"""Job controller (pkg/controller/job/job_controller.go).

syncJob (:431-560) on the job's pods:
  * active = pods neither terminal nor being deleted; succeeded / failed counted from pods, the
    failed count never goes down (status.failed is kept when failed pods are garbage-collected);
  * a NEW failure with the key already requeued `backoffLimit` times fails the Job
    (BackoffLimitExceeded); a Job active longer than spec.activeDeadlineSeconds fails
    (DeadlineExceeded, :601-610). Either way its active pods are deleted — a GPU Job's devices
    are released — and they count as failed;
  * otherwise manageJob (:636-763): more active than parallelism deletes the surplus (the
    least established pods first, controller.ActivePods); fewer creates
    min(completions - succeeded, parallelism) - active in slow-start batches 1, 2, 4, …
    (a batch with errors stops the rest); with spec.completions unset (work-queue Job) it keeps
    `parallelism` pods until the first success, then lets the running ones finish;
  * Complete when succeeded reaches completions, or (work queue) once some pod succeeded and
    none is active.
A pod that fails requeues its Job after an exponential back-off of 10 s doubling up to 6 min
(getBackoff :777-790, DefaultJobBackOff / MaxJobBackOff); a sync that saw a new failure returns
an error, so the key's requeue count (the back-off exponent and the backoffLimit budget) grows
until a sync settles without one. Expectations (controller_utils.go ControllerExpectations)
keep a sync from creating or deleting again before the informer has seen its last writes.

The sync itself is `sync_job`: pure over (job, pods, pod control, requeue count, now), which is
what the ported TestControllerSyncJob / TestSyncJobPastDeadline tables drive.
"""
from __future__ import annotations

import asyncio
import time

from ..api import meta as m
from ..api.helpers import is_pod_ready, is_pod_terminal
from ..client.workqueue import ItemExponentialFailureRateLimiter, RateLimitingQueue
from .base import Controller, split_key
from .controller_utils import sort_active_pods

DEFAULT_JOB_BACKOFF, MAX_JOB_BACKOFF = 10.0, 360.0
SLOW_START_INITIAL_BATCH = 1
EXPECTATIONS_TIMEOUT = 300.0


class NewFailure(Exception):
    """syncJob's error for a sync that saw a new pod failure: the key is not forgotten."""


def is_finished(job: dict) -> bool:
    return any(c.get("type") in ("Complete", "Failed") and c.get("status") == "True"
               for c in (job.get("status") or {}).get("conditions") or [])


def _condition(kind: str, reason: str = "", message: str = "") -> dict:
    now = m.now_rfc3339()
    return {"type": kind, "status": "True", "lastProbeTime": now, "lastTransitionTime": now, "reason": reason,
            "message": message}


async def sync_job(job: dict, pods: list, pod_control, previous_retry: int = 0, now: float | None = None,
                   needs_sync: bool = True) -> tuple[dict, bool, Exception | None]:
    """One syncJob: returns (the job with its new status, forget, error). `pod_control` has
    async create(job) and delete(pod); their exceptions are the pod-control errors."""
    now = time.time() if now is None else now
    job = m.deepcopy(job)
    spec, st = job.get("spec") or {}, job.setdefault("status", {})
    active_pods = [p for p in pods if not is_pod_terminal(p) and not (p.get("metadata") or {}).get("deletionTimestamp")]
    active = len(active_pods)
    succeeded = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Succeeded")
    failed = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Failed")
    n_conditions = len(st.get("conditions") or [])
    if not st.get("startTime"):
        st["startTime"] = m.format_time(now)
    prev_failed = int(st.get("failed") or 0)
    new_failure = failed > prev_failed
    failed = max(failed, prev_failed)
    backoff_limit = int(spec.get("backoffLimit", 6))
    ads = spec.get("activeDeadlineSeconds")
    started = m.parse_time(st["startTime"]) or now
    err: Exception | None = None
    reason = message = ""
    if new_failure and previous_retry + 1 > backoff_limit:
        reason, message = "BackoffLimitExceeded", "Job has reach the specified backoff limit"
    elif ads is not None and now - started >= int(ads):
        reason, message = "DeadlineExceeded", "Job was active longer than specified deadline"
    if reason:
        for p in active_pods:
            try:
                await pod_control.delete(p)
            except Exception as e:      # noqa: BLE001 — reported, the Job still fails
                err = err or e
        failed += active
        active = 0
        st.setdefault("conditions", []).append(_condition("Failed", reason, message))
    else:
        if needs_sync and not (job.get("metadata") or {}).get("deletionTimestamp"):
            active, err = await _manage(job, active_pods, succeeded, pod_control)
        completions = spec.get("completions")
        complete = (succeeded > 0 and active == 0) if completions is None else succeeded >= int(completions)
        if complete:
            st.setdefault("conditions", []).append(_condition("Complete"))
            st["completionTime"] = m.format_time(now)
    forget = False
    if (st.get("active"), st.get("succeeded"), st.get("failed"), len(st.get("conditions") or [])) != \
            (active, succeeded, failed, n_conditions):
        st["active"], st["succeeded"], st["failed"] = active, succeeded, failed
        if new_failure and not is_finished(job):
            return job, False, NewFailure(f"failed pod(s) detected for job key {m.key_of(job)!r}")
        forget = True
    return job, forget, err


async def _manage(job: dict, active_pods: list, succeeded: int, pod_control) -> tuple[int, Exception | None]:
    spec = job.get("spec") or {}
    active = len(active_pods)
    parallelism = int(spec.get("parallelism", 1))
    err: Exception | None = None
    if active > parallelism:
        diff = active - parallelism
        for p in sort_active_pods(list(active_pods))[:diff]:
            try:
                await pod_control.delete(p)
                active -= 1
            except Exception as e:      # noqa: BLE001
                err = err or e
        return active, err
    if active < parallelism:
        completions = spec.get("completions")
        if completions is None:
            want = active if succeeded > 0 else parallelism
        else:
            want = min(int(completions) - succeeded, parallelism)
        diff = max(0, want - active)
        batch = min(diff, SLOW_START_INITIAL_BATCH)
        while diff > 0:
            results = await asyncio.gather(*(pod_control.create(job) for _ in range(batch)), return_exceptions=True)
            errors = [r for r in results if isinstance(r, Exception)]
            active += batch - len(errors)
            diff -= batch
            if errors:
                err = err or errors[0]
                break                   # slow start: a batch with errors skips the rest
            batch = min(2 * batch, diff)
    return active, err


class _PodControl:
    def __init__(self, ctl: "JobController"):
        self.ctl = ctl

    async def create(self, job):
        from .controller_utils import pod_from_template as _pod_from_template
        key = m.key_of(job)
        self.ctl._expect(key, adds=1)
        try:
            await self.ctl.client.create(_pod_from_template(job, "batch/v1", "Job", {"job-name": m.name_of(job)}),
                                         m.namespace_of(job))
        except Exception:
            self.ctl._expect(key, adds=-1)
            raise

    async def delete(self, pod):
        ref = m.controller_ref(pod) or {}
        key = f"{m.namespace_of(pod)}/{ref.get('name', '')}"
        self.ctl._expect(key, dels=1)
        try:
            await self.ctl.client.delete("pods", m.name_of(pod), m.namespace_of(pod))
        except m.StatusError as e:
            self.ctl._expect(key, dels=-1)
            if not m.is_not_found(e):
                raise


class JobController(Controller):
    name = "job"
    max_requeues = None            # a failing Job keeps backing off (capped at MAX_JOB_BACKOFF)

    def __init__(self, mgr):
        super().__init__(mgr)
        self.queue = RateLimitingQueue(self.name, ItemExponentialFailureRateLimiter(DEFAULT_JOB_BACKOFF, MAX_JOB_BACKOFF))
        self.expectations: dict[str, list] = {}     # key -> [adds, dels, set at]
        self.pod_control = _PodControl(self)

    def setup(self):
        f = self.mgr.factory
        self.job_inf = f.informer("jobs")
        self.pod_inf = self.mgr.pods
        self.job_inf.add_handler(on_add=self.enqueue, on_update=self._job_update, on_delete=self.enqueue)
        self.pod_inf.add_handler(on_add=self._pod_add, on_update=self._pod_update, on_delete=self._pod_delete)

    # ----------------------------------------------------------- expectations
    def _expect(self, key, adds=0, dels=0):
        e = self.expectations.setdefault(key, [0, 0, time.monotonic()])
        e[0] += adds
        e[1] += dels
        if adds > 0 or dels > 0:
            e[2] = time.monotonic()

    def _satisfied(self, key) -> bool:
        e = self.expectations.get(key)
        return e is None or (e[0] <= 0 and e[1] <= 0) or time.monotonic() - e[2] > EXPECTATIONS_TIMEOUT

    def _observed(self, pod, adds=0, dels=0):
        ref = m.controller_ref(pod)
        if ref and ref.get("kind") == "Job":
            key = f"{m.namespace_of(pod)}/{ref['name']}"
            e = self.expectations.get(key)
            if e is not None:
                e[0] -= adds
                e[1] -= dels
            return key
        return None

    # ----------------------------------------------------------- handlers
    def _backoff(self, key) -> float:
        n = self.queue.num_requeues(key)
        return 0.0 if n <= 0 else min(MAX_JOB_BACKOFF, DEFAULT_JOB_BACKOFF * 2 ** (n - 1))

    def _job_update(self, old, new):
        self.enqueue(new)
        ads, old_ads = (new.get("spec") or {}).get("activeDeadlineSeconds"), (old.get("spec") or {}).get("activeDeadlineSeconds")
        start = m.parse_time((new.get("status") or {}).get("startTime"))
        if ads is not None and ads != old_ads and start:
            self.queue.add_after(m.key_of(new), max(0.0, start + int(ads) - time.time()))

    def _pod_add(self, pod):
        key = self._observed(pod, adds=1)
        if key:
            self.queue.add(key)

    def _pod_update(self, old, pod):
        key = self._observed(pod)
        if not key:
            return
        if (pod.get("metadata") or {}).get("deletionTimestamp") and not (old.get("metadata") or {}).get("deletionTimestamp"):
            self._observed(pod, dels=1)
        # the only time to back off is when the pod failed (updatePod: immediate unless Failed)
        failed = (pod.get("status") or {}).get("phase") == "Failed" and (old.get("status") or {}).get("phase") != "Failed"
        if failed:
            self.queue.add_after(key, self._backoff(key))
        else:
            self.queue.add(key)

    def _pod_delete(self, pod):
        key = self._observed(pod, dels=0 if (pod.get("metadata") or {}).get("deletionTimestamp") else 1)
        if key:
            self.queue.add(key)

    # ----------------------------------------------------------- sync
    async def sync(self, key):
        job = self.job_inf.get(key)
        if job is None:
            self.expectations.pop(key, None)
            return
        if is_finished(job):
            return
        uid = m.uid_of(job)
        pods = [p for p in self.pod_inf.list() if (m.controller_ref(p) or {}).get("uid") == uid]
        new, forget, err = await sync_job(job, pods, self.pod_control, self.queue.num_requeues(key),
                                          needs_sync=self._satisfied(key))
        ads = (new.get("spec") or {}).get("activeDeadlineSeconds")
        if ads is not None and not is_finished(new):
            start = m.parse_time(new["status"]["startTime"]) or time.time()
            self.queue.add_after(key, max(0.0, start + int(ads) - time.time()) + 0.05)
        if new.get("status") != job.get("status"):
            cond = (new["status"].get("conditions") or [{}])[-1]
            recorder = getattr(self.mgr, "recorder", None)
            if recorder is not None and cond.get("reason") in ("DeadlineExceeded", "BackoffLimitExceeded"):
                recorder.event(new, "Warning", cond["reason"], cond["message"])
            _ns, name = split_key(key)
            await self.client.patch("jobs", name, {"status": new["status"]}, m.namespace_of(job), sub="status")
        if err is not None:
            raise err
        # forget=False (a sync that changed nothing) keeps the key's back-off history; only a
        # settled status resets it
        return forget
