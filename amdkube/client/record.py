"""Event recorder with correlation and a non-blocking sink.

Reference: staging/src/k8s.io/client-go/tools/record — event.go (Eventf → broadcaster →
recordToSink: correlate, then patch the stored event when it is a repeat or create it, and
create it afresh when the patch finds it gone; UpdateState with what the server returned) and
events_cache.go (the EventCorrelator: spam filter, aggregation of similar events, counting of
identical ones; client/events_cache.py). Used by the scheduler for `Scheduled` /
`FailedScheduling` (plugin/pkg/scheduler/scheduler.go:194,425), the controllers and the kubelet.
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..api import meta as m
from .rest import Client

log = logging.getLogger("amdkube.record")

NORMAL, WARNING = "Normal", "Warning"


class EventRecorder:
    """`qps`/`burst` bound the rate of writes to the API (--event-qps/--event-burst; 0: no
    bound); the correlator applies the reference's per-object spam filter (a burst of 25
    events, then one per five minutes), aggregation and counting."""

    def __init__(self, client: Client, component: str, host: str = "", max_queue: int = 10000, qps: float = 0,
                 burst: int = 10, clock=time.time):
        from .events_cache import EventCorrelator
        self.client, self.component, self.host = client, component, host
        from .rest import TokenBucket
        self.limiter = TokenBucket(qps, burst) if qps else None
        self.correlator = EventCorrelator(clock=clock)
        self.clock = clock
        self.queue: asyncio.Queue | None = None
        self.max_queue = max_queue
        self._task: asyncio.Task | None = None
        self.enabled = True

    def start(self):
        self.queue = asyncio.Queue()
        self._task = asyncio.create_task(self._run(), name=f"events-{self.component}")
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass

    def event(self, obj: dict, etype: str, reason: str, message: str, field_path: str = ""):
        if not self.enabled or self.queue is None or self.queue.qsize() >= self.max_queue:
            return
        md = obj.get("metadata") or {}
        ref = {"kind": obj.get("kind", ""), "namespace": md.get("namespace", ""), "name": md.get("name", ""),
               "uid": md.get("uid", ""), "apiVersion": obj.get("apiVersion", ""),
               "resourceVersion": md.get("resourceVersion", "")}
        if field_path:
            ref["fieldPath"] = field_path
        self.queue.put_nowait((ref, etype, reason, message, self.clock()))

    def make_event(self, ref, etype, reason, message, ts) -> dict:
        """makeEvent: named <object>.<unix nanos in hex>, in the object's namespace."""
        ns = ref["namespace"] or "default"
        now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(ts))
        return {"apiVersion": "v1", "kind": "Event", "metadata": {"name": f"{ref['name']}.{int(ts * 1e9):x}", "namespace": ns},
                "involvedObject": ref, "reason": reason, "message": message, "type": etype,
                "source": {"component": self.component, "host": self.host}, "count": 1,
                "firstTimestamp": now, "lastTimestamp": now}

    async def _run(self):
        while True:
            ref, etype, reason, message, ts = await self.queue.get()
            try:
                await self.record(self.make_event(ref, etype, reason, message, ts))
            except asyncio.CancelledError:
                raise
            except Exception as e:  # events are best effort
                log.debug("dropping event %s/%s: %r", ref.get("name"), reason, e)

    async def record(self, ev: dict) -> dict | None:
        """recordToSink/recordEvent: correlate; patch a repeat, create otherwise (or when the
        repeat's stored event is gone); remember what the server stored."""
        res = self.correlator.correlate(ev)
        if res.skip:
            return None
        ev = res.event
        ns = (ev.get("metadata") or {}).get("namespace") or "default"
        if self.limiter is not None:
            await self.limiter.wait()
        stored = None
        if int(ev.get("count") or 1) > 1 and res.patch is not None:
            try:
                stored = await self.client.patch("events", ev["metadata"]["name"], res.patch, ns)
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise
        if stored is None:
            body = {**ev, "metadata": {k: v for k, v in ev["metadata"].items() if k != "resourceVersion"}}
            stored = await self.client.create(body, ns)
        self.correlator.update_state(stored)
        return stored
