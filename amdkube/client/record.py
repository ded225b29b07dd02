"""Event recorder with correlation (count aggregation) and a non-blocking sink.

Reference: staging/src/k8s.io/client-go/tools/record (event.go: Eventf → broadcaster →
sink with retries; events_cache.go: identical events are aggregated into one object whose
`count` and `lastTimestamp` are patched). Used by the scheduler for `Scheduled` /
`FailedScheduling` (plugin/pkg/scheduler/scheduler.go:194,425) and by the kubelet.
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..api import meta as m
from .rest import Client

log = logging.getLogger("amdkube.record")

NORMAL, WARNING = "Normal", "Warning"


SPAM_BURST, SPAM_QPS = 25, 1.0 / 300     # events_cache.go EventSourceObjectSpamFilter defaults


class EventRecorder:
    """`qps`/`burst` bound the rate of writes to the API (--event-qps/--event-burst; 0: no
    bound); every (source, involved object) pair also gets the reference's spam filter: a
    burst of 25 events, then one per five minutes."""

    def __init__(self, client: Client, component: str, host: str = "", max_queue: int = 10000, qps: float = 0,
                 burst: int = 10):
        self.client, self.component, self.host = client, component, host
        from .rest import TokenBucket
        self.limiter = TokenBucket(qps, burst) if qps else None
        self._spam: dict[tuple, tuple[float, float]] = {}     # (kind, ns, name, uid) -> (tokens, last refill)
        self.queue: asyncio.Queue | None = None
        self.max_queue = max_queue
        self.cache: dict[tuple, tuple[str, str, int]] = {}  # key -> (ns, name, count)
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

    def event(self, obj: dict, etype: str, reason: str, message: str):
        if not self.enabled or self.queue is None or self.queue.qsize() >= self.max_queue:
            return
        md = obj.get("metadata") or {}
        ref = {"kind": obj.get("kind", ""), "namespace": md.get("namespace", ""), "name": md.get("name", ""),
               "uid": md.get("uid", ""), "apiVersion": obj.get("apiVersion", ""),
               "resourceVersion": md.get("resourceVersion", "")}
        self.queue.put_nowait((ref, etype, reason, message, time.time()))

    def _spam_ok(self, ref) -> bool:
        key = (ref["kind"], ref["namespace"], ref["name"], ref["uid"])
        now = time.monotonic()
        tokens, last = self._spam.get(key, (float(SPAM_BURST), now))
        tokens = min(float(SPAM_BURST), tokens + (now - last) * SPAM_QPS)
        if tokens < 1:
            self._spam[key] = (tokens, now)
            return False
        self._spam[key] = (tokens - 1, now)
        if len(self._spam) > 4096:
            self._spam = {k: v for k, v in self._spam.items() if now - v[1] < 300}
        return True

    async def _run(self):
        while True:
            ref, etype, reason, message, ts = await self.queue.get()
            try:
                if not self._spam_ok(ref):
                    continue
                if self.limiter is not None:
                    await self.limiter.wait()
                await self._write(ref, etype, reason, message, ts)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # events are best effort
                log.debug("dropping event %s/%s: %r", ref.get("name"), reason, e)

    async def _write(self, ref, etype, reason, message, ts):
        ns = ref["namespace"] or "default"
        key = (ref["kind"], ns, ref["name"], ref["uid"], reason, message, etype)
        now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(ts))
        hit = self.cache.get(key)
        if hit:
            ens, ename, count = hit
            try:
                await self.client.patch("events", ename, {"count": count + 1, "lastTimestamp": now}, ens)
                self.cache[key] = (ens, ename, count + 1)
                return
            except m.StatusError:
                self.cache.pop(key, None)
        name = f"{ref['name']}.{int(ts * 1e9):x}"
        ev = {"apiVersion": "v1", "kind": "Event", "metadata": {"name": name, "namespace": ns},
              "involvedObject": ref, "reason": reason, "message": message, "type": etype,
              "source": {"component": self.component, "host": self.host}, "count": 1,
              "firstTimestamp": now, "lastTimestamp": now}
        await self.client.create(ev, ns)
        if len(self.cache) > 4096:
            self.cache.clear()
        self.cache[key] = (ns, name, 1)
