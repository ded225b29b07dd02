"""Controller scaffolding: informer handlers enqueue keys, workers reconcile with
rate-limited retries (client-go workqueue pattern used by every pkg/controller/*)."""
from __future__ import annotations

import asyncio
import logging

from ..api import meta as m
from ..client.workqueue import RateLimitingQueue, ShutDown

log = logging.getLogger("amdkube.controllers")


class Controller:
    name = "controller"
    workers = 2
    max_requeues: int | None = 15      # retries of a failing key before it is dropped (None: no cap)

    def __init__(self, mgr):
        self.mgr = mgr
        self.client = mgr.client
        self.queue = RateLimitingQueue(self.name)
        self.tasks: list[asyncio.Task] = []
        self.syncs = 0

    def enqueue(self, obj_or_key):
        key = obj_or_key if isinstance(obj_or_key, str) else m.key_of(obj_or_key)
        self.queue.add(key)

    def setup(self):
        """Register informer handlers (called before informers start)."""

    async def start(self):
        for i in range(self.workers):
            self.tasks.append(asyncio.create_task(self._worker(), name=f"{self.name}-{i}"))

    async def stop(self):
        self.queue.shutdown()
        for t in self.tasks:
            t.cancel()

    async def _worker(self):
        while True:
            try:
                key = await self.queue.get()
            except ShutDown:
                return
            try:
                # a sync may return False: done, but keep the key's rate-limit history (the
                # reference's syncHandler `forget` result, e.g. the Job controller's back-off)
                if await self.sync(key) is not False:
                    self.queue.forget(key)
                self.syncs += 1
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.debug("%s: sync %s failed: %r", self.name, key, e)
                if self.max_requeues is None or self.queue.num_requeues(key) < self.max_requeues:
                    self.queue.add_rate_limited(key)
            finally:
                self.queue.done(key)

    async def sync(self, key: str):
        raise NotImplementedError


def split_key(key: str) -> tuple[str, str]:
    if "/" in key:
        ns, name = key.split("/", 1)
        return ns, name
    return "", key
