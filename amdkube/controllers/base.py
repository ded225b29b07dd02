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
                await self.sync(key)
                self.queue.forget(key)
                self.syncs += 1
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.debug("%s: sync %s failed: %r", self.name, key, e)
                if self.queue.num_requeues(key) < 15:
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
