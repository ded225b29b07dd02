"""Reflector + Indexer + SharedInformer (client-go tools/cache).

Reference: tools/cache/reflector.go:239 (ListAndWatch: list → Replace → watch from the
list RV; on watch end re-watch from last RV; on 410 Gone re-list), shared_informer.go:188
(Run, handler fan-out, resync), store.go/thread_safe_store.go (indexers).

Handlers run synchronously on the event loop and must be cheap (enqueue into a work
queue). `has_synced` is set after the first complete list has been delivered.
"""
from __future__ import annotations

import asyncio
import logging
import random

from ..api import meta as m
from .rest import Client

log = logging.getLogger("amdkube.informer")


class ResourceEventHandler:
    def __init__(self, on_add=None, on_update=None, on_delete=None, filter_fn=None):
        self.on_add, self.on_update, self.on_delete, self.filter_fn = on_add, on_update, on_delete, filter_fn

    def add(self, obj):
        if self.filter_fn and not self.filter_fn(obj):
            return
        if self.on_add:
            self.on_add(obj)

    def update(self, old, new):
        if self.filter_fn:
            o, n = self.filter_fn(old), self.filter_fn(new)
            if o and not n:
                if self.on_delete:
                    self.on_delete(old)
                return
            if n and not o:
                if self.on_add:
                    self.on_add(new)
                return
            if not n:
                return
        if self.on_update:
            self.on_update(old, new)

    def delete(self, obj):
        if self.filter_fn and not self.filter_fn(obj):
            return
        if self.on_delete:
            self.on_delete(obj)


class Indexer:
    def __init__(self, indexers: dict | None = None):
        self.items: dict[str, dict] = {}
        self.indexers = indexers or {}
        self.indices: dict[str, dict[str, set]] = {n: {} for n in self.indexers}

    def _index(self, key, obj, remove=False):
        for name, fn in self.indexers.items():
            idx = self.indices[name]
            for v in fn(obj) or ():
                s = idx.setdefault(v, set())
                if remove:
                    s.discard(key)
                    if not s:
                        idx.pop(v, None)
                else:
                    s.add(key)

    def upsert(self, obj) -> dict | None:
        key = m.key_of(obj)
        old = self.items.get(key)
        if old is not None:
            self._index(key, old, remove=True)
        self.items[key] = obj
        self._index(key, obj)
        return old

    def delete(self, obj) -> dict | None:
        key = m.key_of(obj)
        old = self.items.pop(key, None)
        if old is not None:
            self._index(key, old, remove=True)
        return old

    def get(self, key: str) -> dict | None:
        return self.items.get(key)

    def list(self) -> list[dict]:
        return list(self.items.values())

    def by_index(self, name: str, value: str) -> list[dict]:
        return [self.items[k] for k in self.indices[name].get(value, ()) if k in self.items]

    def keys(self):
        return list(self.items)


class Informer:
    def __init__(self, client: Client, resource: str, ns: str = "", label_selector: str | None = None,
                 field_selector: str | None = None, resync: float = 0.0, indexers: dict | None = None,
                 watch_timeout: int | None = None):
        self.client, self.resource, self.ns = client, resource, ns
        self.label_selector, self.field_selector = label_selector, field_selector
        self.resync = resync
        self.indexer = Indexer(indexers)
        self.handlers: list[ResourceEventHandler] = []
        self.synced = asyncio.Event()
        self.last_rv = ""
        self._task: asyncio.Task | None = None
        self._resync_task: asyncio.Task | None = None
        self.watch_timeout = watch_timeout or random.randint(300, 600)
        self.relists = 0

    def add_handler(self, h: ResourceEventHandler | None = None, **kw):
        h = h or ResourceEventHandler(**kw)
        self.handlers.append(h)
        for obj in self.indexer.list():
            h.add(obj)
        return h

    def remove_handler(self, h: ResourceEventHandler):
        try:
            self.handlers.remove(h)
        except ValueError:
            pass

    def has_synced(self) -> bool:
        return self.synced.is_set()

    async def wait_synced(self, timeout: float | None = None):
        await asyncio.wait_for(self.synced.wait(), timeout)

    def start(self):
        if self._task is None:
            self._task = asyncio.create_task(self.run(), name=f"informer-{self.resource}")
            if self.resync:
                self._resync_task = asyncio.create_task(self._resync_loop())
        return self

    async def stop(self):
        for t in (self._task, self._resync_task):
            if t is not None:
                t.cancel()
                try:
                    await t
                except (asyncio.CancelledError, Exception):
                    pass
        self._task = self._resync_task = None

    # ------------------------------------------------------------ reflector
    async def _list(self):
        items, rv = await self.client.list(self.resource, self.ns, self.label_selector, self.field_selector)
        self.relists += 1
        seen = set()
        for obj in items:
            key = m.key_of(obj)
            seen.add(key)
            old = self.indexer.upsert(obj)
            for h in self.handlers:
                if old is None:
                    h.add(obj)
                elif m.rv_of(old) != m.rv_of(obj):
                    h.update(old, obj)
        for key in [k for k in self.indexer.keys() if k not in seen]:
            old = self.indexer.items.get(key)
            self.indexer.delete(old)
            for h in self.handlers:
                h.delete(old)
        self.last_rv = rv
        self.synced.set()

    async def run(self):
        backoff = 0.05
        need_list = True
        while True:
            try:
                if need_list:
                    await self._list()
                    need_list = False
                async for typ, obj in self.client.watch(self.resource, self.ns, self.last_rv, self.label_selector,
                                                        self.field_selector, self.watch_timeout):
                    self._dispatch(typ, obj)
                    backoff = 0.05
            except asyncio.CancelledError:
                raise
            except m.StatusError as e:
                if m.is_gone(e):
                    need_list = True
                    continue
                log.warning("informer %s watch error: %s", self.resource, e)
                need_list = True
            except Exception as e:  # connection errors: re-watch from last RV after backoff
                log.debug("informer %s watch interrupted: %r", self.resource, e)
            await asyncio.sleep(backoff)
            backoff = min(backoff * 2, 2.0)

    def _dispatch(self, typ, obj):
        rv = m.rv_of(obj)
        if rv:
            self.last_rv = rv
        if typ in (m.ADDED, m.MODIFIED):
            old = self.indexer.upsert(obj)
            for h in self.handlers:
                if old is None:
                    h.add(obj)
                else:
                    h.update(old, obj)
        elif typ == m.DELETED:
            old = self.indexer.delete(obj)
            for h in self.handlers:
                h.delete(old or obj)

    async def _resync_loop(self):
        while True:
            await asyncio.sleep(self.resync)
            for obj in self.indexer.list():
                for h in self.handlers:
                    h.update(obj, obj)

    # ----------------------------------------------------------- accessors
    def get(self, key: str):
        return self.indexer.get(key)

    def list(self):
        return self.indexer.list()


class SharedInformerFactory:
    def __init__(self, client: Client, resync: float = 0.0):
        self.client, self.resync = client, resync
        self.informers: dict[tuple, Informer] = {}

    def informer(self, resource, ns="", label_selector=None, field_selector=None, indexers=None) -> Informer:
        k = (resource, ns, label_selector, field_selector)
        if k not in self.informers:
            self.informers[k] = Informer(self.client, resource, ns, label_selector, field_selector, self.resync, indexers)
        return self.informers[k]

    def start(self):
        for inf in self.informers.values():
            inf.start()

    async def wait_for_cache_sync(self, timeout: float = 30.0):
        await asyncio.wait_for(asyncio.gather(*(i.synced.wait() for i in self.informers.values())), timeout)

    async def stop(self):
        for inf in self.informers.values():
            await inf.stop()
