"""Embedded MVCC key-value store with revisioned watch, compaction and WAL+snapshot.

Replaces external etcd v3 (reference SURVEY L0/U7: the apiserver's etcd3 adapter does
Create as `Txn(If ModRevision==0).Then(Put)` — staging/.../storage/etcd3/store.go:152-200 —
GuaranteedUpdate as a ModRevision CAS loop (:263) and Watch from a revision (:661)).

Design (single writer, in-process):
  * one global monotonically increasing revision; every KV keeps create/mod revision and
    a per-key version, exactly like etcd;
  * all mutations are compare-and-swap on mod_revision (0 == "must not exist");
  * an in-memory event history ring serves watch-from-revision; reading before the
    compaction point raises Compacted (HTTP 410 "too old resource version" upstream);
  * durability: an append-only WAL (one JSON line per committed revision) plus periodic
    snapshots; recovery = snapshot + WAL replay, revisions preserved;
  * watcher fan-out happens on commit with per-watcher queues; slow watchers whose queue
    exceeds `max_queue` are terminated (cacher.go behaviour) so they re-list.
Values are opaque bytes (the apiserver stores compact JSON).
"""
from __future__ import annotations

import asyncio
import base64
import collections
import fcntl
import json
import os
import random
import threading
import time


class KeyExists(Exception):
    pass


class KeyNotFound(Exception):
    pass


class CASFailed(Exception):
    def __init__(self, current):
        super().__init__("mod revision mismatch")
        self.current = current


class Compacted(Exception):
    def __init__(self, compact_rev):
        super().__init__(f"required revision has been compacted (compacted at {compact_rev})")
        self.compact_rev = compact_rev


class KV:
    # alt: the value in the other wire format (JSON <-> protobuf), filled on first demand by
    # store/storage.py; a KV never changes, so neither does its transcode
    __slots__ = ("key", "value", "create_rev", "mod_rev", "version", "alt")

    def __init__(self, key, value, create_rev, mod_rev, version):
        self.key, self.value, self.create_rev, self.mod_rev, self.version = key, value, create_rev, mod_rev, version
        self.alt = None

    def __repr__(self):
        return f"KV({self.key!r}, rev={self.mod_rev})"


PUT, DELETE = "PUT", "DELETE"


class Event:
    __slots__ = ("type", "kv", "prev", "rev", "cache", "prev_cache", "fields")

    def __init__(self, type_, kv, prev, rev):
        self.type, self.kv, self.prev, self.rev = type_, kv, prev, rev
        self.cache = None       # decoded-object cache shared by all watchers of this event
        self.prev_cache = None  # decoded previous object (filtered watchers)
        self.fields = None      # field-selector sets of cur/prev, computed once per event


class Watcher:
    """One watch. `transform(ev)` (optional) runs at commit time: it returns the item to queue, or
    None to drop the event, so a watcher never wakes up for events its filter rejects (the cacher
    fan-out: 100 kubelets watching spec.nodeName=<self> cost one dict probe each per pod event,
    not a decode + wakeup each)."""
    __slots__ = ("prefix", "exact", "queue", "closed", "store", "_loop", "err", "transform", "trigger")

    def __init__(self, store, prefix, exact, loop, transform=None, trigger=None):
        self.store, self.prefix, self.exact, self.transform = store, prefix, exact, transform
        self.trigger = trigger  # (fn, value): only events whose fn(ev) contains value can match
        self.queue: asyncio.Queue = asyncio.Queue()
        self.closed = False
        self.err = None
        self._loop = loop

    def wants(self, key: str) -> bool:
        return key == self.prefix if self.exact else key.startswith(self.prefix)

    def _deliver(self, ev):
        if self.closed:
            return
        if self.transform is not None:
            try:
                ev = self.transform(ev)
            except Exception as e:  # a broken filter must not break the writer's commit
                self.err = f"watch filter failed: {e!r}"
                self.close()
                return
            if ev is None:
                return
        if self.queue.qsize() >= self.store.max_queue:
            self.err = "watcher too slow"
            self.close()
            return
        self.queue.put_nowait(ev)

    def deliver(self, ev):
        try:
            running = asyncio.get_running_loop()
        except RuntimeError:
            running = None
        if running is self._loop:
            self._deliver(ev)
        else:
            self._loop.call_soon_threadsafe(self._deliver, ev)

    def close(self):
        if not self.closed:
            self.closed = True
            self.store._remove_watcher(self)
            try:
                self.queue.put_nowait(None)
            except Exception:  # pragma: no cover
                pass

    async def next(self, timeout: float | None = None):
        """Next Event, or None when closed/timeout."""
        if self.closed and self.queue.empty():
            return None
        try:
            if timeout is None:
                return await self.queue.get()
            return await asyncio.wait_for(self.queue.get(), timeout)
        except asyncio.TimeoutError:
            return None

    def __aiter__(self):
        return self

    async def __anext__(self):
        ev = await self.next()
        if ev is None:
            raise StopAsyncIteration
        return ev


class DataDirLocked(RuntimeError):
    pass


def lock_data_dir(path: str, wait: float = 10.0):
    """Hold `<path>/LOCK` (flock, exclusive) for as long as the returned file stays open: two
    processes appending one WAL or raft log would interleave records, so the second one
    waits up to `wait` seconds (a restarted static pod while the old process still exits)
    and then refuses (etcd takes the same lock on its WAL files: pkg/fileutil LockFile)."""
    os.makedirs(path, exist_ok=True)
    f = open(os.path.join(path, "LOCK"), "a+")
    deadline = time.monotonic() + wait
    while True:
        try:
            fcntl.flock(f.fileno(), fcntl.LOCK_EX | fcntl.LOCK_NB)
            f.seek(0)
            f.truncate()
            f.write(f"{os.getpid()}\n")
            f.flush()
            return f
        except BlockingIOError:
            if time.monotonic() >= deadline:
                f.seek(0)
                holder = f.read().strip() or "?"
                f.close()
                raise DataDirLocked(f"data directory {path} is in use by another process (pid {holder})") from None
            time.sleep(0.05)


class MVCCStore:
    def __init__(self, data_dir: str | None = None, history: int = 200_000, max_queue: int = 500_000,
                 snapshot_every: int = 50_000, fsync: bool = False, transformer=None, lock_wait: float = 10.0):
        self.kv: dict[str, KV] = {}
        # keys bucketed by their first two path components ("/registry/pods/"), so a range over one
        # resource never scans the others (admission lists quotas/limitranges on every create)
        self.buckets: dict[str, dict[str, KV]] = {}
        self._sorted: dict[str, list[str]] = {}
        self.rev = 0
        self.compact_rev = 0
        self.history: collections.deque[Event] = collections.deque()
        self.history_limit = history
        self.max_queue = max_queue
        self.watchers: list[Watcher] = []
        # trigger index (cacher.go triggerFunc, e.g. pods by spec.nodeName): (prefix, fn) -> value -> watchers.
        # fn(ev) returns every value a filter keyed on it could match (old and new object), so a
        # watcher outside that set is skipped without running its filter.
        self.triggered: dict[tuple, dict[str, list[Watcher]]] = {}
        self._lock = threading.RLock()
        self.data_dir = data_dir
        self.snapshot_every = snapshot_every
        self.fsync = fsync
        self._wal = None
        self._since_snapshot = 0
        self.commit_hooks = []  # fn(Event) called synchronously on commit (apiserver indexes)
        # value transformer between memory and disk (encryption at rest): to_disk(key, bytes),
        # from_disk(key, bytes); None keeps the bytes as they are
        self.transformer = transformer
        # fault injection: this share of conditional writes whose precondition holds
        # fails as if another writer had won the race, so every GuaranteedUpdate-style retry
        # loop above the store gets exercised (apiserver --store-conflict-chance)
        self.conflict_chance = 0.0
        self.injected_conflicts = 0
        self._dir_lock = None
        if data_dir:
            self._dir_lock = lock_data_dir(data_dir, lock_wait)
            try:
                self._recover()
            except BaseException:
                self._dir_lock.close()
                raise
            self._wal = open(os.path.join(data_dir, "wal.log"), "ab", buffering=0)

    # ----------------------------------------------------------------- reads
    def get(self, key: str) -> KV | None:
        return self.kv.get(key)

    @staticmethod
    def _bucket_of(key: str) -> str:
        i = key.find("/", 1)
        j = key.find("/", i + 1) if i >= 0 else -1
        return key[:j + 1] if j >= 0 else key

    def _index_put(self, key: str, kv: KV):
        b = self._bucket_of(key)
        bucket = self.buckets.setdefault(b, {})
        if key not in bucket:
            self._sorted.pop(b, None)
        bucket[key] = kv

    def _index_del(self, key: str):
        b = self._bucket_of(key)
        bucket = self.buckets.get(b)
        if bucket is not None and bucket.pop(key, None) is not None:
            self._sorted.pop(b, None)

    def _candidates(self, prefix: str) -> list[str]:
        b = self._bucket_of(prefix)
        # the bucket holds every match only when the prefix reaches a full "/a/b/" bucket
        if len(b) <= len(prefix) and prefix.startswith(b) and b.endswith("/") and b.count("/") >= 3:
            keys = self._sorted.get(b)
            if keys is None:
                keys = self._sorted[b] = sorted(self.buckets.get(b, ()))
            if b == prefix:
                return keys
            import bisect
            lo = bisect.bisect_left(keys, prefix)
            hi = bisect.bisect_left(keys, prefix + "￿")
            return keys[lo:hi]
        return sorted(k for k in self.kv if k.startswith(prefix))

    def range(self, prefix: str, limit: int = 0, start_after: str | None = None):
        """Keys with `prefix`, sorted; returns (kvs, rev, more)."""
        with self._lock:
            keys = self._candidates(prefix)
            if start_after is not None:
                import bisect
                keys = keys[bisect.bisect_right(keys, start_after):]
            more = False
            if limit and len(keys) > limit:
                keys, more = keys[:limit], True
            return [self.kv[k] for k in keys], self.rev, more

    def count(self, prefix: str) -> int:
        return len(self._candidates(prefix))

    # ------------------------------------------------------------- mutations
    def put(self, key: str, value, expect_mod_rev: int | None = None) -> KV:
        """CAS put. expect_mod_rev: None = unconditional, 0 = must not exist, n = must match.

        `value` may be bytes or a callable rev -> bytes (lets the caller embed the commit
        revision, e.g. metadata.resourceVersion, into the stored bytes).
        """
        with self._lock:
            cur = self.kv.get(key)
            if expect_mod_rev is not None:
                if expect_mod_rev == 0 and cur is not None:
                    raise KeyExists(key)
                if expect_mod_rev and (cur is None or cur.mod_rev != expect_mod_rev):
                    if cur is None:
                        raise KeyNotFound(key)
                    raise CASFailed(cur)
                if expect_mod_rev:
                    self._inject_conflict(cur)
            rev = self.rev + 1
            data = value(rev) if callable(value) else value
            new = KV(key, data, cur.create_rev if cur else rev, rev, (cur.version + 1) if cur else 1)
            self.rev = rev
            self.kv[key] = new
            self._index_put(key, new)
            self._commit(Event(PUT, new, cur, rev), {"r": rev, "o": "p", "k": key, "v": data} if self._wal is not None else None)
            return new

    def _inject_conflict(self, cur):
        if self.conflict_chance and cur is not None and random.random() < self.conflict_chance:
            self.injected_conflicts += 1
            raise CASFailed(cur)

    def delete(self, key: str, expect_mod_rev: int | None = None) -> KV:
        with self._lock:
            cur = self.kv.get(key)
            if cur is None:
                raise KeyNotFound(key)
            if expect_mod_rev and cur.mod_rev != expect_mod_rev:
                raise CASFailed(cur)
            if expect_mod_rev:
                self._inject_conflict(cur)
            rev = self.rev + 1
            self.rev = rev
            del self.kv[key]
            self._index_del(key)
            tomb = KV(key, cur.value, cur.create_rev, rev, 0)
            self._commit(Event(DELETE, tomb, cur, rev), {"r": rev, "o": "d", "k": key})
            return cur

    def batch(self, ops: list[tuple]) -> tuple[int, list]:
        """Apply [("put", key, value) | ("delete", key)] at ONE new revision, as an etcd Txn
        branch does. Returns (revision, [previous KV or None per op]); a batch that changes
        nothing (only deletes of absent keys) does not advance the revision."""
        with self._lock:
            rev = self.rev + 1
            prevs, staged = [], []
            for op in ops:
                key = op[1]
                cur = self.kv.get(key)
                prevs.append(cur)
                if op[0] == "put":
                    data = op[2](rev) if callable(op[2]) else op[2]
                    new = KV(key, data, cur.create_rev if cur else rev, rev, (cur.version + 1) if cur else 1)
                    self.kv[key] = new
                    self._index_put(key, new)
                    staged.append((Event(PUT, new, cur, rev), {"r": rev, "o": "p", "k": key, "v": data} if self._wal is not None else None))
                elif cur is not None:
                    del self.kv[key]
                    self._index_del(key)
                    staged.append((Event(DELETE, KV(key, cur.value, cur.create_rev, rev, 0), cur, rev), {"r": rev, "o": "d", "k": key}))
            if not staged:
                return self.rev, prevs
            self.rev = rev
            for ev, rec in staged:
                self._commit(ev, rec)
            return rev, prevs

    def _disk(self, key: str, data: bytes) -> str:
        return _b(self.transformer.to_disk(key, data) if self.transformer is not None else data)

    def _undisk(self, key: str, s: str) -> bytes:
        data = _unb(s)
        return self.transformer.from_disk(key, data) if self.transformer is not None else data

    def _commit(self, ev: Event, rec: dict | None):
        if self._wal is not None and rec is not None:
            if "v" in rec:
                rec["v"] = self._disk(rec["k"], rec["v"])
            self._wal.write((json.dumps(rec, separators=(",", ":")) + "\n").encode())
            if self.fsync:
                os.fsync(self._wal.fileno())
            self._since_snapshot += 1
            if self._since_snapshot >= self.snapshot_every:
                self.snapshot()
        self.history.append(ev)
        if len(self.history) > self.history_limit:
            old = self.history.popleft()
            self.compact_rev = old.rev
        for h in self.commit_hooks:
            h(ev)
        key = ev.kv.key
        for w in list(self.watchers):
            if w.wants(key):
                w.deliver(ev)
        if self.triggered:
            for (prefix, fn), idx in list(self.triggered.items()):
                if not key.startswith(prefix):
                    continue
                for v in fn(ev):
                    for w in list(idx.get(v, ())):
                        if w.wants(key):
                            w.deliver(ev)

    def compact(self, rev: int):
        """Drop history at or below `rev` (etcd Compact)."""
        with self._lock:
            while self.history and self.history[0].rev <= rev:
                self.history.popleft()
            self.compact_rev = max(self.compact_rev, min(rev, self.rev))

    # ----------------------------------------------------------------- watch
    def watch(self, prefix: str, start_rev: int = 0, exact: bool = False, transform=None, trigger=None) -> Watcher:
        """Events with rev >= start_rev (0 = from now on). `trigger=(fn, value)` indexes the
        watcher (see self.triggered); it is an optimisation only, `transform` stays the filter."""
        loop = asyncio.get_running_loop()
        with self._lock:
            if start_rev and start_rev <= self.compact_rev:
                raise Compacted(self.compact_rev)
            w = Watcher(self, prefix, exact, loop, transform, None if exact else trigger)
            if start_rev:
                for ev in self.history:
                    if ev.rev >= start_rev and w.wants(ev.kv.key):
                        item = ev if transform is None else transform(ev)
                        if item is not None:
                            w.queue.put_nowait(item)
            if w.trigger is not None:
                fn, value = w.trigger
                self.triggered.setdefault((prefix, fn), {}).setdefault(value, []).append(w)
            else:
                self.watchers.append(w)
            return w

    def all_watchers(self) -> list[Watcher]:
        out = list(self.watchers)
        for idx in self.triggered.values():
            for ws in idx.values():
                out.extend(ws)
        return out

    def _remove_watcher(self, w):
        with self._lock:
            if w.trigger is None:
                try:
                    self.watchers.remove(w)
                except ValueError:
                    pass
                return
            fn, value = w.trigger
            idx = self.triggered.get((w.prefix, fn))
            if idx is None:
                return
            ws = idx.get(value)
            if ws and w in ws:
                ws.remove(w)
                if not ws:
                    del idx[value]
                    if not idx:
                        del self.triggered[(w.prefix, fn)]

    # ------------------------------------------------------------ durability
    def snapshot(self):
        if not self.data_dir:
            return
        path = os.path.join(self.data_dir, "snapshot.json")
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"rev": self.rev, "compact_rev": self.compact_rev,
                       "kv": [[k.key, self._disk(k.key, k.value), k.create_rev, k.mod_rev, k.version]
                              for k in self.kv.values()]}, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
        if self._wal is not None:
            self._wal.close()
        self._wal = open(os.path.join(self.data_dir, "wal.log"), "wb", buffering=0)
        self._since_snapshot = 0

    def dump_state(self) -> dict:
        """The whole keyspace at this revision (a raft snapshot of the store)."""
        with self._lock:
            return {"rev": self.rev, "compact_rev": self.compact_rev,
                    "kv": [[k.key, _b(k.value), k.create_rev, k.mod_rev, k.version] for k in self.kv.values()]}

    def load_state(self, st: dict):
        """Replace the keyspace with a dumped one (raft InstallSnapshot): history restarts at its
        revision and every open watch ends (its clients re-list)."""
        with self._lock:
            self.kv.clear()
            self.buckets.clear()
            self._sorted.clear()
            for key, v, cr, mr, ver in st["kv"]:
                kv = self.kv[key] = KV(key, _unb(v), cr, mr, ver)
                self._index_put(key, kv)
            self.rev = st["rev"]
            self.compact_rev = max(st.get("compact_rev", 0), st["rev"])
            self.history.clear()
        for w in self.all_watchers():
            w.err = "store restored from a snapshot"
            w.close()

    def _recover(self):
        snap = os.path.join(self.data_dir, "snapshot.json")
        snap_rev = 0
        if os.path.exists(snap):
            with open(snap) as f:
                s = json.load(f)
            self.rev = s["rev"]
            self.compact_rev = snap_rev = s["rev"]
            for key, v, cr, mr, ver in s["kv"]:
                self.kv[key] = KV(key, self._undisk(key, v), cr, mr, ver)
        wal = os.path.join(self.data_dir, "wal.log")
        if os.path.exists(wal):
            with open(wal, "rb") as f:
                for line in f:
                    try:
                        rec = json.loads(line)
                    except ValueError:
                        break  # torn tail write
                    r = rec["r"]
                    if r <= snap_rev:       # a batch writes several records at one revision
                        continue
                    key = rec["k"]
                    cur = self.kv.get(key)
                    if rec["o"] == "p":
                        self.kv[key] = KV(key, self._undisk(key, rec["v"]), cur.create_rev if cur else r, r,
                                          (cur.version + 1) if cur else 1)
                    else:
                        self.kv.pop(key, None)
                    self.rev = r
            self.compact_rev = self.rev
        for key, kv in self.kv.items():
            self._index_put(key, kv)

    def close(self):
        for w in self.all_watchers():
            w.close()
        if self._wal is not None:
            self._wal.close()
            self._wal = None
        if self._dir_lock is not None:
            self._dir_lock.close()             # releases the flock
            self._dir_lock = None


def _b(v: bytes) -> str:
    try:
        return v.decode()
    except UnicodeDecodeError:
        return "b64:" + base64.b64encode(v).decode()


def _unb(s: str) -> bytes:
    if s.startswith("b64:"):
        return base64.b64decode(s[4:])
    return s.encode()


def now() -> float:
    return time.time()
