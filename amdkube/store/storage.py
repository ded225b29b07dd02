"""storage.Interface over the MVCC store: typed (JSON) objects, preconditions, CAS update
loops, filtered list and watch with in/out-of-filter event translation.

Reference: staging/src/k8s.io/apiserver/pkg/storage/interfaces.go (Interface), etcd3
store.go:152 (Create), :263 (GuaranteedUpdate: read → tryUpdate → CAS, retry on
conflict), :477 (List), :661 (Watch); cacher.go:292/:469 (watch fan-out with filter,
where an object leaving the filter is delivered as DELETED and entering as ADDED).

Objects are stored as compact JSON whose metadata.resourceVersion already equals the
commit revision (embedded at commit time), so GET/LIST/WATCH can stream stored bytes
without re-encoding. With `--storage-media-type application/vnd.kubernetes.protobuf` a
Storage writes the reference's etcd format instead: the `k8s\x00` protobuf envelope
(api/protobuf.py), falling back to JSON for kinds without a protobuf schema and for objects
that would lose amdkube-only fields in the typed encoding. Reads sniff the magic, so a store
may hold both (as one migrating between media types does).
"""
from __future__ import annotations

import json
from typing import Callable

from ..api import meta as m
from .mvcc import CASFailed, Compacted, KeyExists, KeyNotFound, MVCCStore, PUT, DELETE, Event


PROTO_MAGIC = b"k8s\x00"
JSON_MEDIA_TYPE = "application/json"
PROTO_MEDIA_TYPE = "application/vnd.kubernetes.protobuf"


def _with_rv(obj: dict, media_type: str = JSON_MEDIA_TYPE):
    def build(rev: int) -> bytes:
        obj.setdefault("metadata", {})["resourceVersion"] = str(rev)
        if media_type == PROTO_MEDIA_TYPE:
            from ..api import protobuf as pb
            if pb.supports(obj):
                data, ok = pb.encode_checked(obj)
                if ok:
                    return data
        return json.dumps(obj, separators=(",", ":")).encode()
    return build


def decode_kv(value: bytes) -> dict:
    if value[:4] == PROTO_MAGIC:
        from ..api import protobuf as pb
        return pb.decode(value)
    return json.loads(value)


def json_bytes(value: bytes) -> bytes:
    """The stored value as JSON bytes (transcoding a protobuf-stored object)."""
    if value[:4] == PROTO_MAGIC:
        return json.dumps(decode_kv(value), separators=(",", ":")).encode()
    return value


# Serving the format a KV is NOT stored in costs a transcode. A KV is immutable, so the transcode
# is done once and kept on it (the reference's later cachingObject, which memoizes each object's
# serialization per encoding for all watchers and lists: apiserver/pkg/storage/cacher/
# caching_object.go). A LIST in the other format is then a splice of cached bytes.
def kv_json(kv) -> bytes:
    v = kv.value
    if v[:4] != PROTO_MAGIC:
        return v
    alt = kv.alt
    if alt is None:
        alt = kv.alt = json_bytes(v)
    return alt


def kv_proto(kv) -> bytes | None:
    """The KV's object as a `k8s\x00` protobuf envelope; None for kinds without a protobuf schema."""
    v = kv.value
    if v[:4] == PROTO_MAGIC:
        return v
    alt = kv.alt
    if alt is None:
        from ..api import protobuf as pb
        try:
            obj = json.loads(v)
            alt = pb.encode(obj) if isinstance(obj, dict) and pb.supports(obj) else b""
        except (ValueError, pb.ProtoError):
            alt = b""
        kv.alt = alt
    return alt or None


def event_object(ev: Event) -> dict:
    """Decoded object for an event (cached on the event, shared read-only)."""
    if ev.cache is None:
        if ev.type == PUT:
            ev.cache = decode_kv(ev.kv.value)
        else:
            o = decode_kv(ev.prev.value)
            o.setdefault("metadata", {})["resourceVersion"] = str(ev.rev)
            ev.cache = o
    return ev.cache


def event_prev_object(ev: Event) -> dict | None:
    if ev.prev is None:
        return None
    if ev.prev_cache is None:
        ev.prev_cache = decode_kv(ev.prev.value)
    return ev.prev_cache


class Filter:
    """Label/field predicate (storage.SelectionPredicate)."""
    __slots__ = ("label", "field", "fields_fn")

    def __init__(self, label=None, field=None, fields_fn: Callable | None = None):
        self.label, self.field, self.fields_fn = label, field, fields_fn

    def empty(self) -> bool:
        return (self.label is None or self.label.empty()) and (self.field is None or self.field.empty())

    def fields_of(self, obj: dict) -> dict:
        return self.fields_fn(obj) if self.fields_fn else {"metadata.name": m.name_of(obj),
                                                           "metadata.namespace": m.namespace_of(obj)}

    def matches(self, obj: dict, fields: dict | None = None) -> bool:
        if self.label is not None and not self.label.empty():
            if not self.label.matches(m.labels_of(obj)):
                return False
        if self.field is not None and not self.field.empty():
            if not self.field.matches(fields if fields is not None else self.fields_of(obj)):
                return False
        return True

    def matches_event(self, ev: Event, obj: dict, which: int) -> bool:
        """matches() with the field set cached on the event (computed once for all watchers)."""
        if self.field is None or self.field.empty():
            return self.matches(obj)
        key = (which, self.fields_fn)
        fc = ev.fields
        if fc is None:
            fc = ev.fields = {}
        f = fc.get(key)
        if f is None:
            f = fc[key] = self.fields_of(obj)
        return self.matches(obj, f)


_TRIGGERS: dict[tuple, Callable] = {}


def field_trigger(fields_fn: Callable, field: str) -> Callable:
    """Trigger function for exact `field=value` watches: the field's value in the new and the
    old object of an event (one shared function per (fields_fn, field), so the store groups all
    such watchers under one index). Uses the same per-event field cache as Filter.matches_event."""
    key = (fields_fn, field)
    fn = _TRIGGERS.get(key)
    if fn is None:
        def fn(ev: Event, _fields_fn=fields_fn, _field=field):
            fc = ev.fields
            if fc is None:
                fc = ev.fields = {}
            f0 = fc.get((0, _fields_fn))
            if f0 is None:
                f0 = fc[(0, _fields_fn)] = _fields_fn(event_object(ev))
            vals = {f0.get(_field, "")}
            if ev.prev is not None and ev.type == PUT:
                f1 = fc.get((1, _fields_fn))
                if f1 is None:
                    f1 = fc[(1, _fields_fn)] = _fields_fn(event_prev_object(ev))
                vals.add(f1.get(_field, ""))
            return vals
        _TRIGGERS[key] = fn
    return fn


class Storage:
    # fields whose exact-match watches are indexed (cacher.go: pods by spec.nodeName)
    TRIGGER_FIELDS = ("spec.nodeName", "metadata.name")      # + each kubelet's watch of its own Node

    def __init__(self, store: MVCCStore, resource: str = "object", media_type: str = JSON_MEDIA_TYPE):
        self.store = store
        self.resource = resource
        self.media_type = media_type

    # -------------------------------------------------------------- basic ops
    def create(self, key: str, obj: dict) -> dict:
        try:
            self.store.put(key, _with_rv(obj, self.media_type), expect_mod_rev=0)
        except KeyExists:
            raise m.already_exists(self.resource, key.rsplit("/", 1)[-1])
        return obj

    def get(self, key: str, ignore_not_found=False) -> dict | None:
        kv = self.store.get(key)
        if kv is None:
            if ignore_not_found:
                return None
            raise m.not_found(self.resource, key.rsplit("/", 1)[-1])
        return decode_kv(kv.value)

    def get_raw(self, key: str) -> bytes | None:
        """The object as JSON bytes (stored bytes when stored as JSON)."""
        kv = self.store.get(key)
        return kv_json(kv) if kv else None

    def guaranteed_update(self, key: str, try_update: Callable[[dict], dict | None],
                          precond_uid: str | None = None, precond_rv: str | None = None,
                          ignore_not_found=False, max_retries: int = 100) -> dict:
        """Read-modify-CAS loop. try_update returns the new object (or None = no change).

        A precondition on resourceVersion turns a CAS miss into a Conflict error instead of
        a retry (optimistic concurrency for client updates).
        """
        for _ in range(max_retries):
            kv = self.store.get(key)
            if kv is None:
                if not ignore_not_found:
                    raise m.not_found(self.resource, key.rsplit("/", 1)[-1])
                cur, mod = None, 0
            else:
                cur, mod = decode_kv(kv.value), kv.mod_rev
                if precond_uid and m.uid_of(cur) != precond_uid:
                    raise m.conflict(self.resource, m.name_of(cur),
                                     f"Precondition failed: UID in precondition: {precond_uid}, UID in object meta: {m.uid_of(cur)}")
                if precond_rv and precond_rv != str(mod):
                    raise m.conflict(self.resource, m.name_of(cur),
                                     "the object has been modified; please apply your changes to the latest version and try again")
            new = try_update(cur)
            if new is None:
                return cur
            try:
                self.store.put(key, _with_rv(new, self.media_type), expect_mod_rev=mod)
                return new
            except (CASFailed, KeyExists, KeyNotFound):
                continue
        raise m.conflict(self.resource, key, "too many conflicting updates")

    def delete(self, key: str, precond_uid: str | None = None, precond_rv: str | None = None) -> dict:
        while True:
            kv = self.store.get(key)
            if kv is None:
                raise m.not_found(self.resource, key.rsplit("/", 1)[-1])
            cur = decode_kv(kv.value)
            if precond_uid and m.uid_of(cur) != precond_uid:
                raise m.conflict(self.resource, m.name_of(cur), "Precondition failed: UID mismatch")
            if precond_rv and precond_rv != str(kv.mod_rev):
                raise m.conflict(self.resource, m.name_of(cur), "the object has been modified")
            try:
                self.store.delete(key, expect_mod_rev=kv.mod_rev)
            except CASFailed:
                continue
            except KeyNotFound:
                raise m.not_found(self.resource, key.rsplit("/", 1)[-1])
            cur["metadata"]["resourceVersion"] = str(self.store.rev)
            return cur

    def list(self, prefix: str, flt: Filter | None = None, limit: int = 0, continue_key: str | None = None):
        """Returns (items, list_rv, continue_token)."""
        kvs, rev, more = self.store.range(prefix, 0, continue_key)
        items, last = [], None
        for kv in kvs:
            o = decode_kv(kv.value)
            if flt is None or flt.matches(o):
                items.append(o)
                last = kv.key
                if limit and len(items) >= limit:
                    break
        cont = None
        if limit and len(items) >= limit and last is not None and kvs and last != kvs[-1].key:
            cont = last
        return items, rev, cont

    def list_raw(self, prefix: str):
        kvs, rev, _ = self.store.range(prefix)
        return [kv_json(kv) for kv in kvs], rev

    # ------------------------------------------------------------------ watch
    def watch(self, prefix: str, rv: str | int | None, flt: Filter | None = None, exact=False) -> "FilteredWatch":
        start = int(rv) + 1 if rv not in (None, "", "0", 0) else 0
        fw = FilteredWatch(None, flt)
        trigger = None
        if flt is not None and flt.fields_fn is not None and flt.field is not None:
            for f, op, v in flt.field.terms:
                if op == "=" and f in self.TRIGGER_FIELDS:
                    trigger = (field_trigger(flt.fields_fn, f), v)
                    break
        try:
            fw.w = self.store.watch(prefix, start, exact, transform=fw._translate, trigger=trigger)
        except Compacted as e:
            raise m.gone(f"too old resource version: {rv} ({e.compact_rev})")
        return fw


class FilteredWatch:
    """Translates raw KV events into (type, obj, ev) honouring a filter (cacher semantics).

    The translation runs as the store watcher's commit-time transform, so the queue only ever
    holds events this watch delivers, already translated.
    """

    def __init__(self, w, flt: Filter | None):
        self.w, self.flt = w, flt if (flt is not None and not flt.empty()) else None

    def close(self):
        self.w.close()

    @property
    def closed(self):
        return self.w.closed

    def _translate(self, ev: Event):
        obj = event_object(ev)
        if self.flt is None:
            if ev.type == DELETE:
                return m.DELETED, obj, ev
            return (m.ADDED if ev.prev is None else m.MODIFIED), obj, ev
        cur_ok = ev.type == PUT and self.flt.matches_event(ev, obj, 0)
        prev_ok = False
        if ev.prev is not None:
            if ev.type == DELETE:
                prev_ok = self.flt.matches_event(ev, obj, 0)
            else:
                prev_ok = self.flt.matches_event(ev, event_prev_object(ev), 1)
        if ev.type == DELETE:
            return (m.DELETED, obj, ev) if prev_ok else None
        if cur_ok and prev_ok:
            return m.MODIFIED, obj, ev
        if cur_ok:
            return m.ADDED, obj, ev
        if prev_ok:
            return m.DELETED, obj, ev
        return None

    async def next(self, timeout: float | None = None):
        """(type, obj, raw_event) or None when closed / timed out."""
        return await self.w.next(timeout)

    def __aiter__(self):
        return self

    async def __anext__(self):
        r = await self.next()
        if r is None:
            raise StopAsyncIteration
        return r
