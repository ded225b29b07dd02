"""The garbage collector: an ownerReference dependency graph kept current from watch events.

Reference: pkg/controller/garbagecollector/
  * graph.go — a node per object uid: its identity, owners, dependents, and the beingDeleted /
    deletingDependents / virtual flags; blockingDependents (:138).
  * graph_builder.go — one monitor per deletable resource (syncMonitors :222, the ignored
    resources :354); processGraphChanges (:586) inserts and removes nodes, makes a "virtual"
    node for an owner not seen yet (addDependentToOwners :391), diffs ownerReferences on update
    (referencesDiffs :451, addUnblockedOwnersToDeleteQueue :538) and turns the start of a
    foreground or orphan deletion into work (processTransitions :563).
  * garbagecollector.go — attemptToDeleteItem (:363): the owners are classified solid / dangling
    / waitingForDependentsDeletion (:330); dangling and waiting refs are patched out while a
    solid owner remains; with no solid owner the object is deleted with the propagation its
    finalizers ask for; processDeletingDependentsItem (:480) keeps a foreground-deleted owner
    until every blockOwnerDeletion dependent is gone; attemptToOrphanWorker (:538); Sync
    (:169) re-reads discovery and resyncs the monitors when the resource set changes;
    GetDeletableResources (:594).
  * patch.go — deleteOwnerRefPatch (:29), patchToUnblockOwnerReferences (:40).
  * uid_cache.go — the LRU absentOwnerCache.

The graph is updated inline from the informer callbacks (one event loop, so no lock is needed);
the attemptToDelete and attemptToOrphan queues are worked by async workers. Work is per event:
an update that changes no ownerReference costs a dict lookup, and nothing rescans the cluster.
Custom resources have no strategic-merge schema, so their ownerReference patches fall back to a
JSON patch guarded by the object's resourceVersion.
"""
from __future__ import annotations

import asyncio
import collections
import json
import logging

from ..api import meta as m
from ..api.scheme import SCHEME, ResourceInfo
from ..client.informer import Informer, ResourceEventHandler
from ..client.workqueue import RateLimitingQueue, ShutDown
from .base import Controller

log = logging.getLogger("amdkube.controllers.gc")

FINALIZER_ORPHAN = "orphan"
FINALIZER_DELETE_DEPENDENTS = "foregroundDeletion"
ADD, UPDATE, DELETE = "add", "update", "delete"

# graph_builder.go ignoredResources (:354), as (group, resource)
IGNORED_RESOURCES = frozenset({
    ("extensions", "replicationcontrollers"), ("", "bindings"), ("", "componentstatuses"), ("", "events"),
    ("authentication.k8s.io", "tokenreviews"), ("authorization.k8s.io", "subjectaccessreviews"),
    ("authorization.k8s.io", "selfsubjectaccessreviews"), ("authorization.k8s.io", "localsubjectaccessreviews"),
    ("authorization.k8s.io", "selfsubjectrulesreviews"), ("apiregistration.k8s.io", "apiservices"),
    ("apiextensions.k8s.io", "customresourcedefinitions"),
})


class RestMappingError(Exception):
    """errors.go restMappingError: a reference to a kind discovery does not (yet) know."""

    def __init__(self, kind, version):
        super().__init__(f"unable to get REST mapping for kind: {kind}, version: {version}")


# ---------------------------------------------------------------------------- graph
class ObjectReference:
    """graph.go objectReference: an OwnerReference plus the namespace."""
    __slots__ = ("api_version", "kind", "name", "uid", "namespace")

    def __init__(self, api_version="", kind="", name="", uid="", namespace=""):
        self.api_version, self.kind, self.name, self.uid, self.namespace = api_version, kind, name, uid, namespace

    @classmethod
    def from_owner(cls, ref: dict, namespace: str):
        return cls(ref.get("apiVersion", ""), ref.get("kind", ""), ref.get("name", ""), ref.get("uid", ""), namespace)

    def __repr__(self):
        return f"[{self.api_version}/{self.kind}, namespace: {self.namespace}, name: {self.name}, uid: {self.uid}]"


class Node:
    __slots__ = ("identity", "dependents", "owners", "deleting_dependents", "being_deleted", "virtual", "__weakref__")

    def __init__(self, identity: ObjectReference, owners=None, virtual=False, being_deleted=False,
                 deleting_dependents=False):
        self.identity = identity
        self.dependents: set[Node] = set()
        self.owners: list[dict] = list(owners or [])
        self.virtual = virtual
        self.being_deleted = being_deleted
        self.deleting_dependents = deleting_dependents

    def is_observed(self) -> bool:
        return not self.virtual

    def blocking_dependents(self) -> list:
        """Dependents whose reference to this node has blockOwnerDeletion set."""
        uid = self.identity.uid
        return [d for d in self.dependents
                if any(o.get("uid") == uid and o.get("blockOwnerDeletion") is True for o in d.owners)]

    def __repr__(self):
        return f"node{self.identity!r}"


def references_diffs(old: list, new: list):
    """referencesDiffs (:451): (added, removed, changed pairs) keyed by owner uid."""
    o = {r.get("uid"): r for r in old or []}
    n = {r.get("uid"): r for r in new or []}
    added = [r for u, r in n.items() if u not in o]
    removed = [r for u, r in o.items() if u not in n]
    changed = [(o[u], n[u]) for u in n if u in o and o[u] != n[u]]
    return added, removed, changed


def delete_owner_ref_patch(dependent_uid: str, *owner_uids: str) -> dict:
    """deleteOwnerRefPatch: a strategic merge patch deleting the refs; the uid is a precondition."""
    return {"metadata": {"ownerReferences": [{"$patch": "delete", "uid": u} for u in owner_uids], "uid": dependent_uid}}


def patch_to_unblock_owner_references(n: Node) -> dict:
    """patchToUnblockOwnerReferences: every blocking reference re-sent with blockOwnerDeletion false."""
    refs = [dict(o, blockOwnerDeletion=False) for o in n.owners if o.get("blockOwnerDeletion") is True]
    return {"metadata": {"ownerReferences": refs, "uid": n.identity.uid}}


class UIDCache:
    """uid_cache.go: an LRU set of uids (the owners known to be absent)."""

    def __init__(self, max_entries: int):
        self.max = max_entries
        self._d: collections.OrderedDict = collections.OrderedDict()

    def add(self, uid):
        self._d[uid] = None
        self._d.move_to_end(uid)
        while len(self._d) > self.max:
            self._d.popitem(last=False)

    def has(self, uid) -> bool:
        if uid in self._d:
            self._d.move_to_end(uid)
            return True
        return False


def _being_deleted(obj) -> bool:
    return bool((obj.get("metadata") or {}).get("deletionTimestamp"))


def _has_finalizer(obj, f) -> bool:
    return f in ((obj.get("metadata") or {}).get("finalizers") or [])


def _deletion_starts(old, new) -> bool:
    """deletionStarts (:482): the event takes the object into deletion (no old object: it is
    being deleted already)."""
    if old is None:
        return _being_deleted(new)
    return _being_deleted(new) and not _being_deleted(old)


def parse_group_version(gv: str):
    """schema.ParseGroupVersion: '' → core, 'v1' → ('', 'v1'), 'g/v' → (g, v); None if invalid."""
    if not gv:
        return "", ""
    if gv == "v1":
        return "", "v1"
    parts = gv.split("/")
    if len(parts) == 1:
        return "", parts[0]
    if len(parts) == 2 and parts[0] and parts[1]:
        return parts[0], parts[1]
    return None


DELETABLE_VERBS = ("delete", "list", "watch")


def deletable_resources(resource_lists) -> dict:
    """GetDeletableResources (:594) over preferred resource lists: (group, version, resource) →
    the APIResource entry, for every resource supporting delete, list and watch (subresources and
    unparsable group versions skipped)."""
    out = {}
    for rl in resource_lists or []:
        gv = parse_group_version(rl.get("groupVersion", ""))
        if gv is None:
            log.warning("ignoring invalid discovered resource %r", rl.get("groupVersion"))
            continue
        for r in rl.get("resources") or []:
            if "/" in r.get("name", ""):
                continue
            verbs = set(r.get("verbs") or ())
            if all(v in verbs for v in DELETABLE_VERBS):
                out[(gv[0], gv[1], r["name"])] = r
    return out


async def server_preferred_resources(client):
    """discovery ServerPreferredResources: the core v1 list and each group's preferred version.
    Returns (resource lists, errors): a group that fails is reported and the rest still count
    (ErrGroupDiscoveryFailed)."""
    lists, errs = [], []

    async def get(path):
        try:
            return await client.request("GET", path)
        except Exception as e:
            errs.append(f"{path}: {e!r}")
            return None
    core = await get("/api")
    for v in (core or {}).get("versions") or []:
        rl = await get(f"/api/{v}")
        if rl:
            lists.append(rl)
    for g in ((await get("/apis")) or {}).get("groups") or []:
        pv = ((g.get("preferredVersion") or {}).get("groupVersion")) or \
            ((g.get("versions") or [{}])[0].get("groupVersion"))
        if pv:
            rl = await get(f"/apis/{pv}")
            if rl:
                lists.append(rl)
    return lists, errs


# ---------------------------------------------------------------------------- graph builder
class Monitor:
    def __init__(self, ri: ResourceInfo, informer: Informer, handler, owned: bool):
        self.ri, self.informer, self.handler, self.owned = ri, informer, handler, owned

    def has_synced(self) -> bool:
        return self.informer.has_synced()


class GraphBuilder:
    def __init__(self, attempt_to_delete, attempt_to_orphan, absent_owner_cache: UIDCache, client=None,
                 factory=None, ignored=IGNORED_RESOURCES):
        self.uid_to_node: dict[str, Node] = {}
        self.attempt_to_delete = attempt_to_delete
        self.attempt_to_orphan = attempt_to_orphan
        self.absent_owner_cache = absent_owner_cache
        self.client, self.factory, self.ignored = client, factory, ignored
        self.monitors: dict[tuple, Monitor] = {}
        self.running = False
        self.graph_changes: collections.deque = collections.deque()
        self._draining = False
        self.events_processed = 0

    # ------------------------------------------------------------- monitors
    def _canonical(self, key):
        g, v, r = key
        ri = SCHEME.served(g, v, r)
        if ri is None:
            return (g, r)
        return SCHEME.storage_of(ri).group, SCHEME.storage_of(ri).plural

    def sync_monitors(self, resources: dict) -> list:
        """syncMonitors (:222): keep monitors of resources still present, add the new ones, stop
        the rest. An alias version of a resource shares its storage (one monitor per object set).
        Returns the errors of resources that could not be monitored."""
        errs = []
        current: dict[tuple, Monitor] = {}
        seen_storage = {self._canonical(k): k for k in self.monitors if k in resources}
        to_remove = dict(self.monitors)
        for key, r in sorted(resources.items()):
            g, v, plural = key
            if (g, plural) in self.ignored:
                continue
            if key in to_remove:
                current[key] = to_remove.pop(key)
                continue
            canon = self._canonical(key)
            if canon in seen_storage and seen_storage[canon] != key:
                continue
            ri = SCHEME.served(g, v, plural)
            if ri is None:
                if not r.get("kind"):
                    errs.append(f"couldn't look up resource {key}")
                    continue
                ri = ResourceInfo(g, v, r["kind"], plural, bool(r.get("namespaced")), tuple(r.get("shortNames") or ()))
                SCHEME.add(ri)
            seen_storage[canon] = key
            current[key] = self._monitor_for(ri)
        self.monitors = current
        for mon in to_remove.values():
            self._stop_monitor(mon)
        return errs

    def _monitor_for(self, ri: ResourceInfo) -> Monitor:
        gvk = (ri.api_version, ri.kind)
        h = ResourceEventHandler(on_add=lambda o, k=gvk: self.enqueue((ADD, o, None, k)),
                                 on_update=lambda old, o, k=gvk: self.enqueue((UPDATE, o, old, k)),
                                 on_delete=lambda o, k=gvk: self.enqueue((DELETE, o, None, k)))
        shared = None
        if self.factory is not None:
            for name in (ri.plural, ri.group_resource):
                shared = self.factory.informers.get((name, "", None, None))
                named = SCHEME.resolve(name)
                if shared is not None and named is not None and SCHEME.storage_of(named) is SCHEME.storage_of(ri):
                    break
                shared = None
        if shared is not None:
            return Monitor(ri, shared, h, owned=False)
        inf = Informer(self.client, f"{ri.plural}.{ri.group}" if ri.group else ri.plural)
        return Monitor(ri, inf, h, owned=True)

    def start_monitors(self):
        """startMonitors (:275): attach the handler (a shared informer replays its store) and run
        the informers the GC owns."""
        if not self.running:
            return
        for mon in self.monitors.values():
            if mon.handler in mon.informer.handlers:
                continue
            mon.informer.add_handler(mon.handler)
            if mon.owned:
                mon.informer.start()

    def _stop_monitor(self, mon: Monitor):
        mon.informer.remove_handler(mon.handler)
        if mon.owned:
            asyncio.ensure_future(mon.informer.stop())

    def is_synced(self) -> bool:
        return bool(self.monitors) and all(mon.has_synced() for mon in self.monitors.values())

    async def stop(self):
        self.running = False
        for mon in self.monitors.values():
            mon.informer.remove_handler(mon.handler)
            if mon.owned:
                await mon.informer.stop()
        self.monitors = {}

    # ------------------------------------------------------------- graph
    def enqueue(self, event):
        """graphChanges: events are applied in order, as soon as they arrive."""
        self.graph_changes.append(event)
        if self._draining:
            return
        self._draining = True
        try:
            while self.graph_changes:
                self.process_event(self.graph_changes.popleft())
        finally:
            self._draining = False

    def enqueue_virtual_delete_event(self, ref: ObjectReference):
        self.enqueue((DELETE, {"apiVersion": ref.api_version, "kind": ref.kind,
                               "metadata": {"namespace": ref.namespace, "uid": ref.uid, "name": ref.name}}, None,
                      (ref.api_version, ref.kind)))

    def add_dependent_to_owners(self, n: Node, owners):
        for owner in owners:
            on = self.uid_to_node.get(owner.get("uid"))
            virtual = on is None
            if virtual:
                on = Node(ObjectReference.from_owner(owner, n.identity.namespace), virtual=True)
                self.uid_to_node[on.identity.uid] = on
            on.dependents.add(n)
            if virtual:
                # attemptToDeleteItem asks the apiserver whether this owner exists
                self.attempt_to_delete.add(on)

    def insert_node(self, n: Node):
        self.uid_to_node[n.identity.uid] = n
        self.add_dependent_to_owners(n, n.owners)

    def remove_dependent_from_owners(self, n: Node, owners):
        for owner in owners:
            on = self.uid_to_node.get(owner.get("uid"))
            if on is not None:
                on.dependents.discard(n)

    def remove_node(self, n: Node):
        self.uid_to_node.pop(n.identity.uid, None)
        self.remove_dependent_from_owners(n, n.owners)

    def add_unblocked_owners_to_delete_queue(self, removed, changed):
        for ref in removed:
            if ref.get("blockOwnerDeletion") is True:
                n = self.uid_to_node.get(ref.get("uid"))
                if n is not None:
                    self.attempt_to_delete.add(n)
        for old, new in changed:
            if old.get("blockOwnerDeletion") is True and new.get("blockOwnerDeletion") is not True:
                n = self.uid_to_node.get(new.get("uid"))
                if n is not None:
                    self.attempt_to_delete.add(n)

    def process_transitions(self, old, obj, n: Node):
        if _deletion_starts(old, obj) and _has_finalizer(obj, FINALIZER_ORPHAN):
            self.attempt_to_orphan.add(n)
            return
        if _deletion_starts(old, obj) and _has_finalizer(obj, FINALIZER_DELETE_DEPENDENTS):
            n.deleting_dependents = True
            for dep in list(n.dependents):
                self.attempt_to_delete.add(dep)
            self.attempt_to_delete.add(n)

    def process_event(self, event):
        """processGraphChanges (:586) for one event."""
        self.events_processed += 1
        typ, obj, old, gvk = event
        md = obj.get("metadata") or {}
        uid = md.get("uid")
        existing = self.uid_to_node.get(uid)
        if existing is not None:
            existing.virtual = False        # observed through an informer
        owners = md.get("ownerReferences") or []
        if typ in (ADD, UPDATE) and existing is None:
            api_version, kind = gvk if gvk else (obj.get("apiVersion", ""), obj.get("kind", ""))
            n = Node(ObjectReference(api_version, kind, md.get("name", ""), uid, md.get("namespace", "")), owners,
                     being_deleted=_being_deleted(obj),
                     deleting_dependents=_being_deleted(obj) and _has_finalizer(obj, FINALIZER_DELETE_DEPENDENTS))
            self.insert_node(n)
            self.process_transitions(old, obj, n)
        elif typ in (ADD, UPDATE):
            added, removed, changed = references_diffs(existing.owners, owners)
            if added or removed or changed:
                self.add_unblocked_owners_to_delete_queue(removed, changed)
                existing.owners = list(owners)
                self.add_dependent_to_owners(existing, added)
                self.remove_dependent_from_owners(existing, removed)
            if _being_deleted(obj):
                existing.being_deleted = True
            self.process_transitions(old, obj, existing)
        elif typ == DELETE:
            if existing is None:
                return
            self.remove_node(existing)
            if existing.dependents:
                self.absent_owner_cache.add(uid)
            for dep in list(existing.dependents):
                self.attempt_to_delete.add(dep)
            for owner in existing.owners:
                on = self.uid_to_node.get(owner.get("uid"))
                if on is not None and on.deleting_dependents:
                    # the owner may be waiting for exactly this dependent
                    self.attempt_to_delete.add(on)


# ---------------------------------------------------------------------------- controller
class GarbageCollector(Controller):
    """kube-controller-manager's garbagecollector (startGarbageCollectorController,
    cmd/kube-controller-manager/app/core.go): --concurrent-gc-syncs workers over each queue and
    a discovery resync every 30 s."""
    name = "garbagecollector"

    def __init__(self, mgr, workers: int = 8, sync_period: float = 30.0, absent_cache_size: int = 500,
                 ignored=IGNORED_RESOURCES):
        super().__init__(mgr)
        self.workers = workers
        self.sync_period = sync_period
        self.attempt_to_delete = RateLimitingQueue("garbage_collector_attempt_to_delete")
        self.attempt_to_orphan = RateLimitingQueue("garbage_collector_attempt_to_orphan")
        self.absent_owner_cache = UIDCache(absent_cache_size)
        self.graph = GraphBuilder(self.attempt_to_delete, self.attempt_to_orphan, self.absent_owner_cache,
                                  mgr.client, getattr(mgr, "factory", None), ignored)
        self._resources: dict = {}
        self._paused = asyncio.Event()
        self._paused.set()
        self.items_processed = 0
        self.discovery_calls = 0

    # ------------------------------------------------------------- lifecycle
    async def start(self):
        self.graph.running = True
        await self._sync_once()
        await self._wait_synced()
        for i in range(self.workers):
            self.tasks.append(asyncio.create_task(self._delete_worker(), name=f"gc-delete-{i}"))
            self.tasks.append(asyncio.create_task(self._orphan_worker(), name=f"gc-orphan-{i}"))
        self.tasks.append(asyncio.create_task(self._sync_loop(), name="gc-discovery-sync"))

    async def stop(self):
        self.attempt_to_delete.shutdown()
        self.attempt_to_orphan.shutdown()
        for t in self.tasks:
            t.cancel()
        await self.graph.stop()

    async def _wait_synced(self, timeout: float = 30.0):
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while not self.graph.is_synced() and loop.time() < end:
            await asyncio.sleep(0.02)

    async def get_deletable_resources(self) -> dict:
        """GetDeletableResources: discovery errors are all taken as transient; whatever was
        discovered is used (possibly nothing, which Sync skips)."""
        self.discovery_calls += 1
        lists, errs = await server_preferred_resources(self.client)
        if errs:
            log.warning("failed to discover some groups: %s", "; ".join(errs))
        return deletable_resources(lists)

    async def _sync_once(self) -> bool:
        """One step of Sync (:169): re-read discovery; on a change pause the workers, resync the
        monitors and wait for them to sync."""
        new = await self.get_deletable_resources()
        if not new or set(new) == set(self._resources):
            return False
        self._paused.clear()
        try:
            errs = self.graph.sync_monitors(new)
            for e in errs:
                log.warning("garbage collector: %s", e)
            self.graph.start_monitors()
            await self._wait_synced()
            self._resources = new
        finally:
            self._paused.set()
        return True

    async def _sync_loop(self):
        while True:
            await asyncio.sleep(self.sync_period)
            try:
                await self._sync_once()
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.warning("garbage collector sync: %r", e)

    async def _delete_worker(self):
        while True:
            try:
                item = await self.attempt_to_delete.get()
            except ShutDown:
                return
            await self._paused.wait()
            try:
                self.items_processed += 1
                await self.attempt_to_delete_item(item)
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.debug("error syncing item %s: %r", item, e)
                self.attempt_to_delete.add_rate_limited(item)
            else:
                if not item.is_observed():
                    # a virtual node whose object exists: wait for the informer to report it
                    self.attempt_to_delete.add_rate_limited(item)
                else:
                    self.attempt_to_delete.forget(item)
            finally:
                self.attempt_to_delete.done(item)

    async def _orphan_worker(self):
        while True:
            try:
                owner = await self.attempt_to_orphan.get()
            except ShutDown:
                return
            await self._paused.wait()
            try:
                await self.orphan_dependents(owner.identity, list(owner.dependents))
                await self.remove_finalizer(owner, FINALIZER_ORPHAN)
                self.attempt_to_orphan.forget(owner)
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.debug("orphaning dependents of %s: %r", owner, e)
                self.attempt_to_orphan.add_rate_limited(owner)
            finally:
                self.attempt_to_orphan.done(owner)

    # ------------------------------------------------------------- operations (operations.go)
    def _ri(self, api_version: str, kind: str) -> ResourceInfo:
        ri = SCHEME.for_kind(api_version, kind)
        if ri is None:
            raise RestMappingError(kind, api_version)
        return ri

    def _path(self, ref: ObjectReference) -> str:
        ri = self._ri(ref.api_version, ref.kind)
        return self.client.path(ri, ref.namespace if ri.namespaced else "", ref.name)

    async def get_object(self, ref: ObjectReference) -> dict:
        return await self.client.request("GET", self._path(ref))

    async def delete_object(self, ref: ObjectReference, policy: str):
        body = {"kind": "DeleteOptions", "apiVersion": "v1", "preconditions": {"uid": ref.uid},
                "propagationPolicy": policy}
        return await self.client.request("DELETE", self._path(ref), body=body)

    async def patch_object(self, ref: ObjectReference, patch: dict, refs_fn=None):
        """A strategic merge patch; a kind without a strategic schema (custom resources) gets the
        same change as a JSON patch tested against the uid and resourceVersion it was made from."""
        path = self._path(ref)
        try:
            return await self.client.request("PATCH", path, body=patch,
                                             content_type="application/strategic-merge-patch+json")
        except m.StatusError as e:
            if e.code != 415 or refs_fn is None:
                raise
        cur = await self.client.request("GET", path)
        md = cur.get("metadata") or {}
        ops = [{"op": "test", "path": "/metadata/uid", "value": ref.uid},
               {"op": "test", "path": "/metadata/resourceVersion", "value": md.get("resourceVersion")}]
        new = refs_fn(md.get("ownerReferences") or [])
        ops.append({"op": "replace" if "ownerReferences" in md else "add", "path": "/metadata/ownerReferences",
                    "value": new})
        return await self.client.request("PATCH", path, body=ops, content_type="application/json-patch+json")

    async def remove_finalizer(self, owner: Node, target: str):
        """removeFinalizer: get, drop the finalizer, update; retried on conflicts."""
        for _ in range(5):
            try:
                obj = await self.get_object(owner.identity)
            except m.StatusError as e:
                if m.is_not_found(e):
                    return
                raise
            fins = (obj.get("metadata") or {}).get("finalizers") or []
            if target not in fins:
                return
            obj["metadata"]["finalizers"] = [f for f in fins if f != target]
            try:
                await self.client.request("PUT", self._path(owner.identity), body=obj)
                return
            except m.StatusError as e:
                if m.is_not_found(e):
                    return
                if not m.is_conflict(e):
                    raise
        raise RuntimeError(f"updateMaxRetries(5) has reached. The garbage collector will retry later for owner "
                           f"{owner.identity}.")

    # ------------------------------------------------------------- garbagecollector.go
    async def is_dangling(self, ref: dict, item: Node):
        """(dangling, the owner's latest state)."""
        if self.absent_owner_cache.has(ref.get("uid")):
            return True, None
        oref = ObjectReference.from_owner(ref, item.identity.namespace)
        try:
            owner = await self.get_object(oref)
        except m.StatusError as e:
            if m.is_not_found(e):
                self.absent_owner_cache.add(ref.get("uid"))
                return True, None
            raise
        if m.uid_of(owner) != ref.get("uid"):
            self.absent_owner_cache.add(ref.get("uid"))
            return True, None
        return False, owner

    async def classify_references(self, item: Node, refs):
        solid, dangling, waiting = [], [], []
        for ref in refs:
            d, owner = await self.is_dangling(ref, item)
            if d:
                dangling.append(ref)
            elif _being_deleted(owner) and _has_finalizer(owner, FINALIZER_DELETE_DEPENDENTS):
                waiting.append(ref)
            else:
                solid.append(ref)
        return solid, dangling, waiting

    async def attempt_to_delete_item(self, item: Node):
        if item.being_deleted and not item.deleting_dependents:
            return      # on its way out: its dependents are handled when it is gone
        try:
            latest = await self.get_object(item.identity)
        except m.StatusError as e:
            if not m.is_not_found(e):
                raise
            self.graph.enqueue_virtual_delete_event(item.identity)
            item.virtual = False
            return
        if m.uid_of(latest) != item.identity.uid:
            self.graph.enqueue_virtual_delete_event(item.identity)
            item.virtual = False
            return
        if item.deleting_dependents:
            return await self.process_deleting_dependents_item(item)
        refs = (latest.get("metadata") or {}).get("ownerReferences") or []
        if not refs:
            return
        solid, dangling, waiting = await self.classify_references(item, refs)
        if solid:
            if not dangling and not waiting:
                return
            # waiting refs must go too, or their owners stay stuck with foregroundDeletion
            gone = {r.get("uid") for r in dangling + waiting}
            await self.patch_object(item.identity, delete_owner_ref_patch(item.identity.uid, *gone),
                                    lambda rs: [r for r in rs if r.get("uid") not in gone])
            return
        if waiting and item.dependents:
            for dep in list(item.dependents):
                if dep.deleting_dependents:
                    # a possible cycle: unblock our own owners, then delete in the foreground
                    await self.patch_object(item.identity, patch_to_unblock_owner_references(item),
                                            lambda rs: [dict(r, blockOwnerDeletion=False)
                                                        if r.get("blockOwnerDeletion") is True else r for r in rs])
                    break
            await self.delete_object(item.identity, "Foreground")
            return
        if _has_finalizer(latest, FINALIZER_ORPHAN):
            policy = "Orphan"
        elif _has_finalizer(latest, FINALIZER_DELETE_DEPENDENTS):
            policy = "Foreground"
        else:
            policy = "Background"
        await self.delete_object(item.identity, policy)

    async def process_deleting_dependents_item(self, item: Node):
        blocking = item.blocking_dependents()
        if not blocking:
            await self.remove_finalizer(item, FINALIZER_DELETE_DEPENDENTS)
            return
        for dep in blocking:
            if not dep.deleting_dependents:
                self.attempt_to_delete.add(dep)

    async def orphan_dependents(self, owner: ObjectReference, dependents):
        errs = []

        async def one(dep: Node):
            try:
                await self.patch_object(dep.identity, delete_owner_ref_patch(dep.identity.uid, owner.uid),
                                        lambda rs: [r for r in rs if r.get("uid") != owner.uid])
            except m.StatusError as e:
                if not m.is_not_found(e):
                    errs.append(f"orphaning {dep.identity} failed, {e}")
            except RestMappingError as e:
                errs.append(f"orphaning {dep.identity} failed, {e}")
        await asyncio.gather(*(one(d) for d in dependents))
        if errs:
            raise RuntimeError(f"failed to orphan dependents of owner {owner}, got errors: {'; '.join(errs)}")

    # ------------------------------------------------------------- test / debug helpers
    def graph_has_uid(self, uids) -> bool:
        return any(u in self.graph.uid_to_node for u in uids)

    async def sync(self, key):        # the Controller queue is unused: work arrives through the graph
        pass


def dump_graph(gb: GraphBuilder) -> str:
    """A JSON view of the graph (the reference's later /graph debug handler)."""
    return json.dumps({u: {"identity": repr(n.identity), "owners": [o.get("uid") for o in n.owners],
                           "dependents": sorted(d.identity.uid for d in n.dependents), "virtual": n.virtual,
                           "beingDeleted": n.being_deleted, "deletingDependents": n.deleting_dependents}
                       for u, n in gb.uid_to_node.items()}, indent=1, sort_keys=True)
