"""Shared controller machinery (pkg/controller/controller_utils.go, controller_ref_manager.go).

* ControllerExpectations / UIDTrackingControllerExpectations (controller_utils.go:133-370): a
  controller that issued N creates or deletes does not act again for that key until its
  informer has observed them (or 5 minutes passed — ExpectationsTimeout).
* ActivePods ordering (:720-763): the pods a controller deletes first sort first — unassigned,
  then Pending < Unknown < Running, not ready, ready for less time, more container restarts,
  newer.
* ReplicaSet orderings and filters (:814-891) used by the Deployment controller.
* slow_start_batch (replicaset/replica_set.go:673-697): 1, 2, 4, … calls per batch; a failing
  batch skips the rest.
* ControllerRefManager.claim (controller_ref_manager.go ClaimObject): adopt matching orphans
  (after re-checking the owner is not being deleted), keep owned matches, release owned
  objects whose labels no longer match, leave other owners' objects alone.
"""
from __future__ import annotations

import asyncio
import functools
import time

from ..api import meta as m
from ..api.helpers import get_condition, is_pod_ready

EXPECTATIONS_TIMEOUT = 300.0
SLOW_START_INITIAL_BATCH = 1


# ---------------------------------------------------------------------------- expectations
class ControllerExpectations:
    def __init__(self, clock=time.monotonic, ttl: float = EXPECTATIONS_TIMEOUT):
        self.clock, self.ttl = clock, ttl
        self._store: dict[str, list] = {}          # key -> [adds, dels, timestamp]

    def get_expectations(self, key: str):
        e = self._store.get(key)
        return (e[0], e[1]) if e is not None else None

    def delete_expectations(self, key: str):
        self._store.pop(key, None)

    def satisfied_expectations(self, key: str) -> bool:
        """No record, a fulfilled one, or an expired one: the controller may sync."""
        e = self._store.get(key)
        if e is None:
            return True
        if e[0] <= 0 and e[1] <= 0:
            return True
        return self.clock() - e[2] > self.ttl

    def set_expectations(self, key: str, adds: int, dels: int):
        self._store[key] = [adds, dels, self.clock()]

    def expect_creations(self, key: str, adds: int):
        self.set_expectations(key, adds, 0)

    def expect_deletions(self, key: str, dels: int):
        self.set_expectations(key, 0, dels)

    def lower_expectations(self, key: str, adds: int = 0, dels: int = 0):
        e = self._store.get(key)
        if e is not None:
            e[0] -= adds
            e[1] -= dels

    def raise_expectations(self, key: str, adds: int = 0, dels: int = 0):
        e = self._store.get(key)
        if e is not None:
            e[0] += adds
            e[1] += dels

    def creation_observed(self, key: str):
        self.lower_expectations(key, 1, 0)

    def deletion_observed(self, key: str):
        self.lower_expectations(key, 0, 1)


class UIDTrackingControllerExpectations(ControllerExpectations):
    """Deletions are tracked by pod key, so a deletion observed twice (an update carrying a
    deletionTimestamp, then the delete) lowers the count once."""

    def __init__(self, clock=time.monotonic, ttl: float = EXPECTATIONS_TIMEOUT):
        super().__init__(clock, ttl)
        self._uids: dict[str, set] = {}

    def get_uids(self, key: str):
        return self._uids.get(key)

    def expect_deletions(self, key: str, deleted):       # type: ignore[override]
        keys = set(deleted) if not isinstance(deleted, int) else set()
        self._uids[key] = keys
        super().expect_deletions(key, len(keys) if not isinstance(deleted, int) else deleted)

    def deletion_observed(self, key: str, delete_key: str | None = None):   # type: ignore[override]
        uids = self._uids.get(key)
        if uids is not None and delete_key in uids:
            super().deletion_observed(key)
            uids.discard(delete_key)

    def delete_expectations(self, key: str):
        super().delete_expectations(key)
        self._uids.pop(key, None)


def pod_key(pod: dict) -> str:
    return f"{m.namespace_of(pod)}/{m.name_of(pod)}"


# ---------------------------------------------------------------------------- pod ordering
def is_pod_active(p: dict) -> bool:
    return (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed") and \
        not (p.get("metadata") or {}).get("deletionTimestamp")


def filter_active_pods(pods) -> list[dict]:
    return [p for p in pods if is_pod_active(p)]


_PHASE_RANK = {"Pending": 0, "Unknown": 1, "Running": 2}


def _ready_time(p):
    c = get_condition(p, "Ready")
    if c is not None and c.get("status") == "True":
        return m.parse_time(c.get("lastTransitionTime"))
    return None


def _after_or_zero(t1, t2) -> bool:
    """t1 after t2, a zero (missing) time counting as after any other."""
    if not t1 or not t2:
        return not t1
    return t1 > t2


def _max_restarts(p) -> int:
    return max([int(cs.get("restartCount") or 0) for cs in (p.get("status") or {}).get("containerStatuses") or []]
               or [0])


def active_pods_less(a: dict, b: dict) -> bool:
    """ActivePods.Less (controller_utils.go:731-763)."""
    na, nb = (a.get("spec") or {}).get("nodeName") or "", (b.get("spec") or {}).get("nodeName") or ""
    if na != nb and (not na or not nb):
        return not na
    pa, pb = _PHASE_RANK.get((a.get("status") or {}).get("phase"), 0), _PHASE_RANK.get((b.get("status") or {}).get("phase"), 0)
    if pa != pb:
        return pa < pb
    ra, rb = is_pod_ready(a), is_pod_ready(b)
    if ra != rb:
        return not ra
    if ra and rb:
        ta, tb = _ready_time(a), _ready_time(b)
        if ta != tb:
            return _after_or_zero(ta, tb)
    xa, xb = _max_restarts(a), _max_restarts(b)
    if xa != xb:
        return xa > xb
    ca = m.parse_time((a.get("metadata") or {}).get("creationTimestamp"))
    cb = m.parse_time((b.get("metadata") or {}).get("creationTimestamp"))
    if ca != cb:
        return _after_or_zero(ca, cb)
    return False


def sort_active_pods(pods: list) -> list:
    """In place, the pods to remove first at the front."""
    pods.sort(key=functools.cmp_to_key(lambda a, b: -1 if active_pods_less(a, b) else (1 if active_pods_less(b, a) else 0)))
    return pods


# ---------------------------------------------------------------------------- replica sets
def rs_replicas(rs) -> int:
    return int(((rs or {}).get("spec") or {}).get("replicas", 0) or 0)


def filter_active_replica_sets(rss) -> list[dict]:
    return [rs for rs in rss if rs is not None and rs_replicas(rs) > 0]


def _created(o):
    return m.parse_time((o.get("metadata") or {}).get("creationTimestamp")) or 0.0


def by_creation_timestamp(o):
    """ReplicaSetsByCreationTimestamp: older first, the name breaking ties."""
    return (_created(o), m.name_of(o))


def sort_by_size_older(rss: list) -> list:
    """ReplicaSetsBySizeOlder: larger first, then older."""
    rss.sort(key=lambda r: (-rs_replicas(r), _created(r), m.name_of(r)))
    return rss


def sort_by_size_newer(rss: list) -> list:
    """ReplicaSetsBySizeNewer: larger first, then newer."""
    def cmp(a, b):
        if rs_replicas(a) != rs_replicas(b):
            return -1 if rs_replicas(a) > rs_replicas(b) else 1
        ka, kb = by_creation_timestamp(a), by_creation_timestamp(b)
        return -1 if kb < ka else (1 if ka < kb else 0)
    rss.sort(key=functools.cmp_to_key(cmp))
    return rss


# ---------------------------------------------------------------------------- slow start
async def slow_start_batch(count: int, initial: int, fn) -> tuple[int, BaseException | None]:
    """Call `fn` `count` times in batches of initial, 2·initial, …; the calls of a batch run
    concurrently and a batch with a failure ends the run. Returns (successes, first error)."""
    remaining, successes = count, 0
    batch = min(remaining, initial)
    while batch > 0:
        results = await asyncio.gather(*(fn() for _ in range(batch)), return_exceptions=True)
        errs = [r for r in results if isinstance(r, BaseException)]
        successes += batch - len(errs)
        if errs:
            return successes, errs[0]
        remaining -= batch
        batch = min(2 * batch, remaining)
    return successes, None


# ---------------------------------------------------------------------------- ControllerRef
class ControllerRefManager:
    """Claim objects for `owner` (controller_ref_manager.go:35-170). `adopt(obj)` and
    `release(obj)` perform the writes; `can_adopt()` re-checks (uncached) that the owner is not
    being deleted before the first adoption."""

    def __init__(self, owner: dict, selector, adopt, release, can_adopt=None):
        self.owner, self.selector = owner, selector
        self._adopt, self._release, self._can_adopt = adopt, release, can_adopt
        self._can_adopt_err: BaseException | None = None
        self._checked = False

    async def _check(self):
        if not self._checked:
            self._checked = True
            if self._can_adopt is not None:
                try:
                    await self._can_adopt()
                except Exception as e:        # noqa: BLE001 — any failure blocks adoption
                    self._can_adopt_err = e
        if self._can_adopt_err is not None:
            raise self._can_adopt_err

    async def claim(self, objs, filters=()) -> list[dict]:
        claimed, errors = [], []
        uid = m.uid_of(self.owner)
        deleting = bool((self.owner.get("metadata") or {}).get("deletionTimestamp"))
        for obj in objs:
            match = self.selector.matches(m.labels_of(obj)) and all(f(obj) for f in filters)
            ref = m.controller_ref(obj)
            try:
                if ref is not None:
                    if ref.get("uid") != uid:
                        continue                        # someone else's
                    if match:
                        claimed.append(obj)
                        continue
                    if deleting:
                        continue
                    await self._release(obj)            # ours, but no longer selected
                    continue
                if deleting or not match or (obj.get("metadata") or {}).get("deletionTimestamp"):
                    continue
                await self._check()
                await self._adopt(obj)
                claimed.append(obj)
            except m.StatusError as e:
                if not m.is_not_found(e):
                    errors.append(e)
            except Exception as e:                       # noqa: BLE001
                errors.append(e)
        if errors:
            raise errors[0]
        return claimed


def adopt_patch(owner: dict, api_version: str, kind: str, obj: dict) -> dict:
    """The strategic-merge patch that adds `owner` as the controller of `obj` (the object's UID
    is a precondition)."""
    return {"metadata": {"ownerReferences": [m.new_controller_ref(owner, api_version, kind)], "uid": m.uid_of(obj)}}


def release_patch(owner: dict, obj: dict) -> dict:
    return {"metadata": {"ownerReferences": [{"$patch": "delete", "uid": m.uid_of(owner)}], "uid": m.uid_of(obj)}}


def recheck_deletion(get_fresh):
    """RecheckDeletionTimestamp: the owner, read fresh, must still exist under the same UID and
    not be being deleted."""
    async def check():
        fresh = await get_fresh()
        if (fresh.get("metadata") or {}).get("deletionTimestamp"):
            raise RuntimeError(f"{m.namespace_of(fresh)}/{m.name_of(fresh)} has just been deleted at "
                               f"{fresh['metadata']['deletionTimestamp']}")
        return fresh
    return check


def pod_from_template(owner, api_version, kind, extra_labels=None, node=None):
    """GetPodFromTemplate (controller_utils.go): a pod from the owner's template, named after
    the owner (generateName), labelled with the template's labels plus `extra_labels`,
    controlled by the owner, optionally pinned to `node`."""
    import json as _json
    tpl = _json.loads(_json.dumps((owner.get("spec") or {}).get("template") or {}))
    md = tpl.get("metadata") or {}
    labels = dict(md.get("labels") or {})
    labels.update(extra_labels or {})
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"generateName": m.name_of(owner) + "-", "namespace": m.namespace_of(owner), "labels": labels,
                        "annotations": dict(md.get("annotations") or {}),
                        "ownerReferences": [m.new_controller_ref(owner, api_version, kind)]},
           "spec": tpl.get("spec") or {}}
    if node:
        pod["spec"]["nodeName"] = node
    return pod
