"""ControllerRevision history (pkg/controller/history/controller_history.go).

StatefulSets and DaemonSets snapshot their pod template as ControllerRevisions:
  * the revision's data is the patch `{"spec": {"template": {..., "$patch": "replace"}}}`
    that restores the template (stateful_set_utils.go getPatch, daemon update.go getPatch);
  * its name is `<parent>-<SafeEncodeString(hash)>`, the hash an FNV-32 of the data's bytes plus
    the decimal collision count (HashControllerRevision :77-91); the hash is also the
    `controller.kubernetes.io/hash` label, next to the parent's selector labels;
  * revisions are equal when their hash labels (where both parse) and data agree
    (EqualRevision :100-125);
  * creation retries under a bumped collision count while the name is taken (:209-225).
`History` drives the client and an informer of controllerrevisions; tests substitute a fake of
the same five methods (list / create / update / delete / adopt / release).
"""
from __future__ import annotations

import json

from ..api import meta as m
from .controller_utils import adopt_patch, release_patch

HASH_LABEL = "controller.kubernetes.io/hash"
_SAFE = "bcdfghjklmnpqrstvwxz2456789"


def safe_encode(s: str) -> str:
    return "".join(_SAFE[ord(c) % len(_SAFE)] for c in s)


def revision_name(prefix: str, h: int) -> str:
    """ControllerRevisionName: prefixes longer than 223 characters are truncated."""
    return f"{prefix[:223]}-{safe_encode(str(h))}"


def raw(data) -> bytes:
    """The revision's data as the bytes the hash and equality see (canonical JSON)."""
    return json.dumps(data, sort_keys=True, separators=(",", ":")).encode() if data is not None else b""


def fnv32(data: bytes) -> int:
    """hash/fnv New32 (multiply, then xor)."""
    h = 0x811C9DC5
    for b in data:
        h = (h * 0x01000193) & 0xFFFFFFFF
        h ^= b
    return h


def hash_revision(rev: dict, probe: int | None) -> int:
    data = raw(rev.get("data"))
    if probe is not None:
        data += str(int(probe)).encode()
    return fnv32(data)


def new_controller_revision(parent: dict, api_version: str, kind: str, selector_labels: dict, data: dict,
                            revision: int, collision_count: int | None) -> dict:
    """NewControllerRevision: owned by `parent`, labelled with the selector's labels plus the hash."""
    cr = {"apiVersion": "apps/v1", "kind": "ControllerRevision",
          "metadata": {"labels": dict(selector_labels or {}),
                       "ownerReferences": [m.new_controller_ref(parent, api_version, kind)]},
          "data": data, "revision": int(revision)}
    h = hash_revision(cr, collision_count)
    cr["metadata"]["name"] = revision_name(m.name_of(parent), h)
    cr["metadata"]["labels"][HASH_LABEL] = str(h)
    return cr


def revision_of(rev: dict) -> int:
    return int((rev or {}).get("revision") or 0)


def sort_revisions(revs: list) -> list:
    """SortControllerRevisions: ascending revision number (stable)."""
    revs.sort(key=revision_of)
    return revs


def _label_hash(rev):
    v = m.labels_of(rev).get(HASH_LABEL)
    try:
        return int(v) if v is not None else None
    except ValueError:
        return None


def equal_revision(a: dict | None, b: dict | None) -> bool:
    if a is None or b is None:
        return a is b
    ha, hb = _label_hash(a), _label_hash(b)
    if ha is not None and hb is not None and ha != hb:
        return False
    return raw(a.get("data")) == raw(b.get("data"))


def find_equal_revisions(revs: list, needle: dict) -> list:
    return [r for r in revs if equal_revision(r, needle)]


class History:
    """realHistory over the API client; the informer (cache) answers the lists."""

    resource = "controllerrevisions.apps"

    def __init__(self, client, informer):
        self.client, self.informer = client, informer

    def list(self, parent: dict, selector) -> list:
        """ListControllerRevisions: the namespace's revisions that match the selector and are
        owned by the parent or by nobody."""
        out = []
        uid = m.uid_of(parent)
        for r in self.informer.list():
            if m.namespace_of(r) != m.namespace_of(parent) or not selector.matches(m.labels_of(r)):
                continue
            ref = m.controller_ref(r)
            if ref is None or ref.get("uid") == uid:
                out.append(r)
        return out

    async def create(self, parent: dict, rev: dict, collision: list) -> dict:
        """CreateControllerRevision: `collision` is a one-element list (the *int32 the
        reference bumps in place). A name taken by a revision with the same data is that
        revision (the informer had not caught up) — the later upstream fix; 1.9 bumps the
        collision count then too."""
        clone = m.deepcopy(rev)
        clone["metadata"]["namespace"] = m.namespace_of(parent)
        while True:
            h = hash_revision(rev, collision[0])
            clone["metadata"]["name"] = revision_name(m.name_of(parent), h)
            try:
                return await self.client.create(clone, m.namespace_of(parent))
            except m.StatusError as e:
                if not m.is_already_exists(e):
                    raise
                try:
                    existing = await self.client.get(self.resource, m.name_of(clone), m.namespace_of(parent))
                except m.StatusError:
                    existing = None
                if existing is not None and raw(existing.get("data")) == raw(clone.get("data")):
                    return existing
                collision[0] += 1

    async def update(self, rev: dict, new_revision: int) -> dict:
        """UpdateControllerRevision: renumber, retrying conflicts with the cached copy."""
        clone = m.deepcopy(rev)
        for _ in range(5):
            if revision_of(clone) == new_revision:
                return clone
            clone["revision"] = int(new_revision)
            clone.setdefault("apiVersion", "apps/v1")
            clone.setdefault("kind", "ControllerRevision")
            try:
                return await self.client.update(clone)
            except m.StatusError as e:
                if not m.is_conflict(e):
                    raise
                cached = self.informer.get(m.key_of(clone))
                if cached is not None:
                    clone = m.deepcopy(cached)
        raise m.StatusError(409, "Conflict", f"controllerrevision {m.name_of(rev)}: too many conflicts")

    async def delete(self, rev: dict):
        await self.client.delete(self.resource, m.name_of(rev), m.namespace_of(rev))

    async def adopt(self, parent: dict, api_version: str, kind: str, rev: dict) -> dict:
        owner = m.controller_ref(rev)
        if owner is not None:
            raise ValueError(f"attempt to adopt revision owned by {owner}")
        return await self.client.patch(self.resource, m.name_of(rev), adopt_patch(parent, api_version, kind, rev),
                                       m.namespace_of(parent), patch_type="application/strategic-merge-patch+json")

    async def release(self, parent: dict, rev: dict):
        try:
            return await self.client.patch(self.resource, m.name_of(rev), release_patch(parent, rev),
                                           m.namespace_of(rev), patch_type="application/strategic-merge-patch+json")
        except m.StatusError as e:
            if m.is_not_found(e) or e.code == 422:
                return None
            raise
