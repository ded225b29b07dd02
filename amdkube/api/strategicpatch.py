"""Strategic merge patch, driven by per-type patch metadata.

The reference computes and applies strategic merge patches by reflecting over the Go API
structs: a field's `patchStrategy` ("merge", "retainKeys", "merge,retainKeys") and
`patchMergeKey` struct tags decide whether a list is replaced, merged as a set of scalars, or
merged element-by-element on a key (staging/src/k8s.io/apimachinery/pkg/util/strategicpatch/
patch.go: StrategicMergePatch :812, mergeMap :1258, mergeSlice :1389, CreateThreeWayMergePatch
:1999, diffMaps :168). The SAME field name merges differently by type: Container.ports merges by
containerPort, ServiceSpec.ports by port (core/v1/types.go:2102, :3372).

amdkube carries the tags as data (api/patchmeta.py, generated from the reference's types.go by
hack/gen_patch_meta.py) and walks its OpenAPI definitions (api/openapi.py) to know the type of
every nested field, so the metadata applies per path, exactly as in the reference.

Directives (patch.go constants): `$patch: replace|delete|merge` on a map, `{"$patch": "replace"}`
and `{<key>: v, "$patch": "delete"}` inside merge lists, `$retainKeys` (clear the fields of a
retainKeys-strategy struct not listed), `$setElementOrder/<field>` (final order of a merge list)
and `$deleteFromPrimitiveList/<field>` (removals from a merged list of scalars).

Public API:
  schema_for(api_version, kind) -> node       the root definition of a kind (None: unknown)
  apply(original, patch, node) -> dict        server side StrategicMergePatch
  create_two_way(original, modified, node)    CreateTwoWayMergeMapPatch
  create_three_way(original, modified, current, node, overwrite=True)
                                              CreateThreeWayMergePatch (kubectl apply)
  create_three_way_json_merge(original, modified, current)
                                              jsonmergepatch.CreateThreeWayJSONMergePatch (kinds
                                              without a schema: custom resources)
"""
from __future__ import annotations

import copy
import functools
from dataclasses import dataclass, replace

from .patchmeta import PATCH_META

DIRECTIVE = "$patch"
RETAIN_KEYS = "$retainKeys"
DELETE_PRIMITIVE = "$deleteFromPrimitiveList"
SET_ORDER = "$setElementOrder"
REPLACE, DELETE, MERGE = "replace", "delete", "merge"


class PatchError(ValueError):
    pass


class ConflictError(PatchError):
    pass


# ------------------------------------------------------------------------------- schema
@functools.lru_cache(maxsize=1)
def _defs() -> dict:
    from .openapi import definitions
    return definitions()


@functools.lru_cache(maxsize=1)
def _short_meta() -> dict:
    out: dict = {}
    for full, fields in PATCH_META.items():
        out.setdefault(full.rsplit(".", 1)[1], {}).update(fields)
    return out


def _node_of(p: dict):
    if "$ref" in p:
        return p["$ref"].rsplit("/", 1)[1]
    if p.get("type") == "array":
        return _node_of(p.get("items") or {})
    if "additionalProperties" in p:
        return ("map", _node_of(p["additionalProperties"]))
    return None


def _split_strategy(strat: str) -> tuple[str, bool]:
    """extractRetainKeysPatchStrategy: ("merge"|"replace"|"", has retainKeys)."""
    parts = [s for s in strat.split(",") if s]
    others = [s for s in parts if s != "retainKeys"]
    if len(others) > 1 or len(parts) > 2:
        raise PatchError(f"unexpected patch strategy: {strat}")
    return (others[0] if others else ""), "retainKeys" in parts


class StructNode:
    """A schema node given directly as {field: (child node or None, "strategy", "merge key")}
    (the reference's PatchMetaFromStruct over a Go struct), for types outside the API table."""

    def __init__(self, name: str, fields: dict | None = None):
        self.name, self.fields = name, fields or {}

    def lookup(self, key: str) -> tuple:
        child, strat, mk = self.fields.get(key, (None, "", ""))
        s, retain = _split_strategy(strat)
        return child, s, mk, retain

    def __repr__(self):
        return f"StructNode({self.name})"


@functools.lru_cache(maxsize=4096)
def _lookup(node, key: str) -> tuple:
    """(child node, strategy, merge key, retainKeys) of field `key` of `node`. A node is a
    definition id, ("map", element node) for string-keyed maps, a StructNode, or None (no
    schema: maps merge, lists replace — JSON merge semantics)."""
    if node is None:
        return None, "", "", False
    if isinstance(node, StructNode):
        return node.lookup(key)
    if isinstance(node, tuple):
        return node[1], "", "", False
    d = _defs().get(node)
    if d is None:
        return None, "", "", False
    p = (d.get("properties") or {}).get(key)
    if p is None:
        return None, "", "", False
    meta = PATCH_META.get(node)
    if meta is None:
        meta = _short_meta().get(node.rsplit(".", 1)[1], {})
    strat, mk = meta.get(key, ("", ""))
    s, retain = _split_strategy(strat)
    return _node_of(p), s, mk, retain


def schema_for(api_version: str | None, kind: str | None):
    """The definition a kind's patches are interpreted against; None for unknown kinds."""
    if not api_version or not kind:
        return None
    from .openapi import kind_definition
    return kind_definition(api_version, kind)


# ------------------------------------------------------------------------------- helpers
def _kind(v) -> str:
    if isinstance(v, dict):
        return "map"
    if isinstance(v, list):
        return "list"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, (int, float)):
        return "num"
    if v is None:
        return "null"
    return "str"


def _gostr(v) -> str:
    """fmt.Sprintf("%v") of a decoded JSON scalar (how the reference sorts and compares keys)."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return "<nil>"
    if isinstance(v, float) and v.is_integer() and abs(v) < 1e21:
        return str(int(v))
    return str(v)


def _elem_kind(*lists) -> str:
    kind = None
    for lst in lists:
        for v in lst or ():
            k = _kind(v)
            if k == "list":
                raise PatchError("lists of lists are not supported")
            if kind is None:
                kind = k
            elif k != kind:
                raise PatchError(f"list elements have different types: {kind} and {k}")
    if kind is None:
        raise PatchError("no elements in any of the given slices")
    return kind


def _dedup(seq: list) -> list:
    out = []
    for v in seq:
        if v not in out:
            out.append(v)
    return out


def _sort_scalars(seq: list) -> list:
    return sorted(seq, key=_gostr)


def _mk(item, mk: str):
    if not isinstance(item, dict):
        raise PatchError(f"expected a map in a merge list, got {_kind(item)}")
    if mk not in item:
        raise PatchError(f"map: {item} does not contain declared merge key: {mk}")
    return item[mk]


def _index(lst: list, val, mk: str, kind: str) -> int:
    get = (lambda it: it.get(mk) if isinstance(it, dict) else None) if kind == "map" else (lambda it: it)
    want = get(val)
    for i, v in enumerate(lst):
        if get(v) == want:
            return i
    return -1


def _find(lst: list, mk: str, value):
    for i, v in enumerate(lst):
        if not isinstance(v, dict):
            raise PatchError(f"value for key {i} is not a map")
        if mk in v and v[mk] == value:
            return i
    return -1


def _normalize_slice_order(to_sort: list, order: list, mk: str, kind: str) -> list:
    deletes = []
    if kind == "map":
        for it in list(to_sort) + list(order):
            _mk(it, mk)
        keep = []
        for it in to_sort:
            (deletes if it.get(DIRECTIVE) == DELETE else keep).append(it)
        to_sort = keep
    pos = [(_index(order, it, mk, kind), n) for n, it in enumerate(to_sort)]
    big = len(order) + len(to_sort)
    ranked = sorted(range(len(to_sort)), key=lambda i: (pos[i][0] if pos[i][0] >= 0 else big, i))
    return [to_sort[i] for i in ranked] + deletes


def _merge_sorted(left: list, right: list, server_order: list, mk: str, kind: str) -> list:
    """patch.go mergeSortedSlice: interleave server-only items (left) into the patch items
    (right) by their positions in the live list."""
    out, i, j = [], 0, 0
    while i < len(left) or j < len(right):
        if i >= len(left):
            out.append(right[j])
            j += 1
        elif j >= len(right):
            out.append(left[i])
            i += 1
        else:
            li, ri = _index(server_order, left[i], mk, kind), _index(server_order, right[j], mk, kind)
            if li >= 0 and ri >= 0 and li < ri:
                out.append(left[i])
                i += 1
            else:
                out.append(right[j])
                j += 1
    return out


def _normalize_element_order(patch_items, server_only, patch_order, server_order, mk, kind):
    patch_items = _normalize_slice_order(patch_items, patch_order, mk, kind)
    server_only = _normalize_slice_order(server_only, server_order, mk, kind)
    return _merge_sorted(server_only, patch_items, server_order, mk, kind)


def _partition(merged: list, by: list, mk: str):
    inp, srv = [], []
    for v in merged:
        if mk:
            (inp if _find(by, mk, _mk(v, mk)) >= 0 else srv).append(v)
        else:
            (inp if v in by else srv).append(v)
    return inp, srv


def strip_directives(v):
    """The object without patch directives (the reference drops them when it decodes the
    patched JSON into the typed object)."""
    if isinstance(v, dict):
        return {k: strip_directives(x) for k, x in v.items()
                if not (k == DIRECTIVE or k == RETAIN_KEYS or k.startswith(SET_ORDER + "/")
                        or k.startswith(DELETE_PRIMITIVE + "/"))}
    if isinstance(v, list):
        return [strip_directives(x) for x in v if not (isinstance(x, dict) and DIRECTIVE in x and len(x) == 1)]
    return v


# ------------------------------------------------------------------------------- merge
@dataclass(frozen=True)
class _MergeOpts:
    parallel: bool          # MergeParallelList: apply directive lists (server) vs keep them (merging two patches)
    ignore_nulls: bool      # IgnoreUnmatchedNulls


_SERVER = _MergeOpts(parallel=True, ignore_nulls=True)
_PATCHES = _MergeOpts(parallel=False, ignore_nulls=False)


def _retain_keys(original: dict, patch: dict, o: _MergeOpts):
    if RETAIN_KEYS not in patch:
        return
    rk = patch.pop(RETAIN_KEYS)
    if not o.parallel:
        if RETAIN_KEYS in original:
            if original[RETAIN_KEYS] != rk:
                raise PatchError(f"{original[RETAIN_KEYS]} and {rk} are not deep equal")
        else:
            original[RETAIN_KEYS] = rk
        return
    if not isinstance(rk, list):
        raise PatchError("invalid patch: $retainKeys must be a list")
    keep = set(rk)
    for k, v in patch.items():
        if v is None or k.startswith(DELETE_PRIMITIVE + "/") or k.startswith(SET_ORDER + "/"):
            continue
        if k not in keep:
            raise PatchError(f"invalid patch: {k!r} is not listed in $retainKeys")
    for k in [k for k in original if k not in keep]:
        del original[k]


def _field_key(k: str, prefix: str) -> str:
    head, sep, rest = k.partition("/")
    if not sep or head != prefix or not rest:
        raise PatchError(f"invalid patch: malformed {prefix} directive {k!r}")
    return rest


def _set_element_order(original: dict, patch: dict, node, o: _MergeOpts):
    for key in [k for k in patch if k.startswith(SET_ORDER + "/") or k == SET_ORDER]:
        order = patch.pop(key)
        if not o.parallel:
            if key in original:
                if original[key] != order:
                    raise PatchError("invalid patch: conflicting $setElementOrder lists")
            else:
                original[key] = order
        if not isinstance(order, list):
            raise PatchError("invalid patch: $setElementOrder must be a list")
        field = _field_key(key, SET_ORDER)
        child, strat, mk, _ = _lookup(node, field)
        ol, pl = original.get(field), patch.get(field)
        if ol is not None and not isinstance(ol, list) or pl is not None and not isinstance(pl, list):
            raise PatchError(f"invalid patch: {field} is not a list")
        _check_order(pl or [], order, mk)
        if ol is not None and pl is None:
            merged = ol
        elif ol is None and pl is not None:
            merged = pl
        elif ol is not None:
            merged = _merge_slice(ol, pl, child, mk, o, False) if strat == MERGE else pl
        else:
            continue
        patch.pop(field, None)
        if not merged:
            original[field] = merged
            continue
        inp, srv = _partition(merged, order, mk)
        kind = _elem_kind(ol or [], pl or [], merged)
        server_order = ol or []
        if o.parallel and kind == "map" and strat == MERGE and ol and pl:
            server_order = _go_aliased_view(ol, pl, mk)
        original[field] = _normalize_element_order(inp, srv, order, server_order, mk, kind)


def _go_cap(n: int) -> int:
    """Capacity encoding/json gives a decoded n-element array (grow by 1.5x, at least 4)."""
    cap = 0
    while cap < n:
        cap = max(4, cap + cap // 2)
    return cap


def _go_aliased_view(ol: list, pl: list, mk: str) -> list:
    """The live list as the reference's order normalisation sees it after mergeSlice: Go's
    in-place delete (`append(s[:k], s[k+1:]...)`) and append into spare capacity rewrite the
    backing array the live list still points at (patch.go mergePatchIntoOriginal passes that
    slice as the server order). The reference's table expectations bake this in."""
    n, cap = len(ol), _go_cap(len(ol))
    backing, length = list(ol) + [None] * (cap - n), n
    rest = []
    for pv in pl:
        if not isinstance(pv, dict):
            return ol
        d = pv.get(DIRECTIVE)
        if d is None:
            rest.append(pv)
        elif d == DELETE and mk in pv:
            while True:
                k = next((i for i in range(length) if isinstance(backing[i], dict) and backing[i].get(mk) == pv[mk]), -1)
                if k < 0:
                    break
                backing[k:length - 1] = backing[k + 1:length]
                length -= 1
        elif d == REPLACE:
            return backing[:n]
    for pv in rest:
        if any(isinstance(backing[i], dict) and backing[i].get(mk) == pv.get(mk) for i in range(length)):
            continue
        if length >= cap:
            break                   # append reallocates: later writes no longer reach the live list
        backing[length] = pv
        length += 1
    return backing[:n]


def _check_order(plist: list, order: list, mk: str):
    """validatePatchWithSetOrderList: the patch's items appear in $setElementOrder, in order."""
    if not order or not plist:
        return
    items = [x for x in plist if not (isinstance(x, dict) and x.get(DIRECTIVE) == DELETE)] if mk else plist
    pi = oi = 0
    while pi < len(items) and oi < len(order):
        it = items[pi]
        if isinstance(it, dict) and DIRECTIVE in it:
            pi += 1
            continue
        eq = (_mk(it, mk) == _mk(order[oi], mk)) if mk else it == order[oi]
        if eq:
            pi += 1
        oi += 1
    if pi < len(items) and oi >= len(order):
        raise PatchError(f"the order in patch list {plist} doesn't match $setElementOrder list {order}")


def _merge_map(original: dict | None, patch: dict, node, o: _MergeOpts) -> dict:
    if DIRECTIVE in patch:
        d = patch[DIRECTIVE]
        if d == REPLACE:
            p = dict(patch)
            del p[DIRECTIVE]
            return p
        if d == DELETE:
            return {}
        if d != MERGE:
            raise PatchError(f"unknown patch type: {d!r} in map: {patch}")
        patch = {k: v for k, v in patch.items() if k != DIRECTIVE}
    if original is None:
        original = {}
    _retain_keys(original, patch, o)
    _set_element_order(original, patch, node, o)
    for k, pv in list(patch.items()):
        delete_list = False
        if k.startswith(DELETE_PRIMITIVE + "/") or k == DELETE_PRIMITIVE:
            if not o.parallel:
                original[k] = pv
                continue
            k = _field_key(k, DELETE_PRIMITIVE)
            delete_list = True
            if k not in original:
                continue                # nothing to delete from
        if pv is None:
            original.pop(k, None)
            if o.ignore_nulls:
                continue
        if k not in original:
            original[k] = pv
            continue
        ov = original[k]
        if _kind(ov) != _kind(pv):
            original[k] = pv
            continue
        if isinstance(ov, dict):
            child, strat, _, _ = _lookup(node, k)
            original[k] = pv if strat == REPLACE else _merge_map(ov, pv, child, o)
        elif isinstance(ov, list):
            child, strat, mk, _ = _lookup(node, k)
            original[k] = _merge_slice(ov, pv, child, mk, o, delete_list) if strat == MERGE else pv
        else:
            original[k] = pv
    return original


def _merge_slice(original: list, patch: list, node, mk: str, o: _MergeOpts, delete_list: bool) -> list:
    if not original and not patch:
        return original
    kind = _elem_kind(original, patch)
    if kind != "map":
        if o.parallel and delete_list:
            return [v for v in original if v not in patch]
        merged = _dedup(original + patch)
    else:
        if not mk:
            raise PatchError("cannot merge lists without merge key")
        original, patch = _special_elements(list(original), patch, mk)
        merged = list(original)
        for pv in patch:
            i = _find(merged, mk, _mk(pv, mk))
            if i >= 0:
                merged[i] = _merge_map(merged[i], pv, node, o)
            else:
                merged.append(pv)
    inp, srv = _partition(merged, patch, mk if kind == "map" else "")
    return _normalize_element_order(inp, srv, patch, original, mk, kind)


def _special_elements(original: list, patch: list, mk: str):
    rest, replace_all = [], False
    for pv in patch:
        if not isinstance(pv, dict):
            raise PatchError(f"expected a map in a merge list, got {_kind(pv)}")
        if DIRECTIVE not in pv:
            rest.append(pv)
            continue
        d = pv[DIRECTIVE]
        if d == DELETE:
            if mk not in pv:
                raise PatchError(f"map: {pv} does not contain declared merge key: {mk}")
            original = [x for x in original if not (isinstance(x, dict) and mk in x and x[mk] == pv[mk])]
        elif d == REPLACE:
            replace_all = True
        elif d == MERGE:
            raise PatchError("merging lists cannot yet be specified in the patch")
        else:
            raise PatchError(f"unknown patch type: {d!r} in map: {pv}")
    if replace_all:
        return rest, []
    return original, rest


def apply(original: dict, patch: dict, node=None) -> dict:
    """StrategicMergePatch: `patch` applied to `original` (neither is modified)."""
    if not isinstance(patch, dict):
        raise PatchError("a strategic merge patch must be a JSON object")
    out = _merge_map(copy.deepcopy(original), copy.deepcopy(patch), node, _SERVER)
    return strip_directives(out)


def merge_patches(first: dict, second: dict, node=None) -> dict:
    """Two patches merged into one that has the effect of both (directive lists are kept)."""
    return _merge_map(copy.deepcopy(first), copy.deepcopy(second), node, _PATCHES)


# ------------------------------------------------------------------------------- diff
@dataclass(frozen=True)
class _DiffOpts:
    ignore_deletions: bool = False
    ignore_changes: bool = False          # IgnoreChangesAndAdditions
    set_order: bool = False
    build_retain: bool = False


def _diff_maps(original: dict, modified: dict, node, o: _DiffOpts) -> dict:
    patch: dict = {}
    retain = []
    for k, mv in modified.items():
        if o.build_retain and mv is not None:
            retain.append(k)
        if k not in original:
            if not o.ignore_changes:
                patch[k] = mv
            continue
        ov = original[k]
        if k == DIRECTIVE:
            if not isinstance(ov, str) or not isinstance(mv, str):
                raise PatchError(f"invalid value for special key: {DIRECTIVE}")
            if ov != mv:
                patch[k] = mv
            continue
        if _kind(ov) != _kind(mv):
            if not o.ignore_changes:
                patch[k] = mv
            continue
        if isinstance(ov, dict):
            child, strat, _, retain_sub = _lookup(node, k)
            if strat == REPLACE:
                if not o.ignore_changes:
                    patch[k] = mv
            else:
                pv = _diff_maps(ov, mv, child, replace(o, build_retain=retain_sub))
                if pv:
                    patch[k] = pv
        elif isinstance(ov, list):
            child, strat, mk, retain_sub = _lookup(node, k)
            if strat == MERGE:
                add, dele, order = _diff_lists(ov, mv, child, mk, replace(o, build_retain=retain_sub))
                if add:
                    patch[k] = add
                if dele:
                    patch[f"{DELETE_PRIMITIVE}/{k}"] = dele
                if order:
                    patch[f"{SET_ORDER}/{k}"] = order
            elif not o.ignore_changes and ov != mv:
                patch[k] = mv
        elif not o.ignore_changes and ov != mv:
            patch[k] = mv
    if not o.ignore_deletions:
        for k in original:
            if k not in modified:
                patch[k] = None
    if retain and (patch or any(v is not None and k not in modified for k, v in original.items())):
        patch[RETAIN_KEYS] = _sort_scalars(retain)
    return patch


def _diff_lists(original: list, modified: list, node, mk: str, o: _DiffOpts):
    if not original:
        if not modified or o.ignore_changes:
            return None, None, None
        return modified, None, None
    kind = _elem_kind(original, modified)
    order = None
    if kind == "map":
        plist, dlist = _diff_lists_of_maps(original, modified, node, mk, o)
        plist = _normalize_slice_order(plist, modified, mk, kind)
        same = len(original) == len(modified) and all(_mk(a, mk) == _mk(b, mk) for a, b in zip(original, modified))
        plist = plist + dlist
        dlist = None
        if o.set_order and ((not o.ignore_changes and (plist or not same)) or (not o.ignore_deletions and plist)):
            order = [{mk: _mk(v, mk)} for v in modified]
    else:
        plist, dlist = _diff_lists_of_scalars(original, modified, o)
        plist = _normalize_slice_order(plist, modified, mk, kind)
        if o.set_order and ((not o.ignore_deletions and dlist) or (not o.ignore_changes and original != modified)):
            order = modified
    return plist, dlist, order


def _diff_lists_of_scalars(original: list, modified: list, o: _DiffOpts):
    a, b = _sort_scalars(original), _sort_scalars(modified)
    i = j = 0
    add, dele = [], []
    while i < len(a) or j < len(b):
        sa = _gostr(a[i]) if i < len(a) else None
        sb = _gostr(b[j]) if j < len(b) else None
        if sa is not None and sb is not None and sa == sb:
            i += 1
            j += 1
        elif sa is None or (sb is not None and sa > sb):
            if not o.ignore_changes:
                add.append(b[j])
            j += 1
        else:
            if not o.ignore_deletions:
                dele.append(a[i])
            i += 1
    return add, _dedup(dele)


def _diff_lists_of_maps(original: list, modified: list, node, mk: str, o: _DiffOpts):
    a = sorted(original, key=lambda x: _gostr(_mk(x, mk)))
    b = sorted(modified, key=lambda x: _gostr(_mk(x, mk)))
    i = j = 0
    patch, dele = [], []
    while i < len(a) or j < len(b):
        sa = _gostr(_mk(a[i], mk)) if i < len(a) else None
        sb = _gostr(_mk(b[j], mk)) if j < len(b) else None
        if sa is not None and sb is not None and sa == sb:
            pv = _diff_maps(a[i], b[j], node, o)
            if pv:
                pv[mk] = b[j][mk]
                patch.append(pv)
            i += 1
            j += 1
        elif sa is None or (sb is not None and sa > sb):
            if not o.ignore_changes:
                patch.append(b[j])
            j += 1
        else:
            if not o.ignore_deletions:
                dele.append({mk: a[i][mk], DIRECTIVE: DELETE})
            i += 1
    return patch, dele


def create_two_way(original: dict, modified: dict, node=None) -> dict:
    """CreateTwoWayMergeMapPatch: the patch that turns `original` into `modified`."""
    return _diff_maps(original, modified, node, _DiffOpts(set_order=True))


def create_three_way(original: dict | None, modified: dict, current: dict | None, node=None,
                     overwrite: bool = True) -> dict:
    """CreateThreeWayMergePatch (patch.go:1999): current → modified without deletions, plus
    the deletions from original (the last applied configuration) to modified. With
    overwrite=False a key the patch changes differently from how current changed it since
    original is a ConflictError."""
    original, current = original or {}, current or {}
    delta = _diff_maps(current, modified, node, _DiffOpts(ignore_deletions=True, set_order=True))
    deletions = _diff_maps(original, modified, node, _DiffOpts(ignore_changes=True, set_order=True))
    patch = _merge_map(deletions, delta, node, _PATCHES)
    if not overwrite:
        changed = _diff_maps(original, current, node, _DiffOpts())
        if _conflicts(patch, changed, node, "", ""):
            raise ConflictError(f"patch {patch} conflicts with changes made from original to current {changed}")
    return patch


# ------------------------------------------------------------------------------- conflicts
def _conflicts(left, right, node, strat: str, mk: str) -> bool:
    if isinstance(left, dict):
        if not isinstance(right, dict):
            return True
        lm, rm = left.get(DIRECTIVE), right.get(DIRECTIVE)
        if (DIRECTIVE in left) != (DIRECTIVE in right) or lm != rm:
            return True
        if strat == REPLACE:
            return False
        for k, lv in left.items():
            if k in (DIRECTIVE, RETAIN_KEYS) or k not in right:
                continue
            child, s, key = None, "", ""
            if isinstance(lv, (dict, list)):
                child, s, key, _ = _lookup(node, k)
            if _conflicts(lv, right[k], child, s, key):
                return True
        return False
    if isinstance(left, list):
        if not isinstance(right, list):
            return True
        if not left and not right:
            return False
        kind = _elem_kind(left, right)
        if strat == MERGE:
            if kind != "map":
                return False
            lm_ = {_gostr(_mk(x, mk)): x for x in left}
            rm_ = {_gostr(_mk(x, mk)): x for x in right}
            return any(_conflicts(v, rm_[k], node, "", "") for k, v in lm_.items() if k in rm_)
        if len(left) != len(right):
            return True
        if kind != "map":
            left, right = _sort_scalars(_dedup(left)), _sort_scalars(_dedup(right))
        return any(_conflicts(a, b, node, "", "") for a, b in zip(left, right))
    return left != right or _kind(left) != _kind(right)


# ------------------------------------------------------------------------------- JSON merge
def _json_merge_diff(original, modified, deletions_only: bool, additions_only: bool) -> dict:
    patch = {}
    for k, mv in modified.items():
        ov = original.get(k, _MISSING)
        if ov is _MISSING:
            if not deletions_only:
                patch[k] = mv
        elif isinstance(ov, dict) and isinstance(mv, dict):
            sub = _json_merge_diff(ov, mv, deletions_only, additions_only)
            if sub:
                patch[k] = sub
        elif ov != mv and not deletions_only:
            patch[k] = mv
    if not additions_only:
        for k in original:
            if k not in modified:
                patch[k] = None
    return patch


_MISSING = object()


def _json_merge_patches(a: dict, b: dict) -> dict:
    out = dict(a)
    for k, v in b.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _json_merge_patches(out[k], v)
        else:
            out[k] = v
    return out


def create_three_way_json_merge(original: dict | None, modified: dict, current: dict | None) -> dict:
    """jsonmergepatch.CreateThreeWayJSONMergePatch: what kubectl apply sends for kinds it has
    no schema for (custom resources): lists are replaced, maps merged, dropped fields nulled."""
    original, current = original or {}, current or {}
    delta = _json_merge_diff(current, modified, False, True)
    deletions = _json_merge_diff(original, modified, True, False)
    return _json_merge_patches(deletions, delta)
