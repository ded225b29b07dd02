"""CustomResourceDefinitions (apiextensions.k8s.io/v1beta1).

Reference: staging/src/k8s.io/apiextensions-apiserver — pkg/apis/apiextensions/validation
(name = <plural>.<group>, group with a dot, scope Namespaced|Cluster, names), pkg/controller/
status/naming_controller.go (NamesAccepted, acceptedNames), pkg/controller/finalizer/
crd_finalizer.go (finalizer customresourcecleanup.apiextensions.k8s.io: instances are
deleted before the definition goes), pkg/apiserver/customresource_handler.go (a REST store
per served CRD, established once names are accepted, /status subresource when
spec.subresources.status is set) and pkg/apiserver/validation (openAPIV3Schema checked on
create/update, CustomResourceValidation beta).

Custom objects live under /registry/crd/<group>/<plural>/ so they never share a key range
with a built-in resource of the same plural.
"""
from __future__ import annotations

import asyncio
import json
import re

from ..api import meta as m
from ..api.labels import is_dns1123_label, is_dns1123_subdomain
from ..api.scheme import SCHEME, ResourceInfo
from ..store import PUT
from ..store.storage import decode_kv
from ..api.field import go_value

FINALIZER = "customresourcecleanup.apiextensions.k8s.io"
PREFIX = "/registry/customresourcedefinitions/"


# ------------------------------------------------------------------ validation
def validate_crd(crd: dict, old: dict | None = None) -> list[str]:
    errs = []
    md, spec = crd.get("metadata") or {}, crd.get("spec") or {}
    group, names = spec.get("group", ""), spec.get("names") or {}
    plural, kind = names.get("plural", ""), names.get("kind", "")
    if not group or "." not in group or is_dns1123_subdomain(group):
        errs.append("spec.group: Invalid value: should be a domain with at least one dot")
    if not spec.get("version"):
        errs.append("spec.version: Required value")
    if spec.get("scope") not in ("Namespaced", "Cluster"):
        errs.append('spec.scope: Unsupported value: supported values: "Cluster", "Namespaced"')
    if not plural or is_dns1123_label(plural):
        errs.append("spec.names.plural: Invalid value: must be a DNS-1035-style lowercase name")
    if not kind or not re.match(r"^[A-Z][A-Za-z0-9]*$", kind):
        errs.append("spec.names.kind: Invalid value: must be a CamelCase identifier")
    if md.get("name") != f"{plural}.{group}":
        errs.append(f"metadata.name: Invalid value: must be spec.names.plural+\".\"+spec.group")
    for sn in names.get("shortNames") or []:
        if is_dns1123_label(sn):
            errs.append(f"spec.names.shortNames: Invalid value: {go_value(sn)}")
    if old is not None:
        for f in ("group", "scope"):
            if (old.get("spec") or {}).get(f) != spec.get(f):
                errs.append(f"spec.{f}: Invalid value: field is immutable")
    schema = (spec.get("validation") or {}).get("openAPIV3Schema")
    if schema is not None and not isinstance(schema, dict):
        errs.append("spec.validation.openAPIV3Schema: Invalid value: must be an object")
    return errs


_TYPES = {"object": dict, "array": list, "string": str, "boolean": bool}


def validate_schema(v, s: dict, path: str = "") -> list[str]:
    """The openAPIV3Schema subset CRD authors use: type, properties, required,
    additionalProperties, items, enum, minimum/maximum (+exclusive), multipleOf, min/maxLength,
    pattern, min/maxItems, uniqueItems, min/maxProperties, allOf/anyOf/oneOf/not, nullable."""
    errs: list[str] = []
    p = path or "<root>"
    if v is None and s.get("nullable"):
        return errs
    t = s.get("type")
    if t == "integer":
        if not (isinstance(v, int) and not isinstance(v, bool)):
            return [f"{p}: Invalid value: must be of type integer"]
    elif t == "number":
        if not (isinstance(v, (int, float)) and not isinstance(v, bool)):
            return [f"{p}: Invalid value: must be of type number"]
    elif t in _TYPES and not isinstance(v, _TYPES[t]):
        return [f"{p}: Invalid value: must be of type {t}"]
    if "enum" in s and v not in s["enum"]:
        errs.append(f"{p}: Unsupported value: {go_value(v)}: supported values: {', '.join(map(repr, s['enum']))}")
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        if "minimum" in s and (v < s["minimum"] or (s.get("exclusiveMinimum") and v == s["minimum"])):
            errs.append(f"{p}: Invalid value: {v}: should be greater than {'' if s.get('exclusiveMinimum') else 'or equal to '}{s['minimum']}")
        if "maximum" in s and (v > s["maximum"] or (s.get("exclusiveMaximum") and v == s["maximum"])):
            errs.append(f"{p}: Invalid value: {v}: should be less than {'' if s.get('exclusiveMaximum') else 'or equal to '}{s['maximum']}")
        if s.get("multipleOf") and (v / s["multipleOf"]) != int(v / s["multipleOf"]):
            errs.append(f"{p}: Invalid value: {v}: should be a multiple of {s['multipleOf']}")
    if isinstance(v, str):
        if "minLength" in s and len(v) < s["minLength"]:
            errs.append(f"{p}: Invalid value: should be at least {s['minLength']} chars long")
        if "maxLength" in s and len(v) > s["maxLength"]:
            errs.append(f"{p}: Invalid value: should be at most {s['maxLength']} chars long")
        if "pattern" in s and not re.search(s["pattern"], v):
            errs.append(f"{p}: Invalid value: {go_value(v)}: should match {s['pattern']!r}")
    if isinstance(v, list):
        if "minItems" in s and len(v) < s["minItems"]:
            errs.append(f"{p}: Invalid value: should have at least {s['minItems']} items")
        if "maxItems" in s and len(v) > s["maxItems"]:
            errs.append(f"{p}: Invalid value: should have at most {s['maxItems']} items")
        if s.get("uniqueItems") and len({json.dumps(x, sort_keys=True) for x in v}) != len(v):
            errs.append(f"{p}: Duplicate value: items must be unique")
        if isinstance(s.get("items"), dict):
            for i, x in enumerate(v):
                errs += validate_schema(x, s["items"], f"{path}[{i}]")
    if isinstance(v, dict):
        props = s.get("properties") or {}
        for r in s.get("required") or []:
            if r not in v:
                errs.append(f"{path + '.' if path else ''}{r}: Required value")
        if "minProperties" in s and len(v) < s["minProperties"]:
            errs.append(f"{p}: Invalid value: should have at least {s['minProperties']} properties")
        if "maxProperties" in s and len(v) > s["maxProperties"]:
            errs.append(f"{p}: Invalid value: should have at most {s['maxProperties']} properties")
        addl = s.get("additionalProperties", True)
        for k, x in v.items():
            sub = f"{path}.{k}" if path else k
            if k in props:
                errs += validate_schema(x, props[k], sub)
            elif addl is False:
                errs.append(f"{sub}: Forbidden: field not declared in the schema")
            elif isinstance(addl, dict):
                errs += validate_schema(x, addl, sub)
    for sub_s in s.get("allOf") or []:
        errs += validate_schema(v, sub_s, path)
    if s.get("anyOf") and not any(not validate_schema(v, x, path) for x in s["anyOf"]):
        errs.append(f"{p}: Invalid value: must validate against at least one schema (anyOf)")
    if s.get("oneOf") and sum(1 for x in s["oneOf"] if not validate_schema(v, x, path)) != 1:
        errs.append(f"{p}: Invalid value: must validate against exactly one schema (oneOf)")
    if isinstance(s.get("not"), dict) and not validate_schema(v, s["not"], path):
        errs.append(f"{p}: Invalid value: must not validate against the schema (not)")
    return errs


def resource_info(crd: dict) -> ResourceInfo:
    spec = crd["spec"]
    names = spec["names"]
    subs = ("status",) if "status" in (spec.get("subresources") or {}) else ()
    if "scale" in (spec.get("subresources") or {}):
        subs += ("scale",)
    schema = (spec.get("validation") or {}).get("openAPIV3Schema")

    def validator(obj, old=None):
        from ..api.validation import validate_object_meta
        errs = validate_object_meta(obj, spec.get("scope") == "Namespaced")
        if schema:
            body = {k: v for k, v in obj.items() if k not in ("metadata", "apiVersion", "kind")}
            errs += validate_schema(body, {k: v for k, v in schema.items() if k != "properties"} |
                                    {"properties": {k: v for k, v in (schema.get("properties") or {}).items()
                                                    if k not in ("metadata", "apiVersion", "kind")}})
        return errs
    return ResourceInfo(spec["group"], spec["version"], names["kind"], names["plural"], spec.get("scope") == "Namespaced",
                        tuple(names.get("shortNames") or ()) + ((names["singular"],) if names.get("singular") else ()),
                        subs, names.get("listKind") or names["kind"] + "List", validator=validator)


class CRDManager:
    """Serves a REST store for every established CRD and runs the naming and cleanup loops."""

    def __init__(self, registry):
        self.registry = registry
        self.installed: dict[str, ResourceInfo] = {}   # crd name -> resource info
        self._pending: set[str] = set()
        self._wake: asyncio.Event | None = None
        self._task = None
        registry.store.commit_hooks.append(self._on_commit)
        kvs, _, _ = registry.store.range(PREFIX)
        for kv in kvs:
            self._install(decode_kv(kv.value))

    def start(self):
        self._wake = asyncio.Event()
        self._task = asyncio.create_task(self._loop(), name="crd-controllers")
        self._pending.update(self.installed)
        self._wake.set()
        return self

    async def stop(self):
        from ..utils import cancel_and_wait
        await cancel_and_wait([self._task])

    # ------------------------------------------------------------ serving
    def _install(self, crd: dict):
        from .registry import ResourceStore
        name = m.name_of(crd)
        if (crd.get("metadata") or {}).get("deletionTimestamp") and name not in self.installed:
            return
        ri = resource_info(crd)
        old = self.installed.get(name)
        if old is not None and (old.group, old.plural) != (ri.group, ri.plural):
            self._uninstall(name)
        clash = SCHEME.for_plural(ri.group, ri.plural)
        if clash is not None and name not in self.installed:
            return   # a built-in resource already owns this group/plural
        self.installed[name] = ri
        _scheme_replace(ri, old)
        store = ResourceStore(self.registry, ri)
        store.storage_prefix = f"/registry/crd/{ri.group}/{ri.plural}"
        store.has_status = "status" in ri.subresources
        self.registry.resources[(ri.group, ri.plural)] = store

    def _uninstall(self, name: str):
        ri = self.installed.pop(name, None)
        if ri is None:
            return
        self.registry.resources.pop((ri.group, ri.plural), None)
        _scheme_remove(ri)

    def _on_commit(self, ev):
        k = ev.kv.key
        if not k.startswith(PREFIX):
            return
        name = k[len(PREFIX):]
        if ev.type == PUT:
            self._install(decode_kv(ev.kv.value))
        else:
            self._uninstall(name)
        self._pending.add(name)
        if self._wake is not None:
            self._wake.set()

    # ------------------------------------------------------------ controllers
    async def _loop(self):
        while True:
            await self._wake.wait()
            self._wake.clear()
            for name in list(self._pending):
                self._pending.discard(name)
                try:
                    await self._reconcile(name)
                except Exception:
                    self._pending.add(name)
                    asyncio.get_running_loop().call_later(0.5, self._wake.set)

    async def _reconcile(self, name: str):
        rs = self.registry.rs("customresourcedefinitions", "apiextensions.k8s.io")
        try:
            crd = rs.get("", name)
        except m.StatusError:
            return
        md = crd.get("metadata") or {}
        if md.get("deletionTimestamp"):
            ri = self.installed.get(name)
            if ri is not None:   # crd_finalizer: delete every instance, then release the definition
                store = self.registry.resources.get((ri.group, ri.plural))
                if store is not None:
                    objs = store.list()[0]
                    for o in objs:
                        try:
                            store.delete(m.namespace_of(o), m.name_of(o), grace=0)
                        except m.StatusError:
                            pass
            fins = [f for f in md.get("finalizers") or [] if f != FINALIZER]
            rs.update("", name, None, patch=json.dumps({"metadata": {"finalizers": fins or None}}).encode(),
                      content_type="application/merge-patch+json")
            return
        if FINALIZER not in (md.get("finalizers") or []):
            rs.update("", name, None, patch=json.dumps({"metadata": {"finalizers": list(md.get("finalizers") or []) + [FINALIZER]}}).encode(),
                      content_type="application/merge-patch+json")
            crd = rs.get("", name)
        names = (crd.get("spec") or {}).get("names") or {}
        ok = name in self.installed
        now = m.now_rfc3339()
        conds = [{"type": "NamesAccepted", "status": "True" if ok else "False",
                  "reason": "NoConflicts" if ok else "ResourceConflict",
                  "message": "no conflicts found" if ok else "the group/plural is served by a built-in resource",
                  "lastTransitionTime": now},
                 {"type": "Established", "status": "True" if ok else "False",
                  "reason": "InitialNamesAccepted" if ok else "NotAccepted",
                  "message": "the initial names have been accepted" if ok else "not all names are accepted",
                  "lastTransitionTime": now}]
        old = (crd.get("status") or {})
        prev = {c["type"]: c for c in old.get("conditions") or []}
        for c in conds:
            p = prev.get(c["type"])
            if p is not None and p.get("status") == c["status"]:
                c["lastTransitionTime"] = p.get("lastTransitionTime", now)
        st = {"conditions": conds, "acceptedNames": names if ok else {}}
        if old != st:
            crd["status"] = st
            rs.update("", name, crd, subresource="status")


def _scheme_replace(ri: ResourceInfo, old: ResourceInfo | None):
    if old is not None:
        _scheme_remove(old)
    SCHEME.add(ri)


def _scheme_remove(ri: ResourceInfo):
    SCHEME.by_kind.pop((ri.api_version, ri.kind), None)
    SCHEME.by_plural.pop((ri.group, ri.plural), None)
    SCHEME.by_gvr.pop((ri.group, ri.version, ri.plural), None)
    for k in [k for k, v in SCHEME.by_name.items() if v is ri]:
        del SCHEME.by_name[k]
