"""OpenAPI v2 document of the served API, schema validation, and the field explainer.

Reference: the apiserver publishes /swagger.json and /openapi/v2 (staging/src/k8s.io/apiserver/
pkg/server/routes/openapi.go, kube-openapi builder); kubectl 1.9 downloads it for
`kubectl explain` (pkg/kubectl/explain/{explain,model_printer,recursive_fields_printer}.go) and
for client-side `--validate` (pkg/kubectl/cmd/util/openapi/validation, kube-openapi
pkg/util/proto/validation: "unknown field", "missing required field", "invalid type" errors).

The definitions come from the compact table in `openapi_types.py`; the paths and the
x-kubernetes-group-version-kind extensions come from the live Scheme, so every served version
(including the served-only aliases such as extensions/v1beta1 Deployment) points at the
definition of its storage kind.
"""
from __future__ import annotations

import functools
import json

from .scheme import SCHEME
from .openapi_types import TYPES

META = "io.k8s.apimachinery.pkg.apis.meta.v1"
QUANTITY = "io.k8s.apimachinery.pkg.api.resource.Quantity"
INT_OR_STRING = "io.k8s.apimachinery.pkg.util.intstr.IntOrString"
TIME = f"{META}.Time"
MICROTIME = f"{META}.MicroTime"
PRIMS = {"string": {"type": "string"}, "integer": {"type": "integer", "format": "int32"},
         "long": {"type": "integer", "format": "int64"}, "boolean": {"type": "boolean"},
         "number": {"type": "number", "format": "double"}, "byte": {"type": "string", "format": "byte"},
         "object": {"type": "object"}}
KIND_FIELDS = (("apiVersion", "string", "Versioned schema of this representation of the object; the server rewrites it to the version requested."),
               ("kind", "string", "REST resource type of the object, in CamelCase."),
               ("metadata", f"{META}.ObjectMeta", "Standard object metadata."))


def _parse(text: str) -> tuple[dict, dict]:
    """Table → ({definition id: raw definition}, {definition id: prefix})."""
    raw, prefix_of, prefix, cur = {}, {}, "", None
    for line in text.splitlines():
        if not line.strip():
            continue
        if line.startswith("@"):
            prefix = line[1:].strip()
            continue
        if not line.startswith(" "):
            head, _, desc = line.partition("  ")
            name, *flags = head.split()
            cur = f"{prefix}.{name}"
            raw[cur] = {"desc": desc.strip(), "kind": "+kind" in flags, "fields": []}
            prefix_of[cur] = prefix
            if raw[cur]["kind"]:
                # +meta! : the reference marks metadata required on this kind (core/v1 Event)
                raw[cur]["fields"] += [(n, t, n == "metadata" and "+meta!" in flags, d) for n, t, d in KIND_FIELDS]
            continue
        body, _, desc = line.strip().partition("  ")
        fname, ftype = body.split()[:2]
        raw[cur]["fields"].append((fname, ftype.rstrip("!"), ftype.endswith("!"), desc.strip()))
    return raw, prefix_of


def _resolver(raw: dict, prefix_of: dict):
    by_short: dict[str, list[str]] = {}
    for full in raw:
        by_short.setdefault(full.rsplit(".", 1)[1], []).append(full)

    def ref(t: str, home: str) -> dict:
        if t.startswith("[]"):
            return {"type": "array", "items": ref(t[2:], home)}
        if t.startswith("{}"):
            return {"type": "object", "additionalProperties": ref(t[2:], home)}
        if t in PRIMS:
            return dict(PRIMS[t])
        if t == "time":
            return {"$ref": f"#/definitions/{TIME}"}
        if t == "microtime":
            return {"$ref": f"#/definitions/{MICROTIME}"}
        if t == "quantity":
            return {"$ref": f"#/definitions/{QUANTITY}"}
        if t == "ios":
            return {"$ref": f"#/definitions/{INT_OR_STRING}"}
        if t in raw:
            return {"$ref": f"#/definitions/{t}"}
        cands = by_short.get(t, [])
        same = [c for c in cands if prefix_of[c] == home]
        pick = same or cands
        if len(pick) != 1:
            raise ValueError(f"openapi table: cannot resolve type {t!r} from {home} ({cands})")
        return {"$ref": f"#/definitions/{pick[0]}"}
    return ref


def _kind_defs(defs: dict) -> dict:
    """GVK → definition id for every served kind (aliases map to their storage kind's definition)."""
    by_kind: dict[str, list[str]] = {}
    for full in defs:
        by_kind.setdefault(full.rsplit(".", 1)[1], []).append(full)
    out = {}
    for ri in SCHEME.by_kind.values():
        own = f"io.k8s.api.{ri.group.split('.')[0] if ri.group else 'core'}.{ri.version}.{ri.kind}"
        if own in defs:     # a version with its own shape (extensions/v1beta1 Deployment: rollbackTo)
            out[(ri.group, ri.version, ri.kind)] = own
            continue
        canon = SCHEME.storage_of(ri)
        cands = by_kind.get(canon.kind, [])
        grp = canon.group.split(".")[0] if canon.group else "core"
        pick = [c for c in cands if f".{grp}." in c or f"{grp}-" in c]
        if pick:
            out[(ri.group, ri.version, ri.kind)] = pick[0]
    return out


@functools.lru_cache(maxsize=1)
def definitions() -> dict:
    raw, prefix_of = _parse(TYPES)
    ref = _resolver(raw, prefix_of)
    defs = {TIME: {"description": "RFC 3339 timestamp with second precision.", "type": "string", "format": "date-time"},
            MICROTIME: {"description": "RFC 3339 timestamp with microsecond precision.", "type": "string",
                        "format": "date-time"},
            QUANTITY: {"description": "A fixed-point quantity such as 4, 500m, 288Gi or 1e3.", "type": "string"},
            INT_OR_STRING: {"description": "An integer or a string (a port number or name, a count or a percentage).",
                            "type": "string", "format": "int-or-string"}}
    for full, d in raw.items():
        if full == TIME:
            continue
        props, req = {}, []
        for fname, ftype, required, desc in d["fields"]:
            p = ref(ftype, prefix_of[full])
            if desc:
                p["description"] = desc
            props[fname] = p
            if required:
                req.append(fname)
        defs[full] = {"description": d["desc"], "properties": props}
        if req:
            defs[full]["required"] = req
    # the strategic-merge-patch struct tags, as the reference's swagger.json carries them
    from .patchmeta import PATCH_META
    for full, fields in PATCH_META.items():
        for fname, (strategy, key) in fields.items():
            p = (defs.get(full) or {}).get("properties", {}).get(fname)
            if p is not None:
                p["x-kubernetes-patch-strategy"] = strategy
                if key:
                    p["x-kubernetes-patch-merge-key"] = key
    kinds = _kind_defs(defs)
    for (g, v, k), full in sorted(kinds.items()):
        defs[full].setdefault("x-kubernetes-group-version-kind", []).append({"group": g, "version": v, "kind": k})
        ri = SCHEME.for_kind(f"{g}/{v}" if g else v, k)
        list_id = f"{full}List"
        if ri is None or not raw.get(full, {}).get("kind"):
            continue
        if list_id not in defs:
            defs[list_id] = {"description": f"A list of {k} objects.", "required": ["items"], "properties": {
                "apiVersion": {"type": "string", "description": KIND_FIELDS[0][2]},
                "items": {"type": "array", "items": {"$ref": f"#/definitions/{full}"}, "description": f"The {k} objects."},
                "kind": {"type": "string", "description": KIND_FIELDS[1][2]},
                "metadata": {"$ref": f"#/definitions/{META}.ListMeta", "description": "Standard list metadata."}}}
        defs[list_id].setdefault("x-kubernetes-group-version-kind", []).append({"group": g, "version": v, "kind": ri.list_kind})
    return defs


def kind_definition(api_version: str, kind: str) -> str | None:
    g, _, v = api_version.rpartition("/")
    defs = definitions()
    hit = _kind_defs(defs).get((g, v, kind))
    if hit:
        return hit
    for full, d in defs.items():
        for gvk in d.get("x-kubernetes-group-version-kind", ()):
            if (gvk["group"], gvk["version"], gvk["kind"]) == (g, v, kind):
                return full
    return None


def _params(ri) -> list[dict]:
    out = [{"name": "pretty", "in": "query", "type": "string", "uniqueItems": True,
            "description": "If 'true', the output is pretty printed."}]
    if ri.namespaced:
        out.append({"name": "namespace", "in": "path", "required": True, "type": "string", "uniqueItems": True,
                    "description": "object name and auth scope"})
    return out


_LIST_Q = [{"name": n, "in": "query", "type": t, "uniqueItems": True} for n, t in
           (("labelSelector", "string"), ("fieldSelector", "string"), ("resourceVersion", "string"),
            ("timeoutSeconds", "integer"), ("watch", "boolean"), ("limit", "integer"), ("continue", "string"),
            ("includeUninitialized", "boolean"))]


def document(version: str = "v1.9.11-amdkube") -> dict:
    """The Swagger 2.0 document (/openapi/v2, /swagger.json)."""
    defs = definitions()
    paths: dict[str, dict] = {}
    for ri in sorted(SCHEME.by_kind.values(), key=lambda r: (r.group, r.version, r.plural)):
        full = kind_definition(ri.api_version, ri.kind)
        if full is None:
            continue
        ref = {"$ref": f"#/definitions/{full}"}
        lref = {"$ref": f"#/definitions/{full}List"} if f"{full}List" in defs else {"type": "object"}
        gvk = {"group": ri.group, "version": ri.version, "kind": ri.kind}
        tag = (ri.group.replace(".k8s.io", "").replace(".", "_") or "core") + "_" + ri.version
        op = f"{ri.version[0].upper()}{ri.version[1:]}"
        cap = lambda s: s[:1].upper() + s[1:]   # noqa: E731
        grp = "".join(cap(p) for p in (ri.group.replace(".k8s.io", "").split(".") if ri.group else ["core"]))
        ns_part = "Namespaced" if ri.namespaced else ""
        base = ri.api_prefix() + ("/namespaces/{namespace}" if ri.namespaced else "") + f"/{ri.plural}"
        verbs = set(ri.verbs)

        def o(action, name, resp, params=(), body=None, consumes=None):
            d = {"description": f"{action} {ri.kind}", "operationId": f"{name}{grp}{op}{ns_part}{ri.kind}",
                 "tags": [tag], "produces": ["application/json", "application/yaml", "application/vnd.kubernetes.protobuf"],
                 "schemes": ["https"], "x-kubernetes-action": action, "x-kubernetes-group-version-kind": gvk,
                 "responses": {"200": {"description": "OK", "schema": resp}, "401": {"description": "Unauthorized"}}}
            if params or body:
                d["parameters"] = list(params) + ([{"name": "body", "in": "body", "required": True, "schema": body}] if body else [])
            if consumes:
                d["consumes"] = consumes
            return d
        coll = {"parameters": _params(ri)}
        if "list" in verbs:
            coll["get"] = o("list", "list", lref, _LIST_Q)
        if "create" in verbs:
            coll["post"] = o("post", "create", ref, body=ref)
        if "deletecollection" in verbs:
            coll["delete"] = o("deletecollection", "deleteCollection", {"$ref": f"#/definitions/{META}.Status"}, _LIST_Q)
        paths[base] = coll
        item = {"parameters": [{"name": "name", "in": "path", "required": True, "type": "string", "uniqueItems": True,
                                "description": f"name of the {ri.kind}"}] + _params(ri)}
        if "get" in verbs:
            item["get"] = o("get", "read", ref)
        if "update" in verbs:
            item["put"] = o("put", "replace", ref, body=ref)
        if "patch" in verbs:
            item["patch"] = o("patch", "patch", ref, body={"type": "object"},
                              consumes=["application/json-patch+json", "application/merge-patch+json",
                                        "application/strategic-merge-patch+json"])
        if "delete" in verbs:
            item["delete"] = o("delete", "delete", {"$ref": f"#/definitions/{META}.Status"},
                               body={"$ref": f"#/definitions/{META}.DeleteOptions"})
        paths[base + "/{name}"] = item
        if "watch" in verbs:
            wbase = ri.api_prefix() + "/watch" + ("/namespaces/{namespace}" if ri.namespaced else "") + f"/{ri.plural}"
            paths[wbase] = {"parameters": _params(ri) + _LIST_Q,
                            "get": o("watchList", "watch", {"$ref": f"#/definitions/{META}.WatchEvent"})}
        for sub in ri.subresources:
            if sub in ("status", "scale"):
                sref = ref if sub == "status" else {"$ref": "#/definitions/io.k8s.api.autoscaling.v1.Scale"}
                paths[base + "/{name}/" + sub] = {"parameters": item["parameters"],
                                                  "get": o("get", f"read{cap(sub)}", sref),
                                                  "put": o("put", f"replace{cap(sub)}", sref, body=sref)}
    for p, d in (("/version/", "get the code version"), ("/api/", "get available API versions"),
                 ("/apis/", "get available API groups"), ("/healthz", "liveness")):
        paths[p] = {"get": {"description": d, "operationId": "get" + "".join(cap(x) for x in p.strip("/").split("/")) + "Info",
                            "produces": ["application/json"], "schemes": ["https"],
                            "responses": {"200": {"description": "OK"}}}}
    return {"swagger": "2.0", "info": {"title": "Kubernetes", "version": version}, "paths": paths,
            "definitions": defs, "securityDefinitions": {"BearerToken": {"type": "apiKey", "name": "authorization",
                                                                           "in": "header"}},
            "security": [{"BearerToken": []}]}


@functools.lru_cache(maxsize=4)
def document_bytes(version: str = "v1.9.11-amdkube") -> bytes:
    return json.dumps(document(version), separators=(",", ":"), sort_keys=True).encode()


# ------------------------------------------------------------------------------ validation
def _deref(defs: dict, schema: dict) -> tuple[str | None, dict]:
    if "$ref" in schema:
        name = schema["$ref"].rsplit("/", 1)[1]
        return name, defs.get(name, {})
    return None, schema


def _json_type(v) -> str:
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, int):
        return "integer"
    if isinstance(v, float):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, list):
        return "array"
    if isinstance(v, dict):
        return "object"
    return "null"


def _check(defs: dict, schema: dict, v, path: str, errs: list, owner: str | None, fname: str | None):
    name, s = _deref(defs, schema)
    if v is None:
        return
    t, fmt = s.get("type"), s.get("format")
    got = _json_type(v)
    where = f"{owner}.{fname}" if owner and fname else (name or path)

    def bad(expected):
        errs.append(f'ValidationError({path}): invalid type for {where}: got "{got}", expected "{expected}"')
    if fmt == "int-or-string":
        if got not in ("integer", "string"):
            bad("integer or string")
        return
    if name == QUANTITY:
        if got not in ("integer", "number", "string"):
            bad("string")
        return
    if t == "array":
        if got != "array":
            bad("array")
            return
        for i, item in enumerate(v):
            _check(defs, s.get("items", {}), item, f"{path}[{i}]", errs, owner, fname)
        return
    if "properties" in s:
        if got != "object":
            bad("map" if name is None else "object")
            return
        props = s["properties"]
        for k, sub in v.items():
            if k not in props:
                errs.append(f'ValidationError({path}): unknown field "{k}" in {name}')
                continue
            _check(defs, props[k], sub, f"{path}.{k}", errs, name, k)
        for k in s.get("required", ()):
            if k not in v:
                errs.append(f'ValidationError({path}): missing required field "{k}" in {name}')
        return
    if t == "object":
        if got != "object":
            bad("map" if "additionalProperties" in s else "object")
            return
        if "additionalProperties" in s:
            for k, sub in v.items():
                _check(defs, s["additionalProperties"], sub, f"{path}.{k}", errs, owner, fname)
        return
    if t == "integer" and got != "integer":
        bad("integer")
    elif t == "number" and got not in ("integer", "number"):
        bad("number")
    elif t == "string" and got != "string":
        bad("string")
    elif t == "boolean" and got != "boolean":
        bad("boolean")


def validate(obj: dict, defs: dict | None = None) -> list[str]:
    """kubectl --validate: errors of one object against the schema of its kind; [] for kinds the
    document does not describe (custom resources) and for valid objects."""
    defs = defs if defs is not None else definitions()
    if not isinstance(obj, dict):
        return ["ValidationError: the document is not an object"]
    av, kind = obj.get("apiVersion"), obj.get("kind")
    errs = []
    if not av:
        errs.append('ValidationError(Object): missing required field "apiVersion"')
    if not kind:
        errs.append('ValidationError(Object): missing required field "kind"')
    if errs:
        return errs
    if kind == "List" and av == "v1":
        for i, item in enumerate(obj.get("items") or []):
            errs += [e.replace("ValidationError(", f"ValidationError(List.items[{i}].", 1) for e in validate(item, defs)]
        return errs
    full = _gvk_definition(defs, av, kind)
    if full is None:
        return []
    _check(defs, {"$ref": f"#/definitions/{full}"}, obj, kind, errs, None, None)
    ri = SCHEME.for_kind(av, kind)
    if ri is not None and ri.storage is not None:
        # a served-only version shares its storage kind's definition; that version's own
        # defaulting (e.g. extensions/v1beta1 selector from the template) fills required fields
        errs = [e for e in errs if "missing required field" not in e]
    return errs


def _gvk_definition(defs: dict, api_version: str, kind: str) -> str | None:
    g, _, v = api_version.rpartition("/")
    for name, d in defs.items():
        if any((x["group"], x["version"], x["kind"]) == (g, v, kind) for x in d.get("x-kubernetes-group-version-kind", ())):
            return name
    return None


# ------------------------------------------------------------------------------ explain
def _type_name(defs: dict, schema: dict) -> str:
    name, s = _deref(defs, schema)
    if name in (QUANTITY, INT_OR_STRING, TIME):
        return "string"
    t = s.get("type")
    if t == "array":
        return "[]" + _type_name(defs, s.get("items", {}))
    if "properties" in s:
        return "Object"
    if t == "object" and "additionalProperties" in s:
        return "map[string]" + _type_name(defs, s["additionalProperties"])
    if t == "object":
        return "Object"
    return t or "Object"


def _element(defs: dict, schema: dict) -> tuple[str | None, dict]:
    """The definition behind a field (through arrays and maps)."""
    name, s = _deref(defs, schema)
    while s.get("type") == "array" or ("additionalProperties" in s and "properties" not in s):
        name, s = _deref(defs, s.get("items") or s.get("additionalProperties"))
    return name, s


def _indent(text: str, n: int) -> list[str]:
    import textwrap
    out = []
    for para in text.split("\n"):
        out += textwrap.wrap(para, 80 - n, initial_indent=" " * n, subsequent_indent=" " * n) or [""]
    return out


def explain(defs: dict, api_version: str, kind: str, field_path: list[str], recursive: bool = False) -> str:
    """kubectl explain output for <kind>[.field...]."""
    full = _gvk_definition(defs, api_version, kind)
    if full is None:
        raise KeyError(f"couldn't find resource for \"{api_version}, Kind={kind}\"")
    lines = [f"KIND:     {kind}", f"VERSION:  {api_version}", ""]
    schema, s, field_desc = {"$ref": f"#/definitions/{full}"}, defs[full], None
    for i, f in enumerate(field_path):
        _, elem = _element(defs, schema)
        props = elem.get("properties") or {}
        if f not in props:
            raise KeyError(f'field "{f}" does not exist')
        schema = props[f]
        field_desc = schema.get("description", "")
    name, s = _element(defs, schema)
    if field_path:
        tn = _type_name(defs, schema)
        label = "RESOURCE" if "properties" in s else "FIELD"
        lines += [f"{label}: {field_path[-1]} <{tn}>" if label == "RESOURCE" else f"FIELD:    {field_path[-1]} <{tn}>", ""]
    lines.append("DESCRIPTION:")
    descs = [d for d in ((field_desc if field_path else None), s.get("description") if "properties" in s or not field_path else None) if d]
    if not descs and field_path and name in defs:
        descs = [defs[name].get("description", "")]
    for j, d in enumerate(descs):
        if j:
            lines.append("")
        lines += _indent(d, 5)
    props = s.get("properties")
    if props:
        lines += ["", "FIELDS:"]
        req = set(s.get("required", ()))
        if recursive:
            _recurse(defs, s, 1, lines, set())
        else:
            for k in sorted(props):
                lines.append(f"   {k}\t<{_type_name(defs, props[k])}>" + (" -required-" if k in req else ""))
                d = props[k].get("description")
                if not d:
                    n2, s2 = _element(defs, props[k])
                    d = s2.get("description", "") if "properties" in s2 else ""
                lines += _indent(d, 5) if d else []
                lines.append("")
    return "\n".join(lines).rstrip() + "\n"


def _recurse(defs, s, depth, lines, seen):
    for k in sorted(s.get("properties") or {}):
        sub = s["properties"][k]
        lines.append(f"{'   ' * depth}{k}\t<{_type_name(defs, sub)}>")
        name, el = _element(defs, sub)
        if "properties" in el and name not in seen:
            _recurse(defs, el, depth + 1, lines, seen | {name})
