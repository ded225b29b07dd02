"""kubectl label / annotate, and the resource-argument resolution they share.

Reference:
  * pkg/kubectl/cmd/util/helpers.go GetResourcesAndPairs (:609-627: arguments before the first
    KEY=VALUE / KEY- are resources; a resource after a pair is an error) and ParsePairs
    (:630-665, "invalid annotation format: ...");
  * pkg/kubectl/cmd/label.go — parseLabels (:321-346: one `=`, a valid label value, `KEY-`
    removals, never both for one key), validateNoOverwrites (:311-319), labelFunc (:348-376),
    RunLabel (:185-309: every object is read fresh, a merge patch carries the change, `label "x"
    not found.` for a removal of an absent key, `labeled` / `not labeled`, --list, --dry-run,
    --local, --resource-version only for a single resource);
  * pkg/kubectl/cmd/annotate.go — validateAnnotations (:296-311), validateNoAnnotationOverwrites
    (:314-332, the change-cause annotation may always be overwritten), updateAnnotations
    (:335-363), RunAnnotate (:183-288);
  * pkg/kubectl/resource/builder.go ResourceTypeOrNameArgs: `TYPE NAME...`, `TYPE/NAME...`,
    `TYPE[,TYPE]` with -l or --all ("resource(s) were provided, but no name, label selector, or
    --all flag specified").
"""
from __future__ import annotations

import json
import sys

from ..api import meta as m
from ..api.labels import is_valid_label_value
from ..api.scheme import SCHEME

CHANGE_CAUSE = "kubernetes.io/change-cause"


class UsageError(Exception):
    pass


def get_resources_and_pairs(args, pair_type: str):
    resources, pairs, found = [], [], False
    for s in args:
        non_resource = ("=" in s and not s.startswith("=")) or (s.endswith("-") and s != "-")
        if non_resource:
            found = True
            pairs.append(s)
        elif found:
            raise UsageError(f"all resources must be specified before {pair_type} changes: {s}")
        else:
            resources.append(s)
    return resources, pairs


def parse_pairs(pair_args, pair_type: str, support_remove: bool):
    new, remove, invalid = {}, ([] if support_remove else None), []
    for a in pair_args:
        if "=" in a and not a.startswith("="):
            k, v = a.split("=", 1)
            new[k] = v
        elif support_remove and a.endswith("-") and a != "-":
            remove.append(a[:-1])
        else:
            invalid.append(a)
    if invalid:
        raise UsageError(f"invalid {pair_type} format: {', '.join(invalid)}")
    return new, remove


def parse_labels(spec):
    labels, remove = {}, []
    for s in spec:
        if "=" in s:
            parts = s.split("=")
            if len(parts) != 2:
                raise UsageError(f"invalid label spec: {s}")
            errs = is_valid_label_value(parts[1])
            if errs:
                raise UsageError(f'invalid label value: "{s}": {";".join(errs)}')
            labels[parts[0]] = parts[1]
        elif s.endswith("-"):
            remove.append(s[:-1])
        else:
            raise UsageError(f"unknown label spec: {s}")
    for r in remove:
        if r in labels:
            raise UsageError("can not both modify and remove a label in the same command")
    return labels, (remove or None)


def _aggregate(errs: list[str]) -> str:
    return errs[0] if len(errs) == 1 else "[" + ", ".join(errs) + "]"


def validate_no_overwrites(obj: dict, labels: dict):
    cur = m.labels_of(obj)
    errs = [f"'{k}' already has a value ({cur[k]}), and --overwrite is false" for k in labels if k in cur]
    if errs:
        raise UsageError(_aggregate(errs))


def label_func(obj: dict, overwrite: bool, resource_version: str, labels: dict, remove):
    if not overwrite:
        validate_no_overwrites(obj, labels)
    md = obj.setdefault("metadata", {})
    cur = dict(md.get("labels") or {})
    cur.update(labels)
    for k in remove or ():
        cur.pop(k, None)
    md["labels"] = cur
    if resource_version:
        md["resourceVersion"] = resource_version


def validate_annotations(remove, new: dict):
    both = [r for r in remove or () if r in new]
    if both:
        raise UsageError(f"can not both modify and remove the following annotation(s) in the same command: {', '.join(both)}")


def validate_no_annotation_overwrites(obj: dict, annotations: dict):
    cur = m.annotations_of(obj)
    found = [f"'{k}' already has a value ({cur[k]})" for k in annotations if k != CHANGE_CAUSE and k in cur]
    if found:
        raise UsageError(f"--overwrite is false but found the following declared annotation(s): {'; '.join(found)}")


def update_annotations(obj: dict, overwrite: bool, resource_version: str, annotations: dict, remove):
    if not overwrite:
        validate_no_annotation_overwrites(obj, annotations)
    md = obj.setdefault("metadata", {})
    cur = dict(md.get("annotations") or {})
    cur.update(annotations)
    for k in remove or ():
        cur.pop(k, None)
    md["annotations"] = cur
    if resource_version:
        md["resourceVersion"] = resource_version


def merge_patch(old, new):
    """jsonpatch.CreateMergePatch (RFC 7386): the keys that changed, null for removals."""
    if not isinstance(old, dict) or not isinstance(new, dict):
        return new
    out = {}
    for k in old:
        if k not in new:
            out[k] = None
    for k, v in new.items():
        if k not in old:
            out[k] = v
        elif old[k] != v:
            out[k] = merge_patch(old[k], v) if isinstance(v, dict) and isinstance(old[k], dict) else v
    return out


def resource_arg(ri) -> str:
    return f"{ri.plural}.{ri.group}" if ri.group else ri.plural


async def resolve_targets(c, a, resources: list[str], namespace: str, all_flag: bool = False):
    """ResourceTypeOrNameArgs + FilenameParam: [(ri, obj)] read fresh from the server."""
    from .main import _read_files
    out = []
    for d in _read_files(a.filename) if getattr(a, "filename", None) else []:
        ri = SCHEME.for_object(d)
        ns = m.namespace_of(d) or namespace
        out.append((ri, await c.get(resource_arg(ri), m.name_of(d), ns if ri.namespaced else "")))
    if not resources:
        return out
    if all("/" in r for r in resources):
        for r in resources:
            kind, name = r.split("/", 1)
            ri = SCHEME.resolve(kind)
            if ri is None:
                raise UsageError(f'the server doesn\'t have a resource type "{kind}"')
            out.append((ri, await c.get(resource_arg(ri), name, namespace if ri.namespaced else "")))
        return out
    types, names = resources[0].split(","), resources[1:]
    if any("/" in n for n in names):
        raise UsageError("there is no need to specify a resource type as a separate argument when passing "
                         "arguments in resource/name form")
    ris = []
    for t in types:
        ri = SCHEME.resolve(t)
        if ri is None:
            raise UsageError(f'the server doesn\'t have a resource type "{t}"')
        ris.append(ri)
    if names:
        for ri in ris:
            for n in names:
                out.append((ri, await c.get(resource_arg(ri), n, namespace if ri.namespaced else "")))
        return out
    if not (a.selector or all_flag):
        raise UsageError("resource(s) were provided, but no name, label selector, or --all flag specified")
    for ri in ris:
        items, _ = await c.list(resource_arg(ri), namespace if ri.namespaced else "", a.selector)
        out += [(ri, dict(i, apiVersion=i.get("apiVersion") or ri.api_version, kind=i.get("kind") or ri.kind)) for i in items]
    return out


def _print_obj(obj, fmt):
    if fmt == "json":
        print(json.dumps(obj, indent=4))
    elif fmt == "yaml":
        import yaml
        print(yaml.safe_dump(obj, default_flow_style=False).rstrip())
    elif fmt == "name":
        print(f"{obj.get('kind', '').lower()}/{m.name_of(obj)}")
    else:
        raise UsageError(f"output format {fmt!r} not supported here")


async def _run_meta(c, a, kind: str):
    """RunLabel / RunAnnotate."""
    from .drain import print_success
    pair_type = "label" if kind == "labels" else "annotation"
    resources, pairs = get_resources_and_pairs(a.args, pair_type)
    if kind == "labels":
        new, remove = parse_labels(pairs)
        if getattr(a, "list", False) and a.output:
            raise UsageError("--list and --output may not be specified together")
    else:
        new, remove = parse_pairs(pairs, pair_type, True)
    if not resources and not a.filename:
        raise UsageError("one or more resources must be specified as <resource> <name> or <resource>/<name>")
    if not new and not remove and not (kind == "labels" and getattr(a, "list", False)):
        raise UsageError(f"at least one {pair_type} update is required")
    if kind != "labels":
        validate_annotations(remove, new)
        if getattr(a, "record", False):
            new[CHANGE_CAUSE] = "kubectl " + " ".join(sys.argv[1:]) if sys.argv[1:] else "kubectl annotate"
    ns = a.namespace or "default"
    if getattr(a, "local", False):
        from .main import _read_files
        targets = [(SCHEME.for_object(d), d) for d in _read_files(a.filename)]
    else:
        targets = await resolve_targets(c, a, resources, ns, bool(a.all))
    rv = getattr(a, "resource_version", None) or ""
    single = len(targets) == 1 and not (a.selector or a.all)      # IntoSingleItemImplied
    if rv and not single:
        raise UsageError("--resource-version may only be used with a single resource")
    func = label_func if kind == "labels" else update_annotations
    verb = "labeled" if kind == "labels" else "annotated"
    for ri, obj in targets:
        name = m.name_of(obj)
        if a.dry_run or getattr(a, "local", False) or getattr(a, "list", False):
            func(obj, a.overwrite, rv, new, remove)
            out, msg = obj, verb
        else:
            if kind == "labels":
                for r in remove or ():
                    if r not in m.labels_of(obj):
                        print(f'label "{r}" not found.')
            before = m.deepcopy(obj)
            func(obj, a.overwrite, rv, new, remove)
            patch = merge_patch(before, obj)
            msg = verb if (kind != "labels" or patch) else "not labeled"
            out = await c.patch(resource_arg(ri), name, patch, m.namespace_of(obj) if ri.namespaced else "",
                                patch_type="application/merge-patch+json") if patch else before
        if getattr(a, "list", False):
            for k, v in m.labels_of(out).items():
                print(f"{k}={v}")
            continue
        if a.output:
            _print_obj(out, a.output)
            continue
        print_success(ri.kind.lower(), name, msg, a.dry_run)


async def cmd_label(c, a):
    try:
        await _run_meta(c, a, "labels")
    except UsageError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    return 0


async def cmd_annotate(c, a):
    try:
        await _run_meta(c, a, "annotations")
    except UsageError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    return 0


def add_arguments(sp):
    sp.add_argument("--list", action="store_true")
    sp.add_argument("--local", action="store_true")
    sp.add_argument("--resource-version", default=None)
