"""kubectl taint.

Reference: pkg/kubectl/cmd/taint.go (Complete/Validate :120-220, RunTaint :223-285,
updateTaints :288-304) and pkg/util/taints/taints.go —
  * ParseTaints (:119-162): `key=value:Effect` adds (the key a qualified name, the value a label
    value, the effect NoSchedule|PreferNoSchedule|NoExecute), `key:Effect-` / `key-` removes; a
    key+effect given twice is refused; anything else is "unknown taint spec";
  * a taint both added and removed is refused; without --overwrite, adding a taint whose key and
    effect the node already has is "Node X already has K taint(s) with same effect(s) and
    --overwrite is false";
  * ReorganizeTaints (:166-178): the new list is the added taints then every old taint they do
    not replace (same key and effect); removals by key+effect or by key; a removal that matches
    nothing is an error ("taint "k:Effect" not found") but the rest still applies; the operation
    reported is "modified" (something added and the last removal removed something, or
    --overwrite), "tainted" (the list grew) or "untainted";
  * a node whose update fails (existing taint without --overwrite, a removal that matches
    nothing) is left alone and its error reported; the other nodes are still updated
    (ContinueOnError);
  * only `node`, `nodes` or `no` followed by names, or -l selector / --all (not both).
"""
from __future__ import annotations

import sys

from ..api import meta as m
from ..api.labels import is_qualified_name, is_valid_label_value
from .drain import print_success
from .metacmds import UsageError

EFFECTS = ("NoSchedule", "PreferNoSchedule", "NoExecute")
MODIFIED, TAINTED, UNTAINTED = "modified", "tainted", "untainted"
VALID_RESOURCES = ("nodes", "no", "node")      # ResourceAliases(["node"]) + "node"


def _quoted(xs) -> str:
    return "[" + " ".join(f'"{x}"' for x in xs) + "]"


def _effect_ok(effect: str):
    if effect not in EFFECTS:
        raise UsageError(f"invalid taint effect: {effect}, unsupported taint effect")


def parse_taint(spec: str) -> dict:
    parts = spec.split("=")
    if len(parts) != 2 or not parts[1] or is_qualified_name(parts[0]):
        raise UsageError(f"invalid taint spec: {spec}")
    p2 = parts[1].split(":")
    errs = is_valid_label_value(p2[0])
    if len(p2) != 2 or errs:
        raise UsageError(f"invalid taint spec: {spec}, {'; '.join(errs)}")
    _effect_ok(p2[1])
    return {"key": parts[0], "value": p2[0], "effect": p2[1]}


def parse_taints(specs) -> tuple[list[dict], list[dict]]:
    add, remove, unique = [], [], {}
    for s in specs:
        if "=" in s and ":" in s:
            t = parse_taint(s)
            if t["key"] in unique.get(t["effect"], set()):
                raise UsageError(f"duplicated taints with the same key and effect: {{{t['key']} {t['value']} {t['effect']} <nil>}}")
            unique.setdefault(t["effect"], set()).add(t["key"])
            add.append(t)
        elif s.endswith("-"):
            key, effect = s[:-1], ""
            if ":" in key:
                key, effect = key.split(":")[0], key.split(":")[1]
            if effect:
                _effect_ok(effect)
            remove.append({"key": key, **({"effect": effect} if effect else {})})
        else:
            raise UsageError(f"unknown taint spec: {s}")
    return add, remove


def to_string(t: dict) -> str:
    """Taint.ToString: key=value:effect, key=value, key:effect or key."""
    s = t.get("key", "")
    if t.get("value"):
        s += "=" + t["value"]
    if t.get("effect"):
        s += ":" + t["effect"]
    return s


def _match(a: dict, b: dict) -> bool:
    return a.get("key") == b.get("key") and (a.get("effect") or "") == (b.get("effect") or "")


def reorganize(old: list[dict], overwrite: bool, to_add: list[dict], to_remove: list[dict]) -> tuple[str, list[dict], list[str]]:
    new = list(to_add)
    for o in old:
        if not any(_match(t, o) for t in new):
            new.append(o)
    added = len(old) != len(new)
    errors, removed = [], False
    for r in to_remove:
        before = len(new)
        if r.get("effect"):
            new = [t for t in new if not _match(r, t)]
        else:
            new = [t for t in new if t.get("key") != r.get("key")]
        removed = len(new) != before
        if not removed:
            errors.append(f'taint "{to_string(r)}" not found')
    if (added and removed) or overwrite:
        return MODIFIED, new, errors
    if added:
        return TAINTED, new, errors
    return UNTAINTED, new, errors


def already_exists(old: list[dict], add: list[dict]) -> str:
    return ",".join(t["key"] for t in add for o in old if t["key"] == o.get("key") and t["effect"] == o.get("effect"))


async def cmd_taint(c, a):
    try:
        resources, specs = [], []
        for s in a.args:
            if "=" in s or s.endswith("-"):
                specs.append(s)
            elif specs:
                raise UsageError(f"all resources must be specified before taint changes: {s}")
            else:
                resources.append(s)
        if not resources:
            raise UsageError("one or more resources must be specified as <resource> <name>")
        if not specs:
            raise UsageError("at least one taint update is required")
        add, remove = parse_taints(specs)
        kind, names = resources[0], resources[1:]
        if kind.lower() not in VALID_RESOURCES:
            raise UsageError(f"invalid resource type {kind}, only {_quoted(VALID_RESOURCES)} are supported")
        both = [f'{{"{r["key"]}":"{r.get("effect", "")}"}}' for t in add for r in remove
                if t["key"] == r["key"] and (not r.get("effect") or t["effect"] == r["effect"])]
        if both:
            raise UsageError(f"can not both modify and remove the following taint(s) in the same command: {', '.join(both)}")
        if a.all and a.selector:
            raise UsageError("setting 'all' parameter with a non empty selector is prohibited.")
        if not a.all and not a.selector and not names:
            raise UsageError("at least one resource name must be specified since 'all' parameter is not set")
    except UsageError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    errors = []
    if a.all or a.selector:
        nodes = (await c.list("nodes", "", a.selector))[0]
    else:
        nodes = []
        for n in names:
            try:
                nodes.append(await c.get("nodes", n))
            except m.StatusError as e:
                errors.append(f"Error from server ({e.reason}): {e.message}")
    for node in nodes:
        name = m.name_of(node)
        old = list((node.get("spec") or {}).get("taints") or [])
        if not a.overwrite:
            ex = already_exists(old, add)
            if ex:
                errors.append(f"error: Node {name} already has {ex} taint(s) with same effect(s) and --overwrite is false")
                continue
        op, new, errs = reorganize(old, a.overwrite, add, remove)
        if errs:
            errors.append("error: " + (errs[0] if len(errs) == 1 else "[" + ", ".join(errs) + "]"))
            continue
        try:
            out = await c.patch("nodes", name, {"spec": {"taints": new or None}})
        except m.StatusError as e:
            errors.append(f"Error from server ({e.reason}): {e.message}")
            continue
        if a.output:
            from .run import _print
            _print(out, a.output)
        else:
            print_success("node", name, op)
    for e in errors:
        print(e, file=sys.stderr)
    return 1 if errors else 0
