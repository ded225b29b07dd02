"""kubectl patch.

Reference: pkg/kubectl/cmd/patch.go RunPatch (:118-262) —
  * `--type` json|merge|strategic (default strategic; anything else: `--type must be one of
    [json merge strategic], not "x"`); `-p` is required and may be YAML or JSON;
  * targets from -f, `TYPE NAME...` or `TYPE/NAME...` (ContinueOnError); none is "no objects
    passed to patch";
  * each object is patched on the server and reported `kind "name" patched`, or `... not
    patched` (exit status 1) when the patch changed nothing; -o name prints `kind/name`, another
    -o prints the object; --record annotates the change cause;
  * --local applies the patch to the -f objects without contacting the server and prints them.
"""
from __future__ import annotations

import json
import sys

import yaml

from ..api import meta as m
from .drain import print_success
from .metacmds import UsageError, resource_arg

PATCH_TYPES = {"json": "application/json-patch+json", "merge": "application/merge-patch+json",
               "strategic": "application/strategic-merge-patch+json"}


def parse_patch(text: str):
    try:
        return yaml.safe_load(text) if text.strip() else None
    except yaml.YAMLError as e:
        raise UsageError(f"unable to parse {json.dumps(text)}: {e}") from None


async def cmd_patch(c, a):
    from .main import _read_files
    from .metacmds import resolve_targets
    from .run import _print
    from ..apiserver.registry import apply_patch
    args = list(a.args)
    try:
        if getattr(a, "local", False) and args:
            raise UsageError("cannot specify --local and server resources")
        ptype = (a.type or "strategic").lower()
        if ptype not in PATCH_TYPES:
            raise UsageError(f'--type must be one of [json merge strategic], not "{ptype}"')
        if not a.patch:
            raise UsageError("Must specify -p to patch")
        patch = parse_patch(a.patch)
        body = json.dumps(patch).encode()
        ns = a.namespace or "default"
        if getattr(a, "local", False):
            objs = _read_files(a.filename) if a.filename else []
            if not objs:
                raise UsageError("no objects passed to patch")
            for obj in objs:
                _print(apply_patch(obj, body, PATCH_TYPES[ptype]), a.output or "yaml")
            return 0
        targets = await resolve_targets(c, a, args, ns)
        if not targets:
            raise UsageError("no objects passed to patch")
    except UsageError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    except m.StatusError as e:
        print(f"Error from server ({e.reason}): {e.message}", file=sys.stderr)
        return 1
    rc = 0
    for ri, obj in targets:
        name, nsx = m.name_of(obj), (m.namespace_of(obj) or ns) if ri.namespaced else ""
        try:
            out = await c.patch(resource_arg(ri), name, patch, nsx, patch_type=PATCH_TYPES[ptype])
            if getattr(a, "record", False):
                cause = "kubectl " + " ".join(sys.argv[1:])
                out = await c.patch(resource_arg(ri), name, {"metadata": {"annotations": {"kubernetes.io/change-cause": cause}}},
                                    nsx, patch_type=PATCH_TYPES["merge"])
        except m.StatusError as e:
            print(f"Error from server ({e.reason}): {e.message}", file=sys.stderr)
            rc = 1
            continue
        changed = json.dumps(out, sort_keys=True) != json.dumps(obj, sort_keys=True)
        if a.output and a.output != "name":
            _print(out, a.output)
        else:
            print_success(ri.kind.lower(), name, "patched" if changed else "not patched", short=a.output == "name")
        if not changed:
            rc = 1
    return rc

