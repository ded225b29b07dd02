"""kubectl replace.

Reference: pkg/kubectl/cmd/replace.go RunReplace (:95-165) and forceReplace (:167-265) —
  * -f is required ("Must specify --filename to replace"); --grace-period and --timeout need
    --force;
  * each object is PUT unconditionally: without a resourceVersion in the file the server's
    current one is used (resource.Helper.Replace with overwrite), with one a stale file is a
    conflict; --save-config writes the last-applied annotation, --record the change cause;
  * `kind "name" replaced` (`kind/name` with -o name); errors name the file ("error when
    replacing "f.yaml": ...") and do not stop the other objects;
  * --force deletes every object (grace period 0 becomes 1), prints `kind "name" deleted`,
    waits until each is gone (--timeout, default 5 minutes), then creates them again.
"""
from __future__ import annotations

import asyncio
import json
import sys
import time

from ..api import meta as m
from ..api.scheme import SCHEME
from .drain import print_success
from .metacmds import resource_arg

LAST_APPLIED = "kubectl.kubernetes.io/last-applied-configuration"


def _prepare(a, doc):
    md = doc.setdefault("metadata", {})
    if getattr(a, "save_config", False):
        body = json.loads(json.dumps(doc))
        (body.get("metadata") or {}).get("annotations", {}).pop(LAST_APPLIED, None)
        md.setdefault("annotations", {})[LAST_APPLIED] = json.dumps(body, sort_keys=True, separators=(",", ":")) + "\n"
    if getattr(a, "record", False):
        md.setdefault("annotations", {})["kubernetes.io/change-cause"] = "kubectl " + " ".join(sys.argv[1:])


async def cmd_replace(c, a):
    from .main import _read_files, timeout_of
    if not a.filename:
        print("error: Must specify --filename to replace", file=sys.stderr)
        return 1
    short = a.output == "name"
    if not a.force:
        if a.grace_period >= 0:
            print("error: --grace-period must have --force specified", file=sys.stderr)
            return 1
        if timeout_of(a, 0.0):
            print("error: --timeout must have --force specified", file=sys.stderr)
            return 1
    docs = []
    for path in a.filename:
        for d in _read_files([path]):
            docs.append((path, d))
    if not docs:
        print("error: no objects passed to replace", file=sys.stderr)
        return 1
    errors = []

    def target(doc):
        ri = SCHEME.for_object(doc)
        ns = (m.namespace_of(doc) or a.namespace or "default") if ri.namespaced else ""
        return ri, ns

    if a.force:
        grace = 1 if a.grace_period == 0 else (a.grace_period if a.grace_period > 0 else None)
        for path, doc in docs:
            ri, ns = target(doc)
            try:
                await c.delete(resource_arg(ri), m.name_of(doc), ns, grace=grace)
                print_success(ri.kind.lower(), m.name_of(doc), "deleted", short=short)
            except m.StatusError as e:
                if not m.is_not_found(e):
                    errors.append(f'error when deleting "{path}": {e.message}')
        end = time.monotonic() + (timeout_of(a, 0.0) or 300.0)
        for path, doc in docs:
            ri, ns = target(doc)
            while await c.get_or_none(resource_arg(ri), m.name_of(doc), ns) is not None:
                if time.monotonic() > end:
                    errors.append("timed out waiting for the condition")
                    break
                await asyncio.sleep(0.1)
    for path, doc in docs:
        ri, ns = target(doc)
        _prepare(a, doc)
        if ri.namespaced:
            doc["metadata"]["namespace"] = ns
        try:
            if a.force:
                doc["metadata"].pop("resourceVersion", None)
                await c.create(doc, ns)
            else:
                if not doc["metadata"].get("resourceVersion"):
                    cur = await c.get(resource_arg(ri), m.name_of(doc), ns)
                    doc["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
                await c.update(doc)
            print_success(ri.kind.lower(), m.name_of(doc), "replaced", short=short)
        except m.StatusError as e:
            errors.append(f'error when replacing "{path}": {e.message}')
    for e in errors:
        print(f"Error from server: {e}" if e.startswith("error when") else f"error: {e}", file=sys.stderr)
    return 1 if errors else 0
