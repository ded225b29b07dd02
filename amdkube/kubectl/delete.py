"""kubectl delete.

Reference: pkg/kubectl/cmd/delete.go —
  * targets: -f files, `TYPE NAME...`, `TYPE/NAME...`, or a type with -l / --all (the builder's
    "resource(s) were provided, but no name, label selector, or --all flag specified"); no
    arguments at all is "You must provide one or more resources by argument or filename.";
  * Validate (:196-221): --all turns on --ignore-not-found unless that was given; --now is
    --grace-period=1 (never together with --grace-period); --grace-period=0 without --force
    becomes 1 and waits for the object to be gone, with --force it stays 0 after the
    "warning: Immediate deletion does not wait for confirmation ..." line;
  * RunDelete: --cascade (default) goes through the reapers of pkg/kubectl/delete.go for
    ReplicationControllers, ReplicaSets, Deployments, DaemonSets, StatefulSets and Jobs — the
    workload is emptied before it is deleted and the command returns once its pods are gone —
    and deletes everything else with orphanDependents=false; --cascade=false orphans;
  * `pod "x" deleted` (or `pod/x` with -o name) per object, "No resources found" when nothing
    matched; errors of individual objects are reported at the end (ContinueOnError).
amdkube's reaper is the garbage collector: the workload is deleted with Foreground propagation
(its pods first, ownerReferences with blockOwnerDeletion) and the command waits for it to
disappear, bounded by --timeout (default: 5 minutes + 10 s per replica, as the reapers).
"""
from __future__ import annotations

import asyncio
import sys
import time

from ..api import meta as m
from ..api.scheme import SCHEME
from .drain import print_success
from .metacmds import UsageError, resource_arg

REAPED = {"ReplicationController", "ReplicaSet", "Deployment", "DaemonSet", "StatefulSet", "Job"}
NO_ARGS = ("You must provide one or more resources by argument or filename.\nExample resource specifications include:\n"
           "   '-f rsrc.yaml'\n   '--filename=rsrc.json'\n   '<resource> <name>'\n   '<resource>'")
IMMEDIATE_WARNING = ("warning: Immediate deletion does not wait for confirmation that the running resource has been "
                     "terminated. The resource may continue to run on the cluster indefinitely.")


async def targets(c, a, ns: str) -> list[tuple]:
    """[(ri, name, namespace)] in argument order; selectors and --all list the server."""
    from .main import _read_files
    out = []
    for d in _read_files(a.filename) if a.filename else []:
        ri = SCHEME.for_object(d)
        out.append((ri, m.name_of(d), (m.namespace_of(d) or ns) if ri.namespaced else ""))
    args = list(a.args)
    if not args:
        if not a.filename:
            raise UsageError(NO_ARGS)
        return out
    if all("/" in x for x in args):
        for x in args:
            kind, name = x.split("/", 1)
            ri = SCHEME.resolve(kind)
            if ri is None:
                raise UsageError(f'the server doesn\'t have a resource type "{kind}"')
            out.append((ri, name, ns if ri.namespaced else ""))
        return out
    ris = []
    for t in args[0].split(","):
        ri = SCHEME.resolve(t)
        if ri is None:
            raise UsageError(f'the server doesn\'t have a resource type "{t}"')
        ris.append(ri)
    names = args[1:]
    if names:
        if a.selector or a.all:
            raise UsageError("name cannot be provided when a selector is specified" if a.selector
                             else "setting 'all' parameter but found a non empty resource name")
        return out + [(ri, n, ns if ri.namespaced else "") for ri in ris for n in names]
    if not (a.selector or a.all):
        raise UsageError("resource(s) were provided, but no name, label selector, or --all flag specified")
    for ri in ris:
        nsx = "" if getattr(a, "all_namespaces", False) else (ns if ri.namespaced else "")
        items, _ = await c.list(resource_arg(ri), nsx, a.selector)
        out += [(ri, m.name_of(i), m.namespace_of(i) if ri.namespaced else "") for i in items]
    return out


async def _wait_gone(c, ri, name, ns, timeout: float | None):
    end = None if timeout is None else time.monotonic() + timeout
    while True:
        if await c.get_or_none(resource_arg(ri), name, ns) is None:
            return
        if end is not None and time.monotonic() >= end:
            raise UsageError("timed out waiting for the condition")
        await asyncio.sleep(0.2)


async def cmd_delete(c, a):
    from .main import timeout_of
    ns = a.namespace or "default"
    ignore_nf = a.ignore_not_found if a.ignore_not_found is not None else bool(a.all)
    grace = a.grace_period
    wait = False
    try:
        if getattr(a, "now", False):
            if grace != -1:
                raise UsageError("--now and --grace-period cannot be specified together")
            grace = 1
        if grace == 0:
            if getattr(a, "force", False):
                print(IMMEDIATE_WARNING, file=sys.stderr)
            else:
                wait, grace = True, 1
        found = await targets(c, a, ns)
    except UsageError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    errors = []
    done = 0
    for ri, name, nsx in found:
        res = resource_arg(ri)
        reaped = a.cascade and ri.kind in REAPED
        try:
            obj = await c.get_or_none(res, name, nsx) if reaped else None
            if reaped and obj is None:
                raise m.not_found(res if not ri.group else f"{ri.plural}.{ri.group}", name)
            propagation = "Orphan" if not a.cascade else ("Foreground" if reaped else "Background")
            await c.delete(res, name, nsx, grace=grace if grace >= 0 else None, propagation=propagation)
            if reaped:
                replicas = int(((obj or {}).get("spec") or {}).get("replicas") or 0)
                t = timeout_of(a, 0.0) or (300.0 + 10.0 * replicas)
                await _wait_gone(c, ri, name, nsx, t)
            elif wait:
                await _wait_gone(c, ri, name, nsx, timeout_of(a, 0.0) or None)
            done += 1
            print_success(ri.kind.lower(), name, "deleted", short=a.output == "name")
        except m.StatusError as e:
            if ignore_nf and m.is_not_found(e):
                continue
            errors.append(f"Error from server ({e.reason}): {e.message}")
        except UsageError as e:
            errors.append(f"error: {e}")
    if done == 0 and not errors:
        print("No resources found")
    for e in errors:
        print(e, file=sys.stderr)
    return 1 if errors else 0


def add_arguments(sp):
    sp.add_argument("--now", action="store_true")
