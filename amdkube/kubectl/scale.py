"""kubectl scale.

Reference: pkg/kubectl/cmd/scale.go RunScale (:97-193) and pkg/kubectl/scale.go —
  * --replicas is required and ≥ 0; --resource-version only with one resource;
  * a scaler per kind (ScalerFor :53-67): ReplicationController, ReplicaSet, Deployment,
    StatefulSet scale spec.replicas, Job scales spec.parallelism; anything else "no scaler has
    been implemented for ...";
  * ScaleSimple: read, check the preconditions (--current-replicas, --resource-version:
    PreconditionError "Expected replicas to be N, was M"), write the object back with its
    resourceVersion; ScaleCondition retries only update conflicts, every kubectl.Interval (1 s)
    for up to kubectl.Timeout (5 min);
  * --timeout: wait until the controller has observed and reached the new size
    (ControllerHasDesiredReplicas, ReplicaSetHasDesiredReplicas, DeploymentHasDesiredReplicas,
    StatefulSetHasDesiredReplicas, JobHasDesiredParallelism): "timed out waiting for "x" to be
    synced";
  * `deployment "x" scaled` per object; "no objects passed to scale" when none matched.
"""
from __future__ import annotations

import asyncio
import sys
import time

from ..api import meta as m
from .metacmds import UsageError, resolve_targets, resource_arg

INTERVAL = 1.0
RETRY_TIMEOUT = 300.0
SCALABLE = {"ReplicationController", "ReplicaSet", "Deployment", "StatefulSet", "Job"}


class PreconditionError(Exception):
    def __init__(self, precondition, expected, actual):
        super().__init__(f"Expected {precondition} to be {expected}, was {actual}")


class ScaleError(Exception):
    GET, UPDATE, CONFLICT = range(3)

    def __init__(self, kind, rv, err):
        self.kind = kind
        msg = f"Scaling the resource failed with: {err}"
        if rv:
            msg += f"; Current resource version {rv}"
        super().__init__(msg)


def _size_field(kind):
    return "parallelism" if kind == "Job" else "replicas"


def validate_preconditions(obj: dict, size: int, resource_version: str):
    kind = obj.get("kind", "")
    spec = obj.get("spec") or {}
    if size != -1:
        if kind == "Job":
            cur = spec.get("parallelism")
            if cur is None:
                raise PreconditionError("parallelism", str(size), "nil")
            if int(cur) != size:
                raise PreconditionError("parallelism", str(size), str(cur))
        elif int(spec.get("replicas", 1)) != size:
            raise PreconditionError("replicas", str(size), str(spec.get("replicas", 1)))
    cur_rv = (obj.get("metadata") or {}).get("resourceVersion", "")
    if resource_version and cur_rv != resource_version:
        raise PreconditionError("resource version", resource_version, cur_rv)


async def scale_simple(c, ri, ns: str, name: str, size: int, resource_version: str, count: int) -> str:
    """One attempt: the new resourceVersion, or ScaleError/PreconditionError."""
    try:
        obj = await c.get(resource_arg(ri), name, ns)
    except m.StatusError as e:
        raise ScaleError(ScaleError.GET, "", e.message) from None
    obj.setdefault("kind", ri.kind)
    obj.setdefault("apiVersion", ri.api_version)
    validate_preconditions(obj, size, resource_version)
    obj.setdefault("spec", {})[_size_field(ri.kind)] = count
    try:
        out = await c.update(obj)
    except m.StatusError as e:
        kind = ScaleError.CONFLICT if e.code == 409 else ScaleError.UPDATE
        raise ScaleError(kind, (obj.get("metadata") or {}).get("resourceVersion", ""), e.message) from None
    return (out.get("metadata") or {}).get("resourceVersion", "")


def has_desired(obj: dict, count: int) -> bool:
    """The *HasDesiredReplicas conditions."""
    kind = obj.get("kind", "")
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    gen = (obj.get("metadata") or {}).get("generation", 0)
    observed = st.get("observedGeneration", 0) >= gen
    if kind == "Job":
        return int(st.get("active", 0)) == int(spec.get("parallelism", count))
    if kind == "Deployment":
        return observed and int(st.get("updatedReplicas", 0)) == count
    if kind == "StatefulSet":
        return observed and int(st.get("replicas", 0)) == count
    return observed and int(st.get("replicas", 0)) == count


async def scale(c, ri, ns: str, name: str, count: int, size: int = -1, resource_version: str = "",
                wait: float | None = None, interval: float = INTERVAL, retry_timeout: float = RETRY_TIMEOUT):
    """Scaler.Scale: conflicts retried, preconditions and other failures returned at once."""
    if ri.kind not in SCALABLE:
        raise UsageError(f'no scaler has been implemented for {{{ri.group} {ri.kind}}}')
    end = time.monotonic() + retry_timeout
    while True:
        try:
            await scale_simple(c, ri, ns, name, size, resource_version, count)
            break
        except ScaleError as e:
            if e.kind != ScaleError.CONFLICT or time.monotonic() >= end:
                raise
            await asyncio.sleep(interval)
    if wait:
        deadline = time.monotonic() + wait
        while True:
            obj = await c.get(resource_arg(ri), name, ns)
            obj.setdefault("kind", ri.kind)
            if has_desired(obj, count):
                return
            if time.monotonic() >= deadline:
                raise UsageError(f'timed out waiting for "{name}" to be synced')
            await asyncio.sleep(min(interval, 0.2))


async def cmd_scale(c, a):
    from .drain import print_success
    from .main import timeout_of
    try:
        count = a.replicas if a.replicas is not None else -1
        targets = await resolve_targets(c, a, list(a.args), a.namespace or "default", bool(a.all))
        if count < 0:
            raise UsageError("The --replicas=COUNT flag is required, and COUNT must be greater than or equal to 0")
        rv = getattr(a, "resource_version", None) or ""
        if rv and len(targets) > 1:
            raise UsageError("cannot use --resource-version with multiple resources")
        if not targets:
            raise UsageError("no objects passed to scale")
        for ri, obj in targets:
            name = m.name_of(obj)
            await scale(c, ri, m.namespace_of(obj) or (a.namespace or "default"), name, count,
                        int(getattr(a, "current_replicas", -1)), rv, timeout_of(a, 0.0) or None)
            print_success(ri.kind.lower(), name, "scaled", short=a.output == "name")
    except (UsageError, PreconditionError, ScaleError) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    return 0


def add_arguments(sp):
    sp.add_argument("--current-replicas", type=int, default=-1)
