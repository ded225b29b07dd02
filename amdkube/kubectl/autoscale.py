"""kubectl autoscale and the horizontalpodautoscaler/v1 generator.

Reference: pkg/kubectl/cmd/autoscale.go (RunAutoscale :82-185, validateFlags :196-206) and
pkg/kubectl/autoscale.go generateHPA (:47-116):
  * --max is required and at least 1, and not below --min ("--max=MAXPODS is required and must
    be at least 1, max: N", "--max=MAXPODS must be larger or equal to --min=MINPODS, ...");
  * only ReplicationControllers, ReplicaSets and Deployments ("cannot autoscale a Kind[.group]");
  * the HPA is named --name or after the target; minReplicas only when positive,
    targetCPUUtilizationPercentage only when not negative;
  * --dry-run / -o print the object; otherwise PrintSuccess names the target resource:
    `deployment "x" autoscaled`.
"""
from __future__ import annotations

import sys

from ..api import meta as m
from .drain import print_success
from .metacmds import UsageError

AUTOSCALABLE = {("", "ReplicationController"), ("extensions", "ReplicaSet"), ("extensions", "Deployment"),
                ("apps", "Deployment"), ("apps", "ReplicaSet")}


class GenerateError(Exception):
    pass


def _atoi(s: str) -> int:
    try:
        return int(s, 10)
    except ValueError:
        raise GenerateError(f'strconv.Atoi: parsing "{s}": invalid syntax') from None


def generate_hpa(params: dict) -> dict:
    name = params.get("name") or params.get("default-name")
    if not name:
        raise GenerateError("'name' is a required parameter.")
    lo = _atoi(params["min"]) if "min" in params else -1
    if "max" not in params:
        raise GenerateError("'max' is a required parameter.")
    hi = _atoi(params["max"])
    if lo > hi:
        raise GenerateError("'max' must be greater than or equal to 'min'.")
    cpu = _atoi(params["cpu-percent"]) if "cpu-percent" in params else -1
    spec = {"scaleTargetRef": {"kind": params.get("scaleRef-kind", ""), "name": params.get("scaleRef-name", ""),
                               "apiVersion": params.get("scaleRef-apiVersion", "")},
            "maxReplicas": hi}
    if lo > 0:
        spec["minReplicas"] = lo
    if cpu >= 0:
        spec["targetCPUUtilizationPercentage"] = cpu
    return {"apiVersion": "autoscaling/v1", "kind": "HorizontalPodAutoscaler", "metadata": {"name": name}, "spec": spec}


def validate_flags(lo: int, hi: int) -> list[str]:
    errs = []
    if hi < 1:
        errs.append(f"--max=MAXPODS is required and must be at least 1, max: {hi}")
    if hi < lo:
        errs.append(f"--max=MAXPODS must be larger or equal to --min=MINPODS, max: {hi}, min: {lo}")
    return errs


async def cmd_autoscale(c, a):
    from .metacmds import resolve_targets
    from .run import _print
    hi = -1 if a.max is None else a.max
    lo = -1 if a.min is None else a.min
    errs = validate_flags(lo, hi)
    if errs:
        print("error: " + (errs[0] if len(errs) == 1 else "[" + ", ".join(errs) + "]"), file=sys.stderr)
        return 1
    ns = a.namespace or "default"
    try:
        targets = await resolve_targets(c, a, list(a.args), ns)
        if not targets:
            raise UsageError("error: You must provide one or more resources by argument or filename.")
        for ri, obj in targets:
            if (ri.group, ri.kind) not in AUTOSCALABLE:
                raise UsageError(f"cannot autoscale a {ri.kind}{'.' + ri.group if ri.group else ''}")
            name = m.name_of(obj)
            params = {"default-name": name, "scaleRef-kind": ri.kind, "scaleRef-name": name,
                      "scaleRef-apiVersion": ri.api_version, "max": str(hi), "min": str(lo),
                      "cpu-percent": str(a.cpu_percent if a.cpu_percent is not None else -1)}
            if a.name:
                params["name"] = a.name
            hpa = generate_hpa(params)
            if getattr(a, "record", False):
                hpa["metadata"].setdefault("annotations", {})["kubernetes.io/change-cause"] = "kubectl " + " ".join(sys.argv[1:])
            if a.dry_run:
                _print(hpa, a.output or "yaml")
                continue
            out = await c.create(hpa, ns)
            if a.output:
                _print(out, a.output)
            else:
                print_success(ri.kind.lower(), name, "autoscaled")
    except (UsageError, GenerateError) as e:
        print(f"error: {e}" if not str(e).startswith("error: ") else str(e), file=sys.stderr)
        return 1
    except m.StatusError as e:
        print(f"Error from server ({e.reason}): {e.message}", file=sys.stderr)
        return 1
    return 0
