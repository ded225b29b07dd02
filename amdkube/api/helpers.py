"""Object helpers shared by apiserver, scheduler, kubelet and kubectl.

Fork helpers: pkg/apis/core/v1/helper/helpers.go:465-534 —
ExtendedRequirementsAsSelector, PodExtendedResourceName (exactly one limit key),
PodExtendedResource (lookup by name), PodExtendedResourceAssigned (devices a container
gets). Upstream helpers: IsExtendedResourceName (helpers.go), resource request sums
(pkg/scheduler predicates GetResourceRequest), taint/toleration matching
(pkg/apis/core/v1/helper ToleratesTaint).
"""
from __future__ import annotations

import re

from .labels import is_qualified_name, node_requirements_as_selector, Selector
from .quantity import Quantity

GPU_RESOURCE = "amd.com/gpu"
NVIDIA_GPU = "nvidia.com/gpu"

POD_PENDING, POD_RUNNING, POD_SUCCEEDED, POD_FAILED, POD_UNKNOWN = "Pending", "Running", "Succeeded", "Failed", "Unknown"
HEALTHY, UNHEALTHY = "Healthy", "Unhealthy"


# ----------------------------------------------------------- resource names
def is_default_namespace_resource(name: str) -> bool:
    return "/" not in name or "kubernetes.io/" in name


def is_extended_resource_name(name: str) -> bool:
    """helpers.go IsExtendedResourceName: vendor-domain qualified names only."""
    if is_default_namespace_resource(name) or name.startswith("requests."):
        return False
    return not is_qualified_name("requests." + name)


def is_native_resource(name: str) -> bool:
    return is_default_namespace_resource(name)


# ------------------------------------------------------- fork ExtendedResources
class ExtendedResourceError(ValueError):
    pass


def pod_extended_resource_name(pres: dict) -> str:
    """Exactly one limits key (helpers.go:500-510)."""
    limits = (pres.get("resources") or {}).get("limits") or {}
    if len(limits) != 1:
        raise ExtendedResourceError(f"extended resource {pres.get('name')!r} has unexpected limits length {len(limits)} != 1")
    return next(iter(limits))


def pod_extended_resource_count(pres: dict) -> int:
    rname = pod_extended_resource_name(pres)
    return Quantity(pres["resources"]["limits"][rname]).value()


def pod_extended_resource(pod: dict, name: str) -> dict | None:
    for r in (pod.get("spec") or {}).get("extendedResources") or []:
        if r.get("name") == name:
            return r
    return None


def pod_extended_resource_assigned(rname: str, container: dict, pod: dict) -> list[str]:
    """Device IDs of resource `rname` referenced by `container` (helpers.go:522-534)."""
    out = []
    for ref in container.get("extendedResourceRequests") or []:
        pres = pod_extended_resource(pod, ref)
        if pres is None:
            continue
        try:
            if pod_extended_resource_name(pres) != rname:
                continue
        except ExtendedResourceError:
            continue
        out.extend(pres.get("assigned") or [])
    return out


def extended_requirements_as_selector(reqs: list[dict] | None) -> Selector:
    return node_requirements_as_selector(reqs)


def pod_assigned_devices(pod: dict) -> dict[str, set[str]]:
    """resourceName -> set(device IDs) assigned to this pod (all ExtendedResources)."""
    out: dict[str, set[str]] = {}
    for pres in (pod.get("spec") or {}).get("extendedResources") or []:
        ids = pres.get("assigned") or []
        if not ids:
            continue
        try:
            rname = pod_extended_resource_name(pres)
        except ExtendedResourceError:
            continue
        out.setdefault(rname, set()).update(ids)
    return out


_PARTITION_RE = re.compile(r"^amd\.com/(spx|dpx|qpx|cpx)_nps[12]$")


def is_gpu_resource(rname: str) -> bool:
    """amd.com/gpu or one of the MI355X partition resources (amd.com/cpx_nps2, ...)."""
    return rname == GPU_RESOURCE or bool(_PARTITION_RE.match(rname))


def pod_gpu_request(pod: dict, rname: str | None = None) -> int:
    """GPUs (or GPU partitions) the pod asks for; rname=None counts every GPU resource."""
    match = is_gpu_resource if rname is None else (lambda r: r == rname)
    n = 0
    for pres in (pod.get("spec") or {}).get("extendedResources") or []:
        lim = (pres.get("resources") or {}).get("limits") or {}
        n += sum(Quantity(v).value() for r, v in lim.items() if match(r))
    for c in (pod.get("spec") or {}).get("containers") or []:
        lim = (c.get("resources") or {}).get("limits") or {}
        n += sum(Quantity(v).value() for r, v in lim.items() if match(r))
    return n


# --------------------------------------------------------------- pod resources
def _add(acc: dict, rl: dict | None):
    for k, v in (rl or {}).items():
        acc[k] = acc.get(k, 0) + (Quantity(v).milli_value() if k == "cpu" else Quantity(v).value())


def pod_requests(pod: dict) -> dict[str, int]:
    """Effective requests: sum(containers) max-merged with each init container.

    cpu in millicores, everything else in base units (predicates.go GetResourceRequest).
    """
    spec = pod.get("spec") or {}
    acc: dict[str, int] = {}
    for c in spec.get("containers") or []:
        _add(acc, (c.get("resources") or {}).get("requests"))
    for c in spec.get("initContainers") or []:
        one: dict[str, int] = {}
        _add(one, (c.get("resources") or {}).get("requests"))
        for k, v in one.items():
            if v > acc.get(k, 0):
                acc[k] = v
    return acc


def node_allocatable(node: dict) -> dict[str, int]:
    st = node.get("status") or {}
    src = st.get("allocatable") or st.get("capacity") or {}
    return {k: (Quantity(v).milli_value() if k == "cpu" else Quantity(v).value()) for k, v in src.items()}


def pod_host_ports(pod: dict) -> list[tuple[str, str, int]]:
    out = []
    for c in (pod.get("spec") or {}).get("containers") or []:
        for p in c.get("ports") or []:
            hp = p.get("hostPort") or 0
            if hp:
                out.append((p.get("hostIP") or "0.0.0.0", p.get("protocol") or "TCP", int(hp)))
    return out


# ------------------------------------------------------------- phases/conditions
def is_pod_terminal(pod: dict) -> bool:
    return ((pod.get("status") or {}).get("phase")) in (POD_SUCCEEDED, POD_FAILED)


def pod_phase(pod: dict) -> str:
    return (pod.get("status") or {}).get("phase") or POD_PENDING


def get_condition(obj: dict, ctype: str) -> dict | None:
    for c in (obj.get("status") or {}).get("conditions") or []:
        if c.get("type") == ctype:
            return c
    return None


def set_condition(obj: dict, cond: dict, now: str) -> bool:
    """Upsert a condition; lastTransitionTime only moves when status flips. Returns changed."""
    conds = obj.setdefault("status", {}).setdefault("conditions", [])
    for i, c in enumerate(conds):
        if c.get("type") == cond["type"]:
            changed = c.get("status") != cond.get("status") or c.get("reason") != cond.get("reason")
            new = dict(c)
            new.update(cond)
            new["lastTransitionTime"] = now if c.get("status") != cond.get("status") else c.get("lastTransitionTime", now)
            conds[i] = new
            return changed
    c = dict(cond)
    c.setdefault("lastTransitionTime", now)
    conds.append(c)
    return True


def is_pod_ready(pod: dict) -> bool:
    c = get_condition(pod, "Ready")
    return bool(c and c.get("status") == "True")


def is_node_ready(node: dict) -> bool:
    c = get_condition(node, "Ready")
    return bool(c and c.get("status") == "True")


# --------------------------------------------------------------- taints
def toleration_tolerates_taint(tol: dict, taint: dict) -> bool:
    """ToleratesTaint (pkg/apis/core/v1/helper/helpers.go)."""
    if tol.get("effect") and tol.get("effect") != taint.get("effect"):
        return False
    if tol.get("key") != taint.get("key"):
        # empty key + Exists matches all keys
        if not (not tol.get("key") and tol.get("operator") == "Exists"):
            return False
    op = tol.get("operator") or "Equal"
    if op == "Exists":
        return True
    if op == "Equal":
        return (tol.get("value") or "") == (taint.get("value") or "")
    return False


def tolerations_tolerate_taint(tols: list[dict] | None, taint: dict) -> bool:
    return any(toleration_tolerates_taint(t, taint) for t in tols or [])


def find_untolerated_taint(taints, tols, effects=("NoSchedule", "NoExecute")):
    for t in taints or []:
        if t.get("effect") not in effects:
            continue
        if not tolerations_tolerate_taint(tols, t):
            return t
    return None


# --------------------------------------------------------------- node devices
def node_extended_resources(node: dict) -> dict:
    """NodeStatus.extendedResources: {rname: {resources: {id: {id, health, attributes}}}}."""
    return (node.get("status") or {}).get("extendedResources") or {}


def node_device_ids(node: dict, rname: str, healthy_only: bool = True) -> list[str]:
    dom = node_extended_resources(node).get(rname) or {}
    out = []
    for did, d in (dom.get("resources") or {}).items():
        if healthy_only and (d.get("health") or HEALTHY) != HEALTHY:
            continue
        out.append(did)
    return out
