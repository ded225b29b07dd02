"""Pod QoS classes, OOM score adjustment and the QoS cgroup hierarchy.

Reference: pkg/apis/core/helper/qos/qos.go GetPodQOS (Guaranteed: every container has cpu
and memory limits with requests equal to them; BestEffort: no requests or limits at all;
Burstable otherwise), pkg/kubelet/qos/policy.go GetContainerOOMScoreAdjust (Guaranteed
−998, BestEffort 1000, Burstable 1000 − 1000·memoryRequest/memoryCapacity clamped to
[2, 999] from the memory request), pkg/kubelet/cm/qos_container_manager_linux.go +
pod_container_manager_linux.go (cgroup parent kubepods/[burstable|besteffort]/pod<uid>).
"""
from __future__ import annotations

from ..api.quantity import Quantity

GUARANTEED, BURSTABLE, BEST_EFFORT = "Guaranteed", "Burstable", "BestEffort"
CRITICAL_ANNOTATION = "scheduler.alpha.kubernetes.io/critical-pod"
GUARANTEED_OOM, BEST_EFFORT_OOM = -998, 1000


def _qos_resource(name: str) -> bool:
    """isSupportedQoSComputeResource: cpu, memory and the hugepages-<size> resources."""
    return name in ("cpu", "memory") or name.startswith("hugepages-")


def pod_qos(pod: dict) -> str:
    """GetPodQOS over the app containers of an API-defaulted pod (requests already filled from
    limits): positive quantities are summed per resource across containers; Guaranteed needs a cpu
    and a memory limit in every container and equal summed requests and limits."""
    requests, limits = {}, {}
    guaranteed = True
    for c in (pod.get("spec") or {}).get("containers") or []:
        r = c.get("resources") or {}
        for k, v in (r.get("requests") or {}).items():
            q = Quantity(str(v)).as_fraction()
            if _qos_resource(k) and q > 0:
                requests[k] = requests.get(k, 0) + q
        found = set()
        for k, v in (r.get("limits") or {}).items():
            q = Quantity(str(v)).as_fraction()
            if _qos_resource(k) and q > 0:
                found.add(k)
                limits[k] = limits.get(k, 0) + q
        if not {"cpu", "memory"} <= found:
            guaranteed = False
    if not requests and not limits:
        return BEST_EFFORT
    if guaranteed and all(k in limits and limits[k] == v for k, v in requests.items()) and len(requests) == len(limits):
        return GUARANTEED
    return BURSTABLE


def oom_score_adj(pod: dict, container: dict, memory_capacity: int) -> int:
    """GetContainerOOMScoreAdjust: Burstable containers get 1000 − 1000·memoryRequest/capacity
    from the container's memory request alone, floored at 2 and kept below BestEffort's 1000."""
    q = pod_qos(pod)
    if q == GUARANTEED:
        return GUARANTEED_OOM
    if q == BEST_EFFORT:
        return BEST_EFFORT_OOM
    mem = ((container.get("resources") or {}).get("requests") or {}).get("memory")
    req = Quantity(str(mem)).value() if mem is not None else 0
    adj = 1000 - (1000 * req) // memory_capacity
    if adj < 1000 + GUARANTEED_OOM:
        return 1000 + GUARANTEED_OOM
    return adj - 1 if adj == BEST_EFFORT_OOM else adj


def pod_cgroup_name(pod: dict) -> str:
    """The internal name of the pod's cgroup (pod_container_manager_linux.go GetPodContainerName)."""
    uid = (pod.get("metadata") or {}).get("uid", "")
    q = pod_qos(pod)
    if q == GUARANTEED:
        return f"/kubepods/pod{uid}"
    return f"/kubepods/{q.lower()}/pod{uid}"


def cgroup_parent(pod: dict, driver: str = "cgroupfs") -> str:
    """The CRI sandbox's cgroup parent: the driver's literal name (cgroupManager.Name) — a
    relative path for cgroupfs, the expanded slice path for systemd
    (kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod<uid>.slice/)."""
    name = pod_cgroup_name(pod)
    if driver == "systemd":
        from .cgroups import to_systemd
        return to_systemd(name, True)
    return name.lstrip("/")
