"""Pod QoS classes, OOM score adjustment and the QoS cgroup hierarchy.

Reference: pkg/apis/core/helper/qos/qos.go GetPodQOS (Guaranteed: every container has cpu
and memory limits with requests equal to them; BestEffort: no requests or limits at all;
Burstable otherwise), pkg/kubelet/qos/policy.go GetContainerOOMScoreAdjust (Guaranteed
−998, BestEffort 1000, Burstable 1000 − 1000·memoryRequest/memoryCapacity clamped to
[2, 999]; critical pods −998), pkg/kubelet/cm/qos_container_manager_linux.go +
pod_container_manager_linux.go (cgroup parent kubepods/[burstable|besteffort]/pod<uid>).
"""
from __future__ import annotations

from ..api.quantity import Quantity

GUARANTEED, BURSTABLE, BEST_EFFORT = "Guaranteed", "Burstable", "BestEffort"
CRITICAL_ANNOTATION = "scheduler.alpha.kubernetes.io/critical-pod"
GUARANTEED_OOM, BEST_EFFORT_OOM, CRITICAL_OOM = -998, 1000, -998


def pod_qos(pod: dict) -> str:
    spec = pod.get("spec") or {}
    requests, limits, any_set = {}, {}, False
    guaranteed = True
    for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
        r = c.get("resources") or {}
        rq, li = dict(r.get("requests") or {}), dict(r.get("limits") or {})
        for k, v in li.items():   # requests default to limits
            rq.setdefault(k, v)
        for k in ("cpu", "memory"):
            if k in rq and Quantity(rq[k]).as_fraction() > 0:
                any_set = True
                requests[k] = True
            if k in li and Quantity(li[k]).as_fraction() > 0:
                any_set = True
                limits[k] = True
            if k not in li or k not in rq or Quantity(rq[k]) != Quantity(li[k]):
                guaranteed = False
    if not any_set:
        return BEST_EFFORT
    return GUARANTEED if guaranteed and set(limits) == {"cpu", "memory"} else BURSTABLE


def oom_score_adj(pod: dict, container: dict, memory_capacity: int) -> int:
    if ((pod.get("metadata") or {}).get("annotations") or {}).get(CRITICAL_ANNOTATION) is not None and \
            ((pod.get("metadata") or {}).get("namespace") == "kube-system"):
        return CRITICAL_OOM
    q = pod_qos(pod)
    if q == GUARANTEED:
        return GUARANTEED_OOM
    if q == BEST_EFFORT:
        return BEST_EFFORT_OOM
    res = container.get("resources") or {}
    mem = (res.get("requests") or {}).get("memory") or (res.get("limits") or {}).get("memory")
    req = Quantity(mem).value() if mem else 0
    adj = 1000 - (1000 * req) // max(1, memory_capacity)
    return int(min(999, max(2, adj)))


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
