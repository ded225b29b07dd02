"""Critical-pod admission preemption (pkg/kubelet/preemption/preemption.go).

When a critical pod (kube-system + the scheduler.alpha.kubernetes.io/critical-pod annotation,
ExperimentalCriticalPodAnnotation gate) fails admission only for lack of resources, the kubelet
evicts non-critical pods to make room: first the guaranteed pods that would still be needed
after evicting every burstable and best-effort pod, then the burstable pods needed after the
best-effort ones and those guaranteed, then the best-effort pods; within a class pods are picked
greedily by the smallest squared distance to the remaining requirement (ties: smaller GPU, then
memory, then CPU request). Victims end Failed with reason Preempting.
"""
from __future__ import annotations

from ..api.helpers import pod_requests
from .qos import CRITICAL_ANNOTATION, pod_qos


def is_critical(pod: dict) -> bool:
    md = pod.get("metadata") or {}
    return md.get("namespace") == "kube-system" and (md.get("annotations") or {}).get(CRITICAL_ANNOTATION) == ""


def request(pod: dict, res: str) -> int:
    """resource.GetResourceRequest: 1 for pods, millicores for cpu, base units otherwise, from the
    containers' requests (API-defaulted), plus the pod's device-granular extended resources."""
    if res == "pods":
        return 1
    from ..api.helpers import ExtendedResourceError, pod_extended_resource_count, pod_extended_resource_name
    v = pod_requests(pod).get(res, 0)
    for pres in (pod.get("spec") or {}).get("extendedResources") or []:
        try:
            if pod_extended_resource_name(pres) == res:
                v += pod_extended_resource_count(pres)
        except (ExtendedResourceError, KeyError):
            pass
    return int(v)


def subtract(reqs: dict[str, int], pods) -> dict[str, int]:
    out = {}
    for r, q in reqs.items():
        q -= sum(request(p, r) for p in pods)
        if q > 0:
            out[r] = q
    return out


def distance(reqs: dict[str, int], pod: dict) -> float:
    return sum((max(0, q - request(pod, r)) / q) ** 2 for r, q in reqs.items())


def _smaller(a: dict, b: dict) -> bool:
    for r in ("amd.com/gpu", "memory", "cpu"):
        x, y = request(a, r), request(b, r)
        if x != y:
            return x < y
    return True


def by_distance(pods: list[dict], reqs: dict[str, int]) -> list[dict]:
    """getPodsToPreemptByDistance: each round scans in order for the smallest distance (ties go to
    the smaller request), then moves the last pod into the chosen slot, so later rounds see the
    reference's order."""
    pods, out = list(pods), []
    while reqs:
        if not pods:
            raise ValueError(f"no set of running pods found to reclaim resources: {reqs}")
        best_d, best = float(len(reqs) + 1), 0
        for i, p in enumerate(pods):
            d = distance(reqs, p)
            if d < best_d or (d == best_d and _smaller(p, pods[best])):
                best_d, best = d, i
        victim = pods[best]
        reqs = subtract(reqs, [victim])
        out.append(victim)
        pods[best] = pods[-1]
        pods.pop()
    return out


def pods_to_preempt(active: list[dict], reqs: dict[str, int]) -> list[dict]:
    cands = [p for p in active if not is_critical(p)]
    be = [p for p in cands if pod_qos(p) == "BestEffort"]
    bu = [p for p in cands if pod_qos(p) == "Burstable"]
    gu = [p for p in cands if pod_qos(p) == "Guaranteed"]
    if subtract(reqs, be + bu + gu):
        raise ValueError(f"no set of running pods found to reclaim resources: {subtract(reqs, be + bu + gu)}")
    g = by_distance(gu, subtract(reqs, be + bu))
    b = by_distance(bu, subtract(reqs, be + g))
    e = by_distance(be, subtract(reqs, b + g))
    return e + b + g
