"""Kubelet critical-pod preemption held to pkg/kubelet/preemption/preemption_test.go.

Every case of TestEvictPodsToFreeRequests :87 (its victim choice, through `pods_to_preempt`; the
kill itself is the kubelet's `_preempt_for`), TestGetPodsToPreempt :154,
TestAdmissionRequirementsDistance :247 and TestAdmissionRequirementsSubtract :289, with the
reference's getTestPods :337. Requirement lists are {resource: quantity} (cpu in millicores,
memory in bytes, pods as a count), as getAdmissionRequirementList :417 builds them.
"""
from __future__ import annotations

import pytest

from amdkube.kubelet.preemption import distance, pods_to_preempt, subtract


def _pod(name, requests=None, limits=None):
    res = {}
    if requests:
        res["requests"] = requests
    if limits:
        res["limits"] = limits
    return {"metadata": {"generateName": name, "annotations": {}},
            "spec": {"containers": [{"name": f"{name}-container", "resources": res}]}}


def _rl(cpu, mem):
    return {"cpu": cpu, "memory": mem}


PODS = {
    "tinyBurstable": _pod("tinyBurstable", _rl("1m", "1Mi")),
    "bestEffort": _pod("bestEffort"),
    "critical": _pod("critical", _rl("100m", "100Mi")),
    "burstable": _pod("burstable", _rl("100m", "100Mi")),
    "guaranteed": _pod("guaranteed", _rl("100m", "100Mi"), _rl("100m", "100Mi")),
    "highRequestBurstable": _pod("highRequestBurstable", _rl("300m", "300Mi")),
    "highRequestGuaranteed": _pod("highRequestGuaranteed", _rl("300m", "300Mi"), _rl("300m", "300Mi")),
}
PODS["critical"]["metadata"]["namespace"] = "kube-system"
PODS["critical"]["metadata"]["annotations"]["scheduler.alpha.kubernetes.io/critical-pod"] = ""


def reqs(cpu, memory, pods):
    out = {}
    if cpu > 0:
        out["cpu"] = cpu
    if memory > 0:
        out["memory"] = memory << 20
    if pods > 0:
        out["pods"] = pods
    return out


def _names(pods):
    return sorted(p["metadata"]["generateName"] for p in pods)


ALL = ["critical", "bestEffort", "burstable", "highRequestBurstable", "guaranteed", "highRequestGuaranteed"]
FIVE = ["bestEffort", "burstable", "highRequestBurstable", "guaranteed", "highRequestGuaranteed"]
CASES = [
    # TestEvictPodsToFreeRequests
    ("critical pods cannot be preempted", ["critical"], (0, 0, 1), None),
    ("best effort pods are not preempted when attempting to free resources", ["bestEffort"], (0, 1, 0), None),
    ("multiple pods evicted", ALL, (0, 550, 0), ["highRequestBurstable", "highRequestGuaranteed"]),
    # TestGetPodsToPreempt
    ("no requirements", [], (0, 0, 0), []),
    ("no pods", [], (0, 0, 1), None),
    ("equal pods and resources requirements", ["burstable"], (100, 100, 1), ["burstable"]),
    ("higer requirements than pod requests", ["burstable"], (200, 200, 2), None),
    ("choose between bestEffort and burstable", ["burstable", "bestEffort"], (0, 0, 1), ["bestEffort"]),
    ("choose between burstable and guaranteed", ["burstable", "guaranteed"], (0, 0, 1), ["burstable"]),
    ("choose lower request burstable if it meets requirements", ["bestEffort", "highRequestBurstable", "burstable"],
     (100, 100, 0), ["burstable"]),
    ("choose higher request burstable if lower does not meet requirements", ["bestEffort", "burstable", "highRequestBurstable"],
     (150, 150, 0), ["highRequestBurstable"]),
    ("multiple pods required", FIVE, (350, 350, 0), ["burstable", "highRequestBurstable"]),
    ("evict guaranteed when we have to, and dont evict the extra burstable", FIVE, (0, 550, 0),
     ["highRequestBurstable", "highRequestGuaranteed"]),
]


@pytest.mark.parametrize("name,pods,requirement,expected", CASES, ids=[c[0] for c in CASES])
def test_get_pods_to_preempt(name, pods, requirement, expected):
    inputs = [PODS[p] for p in pods]
    if expected is None:
        with pytest.raises(ValueError, match="no set of running pods found to reclaim resources"):
            pods_to_preempt(inputs, reqs(*requirement))
    else:
        assert _names(pods_to_preempt(inputs, reqs(*requirement))) == sorted(expected)


@pytest.mark.parametrize("name,requirement,pod,expected", [
    ("no requirements", (0, 0, 0), "burstable", 0),
    ("no requests, some requirements", (100, 100, 1), "bestEffort", 2),
    ("equal requests and requirements", (100, 100, 1), "burstable", 0),
    ("higher requests than requirements", (50, 50, 0), "burstable", 0),
])
def test_admission_requirements_distance(name, requirement, pod, expected):
    assert distance(reqs(*requirement), PODS[pod]) == expected


@pytest.mark.parametrize("name,initial,pod,expected", [
    ("subtract a pod from no requirements", (0, 0, 0), "burstable", (0, 0, 0)),
    ("subtract no requests from some requirements", (100, 100, 1), "bestEffort", (100, 100, 0)),
    ("equal requests and requirements", (100, 100, 1), "burstable", (0, 0, 0)),
    ("subtract higher requests than requirements", (50, 50, 0), "burstable", (0, 0, 0)),
    ("subtract lower requests than requirements", (200, 200, 1), "burstable", (100, 100, 0)),
])
def test_admission_requirements_subtract(name, initial, pod, expected):
    assert subtract(reqs(*initial), [PODS[pod]]) == reqs(*expected)


def test_tiny_burstable_benchmark_shape():
    """BenchmarkGetPodsToPreempt :139: 110 tiny pods (1m each) cover a 110m requirement."""
    out = pods_to_preempt([PODS["tinyBurstable"]] * 110, {"cpu": 110})
    assert len(out) == 110


@pytest.mark.parametrize("ns,value,expected", [("ns", "", False), ("ns", "abc", False), ("kube-system", "abc", False),
                                               ("kube-system", "", True)])
def test_is_critical_pod(ns, value, expected):
    """pkg/kubelet/types/pod_update_test.go TestIsCriticalPod :117, against every critical-pod
    check in amdkube (kubelet preemption and eviction, DaemonSet controller)."""
    from amdkube.controllers.daemonset import is_critical as ds_critical
    from amdkube.kubelet.eviction import is_critical_pod
    from amdkube.kubelet.preemption import is_critical
    ann = {"scheduler.alpha.kubernetes.io/critical-pod": value}
    p = {"metadata": {"name": "pod", "namespace": ns, "annotations": ann}}
    assert is_critical(p) is expected and is_critical_pod(p) is expected and ds_critical(ns, ann) is expected
