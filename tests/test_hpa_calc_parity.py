"""The HPA replica calculator held to pkg/controller/podautoscaler/replica_calculator_test.go.

Every test of that file is transcribed (TestReplicaCalcDisjointResourcesMetrics :296 through
TestReplicaCalcComputedToleranceAlgImplementation :717) with the reference harness's shapes
(prepareTestClient :84): pods `test-pod-<i>`, Running, Ready per `podReadiness`, two containers each
requesting `requests[i]`; resource metrics report `levels[i]` milli-units per container (so a pod's
usage is 2 × level), custom pod metrics `levels[i]` milli-units per pod, object metrics `levels[0]`.
"""
from __future__ import annotations

import math

import pytest

from amdkube.controllers.autoscaling import (TOLERANCE, get_object_metric_replicas, get_plain_metric_replicas,
                                             get_resource_replicas)

NS, PREFIX, CONTAINERS = "test-namespace", "test-pod", 2


def _pods(current, requests=(), readiness=None):
    out = []
    for i in range(current):
        cts = [{"name": ""}, {"name": ""}]
        if i < len(requests):
            for c in cts:
                c["resources"] = {"requests": {"cpu": requests[i]}}
        out.append({"metadata": {"name": f"{PREFIX}-{i}", "namespace": NS, "labels": {"name": PREFIX}},
                    "spec": {"containers": cts},
                    "status": {"phase": "Running",
                               "conditions": [{"type": "Ready", "status": readiness[i] if readiness else "True"}]}})
    return out


def _resource(current, requests, levels, target, readiness=None, pod_names=()):
    metrics = {(pod_names[i] if i < len(pod_names) else f"{PREFIX}-{i}"): CONTAINERS * lv for i, lv in enumerate(levels)}
    return get_resource_replicas(current, target, "cpu", _pods(current, requests, readiness), metrics, NS)


def _metric(current, levels, target, readiness=None):
    return get_plain_metric_replicas(current, target, _pods(current, (), readiness),
                                     {f"{PREFIX}-{i}": lv for i, lv in enumerate(levels)})


F, T = "False", "True"
ONE = "1.0"

# (test, current, requests, levels, target, readiness, expected replicas, utilization, raw value)
RESOURCE = [
    ("ScaleUp", 3, [ONE] * 3, [300, 500, 700], 30, None, 5, 50, CONTAINERS * 500),
    ("ScaleUpUnreadyLessScale", 3, [ONE] * 3, [300, 500, 700], 30, [F, T, T], 4, 60, CONTAINERS * 600),
    ("ScaleUpUnreadyNoScale", 3, [ONE] * 3, [400, 500, 700], 30, [T, F, F], 3, 40, CONTAINERS * 400),
    ("ScaleDown", 5, [ONE] * 5, [100, 300, 500, 250, 250], 50, None, 3, 28, CONTAINERS * 280),
    ("ScaleDownIgnoresUnreadyPods", 5, [ONE] * 5, [100, 300, 500, 250, 250], 50, [T, T, T, F, F], 2, 30, CONTAINERS * 300),
    ("Tolerance", 3, ["0.9", "1.0", "1.1"], [1010, 1030, 1020], 100, None, 3, 102, CONTAINERS * 1020),
    ("SuperfluousMetrics", 4, [ONE] * 4, [4000, 9500, 3000, 7000, 3200, 2000], 100, None, 24, 587, CONTAINERS * 5875),
    ("MissingMetrics", 4, [ONE] * 4, [400, 95], 100, None, 3, 24, 495),
    ("MissingMetricsNoChangeEq", 2, [ONE] * 2, [1000], 100, None, 2, 100, CONTAINERS * 1000),
    ("MissingMetricsNoChangeGt", 2, [ONE] * 2, [1900], 100, None, 2, 190, CONTAINERS * 1900),
    ("MissingMetricsNoChangeLt", 2, [ONE] * 2, [600], 100, None, 2, 60, CONTAINERS * 600),
    ("MissingMetricsUnreadyNoChange", 3, [ONE] * 3, [100, 450], 50, [F, T, T], 3, 45, CONTAINERS * 450),
    ("MissingMetricsUnreadyScaleUp", 3, [ONE] * 3, [100, 2000], 50, [F, T, T], 4, 200, CONTAINERS * 2000),
    ("MissingMetricsUnreadyScaleDown", 4, [ONE] * 4, [100, 100, 100], 50, [F, T, T, T], 3, 10, CONTAINERS * 100),
]


@pytest.mark.parametrize("name,current,requests,levels,target,readiness,replicas,util,raw", RESOURCE,
                         ids=[r[0] for r in RESOURCE])
def test_resource_replicas(name, current, requests, levels, target, readiness, replicas, util, raw):
    assert _resource(current, requests, levels, target, readiness) == (replicas, util, raw)


@pytest.mark.parametrize("name,current,requests,levels,target,pod_names,error", [
    ("DisjointResourcesMetrics", 1, [ONE], [100], 100, ["an-older-pod-name"], "no metrics returned matched known pods"),
    ("EmptyMetrics", 4, [ONE] * 3, [], 100, (), "unable to get metrics for resource cpu: no metrics returned from heapster"),
    ("EmptyCPURequest", 1, [], [200], 100, (), "missing request for"),
])
def test_resource_replica_errors(name, current, requests, levels, target, pod_names, error):
    with pytest.raises(LookupError) as e:
        _resource(current, requests, levels, target, pod_names=pod_names)
    assert error in str(e.value)


# (test, current, levels, target, readiness, expected replicas, utilization)
CUSTOM = [
    ("ScaleUpCM", 3, [20000, 10000, 30000], 15000, None, 4, 20000),
    ("ScaleUpCMUnreadyLessScale", 3, [50000, 10000, 30000], 15000, [T, T, F], 4, 30000),
    ("ScaleUpCMUnreadyNoScaleWouldScaleDown", 3, [50000, 15000, 30000], 15000, [F, T, F], 3, 15000),
    ("ScaleDownCM", 5, [12000] * 5, 20000, None, 3, 12000),
    ("ToleranceCM", 3, [20000, 21000, 21000], 20000, None, 3, 20666),
]


@pytest.mark.parametrize("name,current,levels,target,readiness,replicas,util", CUSTOM, ids=[c[0] for c in CUSTOM])
def test_pod_metric_replicas(name, current, levels, target, readiness, replicas, util):
    assert _metric(current, levels, target, readiness) == (replicas, util)


@pytest.mark.parametrize("name,current,level,target,replicas", [
    ("ScaleUpCMObject", 3, 20000, 15000, 4),
    ("ScaleDownCMObject", 5, 12000, 20000, 3),
    ("ToleranceCMObject", 3, 20666, 20000, 3),
])
def test_object_metric_replicas(name, current, level, target, replicas):
    assert get_object_metric_replicas(current, target, level) == replicas


def test_computed_tolerance_alg_implementation():
    """TestReplicaCalcComputedToleranceAlgImplementation, with the reference's int32/float64 steps."""
    start = 10
    used = start * 150
    requested = 2 * used
    requested_to_used = float(requested // used)
    per_pod = requested // start
    target = abs(1 / (requested_to_used * (1 - TOLERANCE))) + .01
    pct = int(target * 100)
    final = int(math.ceil(used / (requested * target) * start))
    requests = [f"{per_pod + d}m" for d in (100, -100, 10, -10, 2, -2, 1, -1, 0, 0)]
    levels = [used // 10] * 10
    expect_util, expect_raw = used * 100 // requested, CONTAINERS * used // 10
    assert final == 9
    assert _resource(start, requests, levels, pct) == (final, expect_util, expect_raw)
    # just inside the tolerance margin nothing scales
    pct = int((abs(1 / (requested_to_used * (1 - TOLERANCE))) + .004) * 100)
    assert _resource(start, requests, levels, pct) == (start, expect_util, expect_raw)


def test_missing_pods_at_exact_target():
    """Not in the reference tests; read off replica_calculator.go: at a usage ratio of exactly 1.0
    a plain metric still zero-fills missing pods (the `else` at :244) and so scales down, while a
    resource metric leaves them out (`else if usageRatio > 1.0` at :131) and keeps the count."""
    assert _metric(2, [15000], 15000) == (1, 15000)
    assert _resource(2, [ONE] * 2, [1000], 100) == (2, 100, CONTAINERS * 1000)
