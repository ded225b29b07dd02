"""Kubelet eviction manager held to the reference's tests.

* pkg/kubelet/eviction/helpers_test.go — the data tables (TestParseThresholdConfig,
  TestThresholdsMet, TestThresholdsUpdatedStats, TestPercentageThresholdsMet, TestNodeConditions,
  TestHasNodeConditions, TestGetStarvedResources) and the eleven TestOrdered* ranking tests are
  extracted by hack/extract_eviction_cases.py into tests/fixtures/eviction_cases.json and
  replayed; the tests built from times relative to `now` (TestThresholdsFirstObservedAt,
  TestThresholdsMetGracePeriod, TestNodeConditionsLastObservedAt, TestNodeConditionsObservedSince),
  TestMakeSignalObservations and testParsePercentage / testCompareThresholdValue are transcribed
  here, cited by line.
* pkg/kubelet/eviction/eviction_manager_test.go — the seven manager scenarios (memory pressure,
  nodefs disk pressure, min-reclaim, node-level reclaim, inode pressure, critical pods,
  allocatable memory) are transcribed step by step with the same fake clock, summary provider,
  pod killer and disk GC.
* A LocalCluster run: memory pressure from the kubelet's own stats summary evicts the BestEffort
  pod, turns MemoryPressure on and rejects a new BestEffort pod.
"""
from __future__ import annotations

import asyncio
import json
import os

import numpy as np
import pytest

from amdkube.kubelet import eviction as E
from amdkube.kubelet.eviction import (ALLOCATABLE_MEMORY, MEMORY, NODEFS, NODEFS_INODES, CapacityProvider, Config,
                                      EvictionManager, Observation, Threshold, ThresholdValue)
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "eviction_cases.json")))
GI, MI = 1 << 30, 1 << 20


def cases(test):
    return [pytest.param(c, id=c["name"]) for c in FIX[test]["cases"]]


def tv(d):
    if d is None:
        return None
    return ThresholdValue(quantity=d.get("quantity"), percentage=d.get("percentage", 0.0))


def threshold(d) -> Threshold:
    return Threshold(d.get("signal", ""), tv(d.get("value")) or ThresholdValue(), float(d.get("gracePeriod", 0.0)),
                     tv(d.get("minReclaim")), d.get("operator", "LessThan"))


def observations(d) -> dict:
    return {sig: Observation(o.get("available", 0), o.get("capacity", 0), o.get("time")) for sig, o in (d or {}).items()}


def same_thresholds(a, b) -> bool:
    """thresholdList.Equal: the same thresholds in any order (hasThreshold: value, grace, operator,
    signal) — and, as thresholdEqual in TestParseThresholdConfig, the same min reclaim."""
    def eq(x, y):
        mr = (x.min_reclaim is None and y.min_reclaim is None) or (
            x.min_reclaim is not None and y.min_reclaim is not None and x.min_reclaim.same(y.min_reclaim))
        return E.has_threshold([x], y) and mr
    return len(a) == len(b) and all(any(eq(x, y) for y in b) for x in a) and all(any(eq(x, y) for x in a) for y in b)


# ------------------------------------------------------------------ helpers_test.go tables
@pytest.mark.parametrize("c", cases("TestParseThresholdConfig"))
def test_parse_threshold_config(c):
    try:
        got = E.parse_threshold_config(c["allocatableConfig"], c["evictionHard"], c["evictionSoft"],
                                       c["evictionSoftGracePeriod"], c["evictionMinReclaim"])
    except ValueError:
        assert c["expectErr"], c["name"]
        return
    assert not c["expectErr"], c["name"]
    want = [threshold(t) for t in c["expectThresholds"]]
    # the reference's expected thresholds carry MinReclaim only where configured
    assert same_thresholds(got, want), (got, want)


@pytest.mark.parametrize("c", cases("TestThresholdsMet") + cases("TestPercentageThresholdsMet"))
def test_thresholds_met(c):
    ts = [threshold(t) for t in c["thresholds"]]
    got = E.thresholds_met(ts, observations(c["observations"]), c.get("enforceMinReclaim", c.get("enforceMinRelaim")))
    want = [threshold(t) for t in c["result"]]
    assert len(got) == len(want) and all(E.has_threshold(want, t) for t in got)


@pytest.mark.parametrize("c", cases("TestThresholdsUpdatedStats"))
def test_thresholds_updated_stats(c):
    ts = [threshold(t) for t in c["thresholds"]]
    got = E.thresholds_updated_stats(ts, observations(c["observations"]), observations(c["last"]))
    assert len(got) == len(c["result"])


@pytest.mark.parametrize("c", cases("TestNodeConditions"))
def test_node_conditions(c):
    assert sorted(E.node_conditions([threshold(t) for t in c["inputs"]])) == sorted(c["result"])


@pytest.mark.parametrize("c", cases("TestHasNodeConditions"))
def test_has_node_condition(c):
    assert (c["item"] in c["inputs"]) == c["result"]


@pytest.mark.parametrize("c", cases("TestGetStarvedResources"))
def test_get_starved_resources(c):
    assert set(E.get_starved_resources([threshold(t) for t in c["inputs"]])) == set(c["result"])


@pytest.mark.parametrize("name", sorted(FIX["ordering"]))
def test_ordered_by(name):
    t = FIX["ordering"][name]
    pods = [json.loads(json.dumps(p)) for p in t["pods"]]
    by_uid = {s["podRef"]["uid"]: s for s in t["stats"]}
    stats = lambda pod: by_uid.get(pod["metadata"]["uid"])    # noqa: E731
    gates = t["gates"]
    local = gates.get("LocalStorageCapacityIsolation", True)
    cmps = []
    for c in t["chain"]:
        if c[0] == "priority":
            cmps.append(E.priority(gates.get("PodPriority", True)))
        elif c[0] == "exceedMemoryRequests":
            cmps.append(E.exceed_memory_requests(stats))
        elif c[0] == "memory":
            cmps.append(E.memory(stats))
        elif c[0] == "exceedDiskRequests":
            cmps.append(E.exceed_disk_requests(stats, c[1], c[2], local))
        elif c[0] == "disk":
            cmps.append(E.disk(stats, c[1], c[2], local))
    E.ordered_by(pods, *cmps)
    assert [p["metadata"]["name"] for p in pods] == t["expected"]


# ------------------------------------------------------------------ transcribed helpers tests
HARD = Threshold(MEMORY, ThresholdValue(quantity=GI), min_reclaim=ThresholdValue(quantity=500 * MI))
SOFT = Threshold(MEMORY, ThresholdValue(quantity=2 * GI), grace=60.0, min_reclaim=ThresholdValue(quantity=500 * MI))


def test_thresholds_first_observed_at():
    """helpers_test.go:1372-1420."""
    now, old = 1000.0, 940.0
    assert E.thresholds_first_observed_at([], {}, now) == {}
    assert E.thresholds_first_observed_at([HARD], {}, now) == {HARD: now}
    assert E.thresholds_first_observed_at([HARD], {HARD: old}, now) == {HARD: old}


def test_thresholds_met_grace_period():
    """helpers_test.go:1421-1478 (soft grace 1m, observed 2m ago)."""
    now, old = 1000.0, 880.0
    assert E.thresholds_met_grace_period({}, now) == []
    assert E.thresholds_met_grace_period({HARD: now}, now) == [HARD]
    assert E.thresholds_met_grace_period({SOFT: now}, now) == []
    assert E.thresholds_met_grace_period({SOFT: old}, now) == [SOFT]


def test_node_conditions_last_observed_at():
    """helpers_test.go:1503-1548."""
    now, old = 1000.0, 940.0
    assert E.node_conditions_last_observed_at(["MemoryPressure"], {}, now) == {"MemoryPressure": now}
    assert E.node_conditions_last_observed_at(["MemoryPressure"], {"MemoryPressure": old}, now) == {"MemoryPressure": now}
    assert E.node_conditions_last_observed_at([], {"MemoryPressure": old}, now) == {"MemoryPressure": old}


def test_node_conditions_observed_since():
    """helpers_test.go:1549-1582 (observed 1m ago; within 2m, not within 30s)."""
    now, at = 1000.0, 940.0
    assert E.node_conditions_observed_since({"MemoryPressure": at}, 120.0, now) == ["MemoryPressure"]
    assert E.node_conditions_observed_since({"MemoryPressure": at}, 30.0, now) == []


def test_parse_percentage_and_compare_threshold_value():
    """testParsePercentage / testCompareThresholdValue (helpers_test.go:1640-1735)."""
    assert E._float32_fraction("25.5") == float(np.float32(np.float32(25.5) / np.float32(100)))
    for bad in ("blah", "foo", "12%345"):
        with pytest.raises(ValueError):
            E._float32_fraction(bad)
    q = lambda v: ThresholdValue(quantity=v)                          # noqa: E731
    p = lambda v: ThresholdValue(percentage=float(np.float32(v)))     # noqa: E731
    for a, b, eq in ((q(123), q(123), True), (q(123), q(456), False), (q(123), p(0.1), False), (p(0.1), p(0.1), True),
                     (p(0.2), p(0.1), False)):
        assert a.same(b) is eq and b.same(a) is eq


def test_make_signal_observations():
    """helpers_test.go:948-1091: node memory (capacity = available + working set), node fs and
    imagefs bytes/inodes, allocatable memory = capacity - reservation - pods' working set."""
    pods = [{"metadata": {"name": f"pod{i}", "namespace": "ns", "uid": f"uid{i}"}, "spec": {"containers": [{}, {}]}}
            for i in range(3)]
    summary = {"node": {"memory": {"availableBytes": 1024, "workingSetBytes": 1000},
                        "fs": {"availableBytes": 2000, "capacityBytes": 3000, "inodesFree": 1000, "inodes": 2000},
                        "runtime": {"imageFs": {"availableBytes": 4000, "capacityBytes": 5000, "inodesFree": 6000,
                                                "inodes": 7000}}},
               "pods": [{"podRef": {"name": p["metadata"]["name"], "namespace": "ns", "uid": p["metadata"]["uid"]},
                         "containers": [{"memory": {"workingSetBytes": 1 << 30}}] * 2} for p in pods]}
    obs, stats = E.make_signal_observations(summary, CapacityProvider({"memory": 10 * GI}, {"memory": 0}), pods)
    assert (obs[MEMORY].available, obs[MEMORY].capacity) == (1024, 2024)
    assert (obs[NODEFS].available, obs[NODEFS].capacity) == (2000, 3000)
    assert (obs[NODEFS_INODES].available, obs[NODEFS_INODES].capacity) == (1000, 2000)
    assert (obs[E.IMAGEFS].available, obs[E.IMAGEFS].capacity) == (4000, 5000)
    assert (obs[E.IMAGEFS_INODES].available, obs[E.IMAGEFS_INODES].capacity) == (6000, 7000)
    assert (obs[ALLOCATABLE_MEMORY].available, obs[ALLOCATABLE_MEMORY].capacity) == (4 * GI, 10 * GI)
    for p in pods:
        assert stats(p)["podRef"]["uid"] == p["metadata"]["uid"]


# ------------------------------------------------------------------ eviction_manager_test.go
LOW, DEFAULT, HIGH = -1, 0, 1


def _rl(cpu="", mem="", disk=""):
    return {k: v for k, v in (("cpu", cpu), ("memory", mem), ("ephemeral-storage", disk)) if v}


def new_pod(name, priority, requests, limits, volumes=None):
    res = {}
    if requests:
        res["requests"] = requests
    if limits:
        res["limits"] = limits
    return {"metadata": {"name": name, "uid": name, "namespace": ""},
            "spec": {"priority": priority, "containers": [{"name": name, "resources": res}], "volumes": volumes or []}}


def _q(v):
    from amdkube.api.quantity import Quantity
    return Quantity(v or "0").value()


def memory_pod(name, prio, req, lim, working_set):
    pod = new_pod(name, prio, req, lim)
    return pod, {"podRef": {"name": name, "uid": name}, "containers": [{"memory": {"workingSetBytes": _q(working_set)}}]}


def disk_pod(name, prio, req, lim, rootfs="", logs="", per_volume="", key="usedBytes"):
    pod = new_pod(name, prio, req, lim)
    vols = [{"name": n, key: _q(per_volume)} for n in E.local_volume_names(pod)]
    return pod, {"podRef": {"name": name, "uid": name}, "volume": vols,
                 "containers": [{"rootfs": {key: _q(rootfs)}, "logs": {key: _q(logs)}}]}


def memory_stats(available, pod_stats):
    v = _q(available)
    return {"node": {"memory": {"availableBytes": v, "workingSetBytes": v}}, "pods": list(pod_stats.values())}


def disk_stats(rootfs_available, imagefs_available, pod_stats):
    r, i = _q(rootfs_available), _q(imagefs_available)
    return {"node": {"fs": {"availableBytes": r, "capacityBytes": 2 * r},
                     "runtime": {"imageFs": {"availableBytes": i, "capacityBytes": 2 * i}}},
            "pods": list(pod_stats.values())}


class Harness:
    """fakeClock + fakeSummaryProvider + mockPodKiller + mockDiskGC + mockDiskInfoProvider."""

    def __init__(self, thresholds, summary, pods, gates=None, image_bytes_freed=0):
        self.now = 0.0
        self.summary = summary
        self.pods = pods
        self.killed = None
        self.grace = None
        self.image_gc_invoked = self.container_gc_invoked = False
        self.image_bytes_freed = image_bytes_freed
        self.gates = {"PodPriority": True, **(gates or {})}
        h = self

        class GC:
            def delete_unused_images(self):
                h.image_gc_invoked = True
                return h.image_bytes_freed

            def delete_all_unused_containers(self):
                h.container_gc_invoked = True

        def kill(pod, status, grace):
            h.killed, h.grace, h.status = pod, grace, status
        self.m = EvictionManager(Config(thresholds, 300.0, 5), kill_pod=kill, summary=lambda: h.summary,
                                 image_gc=GC(), container_gc=GC(), clock=lambda: h.now,
                                 gates=lambda name: h.gates.get(name, False))
        self.capacity = CapacityProvider({"memory": 3 * GI}, {"memory": GI})

    def step(self, seconds, summary=None):
        self.now += seconds
        if summary is not None:
            self.summary = summary
        self.killed = None
        run(self.m.synchronize(lambda: False, lambda: self.pods, self.capacity))

    def admits(self, *pods):
        return [self.m.admit(p)[0] for p in pods]


def _memory_setup():
    specs = [("guaranteed-low-priority-high-usage", LOW, _rl("100m", "1Gi"), _rl("100m", "1Gi"), "900Mi"),
             ("burstable-below-requests", DEFAULT, _rl("100m", "100Mi"), _rl("200m", "1Gi"), "50Mi"),
             ("burstable-above-requests", DEFAULT, _rl("100m", "100Mi"), _rl("200m", "1Gi"), "400Mi"),
             ("best-effort-high-priority-high-usage", HIGH, {}, {}, "400Mi"),
             ("best-effort-low-priority-low-usage", LOW, {}, {}, "100Mi")]
    pods, stats = [], {}
    for s in specs:
        p, st = memory_pod(*s)
        pods.append(p)
        stats[p["metadata"]["name"]] = st
    return pods, stats


def test_memory_pressure():
    """TestMemoryPressure (eviction_manager_test.go:187-395)."""
    pods, stats = _memory_setup()
    evict = pods[4]
    h = Harness([Threshold(MEMORY, ThresholdValue(quantity=GI)),
                 Threshold(MEMORY, ThresholdValue(quantity=2 * GI), grace=120.0)], memory_stats("2Gi", stats), pods)
    be, _ = memory_pod("best-admit", DEFAULT, {}, {}, "0Gi")
    burst, _ = memory_pod("burst-admit", DEFAULT, _rl("100m", "100Mi"), _rl("200m", "200Mi"), "0Gi")
    h.step(0)
    assert not h.m.is_under_memory_pressure() and h.admits(be, burst) == [True, True]
    h.step(60, memory_stats("1500Mi", stats))                # soft threshold
    assert h.m.is_under_memory_pressure() and h.killed is None
    h.step(180, memory_stats("1500Mi", stats))               # past the grace period
    assert h.m.is_under_memory_pressure() and h.killed is evict and h.grace == 5
    assert h.status == {"phase": "Failed", "reason": "Evicted", "message": "The node was low on resource: memory."}
    h.step(1200, memory_stats("3Gi", stats))
    assert not h.m.is_under_memory_pressure()
    h.step(60, memory_stats("500Mi", stats))                 # hard threshold
    assert h.m.is_under_memory_pressure() and h.killed is evict and h.grace == 0
    assert h.admits(be, burst) == [False, True]
    h.step(60, memory_stats("2Gi", stats))
    assert h.m.is_under_memory_pressure() and h.killed is None     # transition period
    assert h.admits(be, burst) == [False, True]
    h.step(300, memory_stats("2Gi", stats))
    assert not h.m.is_under_memory_pressure() and h.killed is None
    assert h.admits(be, burst) == [True, True]


def _disk_setup(key="usedBytes"):
    specs = [("low-priority-high-usage", LOW, _rl("100m", "1Gi"), _rl("100m", "1Gi"), "900Mi", "", ""),
             ("below-requests", DEFAULT, _rl("100m", "100Mi"), _rl("200m", "1Gi"), "", "50Mi", ""),
             ("above-requests", DEFAULT, _rl("100m", "100Mi"), _rl("200m", "1Gi"), "400Mi", "", ""),
             ("high-priority-high-usage", HIGH, {}, {}, "", "", "400Mi"),
             ("low-priority-low-usage", LOW, {}, {}, "100Mi", "", "")]
    pods, stats = [], {}
    for s in specs:
        p, st = disk_pod(*s, key=key)
        pods.append(p)
        stats[p["metadata"]["name"]] = st
    return pods, stats


def test_disk_pressure_nodefs():
    """TestDiskPressureNodeFs (eviction_manager_test.go:405-604)."""
    pods, stats = _disk_setup()
    evict = pods[0]
    h = Harness([Threshold(NODEFS, ThresholdValue(quantity=GI)), Threshold(NODEFS, ThresholdValue(quantity=2 * GI), grace=120.0)],
                disk_stats("16Gi", "200Gi", stats), pods, gates={"LocalStorageCapacityIsolation": True})
    admit, _ = disk_pod("pod-to-admit", DEFAULT, {}, {}, "0Gi", "0Gi", "0Gi")
    h.step(0)
    assert not h.m.is_under_disk_pressure() and h.admits(admit) == [True]
    h.step(60, disk_stats("1.5Gi", "200Gi", stats))
    assert h.m.is_under_disk_pressure() and h.killed is None
    h.step(180, disk_stats("1.5Gi", "200Gi", stats))
    assert h.m.is_under_disk_pressure() and h.killed is evict and h.grace == 5
    assert h.status["message"] == "The node was low on resource: nodefs."
    h.step(1200, disk_stats("16Gi", "200Gi", stats))
    assert not h.m.is_under_disk_pressure()
    h.step(60, disk_stats("500Mi", "200Gi", stats))
    assert h.m.is_under_disk_pressure() and h.killed is evict and h.grace == 0
    assert h.admits(admit) == [False]
    h.step(60, disk_stats("16Gi", "200Gi", stats))
    assert h.m.is_under_disk_pressure() and h.killed is None and h.admits(admit) == [False]
    h.step(300, disk_stats("16Gi", "200Gi", stats))
    assert not h.m.is_under_disk_pressure() and h.killed is None and h.admits(admit) == [True]


def test_min_reclaim():
    """TestMinReclaim (eviction_manager_test.go:607-745)."""
    pods, stats = _memory_setup()
    evict = pods[4]
    h = Harness([Threshold(MEMORY, ThresholdValue(quantity=GI), min_reclaim=ThresholdValue(quantity=500 * MI))],
                memory_stats("2Gi", stats), pods)
    h.step(0)
    assert not h.m.is_under_memory_pressure()
    h.step(60, memory_stats("500Mi", stats))
    assert h.m.is_under_memory_pressure() and h.killed is evict and h.grace == 0
    h.step(60, memory_stats("1.2Gi", stats))                 # above the threshold, below threshold + reclaim
    assert h.m.is_under_memory_pressure() and h.killed is evict and h.grace == 0
    h.step(60, memory_stats("2Gi", stats))
    assert h.m.is_under_memory_pressure() and h.killed is None
    h.step(300, memory_stats("2Gi", stats))
    assert not h.m.is_under_memory_pressure() and h.killed is None


def test_node_reclaim_funcs():
    """TestNodeReclaimFuncs (eviction_manager_test.go:747-922): image GC freeing 700Mi resolves
    .9Gi < 1Gi (+500Mi reclaim) without an eviction; at 400Mi it does not."""
    pods, stats = _disk_setup()
    evict = pods[0]
    h = Harness([Threshold(NODEFS, ThresholdValue(quantity=GI), min_reclaim=ThresholdValue(quantity=500 * MI))],
                disk_stats("16Gi", "200Gi", stats), pods, gates={"LocalStorageCapacityIsolation": True},
                image_bytes_freed=700 * MI)
    h.step(0)
    assert not h.m.is_under_disk_pressure()
    h.step(60, disk_stats(".9Gi", "200Gi", stats))
    assert h.m.is_under_disk_pressure() and h.image_gc_invoked and h.container_gc_invoked and h.killed is None
    h.image_gc_invoked = h.container_gc_invoked = False
    h.step(1200, disk_stats("16Gi", "200Gi", stats))
    assert not h.m.is_under_disk_pressure()
    h.step(60, disk_stats("400Mi", "200Gi", stats))
    assert h.m.is_under_disk_pressure() and h.image_gc_invoked and h.container_gc_invoked
    assert h.killed is evict and h.grace == 0
    h.image_gc_invoked = h.container_gc_invoked = False
    h.step(60, disk_stats("16Gi", "200Gi", stats))
    assert h.m.is_under_disk_pressure() and not (h.image_gc_invoked or h.container_gc_invoked) and h.killed is None
    h.step(300, disk_stats("16Gi", "200Gi", stats))
    assert not h.m.is_under_disk_pressure() and not (h.image_gc_invoked or h.container_gc_invoked) and h.killed is None


def test_inode_pressure_nodefs_inodes():
    """TestInodePressureNodeFsInodes (eviction_manager_test.go:924-1144)."""
    specs = [("low-priority-high-usage", LOW, _rl("100m", "1Gi"), _rl("100m", "1Gi"), "900Mi"),
             ("below-requests", DEFAULT, _rl("100m", "100Mi"), _rl("200m", "1Gi"), "50Mi"),
             ("above-requests", DEFAULT, _rl("100m", "100Mi"), _rl("200m", "1Gi"), "400Mi"),
             ("high-priority-high-usage", HIGH, {}, {}, "400Mi"),
             ("low-priority-low-usage", LOW, {}, {}, "100Mi")]
    pods, stats = [], {}
    for name, prio, req, lim, root in specs:
        p, st = disk_pod(name, prio, req, lim, root, "", "", key="inodesUsed")
        pods.append(p)
        stats[name] = st

    def summary(free, total):
        return {"node": {"fs": {"inodesFree": _q(free), "inodes": _q(total)}}, "pods": list(stats.values())}
    evict = pods[0]
    h = Harness([Threshold(NODEFS_INODES, ThresholdValue(quantity=MI)),
                 Threshold(NODEFS_INODES, ThresholdValue(quantity=2 * MI), grace=120.0)], summary("3Mi", "4Mi"), pods)
    admit, _ = disk_pod("pod-to-admit", DEFAULT, {}, {}, "0", "0", "0", key="inodesUsed")
    h.step(0)
    assert not h.m.is_under_disk_pressure() and h.admits(admit) == [True]
    h.step(60, summary("1.5Mi", "4Mi"))
    assert h.m.is_under_disk_pressure() and h.killed is None
    h.step(180, summary("1.5Mi", "4Mi"))
    assert h.m.is_under_disk_pressure() and h.killed is evict and h.grace == 5
    h.step(1200, summary("3Mi", "4Mi"))
    assert not h.m.is_under_disk_pressure()
    h.step(60, summary("0.5Mi", "4Mi"))
    assert h.m.is_under_disk_pressure() and h.killed is evict and h.grace == 0 and h.admits(admit) == [False]
    h.step(60, summary("3Mi", "4Mi"))
    assert h.m.is_under_disk_pressure() and h.killed is None and h.admits(admit) == [False]
    h.step(300, summary("3Mi", "4Mi"))
    assert not h.m.is_under_disk_pressure() and h.killed is None and h.admits(admit) == [True]


def test_critical_pods_are_not_evicted():
    """TestCriticalPodsAreNotEvicted (eviction_manager_test.go:1147-1280): a static critical pod
    in kube-system is skipped while ExperimentalCriticalPodAnnotation is on."""
    pod, st = memory_pod("critical", DEFAULT, _rl("100m", "1Gi"), _rl("100m", "1Gi"), "800Mi")
    pod["metadata"]["annotations"] = {"scheduler.alpha.kubernetes.io/critical-pod": "", "kubernetes.io/config.source": "file"}
    pod["metadata"]["namespace"] = "kube-system"
    stats = {"critical": st}
    h = Harness([Threshold(MEMORY, ThresholdValue(quantity=GI)),
                 Threshold(MEMORY, ThresholdValue(quantity=2 * GI), grace=120.0)], memory_stats("2Gi", stats), [pod])
    h.gates["ExperimentalCriticalPodAnnotation"] = True
    h.step(60, memory_stats("1500Mi", stats))
    assert h.m.is_under_memory_pressure() and h.killed is None
    h.step(180, memory_stats("1500Mi", stats))
    assert h.m.is_under_memory_pressure() and h.killed is None
    h.step(1200, memory_stats("3Gi", stats))
    assert not h.m.is_under_memory_pressure()
    h.gates["ExperimentalCriticalPodAnnotation"] = False
    h.step(60, memory_stats("500Mi", stats))
    assert h.m.is_under_memory_pressure() and h.killed is pod


def test_allocatable_memory_pressure():
    """TestAllocatableMemoryPressure (eviction_manager_test.go:1283-1445): a 1Gi pod the stats
    know of (not an active pod) pushes allocatable memory below 1Ki."""
    pods, stats = _memory_setup()
    evict = pods[4]
    h = Harness([Threshold(ALLOCATABLE_MEMORY, ThresholdValue(quantity=1024))], memory_stats("4Gi", stats), pods)
    be, _ = memory_pod("best-admit", DEFAULT, {}, {}, "0Gi")
    burst, _ = memory_pod("burst-admit", DEFAULT, _rl("100m", "100Mi"), _rl("200m", "200Mi"), "0Gi")
    h.step(0)
    assert not h.m.is_under_memory_pressure() and h.admits(be, burst) == [True, True]
    _, extra = memory_pod("guaranteed-high-2", DEFAULT, _rl("100m", "1Gi"), _rl("100m", "1Gi"), "1Gi")
    stats["guaranteed-high-2"] = extra
    h.step(60, memory_stats("4Gi", stats))
    assert h.m.is_under_memory_pressure() and h.killed is evict and h.grace == 0
    assert h.admits(be, burst) == [False, True]
    del stats["guaranteed-high-2"]
    h.step(60, memory_stats("4Gi", stats))
    assert h.m.is_under_memory_pressure() and h.killed is None and h.admits(be, burst) == [False, True]
    h.step(300, memory_stats("4Gi", stats))
    assert not h.m.is_under_memory_pressure() and h.killed is None and h.admits(be, burst) == [True, True]


def test_kubelet_flags_and_allocatable_threshold():
    """The kubelet's flag syntax, and --enforce-node-allocatable=pods adds the
    allocatableMemory.available<0 threshold (helpers.go:199-217)."""
    ts = E.parse_thresholds("memory.available<1Gi,nodefs.available<10%", "memory.available<2Gi", "memory.available=1m30s",
                            "memory.available=500Mi", ["pods"])
    assert [t.signal for t in ts] == [ALLOCATABLE_MEMORY, MEMORY, NODEFS, MEMORY]
    assert ts[1].value.quantity == GI and ts[2].value.percentage == float(np.float32(0.1)) and ts[3].grace == 90.0
    assert ts[1].min_reclaim.quantity == 500 * MI and ts[3].min_reclaim.quantity == 500 * MI
    with pytest.raises(ValueError):
        E.parse_thresholds("", "memory.available<1Gi")             # a soft threshold needs a grace period
    with pytest.raises(ValueError):
        E.parse_thresholds("memory.available<0")                   # must be positive


# ------------------------------------------------------------------ in a LocalCluster
async def test_memory_pressure_condition_admission_and_eviction():
    async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                            kubelet_kw={"eviction_interval": 3600, "eviction_hard": "memory.available<2Gi"}) as lc:
        c, k = lc.client, lc.kubelet
        for name, res in (("be", {}), ("gu", {"limits": {"cpu": "100m", "memory": "64Mi"}})):
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"],
                                                     "resources": res}]}}, "default")
            await wait_pod(c, "default", name, ("Running",), 20)
        real = k.stats.summary

        async def low_memory():                  # the node's memory below the 2Gi hard threshold
            s = await real()
            s["node"]["memory"] = {"availableBytes": GI, "workingSetBytes": 63 * GI}
            return s
        k.eviction.summary = low_memory
        victim = await k.eviction_pass()
        assert victim["metadata"]["name"] == "be"
        p = await wait_pod(c, "default", "be", ("Failed",), 10)
        assert p["status"]["reason"] == "Evicted" and p["status"]["message"] == "The node was low on resource: memory."
        for _ in range(400):
            node = await c.get("nodes", lc.node_name)
            conds = {x["type"]: x["status"] for x in node["status"]["conditions"]}
            if conds["MemoryPressure"] == "True":
                break
            await asyncio.sleep(0.05)
        assert conds["MemoryPressure"] == "True"
        # a new BestEffort pod is rejected while the node is under memory pressure
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "late"},
                        "spec": {"nodeName": lc.node_name, "containers": [{"name": "c", "image": "busybox", "command": ["true"]}]}},
                       "default")
        p = await wait_pod(c, "default", "late", ("Failed",), 10)
        assert p["status"]["reason"] == "Evicted" and "[MemoryPressure]" in p["status"]["message"]
        assert (await c.get("pods", "gu", "default"))["status"]["phase"] == "Running"
