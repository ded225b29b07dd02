"""Scheduler priorities held to the reference's own test tables.

Each case is the reference's table entry, transcribed (pods, nodes, Services/RCs/RSs/
StatefulSets, expected HostPriority list), cited by file:line:
  plugin/pkg/scheduler/algorithm/priorities/selector_spreading_test.go
    TestSelectorSpreadPriority :43-364, TestZoneSelectorSpreadPriority :373-556,
    TestZoneSpreadPriority (ServiceAntiAffinity) :558-757
  image_locality_test.go TestImageLocalityPriority :30-175
  resource_limits_test.go TestResourceLimistPriority :28-151
  algorithmprovider/defaults/defaults.go:91-115,217-260 (the registered priority names)
Reference tests compare Namespace "" and "default" as distinct namespaces; so do these (the
apiserver always sets one, so the distinction never arises in a cluster).
"""
from __future__ import annotations

import pytest

from amdkube.scheduler.cache import NodeInfo, SchedulerCache
from amdkube.scheduler.generic import Context, GenericScheduler
from amdkube.scheduler.listers import ControllerListers
from amdkube.scheduler.predicates import PodInfo
from amdkube.scheduler import priorities as P
from amdkube.scheduler.policy_args import build, service_anti_affinity

ZONE = "failure-domain.beta.kubernetes.io/zone"
L1 = {"foo": "bar", "baz": "blah"}
L2 = {"bar": "foo", "baz": "blah"}


def pod(node="", labels=None, ns=None):
    md = {}
    if labels is not None:
        md["labels"] = dict(labels)
    if ns is not None:
        md["namespace"] = ns
    return {"metadata": md, "spec": {"nodeName": node} if node else {}}


def svc(sel, ns=None):
    return {"metadata": {"namespace": ns} if ns else {}, "spec": {"selector": dict(sel)}}


def rc(sel):
    return {"metadata": {}, "spec": {"selector": dict(sel)}}


def rs(sel):   # ReplicaSet and StatefulSet: a LabelSelector
    return {"metadata": {}, "spec": {"selector": {"matchLabels": dict(sel)}}}


def node_infos(nodes: dict, pods: list) -> list:
    out = {}
    for name, labels in nodes.items():
        ni = NodeInfo(name)
        ni.set_node({"metadata": {"name": name, "labels": dict(labels or {})}, "status": {}})
        out[name] = ni
    for i, p in enumerate(pods):
        p = {**p, "metadata": {**p["metadata"], "name": f"p{i}"}}
        n = p["spec"].get("nodeName")
        if n in out:
            out[n].add_pod(f"k{i}", p)
    return out


def run_spread(the_pod, pods, nodes, services=(), rcs=(), rss=(), sss=()):
    nis = node_infos(nodes, pods)
    ctx = Context(list(nis.values()), False, listers=ControllerListers(
        services=lambda: list(services), rcs=lambda: list(rcs), rss=lambda: list(rss), sss=lambda: list(sss)))
    order = list(nis.values())
    scores = P.selector_spread(PodInfo(the_pod), order, ctx)
    return {ni.name: int(s) for ni, s in zip(order, scores)}


M12 = {"machine1": {}, "machine2": {}}

# selector_spreading_test.go TestSelectorSpreadPriority (:68-363), in table order
SPREAD = [
    ("nothing scheduled", pod(), [], {}, dict(), [10, 10]),
    ("no services", pod(labels=L1), [pod("machine1")], {}, dict(), [10, 10]),
    ("different services", pod(labels=L1), [pod("machine1", L2)], {}, dict(services=[svc({"key": "value"})]), [10, 10]),
    ("two pods, one service pod", pod(labels=L1), [pod("machine1", L2), pod("machine2", L1)], {},
     dict(services=[svc(L1)]), [10, 0]),
    ("five pods, one service pod in no namespace", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1, "default"), pod("machine1", L1, "ns1"), pod("machine2", L1), pod("machine2", L2)],
     {}, dict(services=[svc(L1)]), [10, 0]),
    ("four pods, one service pod in default namespace", pod(labels=L1, ns="default"),
     [pod("machine1", L1), pod("machine1", L1, "ns1"), pod("machine2", L1, "default"), pod("machine2", L2)],
     {}, dict(services=[svc(L1, "default")]), [10, 0]),
    ("five pods, one service pod in specific namespace", pod(labels=L1, ns="ns1"),
     [pod("machine1", L1), pod("machine1", L1, "default"), pod("machine1", L1, "ns2"), pod("machine2", L1, "ns1"), pod("machine2", L2)],
     {}, dict(services=[svc(L1, "ns1")]), [10, 0]),
    ("three pods, two service pods on different machines", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {}, dict(services=[svc(L1)]), [0, 0]),
    ("four pods, three service pods", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1), pod("machine2", L1)], {}, dict(services=[svc(L1)]), [5, 0]),
    ("service with partial pod label matches", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {}, dict(services=[svc({"baz": "blah"})]), [0, 5]),
    ("service + replication controller", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {},
     dict(rcs=[rc({"foo": "bar"})], services=[svc({"baz": "blah"})]), [0, 5]),
    ("service + replica set", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {},
     dict(services=[svc({"baz": "blah"})], rss=[rs({"foo": "bar"})]), [0, 5]),
    ("service + stateful set", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {},
     dict(services=[svc({"baz": "blah"})], sss=[rs({"foo": "bar"})]), [0, 5]),
    ("disjoined service and replication controller", pod(labels={"foo": "bar", "bar": "foo"}),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {},
     dict(rcs=[rc({"foo": "bar"})], services=[svc({"bar": "foo"})]), [0, 5]),
    ("disjoined service and replica set", pod(labels={"foo": "bar", "bar": "foo"}),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {},
     dict(services=[svc({"bar": "foo"})], rss=[rs({"foo": "bar"})]), [0, 5]),
    ("disjoined service and stateful set", pod(labels={"foo": "bar", "bar": "foo"}),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {},
     dict(services=[svc({"bar": "foo"})], sss=[rs({"foo": "bar"})]), [0, 5]),
    ("Replication controller with partial pod label matches", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {}, dict(rcs=[rc({"foo": "bar"})]), [0, 0]),
    ("Replica set with partial pod label matches", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {}, dict(rss=[rs({"foo": "bar"})]), [0, 0]),
    ("StatefulSet with partial pod label matches", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {}, dict(sss=[rs({"foo": "bar"})]), [0, 0]),
    ("Another replication controller with partial pod label matches", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {}, dict(rcs=[rc({"baz": "blah"})]), [0, 5]),
    ("Another replication set with partial pod label matches", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {}, dict(rss=[rs({"baz": "blah"})]), [0, 5]),
    ("Another stateful set with partial pod label matches", pod(labels=L1),
     [pod("machine1", L2), pod("machine1", L1), pod("machine2", L1)], {}, dict(sss=[rs({"baz": "blah"})]), [0, 5]),
]


@pytest.mark.parametrize("name,the_pod,pods,_unused,listers,expected", SPREAD, ids=[c[0] for c in SPREAD])
def test_selector_spread_priority_table(name, the_pod, pods, _unused, listers, expected):
    got = run_spread(the_pod, pods, M12, **listers)
    assert [got["machine1"], got["machine2"]] == expected, name


# selector_spreading_test.go TestZoneSelectorSpreadPriority (:366-556)
ZL1 = {"label1": "l1", "baz": "blah"}
ZL2 = {"label2": "l2", "baz": "blah"}
ZNODES = {"machine1.zone1": {ZONE: "zone1"}, "machine1.zone2": {ZONE: "zone2"}, "machine2.zone2": {ZONE: "zone2"},
          "machine1.zone3": {ZONE: "zone3"}, "machine2.zone3": {ZONE: "zone3"}, "machine3.zone3": {ZONE: "zone3"}}
ZORDER = ["machine1.zone1", "machine1.zone2", "machine2.zone2", "machine1.zone3", "machine2.zone3", "machine3.zone3"]
ZONE_SPREAD = [
    ("nothing scheduled", pod(), [], {}, [10, 10, 10, 10, 10, 10]),
    ("no services", pod(labels=ZL1), [pod("machine1.zone1")], {}, [10, 10, 10, 10, 10, 10]),
    ("different services", pod(labels=ZL1), [pod("machine1.zone1", ZL2)], dict(services=[svc({"key": "value"})]),
     [10, 10, 10, 10, 10, 10]),
    ("two pods, 0 matching", pod(labels=ZL1), [pod("machine1.zone1", ZL2), pod("machine1.zone2", ZL2)],
     dict(services=[svc(ZL1)]), [10, 10, 10, 10, 10, 10]),
    ("two pods, 1 matching (in z2)", pod(labels=ZL1), [pod("machine1.zone1", ZL2), pod("machine1.zone2", ZL1)],
     dict(services=[svc(ZL1)]), [10, 0, 3, 10, 10, 10]),
    ("five pods, 3 matching (z2=2, z3=1)", pod(labels=ZL1),
     [pod("machine1.zone1", ZL2), pod("machine1.zone2", ZL1), pod("machine2.zone2", ZL1), pod("machine1.zone3", ZL2),
      pod("machine2.zone3", ZL1)], dict(services=[svc(ZL1)]), [10, 0, 0, 6, 3, 6]),
    ("four pods, 3 matching (z1=1, z2=1, z3=1)", pod(labels=ZL1),
     [pod("machine1.zone1", ZL1), pod("machine1.zone2", ZL1), pod("machine2.zone2", ZL2), pod("machine1.zone3", ZL1)],
     dict(services=[svc(ZL1)]), [0, 0, 3, 0, 3, 3]),
    ("four pods, 3 matching (z1=1, z2=1, z3=1) reordered", pod(labels=ZL1),
     [pod("machine1.zone1", ZL1), pod("machine1.zone2", ZL1), pod("machine1.zone3", ZL1), pod("machine2.zone2", ZL2)],
     dict(services=[svc(ZL1)]), [0, 0, 3, 0, 3, 3]),
    ("Replication controller spreading (z1=0, z2=1, z3=2)", pod(labels=ZL1),
     [pod("machine1.zone3", ZL1), pod("machine1.zone2", ZL1), pod("machine1.zone3", ZL1)],
     dict(rcs=[rc(ZL1)]), [10, 5, 6, 0, 3, 3]),
]


@pytest.mark.parametrize("name,the_pod,pods,listers,expected", ZONE_SPREAD, ids=[c[0] for c in ZONE_SPREAD])
def test_zone_selector_spread_priority_table(name, the_pod, pods, listers, expected):
    got = run_spread(the_pod, pods, ZNODES, **listers)
    assert [got[n] for n in ZORDER] == expected, name


# selector_spreading_test.go TestZoneSpreadPriority (:558-757): ServiceAntiAffinity on label "zone"
SNODES = {"machine01": {"name": "value"}, "machine02": {"name": "value"}, "machine11": {"zone": "zone1"},
          "machine12": {"zone": "zone1"}, "machine21": {"zone": "zone2"}, "machine22": {"zone": "zone2"}}
SORDER = ["machine11", "machine12", "machine21", "machine22", "machine01", "machine02"]
SAA = [
    ("nothing scheduled", pod(), [], [], [10, 10, 10, 10, 0, 0]),
    ("no services", pod(labels=L1), [pod("machine11")], [], [10, 10, 10, 10, 0, 0]),
    ("different services", pod(labels=L1), [pod("machine11", L2)], [svc({"key": "value"})], [10, 10, 10, 10, 0, 0]),
    ("three pods, one service pod", pod(labels=L1), [pod("machine01", L2), pod("machine11", L2), pod("machine21", L1)],
     [svc(L1)], [10, 10, 0, 0, 0, 0]),
    ("three pods, two service pods on different machines", pod(labels=L1),
     [pod("machine11", L2), pod("machine11", L1), pod("machine21", L1)], [svc(L1)], [5, 5, 5, 5, 0, 0]),
    ("three service label match pods in different namespaces", pod(labels=L1, ns="default"),
     [pod("machine11", L1), pod("machine11", L1, "default"), pod("machine21", L1), pod("machine21", L1, "ns1")],
     [svc(L1, "default")], [0, 0, 10, 10, 0, 0]),
    ("four pods, three service pods", pod(labels=L1),
     [pod("machine11", L2), pod("machine11", L1), pod("machine21", L1), pod("machine21", L1)], [svc(L1)],
     [6, 6, 3, 3, 0, 0]),
    ("service with partial pod label matches", pod(labels=L1),
     [pod("machine11", L2), pod("machine11", L1), pod("machine21", L1)], [svc({"baz": "blah"})], [3, 3, 6, 6, 0, 0]),
    ("service pod on non-zoned node", pod(labels=L1),
     [pod("machine01", L1), pod("machine11", L1), pod("machine21", L1), pod("machine21", L1)], [svc(L1)],
     [7, 7, 5, 5, 0, 0]),
]


@pytest.mark.parametrize("name,the_pod,pods,services,expected", SAA, ids=[c[0] for c in SAA])
def test_service_anti_affinity_priority_table(name, the_pod, pods, services, expected):
    nis = node_infos(SNODES, pods)
    order = [nis[n] for n in SORDER]
    ctx = Context(list(nis.values()), False, services=lambda: list(services))
    # the reference's namespace matching is literal ("" != "default"); m.namespace_of is too
    got = service_anti_affinity("zone")(PodInfo(the_pod), order, ctx)
    assert [int(s) for s in got] == expected, name


MB = 1024 * 1024
NODE_40_140_2000 = [{"names": ["gcr.io/40", "gcr.io/40:v1", "gcr.io/40:v1"], "sizeBytes": 40 * MB},
                    {"names": ["gcr.io/140", "gcr.io/140:v1"], "sizeBytes": 140 * MB},
                    {"names": ["gcr.io/2000"], "sizeBytes": 2000 * MB}]
NODE_250_10 = [{"names": ["gcr.io/250"], "sizeBytes": 250 * MB},
               {"names": ["gcr.io/10", "gcr.io/10:v1"], "sizeBytes": 10 * MB}]


def image_node(name, images):
    ni = NodeInfo(name)
    ni.set_node({"metadata": {"name": name}, "status": {"images": images}})
    return ni


@pytest.mark.parametrize("images,expected", [
    (["gcr.io/40", "gcr.io/250"], [1, 3]),      # :110 prefer the larger image one
    (["gcr.io/40", "gcr.io/140"], [2, 0]),      # :126 two images on one node
    (["gcr.io/10", "gcr.io/2000"], [10, 0]),    # :142 if exceed limit, use limit
])
def test_image_locality_priority_table(images, expected):
    nodes = [image_node("machine1", NODE_40_140_2000), image_node("machine2", NODE_250_10)]
    the_pod = {"metadata": {"name": "x"}, "spec": {"containers": [{"name": f"c{i}", "image": im} for i, im in enumerate(images)]}}
    assert [int(s) for s in P.image_locality(PodInfo(the_pod), nodes)] == expected


def limits_pod(*lims):
    return {"metadata": {"name": "x"}, "spec": {"containers": [
        {"name": f"c{i}", "resources": {"limits": {"cpu": c, "memory": mm}}} for i, (c, mm) in enumerate(lims)]}}


def alloc_node(name, milli, mem):
    ni = NodeInfo(name)
    ni.set_node({"metadata": {"name": name}, "status": {"allocatable": {"cpu": f"{milli}m", "memory": str(mem)}}})
    return ni


@pytest.mark.parametrize("the_pod,nodes,expected", [
    ({"metadata": {"name": "x"}, "spec": {"containers": []}},
     [("machine1", 4000, 10000), ("machine2", 4000, 0), ("machine3", 0, 10000), ("machine4", 0, 0)], [0, 0, 0, 0]),
    (limits_pod(("1000m", "0"), ("2000m", "0")), [("machine1", 3000, 10000), ("machine2", 2000, 10000)], [1, 0]),
    (limits_pod(("0", "2000"), ("0", "3000")), [("machine1", 4000, 4000), ("machine2", 5000, 10000)], [0, 1]),
    (limits_pod(("1000m", "2000"), ("2000m", "3000")), [("machine1", 4000, 4000), ("machine2", 5000, 10000)], [1, 1]),
    (limits_pod(("1000m", "2000"), ("2000m", "3000")), [("machine1", 0, 0)], [0]),
])
def test_resource_limits_priority_table(the_pod, nodes, expected):
    nis = [alloc_node(*n) for n in nodes]
    assert [int(s) for s in P.resource_limits(PodInfo(the_pod), nis)] == expected


REGISTERED = ["SelectorSpreadPriority", "InterPodAffinityPriority", "LeastRequestedPriority", "BalancedResourceAllocation",
              "NodePreferAvoidPodsPriority", "NodeAffinityPriority", "TaintTolerationPriority", "ServiceSpreadingPriority",
              "EqualPriority", "ImageLocalityPriority", "MostRequestedPriority", "ResourceLimitsPriority"]


def test_policy_naming_every_registered_priority_loads():
    """defaults.go:91-115,217-260: every name the reference registers is accepted by the policy
    loader; ResourceLimitsPriority needs its gate, as in the reference."""
    from amdkube.scheduler.scheduler import Scheduler
    pol = {"kind": "Policy", "apiVersion": "v1", "priorities": [{"name": n, "weight": 1} for n in REGISTERED]}
    _preds, prios, _cp, _cr = build(pol)
    assert set(prios) == set(REGISTERED)

    class _C:
        async def close(self):
            pass
    s = Scheduler(_C(), policy=pol, feature_gates="ResourceLimitsPriorityFunction=true")
    assert {n for n, _f, _w in s.algo.priorities} == set(REGISTERED)
    with pytest.raises(ValueError, match="ResourceLimitsPriorityFunction"):
        Scheduler(_C(), policy=pol)
    pol2 = {"priorities": [{"name": n, "weight": 1} for n in REGISTERED if n != "ResourceLimitsPriority"]}
    s2 = Scheduler(_C(), policy=pol2)
    assert "EqualPriority" in {n for n, _f, _w in s2.algo.priorities}


def _rs_pod(name, rs_labels):
    return {"metadata": {"name": name, "namespace": "default", "labels": dict(rs_labels), "uid": name},
            "spec": {"containers": [{"name": "c", "image": "busybox",
                                     "resources": {"requests": {"cpu": "100m", "memory": "64Mi"}}}]}}


async def test_replicaset_spreads_across_zones_2_1():
    """3 replicas of a ReplicaSet over 2 zones x 2 nodes land 2/1 by zone, never 3/0, and never
    two on one node. Zone a's nodes are 8x larger, so LeastRequestedPriority alone would keep
    choosing zone a: only the selector spreading (with its 2/3 zone weight) moves a replica."""
    cache = SchedulerCache()
    for z in ("a", "b"):
        for i in range(2):
            name = f"n-{z}{i}"
            big = z == "a"
            cache.add_node({"metadata": {"name": name, "labels": {ZONE: z}},
                            "status": {"allocatable": {"cpu": "64" if big else "8", "memory": "256Gi" if big else "32Gi",
                                                       "pods": "110"},
                                       "conditions": [{"type": "Ready", "status": "True"}]}})
    labels = {"app": "web"}
    the_rs = {"metadata": {"name": "web", "namespace": "default"}, "spec": {"selector": {"matchLabels": labels}}}
    listers = ControllerListers(rss=lambda: [the_rs])
    from amdkube.scheduler.predicates import DEFAULT_PREDICATES
    from amdkube.scheduler.priorities import DEFAULT_PRIORITIES
    g = GenericScheduler(cache, list(DEFAULT_PREDICATES), dict(DEFAULT_PRIORITIES), listers=listers)
    placed = []
    for i in range(3):
        p = _rs_pod(f"web-{i}", labels)
        host, _ = await g.schedule(p)
        p["spec"]["nodeName"] = host
        cache.add_pod(p)
        placed.append(host)
    zones = sorted(sum(1 for h in placed if h.startswith(f"n-{z}")) for z in ("a", "b"))
    assert zones == [1, 2], placed
    assert len(set(placed)) == 3, placed


async def test_fit_index_separates_image_classes():
    """Two pods identical but for their image must not share the fit index's cached node-local
    scores while ImageLocalityPriority is on."""
    cache = SchedulerCache()
    for name, images in (("big-a", [{"names": ["img/a"], "sizeBytes": 900 * MB}]),
                         ("big-b", [{"names": ["img/b"], "sizeBytes": 900 * MB}])):
        cache.add_node({"metadata": {"name": name},
                        "status": {"allocatable": {"cpu": "8", "memory": "32Gi", "pods": "110"}, "images": images,
                                   "conditions": [{"type": "Ready", "status": "True"}]}})
    from amdkube.scheduler.predicates import DEFAULT_PREDICATES
    g = GenericScheduler(cache, list(DEFAULT_PREDICATES), {"ImageLocalityPriority": 1})
    for img, want in (("img/a", "big-a"), ("img/b", "big-b"), ("img/a", "big-a"), ("img/b", "big-b")):
        p = {"metadata": {"name": "p", "namespace": "default"}, "spec": {"containers": [{"name": "c", "image": img}]}}
        host, _ = await g.schedule(p)
        assert host == want, (img, host)
