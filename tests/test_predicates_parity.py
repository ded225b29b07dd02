"""Scheduler predicates held to the reference's own test tables.

The tables of plugin/pkg/scheduler/algorithm/predicates/predicates_test.go are extracted by
hack/extract_predicates_cases.py into tests/fixtures/predicates_cases.json (no case retyped by
hand) and replayed here against amdkube.scheduler.predicates with each reference test's
harness: the node it builds (`node := v1.Node{...}` / SetNode), the NodeInfo of the case's pods,
the listers (FakePodLister / FakeServiceLister / FakeNodeInfo) as a scheduler Context, and the
exact failure reasons the test compares (error.go: a predicate's reason is its name).
"""
from __future__ import annotations

import json
import os

import pytest

from amdkube.scheduler import predicates as P
from amdkube.scheduler.cache import NodeInfo
from amdkube.scheduler.generic import Context
from amdkube.scheduler.policy_args import labels_presence, service_affinity
from amdkube.scheduler.predicates import PodInfo

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "predicates_cases.json")))


def cases(key):
    return [pytest.param(c, id=f"L{FIX[key]['line']}-{i}-{(c.get('test') or c.get('name') or '')[:60]}")
            for i, c in enumerate(FIX[key]["cases"])]


def pod(p):
    p = json.loads(json.dumps(p or {}))
    p.setdefault("metadata", {})
    p.setdefault("spec", {})
    return p


def node_info(pods=(), node=None, name=None):
    """schedulercache.NewNodeInfo(pods...) + SetNode(node)."""
    node = node if node is not None else None
    ni = NodeInfo(name or ((node or {}).get("metadata") or {}).get("name") or "")
    if node is not None:
        ni.set_node(node)
    for i, p in enumerate(pods):
        p = pod(p)
        p["metadata"].setdefault("name", f"p{i}")
        ni.add_pod(f"{p['metadata'].get('namespace', '')}/{p['metadata']['name']}/{i}", p)
    return ni


def from_case_node_info(c, node):
    return node_info((c.get("nodeInfo") or {}).get("nodeInfoPods") or [], node)


RES_NODE = {"status": {"allocatable": {"cpu": "10m", "memory": "20", "pods": "32", "alpha.kubernetes.io/nvidia-gpu": "0",
                                       "example.com/aaa": "5", "ephemeral-storage": "20", "hugepages-2Mi": "5"}}}
ONE_POD_NODE = {"status": {"allocatable": {"cpu": "10m", "memory": "20", "pods": "1", "alpha.kubernetes.io/nvidia-gpu": "0",
                                           "example.com/aaa": "0", "ephemeral-storage": "0", "hugepages-2Mi": "0"}}}


# ------------------------------------------------------------------ TestPodFitsResources
@pytest.mark.parametrize("c", cases("PodFitsResources/enough") + cases("PodFitsResources/storage"))
def test_pod_fits_resources(c):
    ni = from_case_node_info(c, RES_NODE)
    fits, reasons = P.pod_fits_resources(PodInfo(pod(c["pod"])), ni)
    assert fits == c["fits"], reasons
    if not fits:
        assert reasons == c["reasons"]


@pytest.mark.parametrize("c", cases("PodFitsResources/notEnoughPods"))
def test_pod_fits_resources_pod_count(c):
    ni = from_case_node_info(c, ONE_POD_NODE)
    fits, reasons = P.pod_fits_resources(PodInfo(pod(c["pod"])), ni)
    assert fits == c["fits"] and reasons == c["reasons"]


# ------------------------------------------------------------------ host / ports / disks
@pytest.mark.parametrize("c", cases("PodFitsHost"))
def test_pod_fits_host(c):
    fits, reasons = P.pod_fits_host(PodInfo(pod(c["pod"])), node_info(node=c["node"]))
    assert fits == c["fits"]
    assert fits or reasons == ["HostName"]


@pytest.mark.parametrize("c", cases("PodFitsHostPorts"))
def test_pod_fits_host_ports(c):
    fits, reasons = P.pod_fits_host_ports(PodInfo(pod(c["pod"])), from_case_node_info(c, None))
    assert fits == c["fits"]
    assert fits or reasons == ["PodFitsHostPorts"]


@pytest.mark.parametrize("c", cases("GetUsedPorts"))
def test_get_used_ports(c):
    from amdkube.api.helpers import pod_host_ports
    used = {f"{proto}/{ip}/{port}" for p in c["pods"] for ip, proto, port in pod_host_ports(pod(p))}
    assert used == set(c["ports"])


@pytest.mark.parametrize("c", cases("DiskConflicts/GCE") + cases("DiskConflicts/AWS") + cases("DiskConflicts/RBD")
                         + cases("DiskConflicts/ISCSI"))
def test_no_disk_conflict(c):
    ok, reasons = P.no_disk_conflict(PodInfo(pod(c["pod"])), from_case_node_info(c, None))
    assert ok == c["isOk"]
    assert ok or reasons == ["NoDiskConflict"]


# ------------------------------------------------------------------ selectors / labels
@pytest.mark.parametrize("c", cases("PodFitsSelector"))
def test_pod_match_node_selector(c):
    ni = node_info(node={"metadata": {"labels": c.get("labels") or {}}})
    fits, reasons = P.pod_match_node_selector(PodInfo(pod(c["pod"])), ni)
    assert fits == c["fits"]
    assert fits or reasons == ["MatchNodeSelector"]


@pytest.mark.parametrize("c", cases("NodeLabelPresence"))
def test_node_label_presence(c):
    ni = node_info(node={"metadata": {"labels": {"foo": "bar", "bar": "foo"}}})
    fits, reasons = labels_presence(c["labels"], c["presence"])(PodInfo(pod(c.get("pod"))), ni)
    assert fits == c["fits"]
    assert fits or reasons == ["CheckNodeLabelPresence"]


@pytest.mark.parametrize("c", cases("ServiceAffinity"))
def test_service_affinity(c):
    nodes = FIX["ServiceAffinity"]["locals"]
    cand = c["node"]["metadata"]["name"]
    infos = []
    for n in nodes.values():
        name = n["metadata"]["name"]
        # the candidate's NodeInfo is empty (FilterOutPods drops the pods that claim it)
        placed = [p for p in c.get("pods") or [] if p["spec"].get("nodeName") == name] if name != cand else []
        infos.append(node_info(placed, n))
    ni = next(i for i in infos if i.name == cand)
    services = [pod(s) for s in c.get("services") or []]
    ctx = Context(infos, False, services=lambda: services)
    fits, reasons = service_affinity(c["labels"])(PodInfo(pod(c["pod"])), ni, ctx)
    assert fits == c["fits"]
    assert fits or reasons == ["CheckServiceAffinity"]


# ------------------------------------------------------------------ GeneralPredicates
@pytest.mark.parametrize("c", cases("GeneralPredicates"))
def test_general_predicates(c):
    ni = from_case_node_info(c, c["node"])
    fits, reasons = P.general_predicates(PodInfo(pod(c["pod"])), ni)
    assert fits == c["fits"], reasons
    if not fits:
        assert reasons == c["reasons"]


# ------------------------------------------------------------------ inter-pod affinity
def _affinity_ctx(c, candidate, lookup):
    """The harness's listers as a Context: every pod of the case on the NodeInfo of the node
    the test's NodeInfo lister resolves its nodeName to (FakeNodeInfo answers the candidate for
    any name; FakeNodeListInfo looks the name up); the candidate holds only its own pods."""
    infos = {}
    cand = node_info([p for p in c.get("pods") or [] if p["spec"].get("nodeName") == candidate["metadata"].get("name")],
                     candidate)
    for p in c.get("pods") or []:
        name = p["spec"].get("nodeName") or ""
        if name == candidate["metadata"].get("name"):
            continue
        n = lookup(name)
        if n is None:
            continue
        ni = infos.setdefault(name, node_info(node={**n, "metadata": {**n["metadata"], "name": name}}))
        q = pod(p)
        q["metadata"].setdefault("name", f"x{len(ni.pods)}")
        ni.add_pod(f"{name}/{len(ni.pods)}", q)
    all_infos = [cand] + list(infos.values())
    any_anti = any((((p.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity")) for p in c.get("pods") or [])
    return cand, Context(all_infos, any_anti)


@pytest.mark.parametrize("c", cases("InterPodAffinity"))
def test_inter_pod_affinity(c):
    node = c["node"]
    cand, ctx = _affinity_ctx(c, node, lambda name: node)
    fits, reasons = P.match_inter_pod_affinity(PodInfo(pod(c["pod"])), cand, ctx)
    assert fits == c["fits"], reasons
    if not fits:
        assert reasons == c["expectFailureReasons"]


@pytest.mark.parametrize("c", cases("InterPodAffinityWithMultipleNodes"))
def test_inter_pod_affinity_multiple_nodes(c):
    by_name = {n["metadata"]["name"]: n for n in c["nodes"]}
    pi = PodInfo(pod(c["pod"]))
    for i, node in enumerate(c["nodes"]):
        cand, ctx = _affinity_ctx(c, node, by_name.get)
        fits, reasons = P.match_inter_pod_affinity(pi, cand, ctx)
        if not fits:
            assert reasons == c["nodesExpectAffinityFailureReasons"][i], node["metadata"]["name"]
        if ((c["pod"].get("spec") or {}).get("affinity") or {}).get("nodeAffinity"):
            fits2, r2 = P.pod_match_node_selector(pi, node_info(node=node))
            assert fits2 or r2 == ["MatchNodeSelector"]
            fits = fits and fits2
        assert fits == c["fits"][node["metadata"]["name"]], (node["metadata"]["name"], reasons)


# ------------------------------------------------------------------ taints / node conditions
@pytest.mark.parametrize("c", cases("PodToleratesTaints"))
def test_pod_tolerates_taints(c):
    fits, reasons = P.pod_tolerates_node_taints(PodInfo(pod(c["pod"])), node_info(node=c["node"]))
    assert fits == c["fits"]
    assert fits or reasons == ["PodToleratesNodeTaints"]


@pytest.mark.parametrize("c", cases("MemoryPressure"))
def test_memory_pressure(c):
    ni = node_info(node=c["nodeInfo"]["node"])
    fits, reasons = P.check_node_memory_pressure(PodInfo(pod(c["pod"])), ni)
    assert fits == c["fits"]
    assert fits or reasons == ["NodeUnderMemoryPressure"]


@pytest.mark.parametrize("c", cases("DiskPressure"))
def test_disk_pressure(c):
    ni = node_info(node=c["nodeInfo"]["node"])
    fits, reasons = P.check_node_disk_pressure(PodInfo(pod(c["pod"])), ni)
    assert fits == c["fits"]
    assert fits or reasons == ["NodeUnderDiskPressure"]


@pytest.mark.parametrize("c", cases("NodeCondition"))
def test_node_condition(c):
    fits, reasons = P.check_node_condition(PodInfo(pod({})), node_info(node=c["node"]))
    assert fits == c["schedulable"], reasons


def test_fit_error_message_is_a_sorted_histogram():
    """FitError.Error: "<n> <reason>" strings sorted as strings, every reason counted."""
    from amdkube.scheduler.generic import FitError
    e = FitError({}, 3, {"a": ["Insufficient cpu"], "b": ["MatchNodeSelector"], "c": ["MatchNodeSelector",
                                                                                  "PodToleratesNodeTaints"]})
    assert str(e) == "0/3 nodes are available: 1 Insufficient cpu, 1 PodToleratesNodeTaints, 2 MatchNodeSelector."


# ------------------------------------------------------------------ volume predicates
def _lister(key):
    from amdkube.scheduler.volumes import VolumeLister
    loc = FIX[key]["locals"]
    pvcs = {f"{(c['metadata'].get('namespace') or '')}/{c['metadata']['name']}": c for c in loc["pvcInfo"]}
    pvs = {v["metadata"]["name"]: v for v in loc["pvInfo"]}
    classes = {c["metadata"]["name"]: c for c in loc.get("classInfo") or []}
    return VolumeLister(pvcs, pvs, classes)


def _vol_pod_info(p, lister):
    from amdkube.scheduler.volumes import pod_volumes
    pi = PodInfo(pod(p))
    pi.lister, pi.volume_scheduling, pi.vol = lister, True, pod_volumes(pi.pod, lister)
    return pi


@pytest.mark.parametrize("c", cases("EBSVolumeCount"))
def test_max_ebs_volume_count(c, monkeypatch):
    monkeypatch.setenv("KUBE_MAX_PD_VOLS", str(c["maxVols"]))
    lister = _lister("EBSVolumeCount")
    ni = node_info(c.get("existingPods") or [])
    fits, reasons = P.PREDICATES["MaxEBSVolumeCount"](_vol_pod_info(c["newPod"], lister), ni)
    assert fits == c["fits"]
    assert fits or reasons == ["MaxVolumeCount"]


@pytest.mark.parametrize("c", cases("VolumeZone") + cases("VolumeZoneMultiZone"))
def test_volume_zone(c):
    key = "VolumeZone" if c in FIX["VolumeZone"]["cases"] else "VolumeZoneMultiZone"
    fits, reasons = P.no_volume_zone_conflict(_vol_pod_info(c["pod"], _lister(key)), node_info(node=c["node"]))
    assert fits == c["fits"], reasons
    assert fits or reasons == ["NoVolumeZoneConflict"]


@pytest.mark.parametrize("c", cases("VolumeZoneWithBinding"))
def test_volume_zone_with_volume_binding(c):
    """An unbound claim without a WaitForFirstConsumer class is an error in the reference; here
    it is a failure reason naming the claim."""
    lister = _lister("VolumeZoneWithBinding")
    for cls in lister._classes.values():      # the apiserver defaults volumeBindingMode
        cls.setdefault("volumeBindingMode", "Immediate")
    fits, reasons = P.no_volume_zone_conflict(_vol_pod_info(c["pod"], lister), node_info(node=c["node"]))
    assert fits == c["fits"], reasons
    if c.get("expectFailure"):
        assert reasons and "PersistentVolumeClaim" in reasons[0]


@pytest.mark.parametrize("c", cases("GetMaxVols"))
def test_get_max_vols(c, monkeypatch):
    from amdkube.scheduler.volumes import max_pd_limit
    monkeypatch.setenv("KUBE_MAX_PD_VOLS", c["rawMaxVols"])
    assert max_pd_limit("awsElasticBlockStore") == c["expected"]


# ------------------------------------------------------------------ utils_test.go (ports)
def _decode(s):
    """decode(): "PROTO/IP/PORT" -> amdkube's (ip, proto, port) host-port tuple."""
    proto, ip, port = s.split("/")
    return ip, proto, int(port)


@pytest.mark.parametrize("s,want", [("UDP/127.0.0.1/80", ("127.0.0.1", "UDP", 80)),
                                    ("TCP/127.0.0.1/80", ("127.0.0.1", "TCP", 80)),
                                    ("TCP/0.0.0.0/80", ("0.0.0.0", "TCP", 80))])
def test_decode_host_port(s, want):
    from amdkube.api.helpers import pod_host_ports
    proto, ip, port = s.split("/")
    p = {"spec": {"containers": [{"ports": [{"protocol": proto, "hostIP": ip, "hostPort": int(port), "containerPort": 1}]}]}}
    assert [tuple(x) for x in pod_host_ports(p)] == [want] == [_decode(s)]


@pytest.mark.parametrize("special,others,want", [
    ("TCP/0.0.0.0/80", ["TCP/127.0.0.2/8080", "TCP/127.0.0.1/80", "UDP/127.0.0.2/8080"], True),
    ("TCP/0.0.0.0/80", ["TCP/127.0.0.2/8080", "UDP/127.0.0.1/80", "UDP/127.0.0.2/8080"], False),
    ("TCP/0.0.0.0/80", ["TCP/127.0.0.2/8080", "TCP/127.0.0.1/8090", "UDP/127.0.0.2/8080"], False),
    ("TCP/0.0.0.0/80", ["UDP/127.0.0.2/8080", "UDP/127.0.0.1/8090", "TCP/127.0.0.2/8080"], False),
], ids=["test-1", "test-2", "test-3", "test-4"])
def test_special_port_conflict_check(special, others, want):
    assert P.ports_conflict({_decode(o) for o in others}, {_decode(special)}) == want


@pytest.mark.parametrize("existing,wanted,want", [
    ("UDP/127.0.0.1/8080", "UDP/127.0.0.1/8080", True), ("UDP/127.0.0.2/8080", "UDP/127.0.0.1/8080", False),
    ("TCP/127.0.0.1/8080", "UDP/127.0.0.1/8080", False), ("TCP/0.0.0.0/8080", "TCP/127.0.0.1/8080", True),
    ("TCP/127.0.0.1/8080", "TCP/0.0.0.0/8080", True),
], ids=["test1", "test2", "test3", "test4", "test5"])
def test_ports_conflict(existing, wanted, want):
    assert P.ports_conflict({_decode(existing)}, {_decode(wanted)}) == want
