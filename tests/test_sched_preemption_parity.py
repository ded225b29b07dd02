"""Scheduler preemption and queue parity, transcribed from the reference's tables:

* plugin/pkg/scheduler/core/generic_scheduler_test.go — TestSelectNodesForPreemption (:666),
  TestPickOneNodeForPreemption (:804), TestNodesWherePreemptionMightHelp (:965), TestPreempt
  (:1083, including the second Preempt call that must not preempt again while the victims
  terminate), with makeNode (:391) and the small/medium/large/veryLarge containers (:614-660);
* plugin/pkg/scheduler/core/scheduling_queue_test.go — TestPriorityQueue_Add, _AddIfNotPresent,
  _AddUnschedulableIfNotPresent, _Pop, _Update, _Delete, _MoveAllToActiveQueue,
  _AssignedPodAdded, _WaitingPodsForNode;
* PDB-aware victim choice (filterPodsWithPDBViolation :889, selectVictimsOnNode :872) and
  nominated pods taking their GPUs before lower-priority pods (addNominatedPods :367).
"""
import asyncio

import pytest

from amdkube.scheduler import generic as G
from amdkube.scheduler.cache import SchedulerCache
from amdkube.scheduler.generic import FitError, GenericScheduler
from amdkube.scheduler.predicates import (ERR_DISK_CONFLICT, ERR_NODE_LABEL_PRESENCE_VIOLATED, ERR_NODE_OUT_OF_DISK,
                                          ERR_NODE_SELECTOR_NOT_MATCH, ERR_NODE_UNSCHEDULABLE, ERR_POD_AFFINITY_NOT_MATCH,
                                          ERR_POD_NOT_MATCH_HOST_NAME, ERR_TAINTS_TOLERATIONS_NOT_MATCH)
from amdkube.scheduler.queue import NOMINATED_NODE_ANNOTATION, SchedulingQueue
from tests.test_scheduler import node as gpu_node, pod as gpu_pod

CPU, MEM = 100, 200 * 1024 * 1024          # priorityutil.DefaultMilliCpuRequest / DefaultMemoryRequest
NEG, LOW, MID, HIGH, VHIGH = -100, 0, 100, 1000, 10000


def containers(mult):
    return [{"name": "c", "image": "x", "resources": {"requests": {"cpu": f"{CPU * mult}m", "memory": str(MEM * mult)}}}]


SMALL, MEDIUM, LARGE, VLARGE = containers(1), containers(2), containers(3), containers(5)


def make_node(name, milli_cpu=CPU * 5, memory=MEM * 5, labels=None):
    res = {"cpu": f"{milli_cpu}m", "memory": str(memory), "pods": "100"}
    return {"metadata": {"name": name, "labels": labels or {}},
            "status": {"capacity": dict(res), "allocatable": dict(res), "conditions": [{"type": "Ready", "status": "True"}]}}


def pod(name, prio=None, node=None, cont=None, labels=None, affinity=None, deleting=False, ann=None, ns="default"):
    spec = {"containers": cont or [{"name": "c", "image": "x"}]}
    if prio is not None:
        spec["priority"] = prio
    if node:
        spec["nodeName"] = node
    if affinity:
        spec["affinity"] = affinity
    md = {"name": name, "namespace": ns, "uid": name, "labels": labels or {}}
    if deleting:
        md["deletionTimestamp"] = "2018-01-01T00:00:00Z"
    if ann:
        md["annotations"] = ann
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec, "status": {"phase": "Running"}}


def true_pred(pi, ni, ctx=None):
    return True, []


def false_pred(pi, ni, ctx=None):
    return False, ["FakePredicateError"]


def matches_pred(pi, ni, ctx=None):
    return (pi.pod["metadata"]["name"] == ni.name), ([] if pi.pod["metadata"]["name"] == ni.name else ["FakePredicateError"])


def build(nodes, pods, pred="PodFitsResources", affinity=False, queue=None):
    c = SchedulerCache()
    for n in nodes:
        c.add_node(n)
    for p in pods:
        c.add_pod(p)
    custom = {}
    preds = [pred]
    if callable(pred):
        custom = {"matches": pred}
        preds = ["matches"]
    if affinity:
        preds.append("MatchInterPodAffinity")
    g = GenericScheduler(c, preds, {}, custom_predicates=custom)
    g.queue = queue
    return c, g


ANTI = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
    {"labelSelector": {"matchExpressions": [{"key": "pod", "operator": "In", "values": ["preemptor", "value2"]}]},
     "topologyKey": "hostname"}]}}

SELECT_CASES = [
    ("a pod that does not fit on any machine", false_pred, pod("new", HIGH),
     [pod("a", MID, "machine1"), pod("b", MID, "machine2")], {}, False),
    ("a pod that fits with no preemption", true_pred, pod("new", HIGH),
     [pod("a", MID, "machine1"), pod("b", MID, "machine2")], {"machine1": set(), "machine2": set()}, False),
    ("a pod that fits on one machine with no preemption", matches_pred, pod("machine1", HIGH),
     [pod("a", MID, "machine1"), pod("b", MID, "machine2")], {"machine1": set()}, False),
    ("a pod that fits on both machines when lower priority pods are preempted", "PodFitsResources",
     pod("machine1", HIGH, cont=LARGE), [pod("a", MID, "machine1", LARGE), pod("b", MID, "machine2", LARGE)],
     {"machine1": {"a"}, "machine2": {"b"}}, False),
    ("a pod that would fit on the machines, but other pods running are higher priority", "PodFitsResources",
     pod("machine1", LOW, cont=LARGE), [pod("a", MID, "machine1", LARGE), pod("b", MID, "machine2", LARGE)], {}, False),
    ("medium priority pod is preempted, but lower priority one stays as it is small", "PodFitsResources",
     pod("machine1", HIGH, cont=LARGE),
     [pod("a", LOW, "machine1", SMALL), pod("b", MID, "machine1", LARGE), pod("c", MID, "machine2", LARGE)],
     {"machine1": {"b"}, "machine2": {"c"}}, False),
    ("mixed priority pods are preempted", "PodFitsResources", pod("machine1", HIGH, cont=LARGE),
     [pod("a", MID, "machine1", SMALL), pod("b", LOW, "machine1", SMALL), pod("c", MID, "machine1", MEDIUM),
      pod("d", HIGH, "machine1", SMALL), pod("e", HIGH, "machine2", LARGE)], {"machine1": {"b", "c"}}, False),
    ("pod with anti-affinity is preempted", "PodFitsResources",
     pod("machine1", HIGH, cont=SMALL, labels={"pod": "preemptor"}),
     [pod("a", LOW, "machine1", SMALL, labels={"service": "securityscan"}, affinity=ANTI),
      pod("b", MID, "machine1", SMALL), pod("d", HIGH, "machine1", SMALL), pod("e", HIGH, "machine2", LARGE)],
     {"machine1": {"a"}, "machine2": set()}, True),
]


@pytest.mark.parametrize("name,pred,p,pods,expected,aff", SELECT_CASES, ids=[c[0][:50] for c in SELECT_CASES])
def test_select_nodes_for_preemption(name, pred, p, pods, expected, aff):
    nodes = [make_node(n, labels={"hostname": n}) for n in ("machine1", "machine2")]
    c, g = build(nodes, pods, pred, aff)
    got = g.select_nodes_for_preemption(G.PodInfo(p), c.ready_nodes())
    assert {k: {v["metadata"]["name"] for v in vs} for k, (vs, _) in got.items()} == expected
    for vs, _ in got.values():     # victims sorted by decreasing priority
        prios = [G.pod_priority(v) for v in vs]
        assert prios == sorted(prios, reverse=True)


PICK_CASES = [
    ("No node needs preemption", ["machine1"], pod("machine1", HIGH, cont=LARGE),
     [pod("m1.1", MID, "machine1", SMALL)], ["machine1"]),
    ("a pod that fits on both machines when lower priority pods are preempted", ["machine1", "machine2"],
     pod("machine1", HIGH, cont=LARGE), [pod("m1.1", MID, "machine1", LARGE), pod("m2.1", MID, "machine2", LARGE)],
     ["machine1", "machine2"]),
    ("a pod that fits on a machine with no preemption", ["machine1", "machine2", "machine3"],
     pod("machine1", HIGH, cont=LARGE), [pod("m1.1", MID, "machine1", LARGE), pod("m2.1", MID, "machine2", LARGE)],
     ["machine3"]),
    ("machine with min highest priority pod is picked", ["machine1", "machine2", "machine3"],
     pod("machine1", HIGH, cont=VLARGE),
     [pod("m1.1", MID, "machine1", MEDIUM), pod("m1.2", MID, "machine1", LARGE),
      pod("m2.1", MID, "machine2", MEDIUM), pod("m2.2", LOW, "machine2", MEDIUM),
      pod("m3.1", LOW, "machine3", MEDIUM), pod("m3.2", LOW, "machine3", MEDIUM)], ["machine3"]),
    ("when highest priorities are the same, minimum sum of priorities is picked", ["machine1", "machine2", "machine3"],
     pod("machine1", HIGH, cont=VLARGE),
     [pod("m1.1", MID, "machine1", MEDIUM), pod("m1.2", MID, "machine1", LARGE),
      pod("m2.1", MID, "machine2", LARGE), pod("m2.2", LOW, "machine2", MEDIUM),
      pod("m3.1", MID, "machine3", MEDIUM), pod("m3.2", MID, "machine3", MEDIUM)], ["machine2"]),
    ("when highest priority and sum are the same, minimum number of pods is picked", ["machine1", "machine2", "machine3"],
     pod("machine1", HIGH, cont=VLARGE),
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", NEG, "machine1", SMALL), pod("m1.3", MID, "machine1", SMALL),
      pod("m1.4", NEG, "machine1", SMALL), pod("m2.1", MID, "machine2", LARGE), pod("m2.2", NEG, "machine2", MEDIUM),
      pod("m3.1", MID, "machine3", MEDIUM), pod("m3.2", NEG, "machine3", SMALL), pod("m3.3", LOW, "machine3", SMALL)],
     ["machine2"]),
    ("sum of adjusted priorities is considered", ["machine1", "machine2", "machine3"], pod("machine1", HIGH, cont=VLARGE),
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", NEG, "machine1", SMALL), pod("m1.3", NEG, "machine1", SMALL),
      pod("m2.1", MID, "machine2", LARGE), pod("m2.2", NEG, "machine2", MEDIUM),
      pod("m3.1", MID, "machine3", MEDIUM), pod("m3.2", NEG, "machine3", SMALL), pod("m3.3", LOW, "machine3", SMALL)],
     ["machine2"]),
    ("non-overlapping lowest high priority, sum priorities, and number of pods",
     ["machine1", "machine2", "machine3", "machine4"], pod("pod1", VHIGH, cont=VLARGE),
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL), pod("m1.3", LOW, "machine1", SMALL),
      pod("m2.1", HIGH, "machine2", LARGE),
      pod("m3.1", MID, "machine3", MEDIUM), pod("m3.2", LOW, "machine3", SMALL), pod("m3.3", LOW, "machine3", SMALL),
      pod("m3.4", LOW, "machine3", MEDIUM),
      pod("m4.1", MID, "machine4", MEDIUM), pod("m4.2", MID, "machine4", SMALL), pod("m4.3", MID, "machine4", SMALL),
      pod("m4.4", NEG, "machine4", SMALL)], ["machine1"]),
]


@pytest.mark.parametrize("name,nodes,p,pods,expected", PICK_CASES, ids=[c[0][:50] for c in PICK_CASES])
def test_pick_one_node_for_preemption(name, nodes, p, pods, expected):
    c, g = build([make_node(n) for n in nodes], pods)
    cand = g.select_nodes_for_preemption(G.PodInfo(p), c.ready_nodes())
    assert G.pick_one_node_for_preemption(cand) in expected


NODES4 = [f"machine{i}" for i in range(1, 5)]
HELP_CASES = [
    ("No node should be attempted", {"machine1": [ERR_NODE_SELECTOR_NOT_MATCH], "machine2": [ERR_POD_NOT_MATCH_HOST_NAME],
                                     "machine3": [ERR_TAINTS_TOLERATIONS_NOT_MATCH],
                                     "machine4": [ERR_NODE_LABEL_PRESENCE_VIOLATED]}, set()),
    ("pod affinity should be tried", {"machine1": [ERR_POD_AFFINITY_NOT_MATCH], "machine2": [ERR_POD_NOT_MATCH_HOST_NAME],
                                      "machine3": [ERR_NODE_UNSCHEDULABLE]}, {"machine1", "machine4"}),
    ("pod with both pod affinity and anti-affinity should be tried",
     {"machine1": [ERR_POD_AFFINITY_NOT_MATCH], "machine2": [ERR_POD_NOT_MATCH_HOST_NAME]},
     {"machine1", "machine3", "machine4"}),
    ("Mix of failed predicates works fine",
     {"machine1": [ERR_NODE_SELECTOR_NOT_MATCH, ERR_NODE_OUT_OF_DISK, "Insufficient memory"],
      "machine2": [ERR_POD_NOT_MATCH_HOST_NAME, ERR_DISK_CONFLICT], "machine3": ["Insufficient memory"], "machine4": []},
     {"machine3", "machine4"}),
]


@pytest.mark.parametrize("name,failed,expected", HELP_CASES, ids=[c[0] for c in HELP_CASES])
def test_nodes_where_preemption_might_help(name, failed, expected):
    assert set(G.nodes_where_preemption_might_help(NODES4, failed)) == expected


class FakeExtender:
    filter_verb, prioritize_verb, bind_verb = "filter", None, None

    def __init__(self, allow):
        self.allow = allow

    async def filter(self, pod, nodes):
        ok = [n["metadata"]["name"] for n in nodes if self.allow(n["metadata"]["name"])]
        return ok, {n["metadata"]["name"]: "fake" for n in nodes if not self.allow(n["metadata"]["name"])}


PREEMPT_FAILED = {"machine1": ["Insufficient memory"], "machine2": [ERR_DISK_CONFLICT], "machine3": ["Insufficient memory"]}
PREEMPT_CASES = [
    ("basic preemption logic", [pod("m1.1", LOW, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL),
                                pod("m2.1", HIGH, "machine2", LARGE), pod("m3.1", MID, "machine3", MEDIUM)],
     [], "machine1", {"m1.1", "m1.2"}),
    ("One node doesn't need any preemption", [pod("m1.1", LOW, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL),
                                              pod("m2.1", HIGH, "machine2", LARGE)], [], "machine3", set()),
    ("Scheduler extenders allow only machine1, otherwise machine3 would have been chosen",
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL), pod("m2.1", MID, "machine2", LARGE)],
     [FakeExtender(lambda n: True), FakeExtender(lambda n: n == "machine1")], "machine1", {"m1.1", "m1.2"}),
    ("Scheduler extenders do not allow any preemption",
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL), pod("m2.1", MID, "machine2", LARGE)],
     [FakeExtender(lambda n: False)], None, set()),
]


@pytest.mark.parametrize("name,pods,exts,exp_node,exp_victims", PREEMPT_CASES, ids=[c[0][:50] for c in PREEMPT_CASES])
async def test_preempt(name, pods, exts, exp_node, exp_victims):
    c, g = build([make_node(f"machine{i}") for i in (1, 2, 3)], pods, queue=SchedulingQueue())
    g.extenders = exts
    preemptor = pod("pod1", HIGH, cont=VLARGE)
    node, victims, _ = await g.preempt_async(preemptor, PREEMPT_FAILED)
    assert node == exp_node and {v["metadata"]["name"] for v in victims} == exp_victims
    # mark the victims terminating and nominate the preemptor: no further preemption
    for v in victims:
        c.remove_pod(v)
        v = dict(v, metadata=dict(v["metadata"], deletionTimestamp="2018-01-01T00:00:00Z"))
        c.add_pod(v)
        preemptor["metadata"]["annotations"] = {NOMINATED_NODE_ANNOTATION: node}
    node2, victims2, _ = await g.preempt_async(preemptor, PREEMPT_FAILED)
    assert not (node2 and victims2)


async def test_preempt_clears_own_nomination_when_nothing_can_help():
    c, g = build([make_node("machine1")], [pod("a", LOW, "machine1", LARGE)], queue=SchedulingQueue())
    p = pod("p", HIGH, cont=LARGE, ann={NOMINATED_NODE_ANNOTATION: "machine1"})
    node, victims, clear = await g.preempt_async(p, {"machine1": [ERR_NODE_SELECTOR_NOT_MATCH]})
    assert node is None and victims == [] and clear == [p]


def test_pdb_violating_victims_are_reprieved_first_and_counted():
    """selectVictimsOnNode tries to keep PDB-protected pods; pickOneNode prefers fewer violations."""
    pdb = {"metadata": {"name": "pdb", "namespace": "default"},
           "spec": {"selector": {"matchLabels": {"app": "db"}}}, "status": {"disruptionsAllowed": 0}}
    m1 = [pod("db1", LOW, "machine1", LARGE, labels={"app": "db"}), pod("x1", LOW, "machine1", SMALL)]
    m2 = [pod("web", LOW, "machine2", LARGE), pod("x2", LOW, "machine2", SMALL)]
    c, g = build([make_node("machine1"), make_node("machine2")], m1 + m2)
    pi = G.PodInfo(pod("p", HIGH, cont=LARGE))
    cand = g.select_nodes_for_preemption(pi, c.ready_nodes(), [pdb])
    assert {v["metadata"]["name"] for v in cand["machine1"][0]} == {"db1"} and cand["machine1"][1] == 1
    assert {v["metadata"]["name"] for v in cand["machine2"][0]} == {"web"} and cand["machine2"][1] == 0
    assert G.pick_one_node_for_preemption(cand) == "machine2"
    # a PDB that still allows disruptions does not protect
    pdb["status"]["disruptionsAllowed"] = 1
    cand = g.select_nodes_for_preemption(pi, c.ready_nodes(), [pdb])
    assert cand["machine1"][1] == 0


async def test_nominated_preemptor_holds_its_gpus_against_lower_priority_pods():
    """addNominatedPods: a 1-GPU priority-0 pod must not take GPUs freed for a nominated
    priority-1000 8-GPU pod; only a higher-priority pod may."""
    q = SchedulingQueue()
    c, g = build([gpu_node("n0", gpus=8)], [], pred="PodFitsResources", queue=q)
    big = gpu_pod("big", 8, prio=1000)
    big["metadata"]["annotations"] = {NOMINATED_NODE_ANNOTATION: "n0"}
    q.add_unschedulable(big, marked=True)
    assert q.waiting_pods_for_node("n0") == [big]
    small = gpu_pod("small", 1, prio=0)
    with pytest.raises(FitError):
        await g.schedule(small)
    # so is one of equal priority (addNominatedPods counts nominees with priority >= the pod's);
    # a higher-priority pod is not held back
    with pytest.raises(FitError):
        await g.schedule(gpu_pod("peer", 1, prio=1000))
    assert (await g.schedule(gpu_pod("vip", 1, prio=1001)))[0] == "n0"
    # once the nominee is moved back and popped for scheduling, its room is its own again
    q.move_all_to_active()
    assert q.pop_nowait()["metadata"]["name"] == "big"
    assert (await g.schedule(big))[0] == "n0"


# ------------------------------------------------------------------ scheduling_queue_test.go
def qpod(name, ns, prio, nominated=None, extra=None, unschedulable=False):
    md = {"name": name, "namespace": ns, "uid": name + ns}
    ann = dict(extra or {})
    if nominated:
        ann[NOMINATED_NODE_ANNOTATION] = nominated
    if ann:
        md["annotations"] = ann
    p = {"metadata": md, "spec": {"priority": prio}}
    if unschedulable:
        p["status"] = {"conditions": [{"type": "PodScheduled", "status": "False", "reason": "Unschedulable"}]}
    return p


MEDIUM_P = (LOW + HIGH) // 2
HPP = qpod("hpp", "ns1", HIGH)
HPN = qpod("hpp", "ns1", HIGH, "node1")
MPP = qpod("mpp", "ns2", MEDIUM_P, "node1", {"annot2": "val2"})
UP = qpod("up", "ns1", LOW, "node1", {"annot2": "val2"}, unschedulable=True)


def names(pods):
    return [p["metadata"]["name"] for p in pods]


def test_queue_add():
    q = SchedulingQueue()
    for p in (MPP, UP, HPP):
        q.add(p)
    assert names(q.waiting_pods_for_node("node1")) == ["mpp", "up"]
    assert names([q.pop_nowait() for _ in range(3)]) == ["hpp", "mpp", "up"]
    assert q.nominated == {}


def test_queue_add_unschedulable_if_not_present():
    q = SchedulingQueue()
    q.add(HPN)
    q.add_unschedulable(HPN)        # already queued: nothing
    q.add_unschedulable(MPP)        # not marked unschedulable: active queue
    q.add_unschedulable(UP)         # marked: unschedulable queue
    assert names(q.waiting_pods_for_node("node1")) == ["hpp", "mpp", "up"]
    assert names([q.pop_nowait(), q.pop_nowait()]) == ["hpp", "mpp"]
    assert len(q.nominated) == 1 and "ns1/up" in q.unschedulable


async def test_queue_pop_blocks_until_add():
    q = SchedulingQueue()
    t = asyncio.ensure_future(q.pop())
    await asyncio.sleep(0)
    q.add(MPP)
    assert (await asyncio.wait_for(t, 1))["metadata"]["name"] == "mpp" and q.nominated == {}


def test_queue_update():
    q = SchedulingQueue()
    q.update(HPN, HPP)            # in no queue: added to the active queue
    assert "ns1/hpp" in q.items
    q.unschedulable["ns2/mpp"] = MPP
    q.update(MPP, MPP)            # unchanged: stays unschedulable
    assert "ns2/mpp" in q.unschedulable
    changed = qpod("mpp", "ns2", MEDIUM_P, "node1", {"annot2": "val2", "new": "x"})
    q.update(changed, MPP)        # changed metadata: may be schedulable now
    assert "ns2/mpp" in q.items and "ns2/mpp" not in q.unschedulable
    q.update(UP, UP)
    assert "ns1/up" in q.items and not q.unschedulable
    assert q.pop_nowait()["metadata"]["name"] == "hpp"


def test_queue_delete():
    q = SchedulingQueue()
    q.update(HPN, HPP)
    q.add(UP)
    q.delete(HPN)
    assert "ns1/up" in q.items and "ns1/hpp" not in q.items
    assert names(q.waiting_pods_for_node("node1")) == ["up"]
    q.delete(UP)
    assert q.nominated == {}


def test_queue_move_all_to_active():
    q = SchedulingQueue()
    q.add(MPP)
    q.unschedulable["ns1/up"] = UP
    q.unschedulable["ns1/hpp"] = HPP
    q.move_all_to_active()
    assert len(q.items) == 3 and not q.unschedulable


def test_queue_assigned_pod_added():
    aff = qpod("afp", "ns1", MEDIUM_P, unschedulable=True)
    aff["spec"]["affinity"] = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchExpressions": [{"key": "service", "operator": "In", "values": ["securityscan", "value2"]}]},
         "topologyKey": "region"}]}}
    label_pod = {"metadata": {"name": "lbp", "namespace": "ns1", "labels": {"service": "securityscan"}},
                 "spec": {"nodeName": "machine1"}}
    q = SchedulingQueue()
    q.add(MPP)
    q.unschedulable["ns1/up"] = UP
    q.unschedulable["ns1/afp"] = aff
    q.assigned_pod_added(label_pod)
    assert "ns1/afp" in q.items and "ns1/afp" not in q.unschedulable
    assert "ns1/up" in q.unschedulable


def test_queue_waiting_pods_for_node():
    q = SchedulingQueue()
    for p in (MPP, UP, HPP):
        q.add(p)
    assert q.pop_nowait()["metadata"]["name"] == "hpp"
    assert names(q.waiting_pods_for_node("node1")) == ["mpp", "up"]
    assert q.waiting_pods_for_node("node2") == []
