"""Scheduler policy arguments and options (plugin/pkg/scheduler/api/types.go PredicateArgument /
PriorityArgument, predicates.go ServiceAffinity/NodeLabelPresence, priorities
selector_spreading.go ServiceAntiAffinity and node_label.go, interpod_affinity.go
hardPodAffinitySymmetricWeight, factory.go policy from a ConfigMap)."""
import asyncio
import json

import pytest

from amdkube.api import SCHEME
from amdkube.localcluster import LocalCluster
from amdkube.scheduler.cache import SchedulerCache
from amdkube.scheduler.generic import FitError, GenericScheduler
from amdkube.scheduler.policy_args import build
from tests.conftest import run


def _node(name, labels):
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": labels},
            "status": {"capacity": {"cpu": "8", "memory": "16Gi", "pods": "20"},
                       "allocatable": {"cpu": "8", "memory": "16Gi", "pods": "20"},
                       "conditions": [{"type": "Ready", "status": "True"}]}}


def _pod(name, labels=None, node=None, sel=None, affinity=None):
    spec = {"containers": [{"name": "c", "image": "x"}]}
    if node:
        spec["nodeName"] = node
    if sel:
        spec["nodeSelector"] = sel
    if affinity:
        spec["affinity"] = affinity
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "uid": name,
                                                         "labels": labels or {}}, "spec": spec, "status": {"phase": "Pending"}}
    SCHEME.default(p)
    return p


SVC = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "train", "namespace": "default"},
       "spec": {"selector": {"app": "train"}}}


def _sched(policy, nodes, pods=(), services=(SVC,), hard=1):
    preds, prios, cp, cr = build(policy)
    c = SchedulerCache()
    for n in nodes:
        c.add_node(n)
    for p in pods:
        c.add_pod(p)
    return GenericScheduler(c, preds, prios, custom_predicates=cp, custom_priorities=cr, services=lambda: list(services),
                            hard_affinity_weight=hard)


def test_labels_presence_and_service_affinity():
    nodes = [_node("a", {"rack": "r1", "gpu": "mi355x"}), _node("b", {"rack": "r2", "gpu": "mi355x"}), _node("c", {"rack": "r2"})]
    pol = {"predicates": [{"name": "PodFitsResources"},
                          {"name": "HasGPU", "argument": {"labelsPresence": {"labels": ["gpu"], "presence": True}}},
                          {"name": "SameRack", "argument": {"serviceAffinity": {"labels": ["rack"]}}}],
           "priorities": [{"name": "LeastRequestedPriority", "weight": 1}]}
    # the first pod of the service may go to any GPU node; the next ones follow its rack
    g = _sched(pol, nodes, pods=[_pod("t0", {"app": "train"}, node="b")])
    for i in range(3):
        host, _ = asyncio.run(g.schedule(_pod(f"t{i + 1}", {"app": "train"})))
        assert host == "b"                                    # r2 ∩ has gpu
    # an explicit node selector for the label wins over the service's placement
    host, _ = asyncio.run(g.schedule(_pod("t9", {"app": "train"}, sel={"rack": "r1"})))
    assert host == "a"
    # without the label nothing fits
    g2 = _sched({"predicates": [{"name": "NoGPU", "argument": {"labelsPresence": {"labels": ["gpu", "rack"], "presence": True}}}]},
                [_node("c", {"rack": "r2"})])
    with pytest.raises(FitError):
        asyncio.run(g2.schedule(_pod("x")))
    with pytest.raises(ValueError, match="unknown predicate"):
        build({"predicates": [{"name": "Nope"}]})


def test_service_anti_affinity_and_label_preference():
    nodes = [_node("a", {"zone": "z1"}), _node("b", {"zone": "z1"}), _node("c", {"zone": "z2"}), _node("d", {})]
    pol = {"predicates": [{"name": "PodFitsResources"}],
           "priorities": [{"name": "ZoneSpread", "weight": 1, "argument": {"serviceAntiAffinity": {"label": "zone"}}}]}
    placed = [_pod("t0", {"app": "train"}, node="a"), _pod("t1", {"app": "train"}, node="b")]
    host, _ = asyncio.run(_sched(pol, nodes, placed).schedule(_pod("t2", {"app": "train"})))
    assert host == "c"            # z2 holds none of the service's pods
    pol2 = {"predicates": [{"name": "PodFitsResources"}],
            "priorities": [{"name": "AvoidZoneless", "weight": 5, "argument": {"labelPreference": {"label": "zone", "presence": False}}}]}
    host, _ = asyncio.run(_sched(pol2, nodes).schedule(_pod("x")))
    assert host == "d"


def test_hard_pod_affinity_symmetric_weight():
    nodes = [_node("a", {"zone": "z1"}), _node("b", {"zone": "z2"}), _node("c", {"zone": "z3"})]
    needs_db = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": "zone"}]}}
    placed = [_pod("web", {"app": "web"}, node="b", affinity=needs_db)]
    pol = {"predicates": [{"name": "PodFitsResources"}], "priorities": [{"name": "InterPodAffinityPriority", "weight": 1}]}
    host, _ = asyncio.run(_sched(pol, nodes, placed, hard=10).schedule(_pod("db", {"app": "db"})))
    assert host == "b"            # the web pod's required affinity pulls the db pod into z2
    pol["hardPodAffinitySymmetricWeight"] = 0
    g = _sched(pol, nodes, placed, hard=0)
    hosts = {asyncio.run(g.schedule(_pod(f"db{i}", {"app": "db"})))[0] for i in range(3)}
    assert hosts != {"b"}         # no pull: round-robin over equal scores


def test_policy_from_configmap():
    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            for n in (_node("gpu-0", {"gpu": "mi355x"}), _node("cpu-0", {})):
                await c.create(n)
            await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "sched-policy", "namespace": "kube-system"},
                            "data": {"policy.cfg": json.dumps({"kind": "Policy", "apiVersion": "v1", "predicates": [
                                {"name": "PodFitsResources"},
                                {"name": "GPUNodesOnly", "argument": {"labelsPresence": {"labels": ["gpu"], "presence": True}}}],
                                "priorities": [{"name": "LeastRequestedPriority", "weight": 1}]})}})
            from amdkube.client import Client
            from amdkube.scheduler import Scheduler
            await lc.scheduler.stop()
            s = await Scheduler(Client(lc.api.url, token=lc.api.loopback_token), "default-scheduler",
                                policy_configmap=("kube-system", "sched-policy")).start()
            try:
                for i in range(4):
                    await c.create(_pod(f"p{i}"), "default")
                for _ in range(100):
                    pods, _ = await c.list("pods", "default")
                    if all((p["spec"].get("nodeName") for p in pods)):
                        break
                    await asyncio.sleep(0.05)
                assert {p["spec"]["nodeName"] for p in pods} == {"gpu-0"}
            finally:
                await s.stop()
    run(go(), 60)
