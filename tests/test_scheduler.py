"""Scheduler units. Ports plugin/pkg/scheduler/core/extended_resources_test.go:58-294
(TestIsDeviceAMatch / TestAllocateResources / TestHasExtendedResources /
TestRemoveFromAvailable semantics) and adds a test per deliberate fix (SURVEY §7.6
#1 reserve-on-assume, #2 event-order independence, #5 zero predicates, #6 unhealthy
devices, #7 device-aware preemption) plus topology placement."""
import json

import pytest

from amdkube.api import SCHEME
from amdkube.scheduler import extended
from amdkube.scheduler.cache import SchedulerCache
from amdkube.scheduler.generic import FitError, GenericScheduler
from amdkube.scheduler.predicates import DEFAULT_PREDICATES, PodInfo
from amdkube.scheduler.priorities import DEFAULT_PRIORITIES
from amdkube.scheduler.queue import SchedulingQueue
from amdkube.scheduler.scheduler import load_policy
from amdkube.benchmark.schedperf import fake_node
from amdkube.smi import FakeBackend
from tests.conftest import run


def node(name="n0", gpus=8, mem=None, unhealthy=(), cpu="64", taints=None, topo=True):
    n = fake_node(0, gpus, FakeBackend())
    n["metadata"]["name"] = name
    n["status"]["capacity"]["cpu"] = n["status"]["allocatable"]["cpu"] = cpu
    devs = n["status"].get("extendedResources", {}).get("amd.com/gpu", {}).get("resources", {})
    for i, (did, d) in enumerate(sorted(devs.items())):
        if mem is not None:
            d["attributes"]["amd.com/gpu-memory"] = str(mem[i] if isinstance(mem, list) else mem)
        if i in unhealthy:
            d["health"] = "Unhealthy"
    if not topo:
        n["metadata"].pop("annotations", None)
    if taints:
        n.setdefault("spec", {})["taints"] = taints
    return n


def pod(name="p", gpus=0, sel=None, prio=0, cpu=None, node_name=None, assigned=None, multi=None):
    c = {"name": "c", "image": "x"}
    if cpu:
        c["resources"] = {"requests": {"cpu": cpu}, "limits": {"cpu": cpu}}
    spec = {"containers": [c], "priority": prio}
    ers = multi or ([("gpus", gpus, sel)] if gpus else [])
    if ers:
        spec["extendedResources"] = []
        c["extendedResourceRequests"] = []
        for i, (nm, n, s) in enumerate(ers):
            pres = {"name": nm, "resources": {"limits": {"amd.com/gpu": str(n)}}, "affinity": {"required": s or []}}
            if assigned and nm in assigned:
                pres["assigned"] = assigned[nm]
            spec["extendedResources"].append(pres)
            c["extendedResourceRequests"].append(nm)
    if node_name:
        spec["nodeName"] = node_name
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "uid": name}, "spec": spec,
         "status": {"phase": "Pending"}}
    SCHEME.default(p)
    return p


def sched(nodes, predicates=DEFAULT_PREDICATES, priorities=DEFAULT_PRIORITIES):
    c = SchedulerCache()
    for n in nodes:
        c.add_node(n)
    return c, GenericScheduler(c, list(predicates), dict(priorities))


def test_device_match_selector_semantics():
    c, _ = sched([node(mem=[4096, 8192, 2048, 16384, 4096, 4096, 4096, 4096])])
    ni = c.nodes["n0"]
    gt = [{"key": "amd.com/gpu-memory", "operator": "Gt", "values": ["4095"]}]
    pi = PodInfo(pod(gpus=1, sel=gt))
    cand = extended.matching_free(pi, ni, "amd.com/gpu", pi.ext[0][3])
    assert len(cand) == 7
    pi = PodInfo(pod(gpus=1, sel=[{"key": "amd.com/gpu-memory", "operator": "Gt", "values": ["8191"]}]))
    assert len(extended.matching_free(pi, ni, "amd.com/gpu", pi.ext[0][3])) == 2
    bad = PodInfo(pod(gpus=1, sel=[{"key": "amd.com/gpu-memory", "operator": "Gt", "values": ["1", "2"]}]))
    assert bad.ext_error  # Gt with two values is an error (reference TestIsDeviceAMatch)
    assert extended.fits(bad, ni)[0] is False


def test_allocate_counts_and_multi_resource_pods():
    c, _ = sched([node()])
    ni = c.nodes["n0"]
    pi = PodInfo(pod(multi=[("a", 3, None), ("b", 4, None)]))
    b = extended.allocate(pi, ni)
    assert len(b["a"]["resources"]) == 3 and len(b["b"]["resources"]) == 4
    assert not set(b["a"]["resources"]) & set(b["b"]["resources"])
    assert extended.fits(PodInfo(pod(multi=[("a", 5, None), ("b", 4, None)])), ni)[0] is False
    assert extended.fits(PodInfo(pod(gpus=9)), ni) == (False, ["Insufficient amd.com/gpu"])


def test_unhealthy_devices_not_allocated():  # fix #6
    c, _ = sched([node(unhealthy=(0, 1, 2))])
    ni = c.nodes["n0"]
    assert len(ni.available_devices("amd.com/gpu")) == 5
    assert extended.fits(PodInfo(pod(gpus=6)), ni)[0] is False
    b = extended.allocate(PodInfo(pod(gpus=5)), ni)
    healthy = {d for d, x in ni.devices["amd.com/gpu"].items() if x["health"] == "Healthy"}
    assert set(b["gpus"]["resources"]) == healthy


def test_reserve_on_assume_prevents_double_allocation():  # fix #1
    def go():
        c, g = sched([node(gpus=2, topo=False)])
        import asyncio
        h1, b1 = asyncio.run(g.schedule(pod("p1", 1)))
        p1 = pod("p1", 1, node_name=h1, assigned={"gpus": b1["gpus"]["resources"]})
        c.assume_pod(p1)
        h2, b2 = asyncio.run(g.schedule(pod("p2", 1)))
        assert b1["gpus"]["resources"] != b2["gpus"]["resources"]
        c.assume_pod(pod("p2", 1, node_name=h2, assigned={"gpus": b2["gpus"]["resources"]}))
        with pytest.raises(FitError):
            asyncio.run(g.schedule(pod("p3", 1)))
        c.forget_pod(p1)  # binding failed → devices return
        asyncio.run(g.schedule(pod("p3", 1)))
    go()


def test_event_order_independence():  # fix #2
    n = node(gpus=4, topo=False)
    ids = sorted(n["status"]["extendedResources"]["amd.com/gpu"]["resources"])
    bound = pod("b", 2, node_name="n0", assigned={"gpus": ids[:2]})
    c1 = SchedulerCache()
    c1.add_pod(bound)
    c1.add_node(n)   # AddPod before SetNode: the reference would mark the devices available again
    c2 = SchedulerCache()
    c2.add_node(n)
    c2.add_pod(bound)
    assert set(c1.nodes["n0"].available_devices("amd.com/gpu")) == set(c2.nodes["n0"].available_devices("amd.com/gpu")) == set(ids[2:])
    c1.remove_pod(bound)
    assert set(c1.nodes["n0"].available_devices("amd.com/gpu")) == set(ids)


def test_zero_predicates_config():  # fix #5
    import asyncio
    c, g = sched([node(), node("n1")], predicates=[], priorities={})
    h, b = asyncio.run(g.schedule(pod(gpus=2)))
    assert h in ("n0", "n1") and len(b["gpus"]["resources"]) == 2


def test_topology_gang_disjoint_numa():
    import asyncio
    c, g = sched([node()])
    placed = []
    for nm in ("a", "b"):
        h, b = asyncio.run(g.schedule(pod(nm, 4)))
        ids = b["gpus"]["resources"]
        c.assume_pod(pod(nm, 4, node_name=h, assigned={"gpus": ids}))
        placed.append(ids)
    devs = c.nodes["n0"].devices["amd.com/gpu"]
    numas = [{devs[d]["attributes"]["amd.com/numa-node"] for d in ids} for ids in placed]
    assert all(len(s) == 1 for s in numas) and numas[0] != numas[1]
    assert not set(placed[0]) & set(placed[1])


def test_best_fit_single_gpu_keeps_numa_block_whole():
    import asyncio
    c, g = sched([node()])
    # occupy one GPU on NUMA 1 → the next 1-GPU pod should also go to NUMA 1 (keep NUMA 0 whole)
    devs = sorted(c.nodes["n0"].devices["amd.com/gpu"])
    numa1 = [d for d in devs if c.nodes["n0"].devices["amd.com/gpu"][d]["attributes"]["amd.com/numa-node"] == "1"]
    c.add_pod(pod("x", 1, node_name="n0", assigned={"gpus": [numa1[0]]}))
    h, b = asyncio.run(g.schedule(pod("y", 1)))
    assert b["gpus"]["resources"][0] in numa1


def test_gpu_pods_prefer_fullest_node_and_cpu_pods_avoid_gpu_nodes():
    import asyncio
    cpu_only = node("cpu", gpus=0)
    c, g = sched([node("g1"), node("g2"), cpu_only])
    ids = sorted(c.nodes["g1"].devices["amd.com/gpu"])
    c.add_pod(pod("x", 2, node_name="g1", assigned={"gpus": ids[:2]}))
    h, _ = asyncio.run(g.schedule(pod("y", 2)))
    assert h == "g1"   # best fit across nodes
    h, _ = asyncio.run(g.schedule(pod("z", 0, cpu="100m")))
    assert h == "cpu"  # CPU-only pods keep GPU nodes free


def test_predicates_taints_selector_resources_condition():
    import asyncio
    t = [{"key": "dedicated", "value": "ml", "effect": "NoSchedule"}]
    n1 = node("tainted", taints=t)
    n2 = node("small", cpu="1")
    n3 = node("notready")
    n3["status"]["conditions"] = [{"type": "Ready", "status": "False"}]
    c, g = sched([n1, n2, n3])
    with pytest.raises(FitError) as ei:
        asyncio.run(g.schedule(pod(cpu="2")))
    msg = str(ei.value)
    assert "PodToleratesNodeTaints" in msg and "Insufficient cpu" in msg and "NodeNotReady" in msg
    p = pod(cpu="500m")
    p["spec"]["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "ml", "effect": "NoSchedule"}]
    p["spec"]["nodeSelector"] = {"kubernetes.io/hostname": "node-0000"}
    h, _ = asyncio.run(g.schedule(p))
    assert h in ("tainted", "small")


def test_preemption_considers_devices():  # fix #7
    c, g = sched([node(gpus=2, topo=False)])
    ids = sorted(c.nodes["n0"].devices["amd.com/gpu"])
    c.add_pod(pod("low1", 1, prio=1, node_name="n0", assigned={"gpus": [ids[0]]}))
    c.add_pod(pod("low2", 1, prio=5, node_name="n0", assigned={"gpus": [ids[1]]}))
    nodename, victims = g.preempt(pod("high", 1, prio=100))
    assert nodename == "n0" and [v["metadata"]["name"] for v in victims] == ["low1"]
    nodename, victims = g.preempt(pod("mid", 2, prio=3))
    assert nodename is None  # would need low2 (prio 5 > 3)


def test_queue_priority_order_and_unschedulable_moves():
    import asyncio

    async def go():
        q = SchedulingQueue()
        q.add(pod("low", prio=1))
        q.add(pod("high", prio=10))
        q.add(pod("mid", prio=5))
        assert [(await q.pop())["metadata"]["name"] for _ in range(3)] == ["high", "mid", "low"]
        q.add_unschedulable(pod("u"), marked=True)
        assert len(q) == 0
        q.move_all_to_active()
        assert (await q.pop())["metadata"]["name"] == "u"
    run(go())


def test_policy_file(tmp_path):
    p = tmp_path / "policy.json"
    p.write_text(json.dumps({"kind": "Policy", "predicates": [{"name": "GeneralPredicates"}],
                             "priorities": [{"name": "GPUTopologyPriority", "weight": 3}]}))
    preds, prios, exts = load_policy(str(p))
    assert preds == ["GeneralPredicates"] and prios == {"GPUTopologyPriority": 3} and exts == []


def test_overlapping_selectors_on_one_resource_name():
    """Two requests of amd.com/gpu whose selectors overlap: the per-request counts fit on node
    'a' (1 big GPU each) but no disjoint assignment exists there; the pod goes to 'b'."""
    big = [{"key": "amd.com/gpu-memory", "operator": "Gt", "values": ["100000"]}]
    a = node("a", gpus=2, mem=[294912, 1024])
    b = node("b", gpus=2, mem=[294912, 294912])
    c, g = sched([a, b])
    p = pod(multi=[("r1", 1, big), ("r2", 1, big)])
    pi = PodInfo(p)
    assert extended.fits(pi, c.nodes["a"]) == (False, ["Insufficient amd.com/gpu"])
    assert extended.fits(pi, c.nodes["b"])[0]
    host, binding = run(g.schedule(p))
    assert host == "b"
    assert {binding["r1"]["resources"][0], binding["r2"]["resources"][0]} == set(c.nodes["b"].available_devices("amd.com/gpu"))
    # a narrow selector next to a wide one on the same node: allocate serves the narrow one first
    wide = PodInfo(pod(multi=[("w", 1, None), ("n", 1, big)]))
    bind = extended.allocate(wide, c.nodes["a"])
    big_id = [d for d, dv in c.nodes["a"].available_devices("amd.com/gpu").items()
              if dv["attributes"]["amd.com/gpu-memory"] == "294912"][0]
    assert bind["n"]["resources"] == [big_id] and bind["w"]["resources"] != [big_id]


def test_allocation_failure_tries_the_next_ranked_host(monkeypatch):
    c, g = sched([node("a", gpus=8), node("b", gpus=8)])
    real = extended.allocate
    tried = []

    def flaky(pi, ni, use_topology=True):
        tried.append(ni.name)
        return None if len(tried) == 1 else real(pi, ni, use_topology)
    monkeypatch.setattr(extended, "allocate", flaky)
    host, binding = run(g.schedule(pod(gpus=2)))
    assert tried[0] != host and len(tried) == 2 and len(binding["gpus"]["resources"]) == 2
    monkeypatch.setattr(extended, "allocate", lambda *a, **k: None)
    with pytest.raises(FitError) as e:
        run(g.schedule(pod("q", gpus=2)))
    assert set(e.value.failed) == {"a", "b"}


def test_fit_index_decides_like_a_full_scan():
    """The incremental per-equivalence-class fit index (only nodes changed since the last pod of
    the class are re-checked) picks the same host, devices and failure as evaluating every node,
    across binds, node updates (taint, removal) and pod removal — with ImageLocalityPriority on and
    pods that differ only in their image (the image is part of the equivalence class)."""
    import asyncio
    import random
    rnd = random.Random(7)
    images = ["img/a", "img/b", "img/c"]

    def world():
        nodes = [node(f"n{i}", gpus=rnd.choice((0, 2, 4, 8)), cpu=str(rnd.choice((2, 4, 8)))) for i in range(24)]
        for n in nodes:
            n["status"]["images"] = [{"names": [im], "sizeBytes": rnd.choice((0, 100, 400, 900)) << 20}
                                     for im in images if rnd.random() < 0.5]
        return sched(nodes, priorities={**DEFAULT_PRIORITIES, "ImageLocalityPriority": 3})

    rnd.seed(7)
    c_fast, g_fast = world()
    rnd.seed(7)
    c_slow, g_slow = world()
    g_slow._uniform_others = lambda pi: False          # always the full scan,
    g_slow._equiv_key = lambda pi: None                 # with no equivalence cache at all
    script = random.Random(11)
    bound = []
    for step in range(160):
        kind = script.random()
        if kind < 0.07 and bound:                      # a pod goes away
            p = bound.pop(script.randrange(len(bound)))
            c_fast.remove_pod(p)
            c_slow.remove_pod(p)
            continue
        if kind < 0.1:                                 # a node is tainted NoSchedule, or comes back
            n = node(f"n{script.randrange(24)}", gpus=8, cpu="8",
                     taints=[{"key": "k", "effect": "NoSchedule"}] if script.random() < 0.5 else None)
            c_fast.update_node(n)
            c_slow.update_node(n)
            continue
        p = pod(f"p{step}", gpus=script.choice((0, 0, 1, 2)), cpu=script.choice(("100m", "500m", "1")))
        p["spec"]["containers"][0]["image"] = script.choice(images)
        results = []
        for c, g in ((c_fast, g_fast), (c_slow, g_slow)):
            try:
                h, b = asyncio.run(g.schedule(p))
                results.append((h, b))
                assigned = {k: v["resources"] for k, v in b.items()} if b else None
                c.assume_pod(pod(p["metadata"]["name"], gpus=len((b or {}).get("gpus", {}).get("resources", [])),
                                 cpu=p["spec"]["containers"][0]["resources"]["requests"]["cpu"],
                                 node_name=h, assigned=assigned))
            except FitError as e:
                results.append(("fit-error", str(e)))
        assert results[0] == results[1], (step, results)
        if results[0][0] != "fit-error":
            bound.append(pod(p["metadata"]["name"], node_name=results[0][0]))
    assert g_fast.findex and g_fast.ecache_hits > 0
