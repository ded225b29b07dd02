"""Kubelet eviction manager (reference pkg/kubelet/eviction/helpers_test.go
ParseThresholdConfig, eviction_manager_test.go (memory pressure: conditions, admission of
BestEffort pods, eviction ranking by QoS, soft thresholds with grace periods, pressure
transition period), rank tests)."""
import asyncio

from amdkube.kubelet.eviction import MEMORY, NODEFS, EvictionManager, parse_thresholds, rank
from amdkube.localcluster import LocalCluster, wait_pod

GI = 1 << 30


def test_threshold_parsing_and_soft_grace():
    ts = parse_thresholds("memory.available<1Gi,nodefs.available<10%", "memory.available<2Gi", "memory.available=1m30s",
                          "memory.available=500Mi")
    hard = {t.signal: t for t in ts if t.hard}
    soft = [t for t in ts if not t.hard][0]
    assert hard[MEMORY].quantity == GI and hard[NODEFS].percentage == 0.10 and soft.grace == 90.0
    assert hard[MEMORY].min_reclaim == 500 * (1 << 20)
    clock = [0.0]
    em = EvictionManager(ts, pressure_transition=300.0, clock=lambda: clock[0])
    obs = {MEMORY: (int(1.5 * GI), 64 * GI), NODEFS: (50 * GI, 100 * GI)}
    assert em.met(obs) == []                        # soft threshold met, grace not yet elapsed
    clock[0] = 91.0
    assert [t.signal for t in em.met(obs)] == [MEMORY]
    assert em.conditions(obs) == {"MemoryPressure"}
    clock[0] = 200.0
    assert em.conditions({MEMORY: (10 * GI, 64 * GI)}) == {"MemoryPressure"}   # held for the transition period
    clock[0] = 400.0
    assert em.conditions({MEMORY: (10 * GI, 64 * GI)}) == set()
    try:
        parse_thresholds("", "memory.available<1Gi")
        raise AssertionError("soft thresholds need a grace period")
    except ValueError:
        pass


def _pod(uid, qos):
    res = {"Guaranteed": {"limits": {"cpu": "1", "memory": "1Gi"}}, "Burstable": {"requests": {"memory": "1Gi"}},
           "BestEffort": {}}[qos]
    return {"metadata": {"uid": uid, "namespace": "default", "name": uid}, "spec": {"containers": [{"name": "c", "resources": res}]}}


def test_rank_and_admit():
    pods = [_pod("g", "Guaranteed"), _pod("b1", "Burstable"), _pod("b2", "Burstable"), _pod("e", "BestEffort")]
    usage = {"b1": GI, "b2": 3 * GI, "g": 5 * GI}
    order = [p["metadata"]["uid"] for p in rank(pods, MEMORY, usage)]
    # helpers.go rankMemoryPressure: no stats first, then pods above their request, then priority,
    # then the larger usage above request (g: 4Gi over, b2: 2Gi over; b1 sits at its request)
    assert order == ["e", "g", "b2", "b1"]
    pods[2]["spec"]["priority"] = -10
    assert [p["metadata"]["uid"] for p in rank(pods, MEMORY, usage)] == ["e", "b2", "g", "b1"]
    assert [p["metadata"]["uid"] for p in rank(pods, MEMORY, usage, use_priority=False)] == ["e", "g", "b2", "b1"]
    em = EvictionManager(parse_thresholds("memory.available<1Gi"))
    assert em.admit(_pod("e", "BestEffort"), {"MemoryPressure"})[0] is False
    assert em.admit(_pod("b1", "Burstable"), {"MemoryPressure"})[0] is True
    assert em.admit(_pod("g", "Guaranteed"), {"DiskPressure"})[0] is False


def test_min_reclaim_keeps_threshold_met_and_soft_grace_override():
    """thresholdsMet(enforceMinReclaim): once met, memory.available<1Gi stays met until
    available ≥ 1Gi + 500Mi; soft evictions use MaxPodGracePeriodSeconds, hard ones 0."""
    ts = parse_thresholds("memory.available<1Gi", "nodefs.available<20%", "nodefs.available=0s", "memory.available=500Mi")
    em = EvictionManager(ts, max_pod_grace=7)
    assert em.met({MEMORY: (int(1.2 * GI), 64 * GI)}) == []
    assert [t.signal for t in em.met({MEMORY: (int(0.9 * GI), 64 * GI)})] == [MEMORY]
    assert [t.signal for t in em.met({MEMORY: (int(1.2 * GI), 64 * GI)})] == [MEMORY]   # not yet reclaimed
    assert em.met({MEMORY: (int(1.6 * GI), 64 * GI)}) == []                            # ≥ 1Gi + 500Mi
    assert em.met({MEMORY: (int(1.2 * GI), 64 * GI)}) == []                            # resolved: plain threshold again
    pct = parse_thresholds("nodefs.available<10%", "", "", "nodefs.available=5%")[0]
    assert pct.reclaim(100 * GI) == 5 * GI
    hard = [t for t in ts if t.hard][0]
    soft = [t for t in ts if not t.hard][0]
    pod = _pod("b1", "Burstable")
    pod["spec"]["terminationGracePeriodSeconds"] = 60
    assert em.grace_for(pod, hard) == 0 and em.grace_for(pod, soft) == 7
    assert EvictionManager(ts).grace_for(pod, soft) == 0


async def test_memory_pressure_condition_admission_and_eviction():
    async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                            kubelet_kw={"eviction_interval": 3600, "eviction_hard": "memory.available<2Gi"}) as lc:
        c, k = lc.client, lc.kubelet
        for name, res in (("be", {}), ("gu", {"limits": {"cpu": "100m", "memory": "64Mi"}})):
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"],
                                                     "resources": res}]}}, "default")
            await wait_pod(c, "default", name, ("Running",), 20)
        k.eviction_observer = lambda: {MEMORY: (GI, 64 * GI)}      # below the 2Gi hard threshold
        victim = await k.eviction_pass()
        assert victim["metadata"]["name"] == "be"
        p = await wait_pod(c, "default", "be", ("Failed",), 10)
        assert p["status"]["reason"] == "Evicted" and "memory" in p["status"]["message"]
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
        assert p["status"]["reason"] == "Evicted" and "MemoryPressure" in p["status"]["message"]
        assert (await c.get("pods", "gu", "default"))["status"]["phase"] == "Running"
