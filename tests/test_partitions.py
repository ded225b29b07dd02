"""MI355X compute/memory partitions (SPX/DPX/QPX/CPX x NPS1/NPS2) as schedulable devices.

The reference has no notion of GPU partitioning (SURVEY §2.5 "Optional extension: CPX/NPS
partitions exposed as separate devices with attributes"); these tests pin the amdkube design:
fixture expansion, device identity/visibility, the parent-aware topology allocator (native ==
Python oracle), scheduler packing, both resource-naming strategies, and an end-to-end pod on a
partitioned node.
"""
import json
import random

import pytest

from amdkube.api import SCHEME
from amdkube.deviceplugin.amd import attributes, make_plugins, resource_groups, topology_label
from amdkube.ops import topology as t
from amdkube.scheduler import extended
from amdkube.scheduler.cache import SchedulerCache
from amdkube.scheduler.predicates import PodInfo
from amdkube.smi import FakeBackend, device_id, visibility_token
from amdkube.smi.backend import _Limited, partition_fixture
from tests.conftest import run


def test_fixture_expansion_modes():
    b = FakeBackend(compute_partition="CPX", memory_partition="NPS2")
    g = b.gpus()
    assert len(g) == 64
    assert {x["num_cu"] for x in g} == {32}
    assert {x["vram_total_bytes"] >> 30 for x in g} == {144}
    assert len({device_id(x) for x in g}) == 64
    assert len({x["render_minor"] for x in g}) == 64
    # partitions share the parent's HIP UUID, so visibility uses the agent ordinal
    assert visibility_token(g[9]) == "9"
    assert device_id(g[9]).endswith("-p1")
    topo = b.topology()
    assert topo[0][1]["type"] == "xcp" and topo[0][8]["type"] == "xgmi"
    d = FakeBackend(compute_partition="DPX")
    assert len(d.gpus()) == 16 and {x["num_cu"] for x in d.gpus()} == {128}
    assert {x["vram_total_bytes"] >> 30 for x in d.gpus()} == {288}
    s = FakeBackend()
    assert len(s.gpus()) == 8 and visibility_token(s.gpus()[0]).startswith("GPU-")
    with pytest.raises(ValueError):
        partition_fixture(s.data, "SPX", "NPS2")
    with pytest.raises(ValueError):
        partition_fixture(s.data, "OCTX", "NPS1")
    # --max-gpus counts physical GPUs: all 8 partitions of each kept GPU stay visible
    lim = _Limited(b, 2)
    assert len(lim.gpus()) == 16 and len(lim.topology()) == 16


def test_attributes_and_naming_strategies():
    b = FakeBackend(compute_partition="CPX", memory_partition="NPS1")
    a = attributes(b.gpus()[10])
    assert a["amd.com/partition"] == "CPX" and a["amd.com/partition-id"] == "2"
    assert a["amd.com/parent-gpu"] == b.gpus()[8]["bdf"].replace(":", "-")
    assert a["amd.com/cu-count"] == "32"
    assert list(resource_groups(b.gpus(), "single")) == ["amd.com/gpu"]
    assert list(resource_groups(b.gpus(), "mixed")) == ["amd.com/cpx_nps1"]
    assert list(resource_groups(FakeBackend().gpus(), "mixed")) == ["amd.com/gpu"]
    with pytest.raises(ValueError):
        resource_groups(b.gpus(), "weird")
    lab = json.loads(topology_label(b.gpus(), b.topology()))
    assert lab["parent"][:9] == [0] * 8 + [1]
    plugins = make_plugins(b, "mixed", plugins_dir="/tmp/unused")
    assert [p.resource_name for p in plugins] == ["amd.com/cpx_nps1"]
    assert plugins[0].labels["amd.com/gpu.count"] == "8"
    assert plugins[0].labels["amd.com/gpu.partition-modes"] == "CPX_NPS1"


def test_partitioned_topology_native_matches_python():
    assert t.NATIVE
    rng = random.Random(11)
    for _ in range(60):
        parts = rng.choice([2, 4, 8])
        n = 8 * parts
        parent = [i // parts for i in range(n)]
        numa = [p // 4 for p in parent]
        link = [[0 if i == j else (5 if parent[i] == parent[j] else (15 if numa[i] == numa[j] else 30)) for j in range(n)]
                for i in range(n)]
        free = sorted(rng.sample(range(n), rng.randint(1, n)))
        k = rng.randint(1, min(len(free), 10))
        a = t.select(free, k, link, numa, free, parent)
        b = t.py_select(free, k, link, numa, free, parent)
        assert a[0] == b[0] and abs(a[1] - b[1]) < 1e-9, (free, k, a, b)
        assert abs(t.score(free, k, link, numa, free, parent) - t.py_score(free, k, link, numa, free, parent)) < 1e-9


def _node(b, name="cpx-0"):
    g = b.gpus()
    devs = {device_id(x): {"id": device_id(x), "health": "Healthy", "attributes": attributes(x)} for x in g}
    return {"apiVersion": "v1", "kind": "Node",
            "metadata": {"name": name, "annotations": {"amd.com/gpu-topology": topology_label(g, b.topology())}},
            "status": {"capacity": {"cpu": "64", "memory": "512Gi", "pods": "110", "amd.com/gpu": str(len(g))},
                       "allocatable": {"cpu": "64", "memory": "512Gi", "pods": "110", "amd.com/gpu": str(len(g))},
                       "extendedResources": {"amd.com/gpu": {"resources": devs}},
                       "conditions": [{"type": "Ready", "status": "True"}]}}


def _pod(name, n, sel=None):
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "uid": name},
         "spec": {"containers": [{"name": "c", "image": "x", "extendedResourceRequests": ["g"]}],
                  "extendedResources": [{"name": "g", "resources": {"limits": {"amd.com/gpu": str(n)}},
                                         "affinity": {"required": sel or []}}]}}
    SCHEME.default(p)
    return p


def _parents(b, ids):
    by = {device_id(x): x["parent_index"] for x in b.gpus()}
    return [by[i] for i in ids]


def test_scheduler_packs_partitions_and_keeps_gpus_whole():
    b = FakeBackend(compute_partition="CPX", memory_partition="NPS1")
    cache = SchedulerCache()
    cache.add_node(_node(b))
    ni = cache.nodes["cpx-0"]
    # a full-GPU-sized request lands on the 8 partitions of ONE physical GPU
    bind = extended.allocate(PodInfo(_pod("big", 8, [{"key": "amd.com/partition", "operator": "In", "values": ["CPX"]}])), ni)
    assert len(set(_parents(b, bind["g"]["resources"]))) == 1
    # small requests pack onto an already-split GPU instead of breaking a whole one
    placed = []
    for i in range(4):
        p = _pod(f"s{i}", 2)
        bind = extended.allocate(PodInfo(p), ni)
        ids = bind["g"]["resources"]
        assert len(set(_parents(b, ids))) == 1, ids
        placed.append(_parents(b, ids)[0])
        p["spec"]["nodeName"] = "cpx-0"
        p["spec"]["extendedResources"][0]["assigned"] = ids
        cache.assume_pod(p)
    assert len(set(placed)) == 1  # 4 x 2 partitions fill exactly one more GPU
    # memory-partition attribute selector (NPS2: 144 GiB per partition)
    b2 = FakeBackend(compute_partition="CPX", memory_partition="NPS2")
    c2 = SchedulerCache()
    c2.add_node(_node(b2, "cpx-1"))
    sel = [{"key": "amd.com/gpu-memory", "operator": "Gt", "values": ["200000"]}]
    assert extended.allocate(PodInfo(_pod("m", 1, sel)), c2.nodes["cpx-1"]) is None


def test_e2e_mixed_naming_partition_pod():
    from amdkube.localcluster import LocalCluster, wait_pod

    async def body():
        lc = await LocalCluster(gpus="fake", n_gpus=2, partition="QPX/NPS1", resource_naming="mixed").start()
        try:
            node = await lc.wait_gpus(8, resource="amd.com/qpx_nps1")
            assert "amd.com/gpu" not in node["status"]["allocatable"]
            from amdkube.kubectl.printers import node_gpu_summary
            assert node_gpu_summary(node) == ("8", "8", "8", "MI355X/QPX")
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "part", "namespace": "default"},
                   "spec": {"restartPolicy": "Never", "containers": [{
                       "name": "c", "image": "busybox", "command": ["sh", "-c", "echo $ROCR_VISIBLE_DEVICES"],
                       "resources": {"limits": {"amd.com/qpx_nps1": "2"}}}]}}
            await lc.client.create(pod)
            got = await wait_pod(lc.client, "default", "part", ("Succeeded", "Failed"), 30)
            assert got["status"]["phase"] == "Succeeded", got["status"]
            er = got["spec"]["extendedResources"][0]
            assert list(er["resources"]["limits"]) == ["amd.com/qpx_nps1"] and len(er["assigned"]) == 2
            # both partitions of one physical GPU
            assert len({a.rsplit("-p", 1)[0] for a in er["assigned"]}) == 1
            log = await lc.client.logs("default", "part", "c")
            assert sorted(log.strip().split(",")) == sorted(
                str(g["hip_id"]) for g in lc.backend.gpus() if device_id(g) in er["assigned"])
        finally:
            await lc.stop()
    run(body(), timeout=90)
