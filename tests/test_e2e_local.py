"""End-to-end on one in-process node (apiserver + scheduler + controllers + rocshim + AMD
plugin on the fake 8×MI355X backend + kubelet): the minimum slice of SURVEY §7.4 and the
BASELINE configs 1-4 at CPU level. GPU-backed variants live in test_gpu.py.
"""
import asyncio

import pytest

from amdkube.api import meta as m
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


def gpu_pod(name, n=1, cmd=None, policy="Never", selectors=None, legacy=True):
    c = {"name": "c", "image": "busybox", "command": cmd or ["sh", "-c", "echo VISIBLE=$ROCR_VISIBLE_DEVICES IDS=$AMD_GPU_DEVICE_IDS"]}
    spec = {"restartPolicy": policy, "containers": [c]}
    if legacy:
        c["resources"] = {"limits": {"amd.com/gpu": str(n)}}
    else:
        c["extendedResourceRequests"] = ["gpus"]
        spec["extendedResources"] = [{"name": "gpus", "resources": {"limits": {"amd.com/gpu": str(n)}},
                                      "affinity": {"required": selectors or []}}]
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"}, "spec": spec}


def test_cpu_pod_runs_and_logs():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "web"},
                            "spec": {"containers": [{"name": "nginx", "image": "nginx", "ports": [{"containerPort": 8080}]}]}})
            p = await wait_pod(c, "default", "web", ("Running",), 20)
            assert p["spec"]["nodeName"] == lc.node_name
            assert p["status"]["containerStatuses"][0]["ready"] is True
            await c.delete("pods", "web", "default")
            for _ in range(200):
                if await c.get_or_none("pods", "web", "default") is None:
                    break
                await asyncio.sleep(0.05)
            assert await c.get_or_none("pods", "web", "default") is None  # kubelet finalized the graceful delete
    run(go(), 60)


def test_gpu_pod_gets_exactly_its_device():
    async def go():
        async with LocalCluster(gpus="fake", relist_period=0.2) as lc:
            c = lc.client
            node = await lc.wait_gpus(8)
            assert node["status"]["capacity"]["amd.com/gpu"] == "8"
            assert "amd.com/gpu-topology" in m.annotations_of(await c.get("nodes", lc.node_name))
            await c.create(gpu_pod("g1", 1))
            p = await wait_pod(c, "default", "g1", ("Succeeded",), 20)
            [pres] = p["spec"]["extendedResources"]
            assert len(pres["assigned"]) == 1
            logs = await c.logs("default", "g1")
            gid = pres["assigned"][0]
            assert f"IDS={gid}" in logs and f"VISIBLE={gid}" in logs, logs
    run(go(), 60)


def test_selectors_and_topology_gang():
    """BASELINE config 3 (gpu-type + gpu-memory selectors, 4 GPUs) and config 4 (2 pods × 4 GPUs
    land on disjoint, NUMA-aligned subsets)."""
    async def go():
        async with LocalCluster(gpus="fake", relist_period=0.2) as lc:
            c = lc.client
            await lc.wait_gpus(8)
            sel = [{"key": "amd.com/gpu-type", "operator": "In", "values": ["MI355X"]},
                   {"key": "amd.com/gpu-memory", "operator": "Gt", "values": ["262143"]}]
            sleep = ["sh", "-c", "sleep 30"]
            await c.create(gpu_pod("a", 4, sleep, legacy=False, selectors=sel))
            await c.create(gpu_pod("b", 4, sleep, legacy=False, selectors=sel))
            pa = await wait_pod(c, "default", "a", ("Running",), 20)
            pb = await wait_pod(c, "default", "b", ("Running",), 20)
            ga = set(pa["spec"]["extendedResources"][0]["assigned"])
            gb = set(pb["spec"]["extendedResources"][0]["assigned"])
            assert len(ga) == 4 and len(gb) == 4 and not (ga & gb)
            node = await c.get("nodes", lc.node_name)
            devs = node["status"]["extendedResources"]["amd.com/gpu"]["resources"]
            numa = lambda s: {devs[d]["attributes"]["amd.com/numa-node"] for d in s}  # noqa: E731
            assert len(numa(ga)) == 1 and len(numa(gb)) == 1 and numa(ga) != numa(gb)
            # a third 1-GPU pod cannot fit; an impossible selector stays pending with a reason
            await c.create(gpu_pod("c", 1, sleep))
            big = [{"key": "amd.com/gpu-memory", "operator": "Gt", "values": ["999999999"]}]
            await c.create(gpu_pod("d", 1, sleep, legacy=False, selectors=big))
            await asyncio.sleep(1.0)
            pc = await c.get("pods", "c", "default")
            assert not pc["spec"].get("nodeName")
            cond = [x for x in pc["status"].get("conditions") or [] if x["type"] == "PodScheduled"]
            assert cond and cond[0]["status"] == "False" and "Insufficient amd.com/gpu" in cond[0]["message"]
            # free a gang → the pending 1-GPU pod schedules onto the freed NUMA node
            await c.delete("pods", "a", "default", grace=1)
            pc = await wait_pod(c, "default", "c", ("Running",), 20)
            assert set(pc["spec"]["extendedResources"][0]["assigned"]) <= ga
    run(go(), 90)


def test_many_gpu_pods_never_double_assigned():
    async def go():
        async with LocalCluster(gpus="fake", n_gpus=4, relist_period=0.2) as lc:
            c = lc.client
            await lc.wait_gpus(4)
            names = [f"p{i}" for i in range(12)]
            for n in names:
                await c.create(gpu_pod(n, 1, ["sh", "-c", "sleep 0.2; echo ok"]))
            done = {}
            for n in names:
                done[n] = await wait_pod(c, "default", n, ("Succeeded",), 40)
            # at no time were two running pods on one GPU: the runtime's own nanosecond start/exit
            # times of every container, grouped by the render node it was given
            spans = {}
            pod_of = {}
            for ct in lc.shim.containers.values():
                render = [d["host_path"] for d in ct.devices if "/dri/render" in d["host_path"]]
                if not render:
                    continue
                assert len(render) == 1 and ct.started_at and ct.finished_at, vars(ct)
                spans.setdefault(render[0], []).append((ct.started_at, ct.finished_at))
                pod_of[ct.id] = ct.sandbox_id
            assert sum(len(v) for v in spans.values()) == 12 and len(spans) <= 4, spans
            for dev, iv in spans.items():
                iv.sort()
                for (s0, e0), (s1, e1) in zip(iv, iv[1:]):
                    assert e0 <= s1, f"two pods ran on {dev} at once: [{s0}, {e0}] overlaps [{s1}, {e1}]"
            # and the API agrees on who had which GPU
            gids = [p["spec"]["extendedResources"][0]["assigned"][0] for p in done.values()]
            assert len(set(gids)) <= 4
    run(go(), 120)
