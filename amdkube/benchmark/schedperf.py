"""scheduler_perf equivalent: in-process apiserver + scheduler + fake nodes (API objects only).

Reference: test/integration/scheduler_perf/scheduler_test.go:35-92 — 100 nodes
(4 CPU / 32 Gi / 110 pods), 3,000 pods, minimum-interval QPS must stay ≥ 30 pods/s
(warn < 100). amdkube's variant gives every fake node 8 MI355X devices (fixture attributes
+ topology annotation) and can make every pod request one GPU, so the device allocator and
xGMI/NUMA scorer are on the measured path.
"""
from __future__ import annotations

import asyncio
import json
import time

from ..apiserver import APIServer
from ..client import Client
from ..deviceplugin.amd import attributes, topology_label
from ..scheduler import Scheduler
from ..smi import FakeBackend, device_id


def m_name(p: dict) -> str:
    return (p.get("metadata") or {}).get("name", "")


def fake_node(i: int, gpus: int, backend: FakeBackend | None):
    st = {"capacity": {"cpu": "4", "memory": "32Gi", "pods": "110"}, "allocatable": {"cpu": "4", "memory": "32Gi", "pods": "110"},
          "conditions": [{"type": "Ready", "status": "True", "lastHeartbeatTime": "2030-01-01T00:00:00Z"}]}
    md = {"name": f"node-{i:04d}", "labels": {"kubernetes.io/hostname": f"node-{i:04d}"}}
    if gpus and backend is not None:
        gl = backend.gpus()[:gpus]
        devs = {}
        for g in gl:
            did = f"{device_id(g)}-n{i}"
            devs[did] = {"id": did, "health": "Healthy", "attributes": attributes(g)}
        st["capacity"]["amd.com/gpu"] = st["allocatable"]["amd.com/gpu"] = str(gpus)
        st["extendedResources"] = {"amd.com/gpu": {"resources": devs}}
        topo = json.loads(topology_label(gl, [r[:gpus] for r in backend.topology()[:gpus]]))
        topo["ids"] = [f"{x}-n{i}" for x in topo["ids"]]
        md["annotations"] = {"amd.com/gpu-topology": json.dumps(topo)}
    return {"apiVersion": "v1", "kind": "Node", "metadata": md, "status": st}


def pod(i: int, gpu: bool):
    c = {"name": "c", "image": "k8s.gcr.io/pause:3.1",
         "resources": {"requests": {"cpu": "10m", "memory": "10Mi"}, "limits": {"cpu": "10m", "memory": "10Mi"}}}
    if gpu:
        c["resources"]["limits"]["amd.com/gpu"] = "1"
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"pod-{i:06d}", "namespace": "default"},
            "spec": {"containers": [c]}}


def bound_pod(i: int, n_nodes: int):
    """An existing pod already running on a node (scheduler_bench_test.go makeBasePod + NodeName):
    it occupies the node's cpu/memory/pod slots the scheduler must account for."""
    p = pod(i, False)
    p["metadata"]["name"] = f"existing-{i:06d}"
    p["spec"]["nodeName"] = f"node-{i % n_nodes:04d}"
    return p


async def run_schedperf(n_nodes=100, n_pods=3000, gpus_per_node=8, gpu_pods=True, create_concurrency=64,
                        existing_pods=0):
    """scheduler_test.go (100 nodes / 3000 pods) and scheduler_bench_test.go:32-55 (100/1000
    nodes × 0/1000 existing pods): `existing_pods` are bound before the clock starts."""
    api = await APIServer(event_ttl=3600).start()
    client = Client(api.url, pool=128)
    fb = FakeBackend()
    try:
        for i in range(n_nodes):
            await client.create(fake_node(i, gpus_per_node, fb))
        if existing_pods:
            esem = asyncio.Semaphore(create_concurrency)

            async def mk_existing(i):
                async with esem:
                    await client.create(bound_pod(i, n_nodes))
            await asyncio.gather(*(mk_existing(i) for i in range(existing_pods)))
        sched = await Scheduler(Client(api.url, pool=256)).start()
        sched.recorder.enabled = False  # events are not on the measured path in scheduler_perf either
        # gpu_pods=True: every pod asks for a GPU (capped at the GPUs there are); "mixed": the
        # density mix, 8 GPU pods in every 30 (one per GPU), the rest CPU-only — the reference's
        # 3000-pod size with the device allocator on the path
        if gpu_pods == "mixed":
            want = n_pods
        else:
            want = min(n_pods, n_nodes * gpus_per_node) if gpu_pods else n_pods
        sem = asyncio.Semaphore(create_concurrency)

        async def mk(i):
            async with sem:
                await client.create(pod(i, (i % 30 < gpus_per_node and i // 30 < n_nodes) if gpu_pods == "mixed" else gpu_pods))
        t0 = time.perf_counter()
        creator = asyncio.ensure_future(asyncio.gather(*(mk(i) for i in range(want))))
        # scheduler_test.go schedulePods: start the pulse once 1 % of the pods are scheduled, then
        # count pods scheduled per 1 s interval; the interval in which the run completes is not
        # counted ("the value is random")
        while sched.scheduled <= want // 100 and time.perf_counter() - t0 < 600:
            await asyncio.sleep(0.05)
        samples = []
        prev, t_start = sched.scheduled, time.perf_counter()
        while sched.scheduled < want:
            await asyncio.sleep(1.0)
            if sched.scheduled >= want or time.perf_counter() - t0 > 600:
                break
            samples.append(sched.scheduled - prev)
            prev = sched.scheduled
        el = time.perf_counter() - t0
        await creator
        # verify: no device handed out twice
        items, _ = await client.list("pods", "default")
        items = [p for p in items if not m_name(p).startswith("existing-")]
        seen, dup = set(), 0
        for p in items:
            for pres in (p.get("spec") or {}).get("extendedResources") or []:
                for d in pres.get("assigned") or []:
                    dup += d in seen
                    seen.add(d)
        # no full interval (everything scheduled within 1 s of the 1 % mark): the run's own rate
        tail_rate = (sched.scheduled - prev) / max(1e-9, time.perf_counter() - t_start) if not samples else None
        res = {"nodes": n_nodes, "existing_pods": existing_pods, "pods": want, "gpu_pods": gpu_pods,
               "gpu_pods_scheduled": sum(1 for p in items if (p.get("spec") or {}).get("extendedResources")),
               "scheduled": sched.scheduled, "elapsed_s": round(el, 3),
               "avg_pods_per_s": round(sched.scheduled / el, 1),
               "min_interval_pods_per_s": round(min(samples), 1) if samples else round(tail_rate, 1),
               "intervals": samples,
               "bind_errors": sched.bind_errors, "double_assigned": dup}
        await sched.stop()
        await sched.client.close()
        return res
    finally:
        await client.close()
        await api.stop()


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser("amdkube scheduler_perf")
    ap.add_argument("--nodes", type=int, default=100)
    ap.add_argument("--pods", type=int, default=3000)
    ap.add_argument("--existing", type=int, default=0, help="pods bound to nodes before the measured run")
    ap.add_argument("--gpu-pods", default="mixed", choices=("mixed", "all", "none"))
    a = ap.parse_args(argv)
    gp = {"mixed": "mixed", "all": True, "none": False}[a.gpu_pods]
    print(json.dumps(asyncio.run(run_schedperf(a.nodes, a.pods, gpu_pods=gp, existing_pods=a.existing))), flush=True)


if __name__ == "__main__":
    main()
