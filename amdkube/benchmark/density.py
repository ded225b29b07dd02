"""Cluster density / saturation benchmark on hollow MI355X nodes (kubemark-style).

Reference: test/e2e/scalability/density.go. It saturates the cluster with replicated pause pods
at 30 pods/node (:55-56, :364-367) and fails below 8 pods/s. It reports pod startup latency
phases from a watch: create→schedule, schedule→run, run→watch, and e2e (:771-819). The SLO is
p50/p90/p99 ≤ 5 s (test/e2e/framework/metrics_util.go:46).

amdkube runs the same experiment with the real control plane:
  * apiserver in this process; scheduler and controller-manager (ReplicaSet controller) as their
    own processes, as in a real deployment (`--in-process` keeps all three here);
  * N hollow nodes in a child process (`python -m amdkube hollow-node --count N`). Each hollow
    node is a real kubelet with the real AMD device plugin over a simulated 8×MI355X and a fake
    CRI runtime. The reference's kubemark had no GPUs at all.

Each node gets `gpus_per_node` GPU pods (`amd.com/gpu: 1`, ResourceV2 → device-granular
binding) plus CPU pause pods up to `pods_per_node`. Two ReplicaSets create them all at once.
Saturation throughput = pods / (first create → last pod observed Running).

  python -m amdkube.benchmark.density --nodes 10 --pods-per-node 30
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import time

from ..api import meta as m
from ..apiserver import APIServer
from ..client import Client
from ..controllers import ControllerManager
from ..scheduler import Scheduler

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, max(0, int(round(q / 100.0 * (len(xs) - 1)))))]


def _rs(name, replicas, gpu):
    c = {"name": "pause", "image": "k8s.gcr.io/pause:3.1",
         "resources": {"requests": {"cpu": "10m", "memory": "10Mi"}, "limits": {"cpu": "10m", "memory": "10Mi"}}}
    if gpu:
        c["resources"]["limits"]["amd.com/gpu"] = "1"
    labels = {"app": name}
    return {"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": name, "namespace": "default"},
            "spec": {"replicas": replicas, "selector": {"matchLabels": labels},
                     "template": {"metadata": {"labels": labels},
                                  "spec": {"terminationGracePeriodSeconds": 0, "containers": [c]}}}}


async def run_density(n_nodes: int = 10, pods_per_node: int = 30, gpus_per_node: int = 8, node_procs: int = 2,
                      timeout: float = 300.0, in_process: bool = False, cm_qps: float = 1000.0, cm_burst: int = 1000) -> dict:
    """cm_qps/cm_burst: the controller-manager's --kube-api-qps/--kube-api-burst. Its default
    of 20 (the reference's) caps ReplicaSet pod creation at 20 pods/s, so density runs raise it
    explicitly, as the reference's kubemark masters do (cluster/kubemark/gce/config-default.sh
    KUBEMARK_MASTER_COMPONENTS_QPS_LIMITS)."""
    api = await APIServer(event_ttl=3600).start()
    client = Client(api.url, pool=128)
    sched = cm = None
    procs = []
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    if in_process:
        sched = await Scheduler(Client(api.url, pool=256)).start()
        cm = await ControllerManager(Client(api.url, pool=128, qps=cm_qps, burst=cm_burst), controllers=["replicaset"]).start()
    else:
        for argv in (["scheduler", "--master", api.url, "--port", "0"],
                     ["controller-manager", "--master", api.url, "--controllers", "replicaset",
                      "--kube-api-qps", str(cm_qps), "--kube-api-burst", str(cm_burst)]):
            procs.append(subprocess.Popen([sys.executable, "-m", "amdkube", *argv], cwd=ROOT, env=env,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
    per = [n_nodes // node_procs + (1 if i < n_nodes % node_procs else 0) for i in range(node_procs)]
    try:
        for i, cnt in enumerate(per):
            if cnt:
                prof = os.environ.get("AMDKUBE_PROFILE_HOLLOW")  # cProfile output path for hollow process 0
                pre = ["-m", "cProfile", "-o", prof] if prof and i == 0 else []
                procs.append(subprocess.Popen(
                    [sys.executable, *pre, "-m", "amdkube", "hollow-node", "--server", api.url, "--count", str(cnt),
                     "--gpus", str(gpus_per_node), "--name-prefix", f"hollow{i}"],
                    cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        loop = asyncio.get_running_loop()
        t_nodes = time.perf_counter()
        while True:
            nodes, _ = await client.list("nodes")
            ready = [n for n in nodes if int((n["status"].get("allocatable") or {}).get("amd.com/gpu", 0) or 0) >= gpus_per_node]
            if len(ready) >= n_nodes:
                break
            if time.perf_counter() - t_nodes > 60 or any(p.poll() is not None for p in procs):
                raise RuntimeError(f"only {len(ready)}/{n_nodes} hollow nodes became ready")
            await asyncio.sleep(0.1)
        node_ready_s = time.perf_counter() - t_nodes

        n_gpu = n_nodes * gpus_per_node
        n_cpu = n_nodes * pods_per_node - n_gpu
        total = n_gpu + n_cpu
        seen: dict[str, dict] = {}
        done = asyncio.Event()
        n_running = [0]
        _, rv = await client.list("pods", "default")

        async def watch():
            async for typ, p in client.watch("pods", "default", resource_version=rv):
                k = m.name_of(p)
                t = time.perf_counter()
                rec = seen.setdefault(k, {"created": t, "gpu": "gpu" in k})
                if "scheduled" not in rec and (p.get("spec") or {}).get("nodeName"):
                    rec["scheduled"] = t
                if "running" not in rec and (p.get("status") or {}).get("phase") == "Running":
                    rec["running"] = t
                    n_running[0] += 1
                    for cs in (p.get("status") or {}).get("containerStatuses") or []:
                        st = ((cs.get("state") or {}).get("running") or {}).get("startedAt")
                        if st:
                            rec["started_at"] = st
                    if n_running[0] >= total:
                        done.set()
                        return
        wt = asyncio.create_task(watch())
        t0 = time.perf_counter()
        await client.create(_rs("density-gpu", n_gpu, True))
        await client.create(_rs("density-cpu", n_cpu, False))
        try:
            await asyncio.wait_for(done.wait(), timeout)
        finally:
            wt.cancel()
        elapsed = time.perf_counter() - t0
        e2e = [(r["running"] - r["created"]) * 1e3 for r in seen.values() if "running" in r]
        sched_lat = [(r["scheduled"] - r["created"]) * 1e3 for r in seen.values() if "scheduled" in r]
        node_lat = [(r["running"] - r["scheduled"]) * 1e3 for r in seen.values() if "running" in r and "scheduled" in r]
        gpu_e2e = [(r["running"] - r["created"]) * 1e3 for r in seen.values() if "running" in r and r["gpu"]]
        pods, _ = await client.list("pods", "default")
        assigned = [(p["spec"].get("nodeName"), d) for p in pods for er in p["spec"].get("extendedResources") or []
                    for d in er.get("assigned") or []]
        return {"nodes": n_nodes, "pods_per_node": pods_per_node, "gpu_pods": n_gpu, "cpu_pods": n_cpu, "pods": total,
                "node_ready_s": round(node_ready_s, 2), "elapsed_s": round(elapsed, 3),
                "saturation_pods_per_s": round(total / elapsed, 1), "controller_manager_qps": cm_qps,
                "startup_ms": {"p50": round(pct(e2e, 50), 1), "p90": round(pct(e2e, 90), 1), "p99": round(pct(e2e, 99), 1)},
                "gpu_startup_ms": {"p50": round(pct(gpu_e2e, 50), 1), "p90": round(pct(gpu_e2e, 90), 1),
                                   "p99": round(pct(gpu_e2e, 99), 1)},
                "create_to_schedule_ms_p50": round(pct(sched_lat, 50), 1),
                "schedule_to_run_ms_p50": round(pct(node_lat, 50), 1),
                "gpu_devices_assigned": len(assigned), "double_assigned": len(assigned) - len(set(assigned))}
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        if cm is not None:
            await cm.stop()
            await cm.client.close()
        if sched is not None:
            await sched.stop()
            await sched.client.close()
        await client.close()
        await api.stop()


def main(argv=None):
    ap = argparse.ArgumentParser("amdkube density benchmark")
    ap.add_argument("--nodes", type=int, default=10)
    ap.add_argument("--pods-per-node", type=int, default=30)
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--node-procs", type=int, default=2)
    ap.add_argument("--in-process", action="store_true", help="scheduler + controller-manager in the apiserver process")
    ap.add_argument("--controller-manager-qps", type=float, default=1000.0,
                    help="controller-manager --kube-api-qps (its default, 20, caps pod creation at 20/s)")
    ap.add_argument("--controller-manager-burst", type=int, default=1000)
    a = ap.parse_args(argv)
    print(json.dumps(asyncio.run(run_density(a.nodes, a.pods_per_node, a.gpus_per_node, a.node_procs,
                                             in_process=a.in_process, cm_qps=a.controller_manager_qps,
                                             cm_burst=a.controller_manager_burst))))


if __name__ == "__main__":
    main()
