"""CPU manager (pkg/kubelet/cm/cpumanager: cpu_assignment_test.go, policy_static_test.go,
state_checkpoint_test.go, cpu_manager_test.go reconcile), plus GPU-NUMA placement."""
import asyncio
import json
import os

import pytest

from amdkube.api import meta as m
from amdkube.kubelet.cpumanager import (CPUManager, CPUTopology, format_cpuset, parse_cpuset, take_by_topology)
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run

# 2 sockets × 4 cores × 2 threads: cpu = t*8 + s*4 + k
TOPO = CPUTopology.synthetic(2, 4, 2)


def test_cpuset_format_roundtrip():
    assert parse_cpuset("0-3,8,10-11") == {0, 1, 2, 3, 8, 10, 11}
    assert format_cpuset({11, 0, 1, 2, 3, 8, 10}) == "0-3,8,10-11"
    assert format_cpuset(set()) == ""


def test_take_by_topology_sockets_cores_threads():
    all_cpus = set(TOPO.cpus)
    sock0 = take_by_topology(TOPO, all_cpus, 8)                    # a whole socket
    assert {TOPO.cpus[c].socket for c in sock0} == {0} and len(sock0) == 8
    two_cores = take_by_topology(TOPO, all_cpus, 4)                # whole cores (both threads)
    assert len({TOPO.cpus[c].core for c in two_cores}) == 2
    avail = all_cpus - {0}                                         # core 0 of socket 0 half used
    one = take_by_topology(TOPO, avail, 1)
    assert one == {8}                                              # the sibling of the used thread first
    with pytest.raises(ValueError):
        take_by_topology(TOPO, {1, 2}, 3)


def test_static_policy_reserved_exclusive_shared_and_checkpoint(tmp_path):
    state = str(tmp_path / "cpu_manager_state")
    cm = CPUManager("static", TOPO, reserved_cpus_milli=1500, state_file=state)
    assert len(cm.reserved) == 2 and cm.reserved == {0, 8}          # ceil(1.5) CPUs = one whole core
    g = {"metadata": {"uid": "u1"}, "spec": {"containers": [
        {"name": "c", "resources": {"requests": {"cpu": "4", "memory": "1Gi"}, "limits": {"cpu": "4", "memory": "1Gi"}}}]}}
    cs = parse_cpuset(cm.allocate(g, g["spec"]["containers"][0]))
    assert len(cs) == 4 and not cs & cm.reserved
    frac = {"metadata": {"uid": "u2"}, "spec": {"containers": [
        {"name": "c", "resources": {"requests": {"cpu": "1500m", "memory": "1Gi"}, "limits": {"cpu": "1500m", "memory": "1Gi"}}}]}}
    assert parse_cpuset(cm.allocate(frac, frac["spec"]["containers"][0])) == cm.default_set()   # not integer: shared
    be = {"metadata": {"uid": "u3"}, "spec": {"containers": [{"name": "c"}]}}
    assert parse_cpuset(cm.allocate(be, be["spec"]["containers"][0])) == set(TOPO.cpus) - cs
    saved = json.load(open(state))
    assert saved["policyName"] == "static" and saved["entries"] == {"u1/c": format_cpuset(cs)}
    again = CPUManager("static", TOPO, reserved_cpus_milli=1500, state_file=state)   # restart keeps assignments
    assert again.assignments == {"u1/c": cs}
    again.release_pod("u1")
    assert again.default_set() == set(TOPO.cpus)
    json.dump({"policyName": "none", "entries": {}}, open(state, "w"))
    with pytest.raises(RuntimeError):                               # checkpoint from another policy
        CPUManager("static", TOPO, reserved_cpus_milli=1000, state_file=state)
    json.dump({"policyName": "static", "entries": {"a/b": "0-1", "c/d": "1-2"}}, open(state, "w"))
    with pytest.raises(RuntimeError):                               # overlapping assignments
        CPUManager("static", TOPO, reserved_cpus_milli=1000, state_file=state)
    with pytest.raises(ValueError):
        CPUManager("static", TOPO, reserved_cpus_milli=0)


def test_gpu_numa_preference():
    topo = CPUTopology.synthetic(2, 8, 2, numa_per_socket=2)       # 4 NUMA nodes of 4 cores
    cm = CPUManager("static", topo, reserved_cpus_milli=1000)
    pod = {"metadata": {"uid": "g"}, "spec": {"containers": [
        {"name": "c", "resources": {"requests": {"cpu": "4", "memory": "1Gi"}, "limits": {"cpu": "4", "memory": "1Gi"}}}]}}
    cs = parse_cpuset(cm.allocate(pod, pod["spec"]["containers"][0], prefer_numa={3}))
    assert {topo.cpus[c].numa for c in cs} == {3}
    big = {"metadata": {"uid": "h"}, "spec": {"containers": [
        {"name": "c", "resources": {"requests": {"cpu": "12", "memory": "1Gi"}, "limits": {"cpu": "12", "memory": "1Gi"}}}]}}
    cs2 = parse_cpuset(cm.allocate(big, big["spec"]["containers"][0], prefer_numa={3}))
    assert len(cs2) == 12 and not cs2 & cs                          # no room on node 3: anywhere


def test_static_cpu_manager_pins_containers_on_node(tmp_path):
    topo = CPUTopology.discover()
    if topo.num_cpus < 4:
        pytest.skip("needs ≥ 4 CPUs")

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"cpu_manager_policy": "static", "kube_reserved": "cpu=1",
                                            "cpu_manager_reconcile_period": 0.2}) as lc:
            c = lc.client
            show = ["sh", "-c", "grep Cpus_allowed_list /proc/self/status; sleep 30"]
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "shared"},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": show}]}}, "default")
            await wait_pod(c, "default", "shared", ("Running",), 20)
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "excl"},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": show,
                                                     "resources": {"limits": {"cpu": "2", "memory": "64Mi"}}}]}}, "default")
            await wait_pod(c, "default", "excl", ("Running",), 20)
            cm = lc.kubelet.cpu_manager
            excl_uid = m.uid_of(await c.get("pods", "excl", "default"))
            mine = cm.assignments[f"{excl_uid}/c"]
            for _ in range(50):
                logs = await c.logs("default", "excl")
                if "Cpus_allowed_list" in logs:
                    break
                await asyncio.sleep(0.1)
            assert parse_cpuset(logs.split()[-1]) == mine and len(mine) == 2 and not mine & cm.reserved
            # reconcile moves the shared container off the exclusive CPUs
            for _ in range(50):
                pid = next((x.pid for x in lc.shim.containers.values()
                            if x.labels.get("io.kubernetes.pod.name") == "shared" and x.state == 1), None)
                if pid and not (os.sched_getaffinity(pid) & mine):
                    break
                await asyncio.sleep(0.1)
            assert pid and not (os.sched_getaffinity(pid) & mine) and os.sched_getaffinity(pid) == cm.default_set()
            await c.delete("pods", "excl", "default", grace=0)
            for _ in range(100):
                if f"{excl_uid}/c" not in cm.assignments:
                    break
                await asyncio.sleep(0.05)
            assert not cm.assignments
    run(go(), 60)
