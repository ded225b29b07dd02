"""Kubelet features beyond the GPU path: activeDeadlineSeconds (pkg/kubelet/active_deadline.go),
node allocatable reservations (cm/node_container_manager.go), pod sysctls
(pkg/kubelet/sysctl/whitelist_test.go, validation.go sysctl annotations), OOM-kill reasons."""
import asyncio
import os

import pytest

from amdkube.api import meta as m
from amdkube.api.validation import validate_pod
from amdkube.kubelet.cm import node_allocatable, parse_reserved
from amdkube.kubelet.eviction import parse_thresholds
from amdkube.kubelet.sysctl import SAFE, SAFE_ANNOTATION, UNSAFE_ANNOTATION, Whitelist, validate_annotations
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


def test_active_deadline_fails_pod():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "dl"},
                            "spec": {"activeDeadlineSeconds": 1, "restartPolicy": "Never",
                                     "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}, "default")
            await wait_pod(c, "default", "dl", ("Running",), 20)
            p = await wait_pod(c, "default", "dl", ("Failed",), 20)
            assert p["status"]["reason"] == "DeadlineExceeded"
            assert "deadline" in p["status"]["message"]
            assert not any(x.state == 1 for x in lc.shim.containers.values())
    run(go(), 60)


def test_node_allocatable_subtracts_reservations_and_hard_eviction():
    cap = {"cpu": "8", "memory": "32Gi", "pods": "110", "amd.com/gpu": "8"}
    th = parse_thresholds("memory.available<100Mi,nodefs.available<10%")
    a = node_allocatable(cap, parse_reserved("cpu=500m,memory=1Gi"), parse_reserved("cpu=1,memory=512Mi"), th)
    assert a["cpu"] == "6500m"
    assert a["memory"] == f"{(32 * 1024 - 1024 - 512 - 100) * 1024}Ki"
    assert a["pods"] == "110" and a["amd.com/gpu"] == "8"
    with pytest.raises(ValueError):
        parse_reserved("amd.com/gpu=1")
    assert node_allocatable({"cpu": "1"}, parse_reserved("cpu=2"), {}, ())["cpu"] == "0"

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"kube_reserved": "cpu=250m,memory=256Mi", "cpu_capacity": 4,
                                            "memory_capacity": 8 << 30}) as lc:
            node = await lc.client.get("nodes", lc.node_name)
            assert node["status"]["capacity"]["cpu"] == "4"
            assert node["status"]["allocatable"]["cpu"] == "3750m"
            assert node["status"]["allocatable"]["memory"] == f"{(8 * 1024 - 256 - 100) * 1024}Ki"
    run(go(), 60)


def test_sysctl_validation_whitelist_and_admission():
    ok = {SAFE_ANNOTATION: "kernel.shm_rmid_forced=1", UNSAFE_ANNOTATION: "net.core.somaxconn=1024"}
    assert validate_annotations(ok) == []
    assert validate_annotations({SAFE_ANNOTATION: "Kernel.Bad=1"})
    assert validate_annotations({SAFE_ANNOTATION: "novalue"})
    assert any("safe and unsafe" in e for e in validate_annotations({SAFE_ANNOTATION: "a.b=1", UNSAFE_ANNOTATION: "a.b=2"}))
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d", "annotations": {SAFE_ANNOTATION: "a..b=1"}},
           "spec": {"containers": [{"name": "c", "image": "x"}]}}
    assert any("sysctls" in e for e in validate_pod(pod))
    with pytest.raises(ValueError):
        Whitelist(["kernel.panic"], UNSAFE_ANNOTATION)          # not namespaced
    safe = Whitelist(SAFE, SAFE_ANNOTATION)
    unsafe = Whitelist(["net.*", "kernel.msgmax"], UNSAFE_ANNOTATION)

    def pod_with(ann, **spec):
        return {"metadata": {"annotations": ann}, "spec": spec}
    assert safe.admit(pod_with({SAFE_ANNOTATION: "net.ipv4.tcp_syncookies=1"}))[0]
    assert safe.admit(pod_with({SAFE_ANNOTATION: "net.core.somaxconn=1"}))[1] == "SysctlForbidden"
    assert safe.admit(pod_with({SAFE_ANNOTATION: "net.ipv4.tcp_syncookies=1"}, hostNetwork=True))[1] == "SysctlForbidden"
    assert unsafe.admit(pod_with({UNSAFE_ANNOTATION: "net.core.somaxconn=1024,kernel.msgmax=1"}))[0]
    assert unsafe.admit(pod_with({UNSAFE_ANNOTATION: "kernel.msgmax=1"}, hostIPC=True))[1] == "SysctlForbidden"
    assert unsafe.admit(pod_with({UNSAFE_ANNOTATION: "kernel.sem=1"}))[1] == "SysctlForbidden"
    assert unsafe.admit(pod_with({UNSAFE_ANNOTATION: "bad"}))[1] == "InvalidSysctlAnnotation"

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False) as lc:
            await lc.client.create({"apiVersion": "v1", "kind": "Pod",
                                    "metadata": {"name": "sc", "annotations": {UNSAFE_ANNOTATION: "net.core.somaxconn=1024"}},
                                    "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "5"]}]}},
                                   "default")
            p = await wait_pod(lc.client, "default", "sc", ("Failed",), 20)
            assert p["status"]["reason"] == "SysctlForbidden", p["status"]
    run(go(), 60)


def test_oom_killed_reason_from_cgroup_memory_events(tmp_path):
    from amdkube.runtime.rocshim import RocShim
    shim = RocShim.__new__(RocShim)
    shim.isolation, shim.cgroup_root = "namespaces", str(tmp_path)

    class C_:
        sandbox_id, id, resources = "sb", "ct", {}
    d = tmp_path / "sb" / "ct"
    d.mkdir(parents=True)
    (d / "memory.events").write_text("low 0\nhigh 0\nmax 3\noom 1\noom_kill 0\n")
    assert not shim._oom_killed(C_())
    (d / "memory.events").write_text("low 0\nhigh 0\nmax 3\noom 1\noom_kill 1\n")
    assert shim._oom_killed(C_())
    shim.isolation = "env"
    assert not shim._oom_killed(C_())
