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


def test_image_gc_frees_unused_images_lru(tmp_path):
    """image_gc_manager_test.go: above the high threshold, unused images go least recently used
    first down to the low threshold; in-use, too-young and preloaded images stay."""
    from amdkube.kubelet.images import ImageGCManager

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False) as lc:
            c, k = lc.client, lc.kubelet
            srcs = []
            for i in range(3):
                d = tmp_path / f"img{i}"
                d.mkdir()
                (d / "run").write_text("#!/bin/sh\nsleep 30\n")
                os.chmod(d / "run", 0o755)
                (d / "payload").write_bytes(os.urandom(64 * 1024))
                srcs.append(str(d))
            for i, s in enumerate(srcs):
                await k.cri.pull_image(f"file://{s}")
            imgs = {i.repo_tags[0]: i for i in await k.cri.list_images()}
            names = [f"file://{s}:latest" for s in srcs]
            assert all(imgs[n].size >= 64 * 1024 for n in names)
            # image 2 is used by a running pod
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "user"},
                            "spec": {"containers": [{"name": "c", "image": f"file://{srcs[2]}"}]}}, "default")
            await wait_pod(c, "default", "user", ("Running",), 20)
            clock = [1000.0]
            gc = ImageGCManager(k.cri, high=90, low=80, min_age=60, clock=lambda: clock[0])
            await gc.detect()
            clock[0] += 30
            assert (await gc.free_space(10 ** 9)) == 0                 # every candidate is younger than min age
            clock[0] += 100
            await gc.detect()                                        # the running pod's image is "used" now
            clock[0] += 10
            gc.records[imgs[names[1]].id].last_used = clock[0] - 5    # image 1 used more recently than image 0
            freed = await gc.free_space(1)
            left = {i.repo_tags[0] for i in await k.cri.list_images()}
            assert freed >= 64 * 1024 and names[0] not in left and names[1] in left and names[2] in left
            freed = await gc.delete_unused()
            left = {i.repo_tags[0] for i in await k.cri.list_images()}
            assert names[1] not in left and names[2] in left and "busybox:latest" in left
            assert len(os.listdir(os.path.join(lc.shim.state_dir, "images"))) == 1   # only the in-use blob remains
            with pytest.raises(ValueError):
                ImageGCManager(k.cri, high=50, low=80)
            out = await ImageGCManager(k.cri, high=100, low=90).garbage_collect()
            assert 0 <= out["usage_percent"] <= 100 and out["freed"] == 0
    run(go(), 60)


def test_critical_pod_preemption_selection_and_admission():
    """preemption_test.go: the minimal victim set, best-effort first, distance-ordered; on a
    node without room a critical kube-system pod is admitted after evicting what it needs."""
    from amdkube.kubelet.preemption import pods_to_preempt

    def p(name, qos, cpu=None, mem=None, critical=False):
        res = {}
        if qos == "Guaranteed":
            res = {"requests": {"cpu": cpu, "memory": mem}, "limits": {"cpu": cpu, "memory": mem}}   # API-defaulted
        elif qos == "Burstable":
            res = {"requests": {k: v for k, v in (("cpu", cpu), ("memory", mem)) if v}}
        md = {"name": name, "namespace": "kube-system" if critical else "default", "uid": name}
        if critical:
            md["annotations"] = {"scheduler.alpha.kubernetes.io/critical-pod": ""}
        return {"metadata": md, "spec": {"containers": [{"name": "c", "resources": res}]}}
    pods = [p("be1", "BestEffort"), p("bu-small", "Burstable", "100m"), p("bu-big", "Burstable", "900m"),
            p("gu", "Guaranteed", "2", "1Gi"), p("crit", "Guaranteed", "4", "1Gi", critical=True)]
    names = lambda vs: sorted(m.name_of(v) for v in vs)   # noqa: E731
    assert names(pods_to_preempt(pods, {"cpu": 800})) == ["bu-big"]          # closest single burstable pod
    assert names(pods_to_preempt(pods, {"cpu": 2500})) == ["bu-big", "gu"]
    assert names(pods_to_preempt(pods, {"pods": 1})) == ["be1"]
    with pytest.raises(ValueError):
        pods_to_preempt(pods, {"cpu": 10000})                               # critical pods are never victims

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"cpu_capacity": 2, "feature_gates": "ExperimentalCriticalPodAnnotation=true"}) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "hog"},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"],
                                                     "resources": {"requests": {"cpu": "1500m"}}}]}}, "default")
            await wait_pod(c, "default", "hog", ("Running",), 20)
            crit = {"apiVersion": "v1", "kind": "Pod", "metadata": {
                "name": "crit", "namespace": "kube-system", "annotations": {"scheduler.alpha.kubernetes.io/critical-pod": ""}},
                "spec": {"nodeName": lc.node_name, "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"],
                                                                  "resources": {"requests": {"cpu": "1"}}}]}}
            await c.create(crit, "kube-system")
            await wait_pod(c, "kube-system", "crit", ("Running",), 40)
            hog = await wait_pod(c, "default", "hog", ("Failed",), 40)
            assert hog["status"]["reason"] == "Preempting"
    run(go(), 120)


def test_stats_summary_and_cadvisor_metrics(tmp_path):
    """server/stats summary: container cpu/memory/rootfs/logs, pod volumes (du) and
    ephemeral storage, node fs / imageFs / rlimit / kubelet system container; /metrics/cadvisor
    container_* families (pkg/kubelet/server/stats/summary_test.go, cadvisor prometheus tests)."""
    import aiohttp

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"volume_reconcile_period": 0.2}) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "writer"}, "spec": {
                "volumes": [{"name": "scratch", "emptyDir": {}}],
                "containers": [{"name": "w", "image": "busybox", "command": [
                    "sh", "-c", "head -c 2097152 /dev/zero > $AMDKUBE_ROOTFS/data/blob; echo logged; sleep 60"],
                    "volumeMounts": [{"name": "scratch", "mountPath": "/data"}]}]}}, "default")
            await wait_pod(c, "default", "writer", timeout=30)
            url = f"http://127.0.0.1:{lc.kubelet.server.port}"
            async with aiohttp.ClientSession() as s:
                pod = None
                for _ in range(100):
                    summ = await (await s.get(url + "/stats/summary")).json()
                    pod = next((p for p in summ["pods"] if p["podRef"]["name"] == "writer"), None)
                    vols = {v["name"]: v for v in (pod or {}).get("volume") or []}
                    if pod and vols.get("scratch", {}).get("usedBytes", 0) >= 2 << 20:
                        break
                    lc.kubelet.stats.du.forget("")      # re-measure (the du cache keeps results 10 s)
                    await asyncio.sleep(0.1)
                assert vols["scratch"]["usedBytes"] >= 2 << 20 and vols["scratch"]["capacityBytes"] > 0
                ctr = pod["containers"][0]
                assert ctr["name"] == "w" and ctr["memory"]["rssBytes"] > 0 and "usedBytes" in ctr["rootfs"]
                assert ctr["logs"]["usedBytes"] > 0
                assert pod["ephemeral-storage"]["usedBytes"] >= vols["scratch"]["usedBytes"]
                node = summ["node"]
                assert node["fs"]["capacityBytes"] > 0 and "usedBytes" in node["runtime"]["imageFs"]
                assert node["rlimit"]["maxpid"] > 0 and node["systemContainers"][0]["name"] == "kubelet"
                text = await (await s.get(url + "/metrics/cadvisor")).text()
            assert 'container_cpu_usage_seconds_total{container_name="w",pod_name="writer",namespace="default",cpu="total"}' in text
            assert "machine_cpu_cores " in text and "container_memory_working_set_bytes{" in text
    run(go(), 60)


def test_local_storage_capacity_isolation_eviction():
    """eviction_manager_test.go TestLocalStorageEviction: emptyDir over its sizeLimit and a
    container over its ephemeral-storage limit are evicted; a pod within its limits stays."""
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"feature_gates": "LocalStorageCapacityIsolation=true", "eviction_interval": 3600,
                                            "volume_reconcile_period": 0.2}) as lc:
            c = lc.client
            fill = "head -c 3145728 /dev/zero > $AMDKUBE_ROOTFS/d/blob; sleep 60"
            specs = {
                "hog": {"volumes": [{"name": "d", "emptyDir": {"sizeLimit": "1Mi"}}],
                        "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", fill],
                                        "volumeMounts": [{"name": "d", "mountPath": "/d"}]}]},
                "chatty": {"containers": [{"name": "c", "image": "busybox",
                                           "command": ["sh", "-c", "head -c 2097152 /dev/zero | tr '\\\\0' x; sleep 60"],
                                           "resources": {"limits": {"ephemeral-storage": "1Mi"}}}]},
                "fine": {"volumes": [{"name": "d", "emptyDir": {"sizeLimit": "100Mi"}}],
                         "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", fill],
                                         "volumeMounts": [{"name": "d", "mountPath": "/d"}],
                                         "resources": {"limits": {"ephemeral-storage": "50Mi"}}}]}}
            for name, spec in specs.items():
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name}, "spec": spec}, "default")
            for name in specs:
                await wait_pod(c, "default", name, timeout=30)
            evicted = set()
            for _ in range(60):          # until the writes have landed (slow under a loaded machine)
                lc.kubelet.stats.du.forget("")
                k = lc.kubelet
                evicted |= {m.name_of(p) for p in await k.eviction.local_storage_eviction(k.active_pods(), await k.stats.summary())}
                if evicted >= {"hog", "chatty"}:
                    break
                await asyncio.sleep(0.25)
            assert evicted == {"hog", "chatty"}, evicted
            # the status names the resource (eviction_manager.go evictPod): EmptyDir / ephemeral-storage
            for name, reason in (("hog", "low on resource: EmptyDir"), ("chatty", "low on resource: ephemeral-storage")):
                p = await wait_pod(c, "default", name, ("Failed",), 20)
                assert p["status"]["reason"] == "Evicted" and reason in p["status"]["message"], p["status"]
            assert (await c.get("pods", "fine", "default"))["status"]["phase"] == "Running"
    run(go(), 90)
