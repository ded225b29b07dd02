"""Kubelet behaviour on an in-process node. Ports the fork's node e2e
(test/e2e_node/gpu_device_plugin.go:45-143): GPU assignment survives a kubelet restart; a
second pod gets a different GPU; after the plugin is removed capacity drops to 0 while running
pods keep their GPUs, also across another kubelet restart. Plus restart policy / init
containers / readiness probes / admission rejection / volumes + downward env."""
import asyncio
import os

import pytest

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.kubelet.kubelet import Kubelet
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


def gpu_sleeper(name, secs=60):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", f"echo $ROCR_VISIBLE_DEVICES; sleep {secs}"],
                                     "resources": {"limits": {"amd.com/gpu": "1"}}}]}}


async def restart_kubelet(lc: LocalCluster):
    cfg = lc.kubelet.cfg
    await lc.kubelet.stop()
    await lc.kubelet.client.close()
    lc.kubelet = await Kubelet(Client(lc.api.url), cfg, smi_backend=lc.backend).start()


def test_gpu_assignment_survives_kubelet_and_plugin_restart():
    async def go():
        async with LocalCluster(gpus="fake", n_gpus=2, relist_period=0.2, node_status_update_frequency=0.5) as lc:
            c = lc.client
            await lc.wait_gpus(2)
            await c.create(gpu_sleeper("p1"))
            p1 = await wait_pod(c, "default", "p1", ("Running",), 20)
            g1 = p1["spec"]["extendedResources"][0]["assigned"]
            cid1 = p1["status"]["containerStatuses"][0]["containerID"]
            await restart_kubelet(lc)
            await asyncio.sleep(1.0)
            p1 = await c.get("pods", "p1", "default")
            assert p1["status"]["phase"] == "Running"
            assert p1["status"]["containerStatuses"][0]["containerID"] == cid1          # not restarted
            assert p1["spec"]["extendedResources"][0]["assigned"] == g1                  # same GPU
            await c.create(gpu_sleeper("p2"))
            p2 = await wait_pod(c, "default", "p2", ("Running",), 20)
            assert p2["spec"]["extendedResources"][0]["assigned"] != g1                  # different GPU
            # delete the device plugin: capacity → 0, running pods keep their GPUs
            await lc.plugin.stop()
            for _ in range(100):
                node = await c.get("nodes", lc.node_name)
                if (node["status"].get("capacity") or {}).get("amd.com/gpu") in (None, "0"):
                    break
                await asyncio.sleep(0.1)
            assert "amd.com/gpu" not in (node["status"].get("extendedResources") or {})
            await restart_kubelet(lc)
            await asyncio.sleep(1.0)
            for name, cid in (("p1", cid1),):
                p = await c.get("pods", name, "default")
                assert p["status"]["phase"] == "Running" and p["status"]["containerStatuses"][0]["containerID"] == cid
    run(go(), 120)


def test_restart_policy_init_containers_probes_and_volumes():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cfg", "namespace": "default"},
                            "data": {"greeting": "hello-cm"}})
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "w", "namespace": "default", "labels": {"app": "w"}},
                   "spec": {"restartPolicy": "OnFailure",
                            "volumes": [{"name": "work", "emptyDir": {}}, {"name": "cfg", "configMap": {"name": "cfg"}}],
                            "initContainers": [{"name": "init", "image": "busybox", "command": ["sh", "-c", "echo ready > $AMDKUBE_ROOTFS/work/flag"],
                                                "volumeMounts": [{"name": "work", "mountPath": "/work"}]}],
                            "containers": [{"name": "main", "image": "busybox",
                                            "command": ["sh", "-c", "cat $AMDKUBE_ROOTFS/work/flag; cat $AMDKUBE_ROOTFS/etc/cfg/greeting; echo; echo POD=$MY_POD; sleep 30"],
                                            "env": [{"name": "MY_POD", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}}],
                                            "volumeMounts": [{"name": "work", "mountPath": "/work"}, {"name": "cfg", "mountPath": "/etc/cfg"}],
                                            "readinessProbe": {"exec": {"command": ["true"]}, "periodSeconds": 1}}]}}
            await c.create(pod)
            p = await wait_pod(c, "default", "w", ("Running",), 20)
            for _ in range(100):
                p = await c.get("pods", "w", "default")
                if p["status"]["containerStatuses"][0]["ready"]:
                    break
                await asyncio.sleep(0.1)
            assert p["status"]["containerStatuses"][0]["ready"]
            assert p["status"]["initContainerStatuses"][0]["state"]["terminated"]["exitCode"] == 0
            logs = (await c.logs("default", "w", "main")).split()
            assert logs == ["ready", "hello-cm", "POD=w"], logs
            # OnFailure: failing container is restarted (restartCount increments)
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "crash", "namespace": "default"},
                            "spec": {"restartPolicy": "OnFailure", "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", "exit 1"]}]}})
            lc.kubelet.runtime.backoff.clear()
            lc.kubelet.runtime.backoff.default = 0.2
            for _ in range(150):
                p = await c.get("pods", "crash", "default")
                cs = (p["status"].get("containerStatuses") or [{}])[0]
                if cs.get("restartCount", 0) >= 1:
                    break
                await asyncio.sleep(0.1)
            assert cs.get("restartCount", 0) >= 1, p["status"]
    run(go(), 120)


def test_admission_rejects_pod_that_does_not_fit():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, kubelet_kw={"cpu_capacity": 2}) as lc:
            c = lc.client
            # bypass the scheduler (nodeName preset) so the kubelet's own admission decides
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "big", "namespace": "default"},
                            "spec": {"nodeName": lc.node_name, "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "5"],
                                                                                "resources": {"requests": {"cpu": "4"}}}]}})
            p = await wait_pod(c, "default", "big", ("Failed",), 20)
            assert p["status"]["reason"] == "OutOfcpu"
            # a GPU pod pinned to a node without an assignment is rejected by the DeviceManager
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "nogpu", "namespace": "default"},
                            "spec": {"nodeName": lc.node_name, "extendedResources": [{"name": "g", "resources": {"limits": {"amd.com/gpu": "1"}}}],
                                     "containers": [{"name": "c", "image": "busybox", "extendedResourceRequests": ["g"]}]}})
            p = await wait_pod(c, "default", "nogpu", ("Failed",), 20)
            assert p["status"]["reason"] == "UnexpectedAdmissionError"
    run(go(), 60)


def test_kubelet_http_api_and_metrics():
    async def go():
        async with LocalCluster(gpus="fake", n_gpus=2, relist_period=0.2) as lc:
            await lc.wait_gpus(2)
            await lc.client.create(gpu_sleeper("s", 20))
            await wait_pod(lc.client, "default", "s", ("Running",), 20)
            import aiohttp
            base = f"http://127.0.0.1:{lc.kubelet.server.port}"
            async with aiohttp.ClientSession() as s:
                assert (await (await s.get(base + "/healthz")).text()) == "ok"
                pods = await (await s.get(base + "/pods")).json()
                assert [p["metadata"]["name"] for p in pods["items"]] == ["s"]
                summ = await (await s.get(base + "/stats/summary")).json()
                assert len(summ["node"]["accelerators"]) == 2
                acc = summ["pods"][0]["containers"][0]["accelerators"]
                assert len(acc) == 1 and acc[0]["make"] == "amd"
                # VRAM is attributed by process: only what the container's own processes hold counts
                # (a partitioned GPU's device-level number would include its neighbours)
                from amdkube.smi import device_id
                smi = lc.kubelet.smi
                fake = getattr(smi, "inner", smi)
                idx = next(g["index"] for g in smi.gpus() if device_id(g) == acc[0]["id"])
                cid = next(x.id for x in await lc.kubelet.cri.list_containers() if x.metadata.name == "c")
                _, info = await lc.kubelet.cri.container_status(cid, verbose=True)
                fake.procs[idx] = [{"pid": int(info["pid"]), "vram_bytes": 123456789}, {"pid": 1, "vram_bytes": 5 << 30}]
                summ = await (await s.get(base + "/stats/summary")).json()
                assert summ["pods"][0]["containers"][0]["accelerators"][0]["memoryUsed"] == 123456789
                cad = await (await s.get(base + "/metrics/cadvisor")).text()
                assert 'container_accelerator_memory_total_bytes{container_name="c",pod_name="s"' in cad
                assert [ln for ln in cad.splitlines() if ln.startswith("container_accelerator_memory_used_bytes")][0] \
                    .endswith(" 123456789")
                met = await (await s.get(base + "/metrics")).text()
                assert "kubelet_device_plugin_registration_count" in met and "kubelet_pod_start_latency_microseconds" in met
                logs = await (await s.get(base + "/containerLogs/default/s/c")).text()
                assert logs.strip().startswith("GPU-")
    run(go(), 60)


def test_legacy_accelerators_gate_whole_gpu_allocation():
    """Accelerators gate (reference pkg/kubelet/gpu/nvidia/nvidia_gpu_manager_test.go):
    alpha.kubernetes.io/amd-gpu capacity from the render nodes, disjoint whole-GPU allocation,
    the shared /dev/kfd control node, request == limit validation, release on deletion."""
    import asyncio
    from amdkube.api import meta as m
    from amdkube.kubelet.gpu_legacy import ANNOTATION, RESOURCE
    from amdkube.localcluster import LocalCluster, wait_pod

    def pod(name, n):
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
                "spec": {"containers": [{"name": "c", "image": "amdkube/pause:3.1",
                                         "resources": {"limits": {RESOURCE: str(n)}}}]}}

    async def go():
        async with LocalCluster(gpus="fake", relist_period=0.2, kubelet_kw={"feature_gates": "Accelerators=true"}) as lc:
            c = lc.client
            for _ in range(100):
                node = await c.get("nodes", lc.node_name)
                if node["status"]["allocatable"].get(RESOURCE) == "8":
                    break
                await asyncio.sleep(0.05)
            assert node["status"]["capacity"][RESOURCE] == "8"
            await c.create(pod("a", 4), "default")
            await c.create(pod("b", 4), "default")
            for n in ("a", "b"):
                await wait_pod(c, "default", n, ("Running",), 20)
            devs = {}
            for ct in lc.shim.containers.values():
                paths = [d["host_path"] for d in ct.devices]
                assert any(p.endswith("/kfd") for p in paths)
                devs[ct.annotations.get("io.kubernetes.pod.name", ct.id)] = {p for p in paths if "renderD" in p}
                assert ct.annotations.get(ANNOTATION)
            sets = list(devs.values())
            assert len(sets) == 2 and all(len(s) == 4 for s in sets) and not (sets[0] & sets[1])
            # no GPUs left: the scheduler keeps the third pod pending
            await c.create(pod("c", 1), "default")
            await asyncio.sleep(0.5)
            assert (await c.get("pods", "c", "default"))["status"]["phase"] == "Pending"
            bad = pod("d", 1)
            bad["spec"]["containers"][0]["resources"]["requests"] = {RESOURCE: "2"}
            try:
                await c.create(bad, "default")
                raise AssertionError("request != limit must be rejected")
            except m.StatusError as e:
                assert e.code == 422
            # deleting a pod frees its GPUs for the pending one
            await c.delete("pods", "a", "default", grace=0)
            await wait_pod(c, "default", "c", ("Running",), 20)

    from tests.conftest import run
    run(go(), 90)


def test_legacy_gpu_manager_rebuild_after_restart():
    """In-use state comes back from running containers' annotations (reference
    nvidia_gpu_manager.go updateAllocatedGPUs), and terminated pods free their GPUs."""
    from amdkube.kubelet.gpu_legacy import ANNOTATION, RESOURCE, AMDGPUManager, LegacyGPUError

    class Smi:
        def gpus(self):
            return [{"render_minor": 128 + i, "uuid": f"GPU-{i}"} for i in range(4)]

    g = AMDGPUManager(Smi()).start()
    assert g.capacity() == 4
    g.rebuild([("u1", "c", {ANNOTATION: "/dev/dri/renderD128,/dev/dri/renderD129"})])
    pod = lambda uid, phase="Running": {"metadata": {"uid": uid, "name": uid}, "status": {"phase": phase}}
    ctr = {"name": "c", "resources": {"limits": {RESOURCE: "2"}}}
    a = g.allocate(pod("u2"), ctr, [pod("u1"), pod("u2")])
    assert a["annotations"][ANNOTATION] == "/dev/dri/renderD130,/dev/dri/renderD131"
    assert a["envs"]["ROCR_VISIBLE_DEVICES"] and a["devices"][0]["host_path"] == "/dev/kfd"
    assert g.allocate(pod("u2"), ctr, [pod("u1"), pod("u2")]) == a      # idempotent on restart
    try:
        g.allocate(pod("u3"), ctr, [pod("u1"), pod("u2"), pod("u3")])
        raise AssertionError("over-allocation")
    except LegacyGPUError:
        pass
    b = g.allocate(pod("u3"), ctr, [pod("u1", "Succeeded"), pod("u2"), pod("u3")])
    assert b["annotations"][ANNOTATION] == "/dev/dri/renderD128,/dev/dri/renderD129"


def test_full_status_event_merges_into_runtime_cache():
    """Evented PLEG with complete pod state (KEP-3386 ContainerEventResponse): one sandbox and
    all its containers are replaced, other sandboxes are kept, a removed sandbox disappears."""
    from amdkube.grpcdesc.cri import CRI as C
    from amdkube.kubelet.kuberuntime import ContainerRuntimeStatus, PodRuntimeStatus, apply_event

    def cs(cid, name, state, created):
        return C.ContainerStatus(id=cid, metadata=C.ContainerMetadata(name=name), state=state, created_at=created,
                                 annotations={"io.kubernetes.container.restartCount": "1"})
    rt = PodRuntimeStatus("u")
    rt.sandboxes = [("old", C.SANDBOX_NOTREADY, 0, 1)]
    rt.containers = {"c": [ContainerRuntimeStatus.from_cri(cs("c0", "c", C.CONTAINER_EXITED, 1), {}, "old")]}
    ev = C.ContainerEventResponse(
        container_id="c1", container_event_type=C.CONTAINER_STARTED_EVENT, created_at=10,
        pod_sandbox_status=C.PodSandboxStatus(id="new", metadata=C.PodSandboxMetadata(uid="u", attempt=1), state=C.SANDBOX_READY,
                                              created_at=5, network=C.PodSandboxNetworkStatus(ip="10.1.0.7")),
        containers_statuses=[cs("c1", "c", C.CONTAINER_RUNNING, 6)])
    ips = {}
    new = apply_event(rt, ev, ips)
    assert [s[0] for s in new.sandboxes] == ["new", "old"] and new.ip == "10.1.0.7" and ips == {"new": "10.1.0.7"}
    assert [c.id for c in new.containers["c"]] == ["c1", "c0"] and new.latest("c").restart_count == 1
    assert rt.sandboxes == [("old", C.SANDBOX_NOTREADY, 0, 1)]          # the input is never mutated
    gone = C.ContainerEventResponse(container_id="old", container_event_type=C.CONTAINER_DELETED_EVENT, created_at=11,
                                    pod_sandbox_status=C.PodSandboxStatus(id="old", metadata=C.PodSandboxMetadata(uid="u")))
    after = apply_event(new, gone, ips)
    assert [s[0] for s in after.sandboxes] == ["new"] and [c.id for c in after.containers["c"]] == ["c1"]


def test_container_gc_keeps_newest_dead_container_per_pod_container():
    """kuberuntime_gc_test.go: per (pod, container) the newest dead container stays for an
    active pod, all go for a deleted pod, dead sandboxes without containers are removed except
    an active pod's newest one, and container logs go with their containers."""
    import asyncio
    import os
    from amdkube.localcluster import LocalCluster, wait_pod

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"gc_period": 3600}) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "crash"},
                            "spec": {"restartPolicy": "OnFailure",
                                     "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", "exit 3"]}]}},
                           "default")
            await wait_pod(c, "default", "crash", ("Running", "Pending", "Failed"), 20)
            uid = (await c.get("pods", "crash", "default"))["metadata"]["uid"]
            # two more attempts of the same container, created the way a restart does; wait for
            # the kubelet's own first (immediate) restart to exit too, so the crash-loop back-off
            # (10 s) keeps it from adding attempts while the GC runs
            for _ in range(100):
                dead = [x for x in lc.shim.containers.values() if x.labels.get("io.kubernetes.pod.uid") == uid and x.state == 2]
                if len(dead) >= 2:
                    break
                await asyncio.sleep(0.05)
            assert len(dead) >= 2
            dead.sort(key=lambda x: x.created_at)
            sid = dead[0].sandbox_id
            import copy
            for i in range(2):
                clone = copy.copy(dead[0])
                clone.id = f"{dead[0].id[:-1]}{i}"
                clone.created_at = dead[0].created_at - (i + 1) * 10**9
                clone.log_path = dead[0].log_path + f".old{i}"
                open(clone.log_path, "w").write("old\n")
                lc.shim.containers[clone.id] = clone
            before = [(x.id, x.state, x.created_at) for x in lc.shim.containers.values() if x.labels.get("io.kubernetes.pod.uid") == uid]
            out = await lc.kubelet.container_gc()
            left = [x for x in lc.shim.containers.values() if x.labels.get("io.kubernetes.pod.uid") == uid]
            dead_before = [b for b in before if b[1] == 2]
            newest = max(dead_before, key=lambda b: b[2])[0]
            running = [b for b in before if b[1] != 2]
            assert out["containers"] == len(dead_before) - 1, (out, before)
            assert {x.id for x in left} == {newest} | {b[0] for b in running}
            assert not any(os.path.exists(dead[0].log_path + f".old{i}") for i in range(2))
            assert sid in lc.shim.sandboxes
            # once the pod is gone from the API, everything of it is collected
            await c.delete("pods", "crash", "default", grace=0)
            for _ in range(100):
                if not [x for x in lc.shim.containers.values() if x.labels.get("io.kubernetes.pod.uid") == uid] \
                        and sid not in lc.shim.sandboxes:
                    break
                await lc.kubelet.container_gc()
                await asyncio.sleep(0.05)
            assert sid not in lc.shim.sandboxes

    from tests.conftest import run
    run(go(), 60)


def test_status_from_events_waits_for_the_calls_final_event():
    """after StopPodSandbox the kubelet's runtime cache must come from the sandbox's
    own STOPPED event (the call's trailer names it), not from the per-container events the
    runtime emits first while the sandbox still shows READY; no-op calls need no event and an
    event that never comes falls back to a re-list."""
    import time
    from amdkube.grpcdesc.cri import CRI as C
    from amdkube.kubelet.cri_client import CURRENT_POD

    async def go():
        async with LocalCluster(gpus="none", relist_period=30, with_controllers=False) as lc:
            k, c = lc.kubelet, lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "ev"},
                            "spec": {"restartPolicy": "Never", "containers": [
                                {"name": n, "image": "busybox", "command": ["sleep", "60"]} for n in ("a", "b")]}}, "default")
            pod = await wait_pod(c, "default", "ev", ("Running",), 20)
            uid = m.uid_of(pod)
            for _ in range(100):
                if k._full_events and all(x.state == C.CONTAINER_RUNNING for x in lc.shim.containers.values()
                                          if x.labels.get("io.kubernetes.pod.uid") == uid):
                    break
                await asyncio.sleep(0.02)
            k.dispatch = lambda u: None          # keep the pod worker out of the way
            await asyncio.sleep(0.2)
            await k._cached_status(uid, fresh=True)
            token = CURRENT_POD.set(uid)
            try:
                k.cri.take_touched(uid)
                before = k.cri.pod_mutations(uid)
                await k.runtime.kill_pod(uid, 0, pod, k._cached_sandboxes(uid))
                assert k.cri.pod_mutations(uid) > before
                touched = k.cri.take_touched(uid)
            finally:
                CURRENT_POD.reset(token)
            assert len(touched) == 1 and all(ts > 0 for ts in touched.values()), touched
            rt = await k._status_from_events(uid, touched)
            assert rt is not None
            assert [sb[1] for sb in rt.sandboxes] == [C.SANDBOX_NOTREADY], rt.sandboxes
            assert all(x.state == C.CONTAINER_EXITED for lst in rt.containers.values() for x in lst)
            # a no-op mutation (stop an exited container) is already covered by the cache
            cid = next(x.id for x in lc.shim.containers.values() if x.labels.get("io.kubernetes.pod.uid") == uid)
            token = CURRENT_POD.set(uid)
            try:
                await k.cri.stop_container(cid, 0)
                noop = k.cri.take_touched(uid)
            finally:
                CURRENT_POD.reset(token)
            t0 = time.perf_counter()
            assert await k._status_from_events(uid, noop) is not None
            assert time.perf_counter() - t0 < 0.1
            # an event that never arrives: bounded wait, then None (the caller re-lists)
            t0 = time.perf_counter()
            assert await k._status_from_events(uid, {"f" * 32: time.time_ns() + 10**12}, timeout=0.05) is None
            assert time.perf_counter() - t0 < 0.5

    run(go(), 60)


def test_gc_treats_unknown_pods_as_deleted_only_when_sources_ready(tmp_path):
    """kuberuntime_gc.go:212-219, 299-309: with sources not ready an unknown pod keeps its
    newest dead container and sandbox; once ready, everything of it goes (and its pod dir);
    MaxContainers first cuts every unit to an equal share."""
    from types import SimpleNamespace as NS
    from amdkube.grpcdesc.cri import CRI as C
    from amdkube.kubelet.kuberuntime import RuntimeManager

    class FakeCRI:
        def __init__(self):
            self.sbs = [NS(id=f"s{i}", labels={"io.kubernetes.pod.uid": u}, state=C.SANDBOX_NOTREADY, created_at=i)
                        for i, u in enumerate(("gone", "gone", "live"))]
            self.conts = [NS(id=f"{u}-{n}-{i}", pod_sandbox_id=sid, labels={"io.kubernetes.pod.uid": u},
                             metadata=NS(name=n), state=C.CONTAINER_EXITED, created_at=100 + i)
                          for u, sid in (("gone", "s1"), ("live", "s2")) for n in ("x", "y") for i in range(3)]

        async def list_pod_sandbox(self):
            return list(self.sbs)

        async def list_containers(self):
            return list(self.conts)

        async def container_status(self, cid):
            return NS(log_path=""), {}

        async def remove_container(self, cid):
            self.conts = [c for c in self.conts if c.id != cid]

        async def remove_pod_sandbox(self, sid):
            self.sbs = [s for s in self.sbs if s.id != sid]

    (tmp_path / "pods" / "gone" / "logs").mkdir(parents=True)
    (tmp_path / "pods" / "live" / "logs").mkdir(parents=True)
    active = {"live"}.__contains__

    async def go():
        cri = FakeCRI()
        rm = RuntimeManager(cri, None, str(tmp_path))
        out = await rm.garbage_collect(active, 1, -1, sources_ready=False)
        assert sorted(c.id for c in cri.conts) == ["gone-x-2", "gone-y-2", "live-x-2", "live-y-2"]
        assert [s.id for s in cri.sbs] == ["s1", "s2"] and out["pod_dirs"] == 0
        assert (tmp_path / "pods" / "gone").exists()
        out = await rm.garbage_collect(active, 1, -1, sources_ready=True)
        assert sorted(c.id for c in cri.conts) == ["live-x-2", "live-y-2"]
        assert [s.id for s in cri.sbs] == ["s2"] and out["pod_dirs"] == 1
        assert not (tmp_path / "pods" / "gone").exists() and (tmp_path / "pods" / "live").exists()
        cri2 = FakeCRI()
        await rm.garbage_collect(lambda u: True, 3, 3, sources_ready=True)   # nothing on cri (rm bound to cri)
        rm2 = RuntimeManager(cri2, None, str(tmp_path))
        await rm2.garbage_collect(lambda u: True, -1, 3, sources_ready=True)
        # 4 units × 3 → share max(1, 3 // 4) = 1 each, then the oldest go until 3 remain
        assert sorted(c.id for c in cri2.conts) == ["gone-y-2", "live-x-2", "live-y-2"]

    run(go(), 30)


async def test_gpu_pod_waiting_on_a_volume_does_not_hold_the_device_start_window():
    """A GPU pod stuck on a missing ConfigMap leaves the kubelet's device-start set, so a
    device-less pod's first start is not delayed by device_pod_start_window (advisor r3)."""
    import time as _t
    from amdkube.localcluster import LocalCluster, wait_pod
    async with LocalCluster(gpus="fake", n_gpus=1, with_controllers=False, relist_period=0.2,
                            kubelet_kw={"device_pod_start_window": 1.0}) as lc:
        c = lc.client
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "gpu-stuck"},
                        "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"],
                                                 "resources": {"limits": {"amd.com/gpu": "1"}},
                                                 "volumeMounts": [{"name": "cfg", "mountPath": "/cfg"}]}],
                                 "volumes": [{"name": "cfg", "configMap": {"name": "does-not-exist"}}]}}, "default")
        end = _t.time() + 10
        seen = False
        while _t.time() < end:
            seen = seen or bool(lc.kubelet._device_starting)
            if seen and not lc.kubelet._device_starting:
                break
            await asyncio.sleep(0.02)
        assert seen and not lc.kubelet._device_starting
        t0 = _t.time()
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "plain"},
                        "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"]}]}}, "default")
        await wait_pod(c, "default", "plain", ("Running",), 20)
        assert _t.time() - t0 < 0.9, "the device-less pod waited out the device-start window"
