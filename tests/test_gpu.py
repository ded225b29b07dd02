"""GPU tier (real MI355X via gpurun). Ordering matters: every test that spawns processes
(pods, probes) runs before the tests that initialise HIP inside this pytest process.

Numerics: the HIP kernels are checked against a host fp32 reference (vector add compares
every element with |c - (a+b)| ≤ 1e-5; the HBM probe re-derives every written word).
"""
import asyncio
import json
import os
import subprocess
import time

import pytest

pytestmark = pytest.mark.gpu

from amdkube.localcluster import LocalCluster, wait_pod  # noqa: E402
from tests.conftest import run  # noqa: E402

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "amdkube", "_native", "bin")


def vadd_pod(name, gpu=True, args=("--print-uuid",)):
    c = {"name": "vadd", "image": "rocm/vector-add", "args": list(args)}
    if gpu:
        c["resources"] = {"limits": {"amd.com/gpu": "1"}}
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {"restartPolicy": "Never", "containers": [c]}}


def test_01_amdsmi_backend_enumerates_mi355x():
    from amdkube.smi import AmdSmiBackend, device_id, visibility_token
    b = AmdSmiBackend()
    gpus = b.gpus()
    assert gpus, "amd-smi found no GPU"
    g = gpus[0]
    assert g["gfx_target"] == "gfx950"
    assert g["vram_total_bytes"] >= 250 * 2 ** 30
    assert g["num_cu"] == 256
    assert visibility_token(g).startswith("GPU-")
    assert device_id(g)
    s = b.sample(0)
    assert "vram_used_bytes" in s
    topo = b.topology()
    assert topo[0][0]["type"] == "self"
    b.close()


def test_01b_ras_queries_and_new_fault_health():
    """The real RAS state reads without error (xGMI error status, bad pages, threshold, ECC
    blocks; "not supported"/"no permission" are legitimate answers on a VM or without root),
    and the delta monitor keeps the healthy part Healthy."""
    from amdkube.smi import AmdSmiBackend
    from amdkube.smi.health import HealthMonitor
    b = AmdSmiBackend()
    try:
        r = b.ras(0)
        print("ras:", r)
        ok_states = ("SUCCESS", "NOT_SUPPORTED", "NO_PERM", "NOT_YET_IMPLEMENTED", "FILE_ERROR")
        for k in ("bad_pages_status", "reserved_pages_status", "bad_page_threshold_status", "ecc_enabled_status",
                  "xgmi_ecc_status"):
            assert any(st in r[k] for st in ok_states), (k, r[k])
        # xGMI health has two sources; the error-status file answers INVAL on the gpurun box, the
        # XGMI_WAFL RAS block counts answer: at least one must
        assert "xgmi_error" in r or "xgmi_ecc_uncorrectable" in r, r
        if "xgmi_error" in r:
            assert r["xgmi_error"] in (0, 1, 2)
        assert "bad_pages" in r or "reserved_pages" in r, r
        hm = HealthMonitor(b)
        hm.snapshot(0)
        assert hm.check(0) == (True, ""), hm.check(0)
    finally:
        b.close()


def test_02_gpu_pod_runs_on_its_assigned_device():
    async def go():
        async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False) as lc:
            node = await lc.wait_gpus(1, 60)
            dev = node["status"]["extendedResources"]["amd.com/gpu"]["resources"]
            [did] = list(dev)
            assert dev[did]["attributes"]["amd.com/gfx"] == "gfx950"
            assert dev[did]["attributes"]["amd.com/gpu-type"] == "MI355X"
            await lc.client.create(vadd_pod("gpu-pod"))
            p = await wait_pod(lc.client, "default", "gpu-pod", ("Succeeded", "Failed"), 120)
            logs = await lc.client.logs("default", "gpu-pod")
            assert p["status"]["phase"] == "Succeeded", (p["status"], logs)
            assert "Test PASSED" in logs
            assert p["spec"]["extendedResources"][0]["assigned"] == [did]
            tok = lc.plugin.by_id[did]["hip_uuid"]
            assert f"uuid={tok}" in logs, logs
            # a pod without amd.com/gpu must not see the GPU (isolation)
            await lc.client.create(vadd_pod("cpu-pod", gpu=False, args=()))
            p = await wait_pod(lc.client, "default", "cpu-pod", ("Succeeded", "Failed"), 120)
            assert p["status"]["phase"] == "Failed", p["status"]
            cpu_logs = await lc.client.logs("default", "cpu-pod")
            assert "no GPU visible" in cpu_logs or "no ROCm-capable device" in cpu_logs, cpu_logs
    run(go(), 300)


def test_02c_device_guard_on_mi355x():
    """Enforced isolation on the real node (rocshim isolation=auto: Landlock on the unprivileged
    gpurun box). A non-GPU pod that unsets every *_VISIBLE_DEVICES still cannot reach the GPU
    (vector-add fails, /dev/kfd and the render node refuse to open); a GPU pod that unsets
    ROCR_VISIBLE_DEVICES still passes on its own device; mknod of a DRM node is refused by the
    kernel guard (EACCES from Landlock, before the capability check's EPERM)."""
    unset = "unset ROCR_VISIBLE_DEVICES HIP_VISIBLE_DEVICES CUDA_VISIBLE_DEVICES GPU_DEVICE_ORDINAL; "
    opener = ("import glob, os\n"
              "for p in ['/dev/kfd'] + sorted(glob.glob('/dev/dri/*')):\n"
              "    try:\n        os.close(os.open(p, os.O_RDWR)); print('OPENED', p)\n"
              "    except OSError as e:\n        print('refused', p, e.strerror)\n"
              "try:\n    os.mknod('/tmp/ak-mknod-226', 0o020600, os.makedev(226, 200)); print('MKNOD OK')\n"
              "except OSError as e:\n    print('mknod', e.strerror)\n")

    def pod(name, gpu, cmd):
        p = vadd_pod(name, gpu=gpu)
        c = p["spec"]["containers"][0]
        c["image"], c["command"], c["args"] = "busybox", ["sh", "-c", cmd], []
        return p

    async def go():
        async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False) as lc:
            assert lc.shim.isolation in ("landlock", "userns", "namespaces"), lc.shim.isolation_probe
            await lc.wait_gpus(1, 60)
            await lc.client.create(pod("escape", False, unset + f"exec {BIN}/rocm-vector-add"))
            await lc.client.create(pod("opener", False, unset + f"exec python3 -c \"{opener}\""))
            for name in ("escape", "opener"):
                await wait_pod(lc.client, "default", name, ("Succeeded", "Failed"), 120)
            p = await lc.client.get("pods", "escape", "default")
            logs = await lc.client.logs("default", "escape")
            assert p["status"]["phase"] == "Failed" and "Test PASSED" not in logs, (p["status"], logs)
            logs = await lc.client.logs("default", "opener")
            assert "OPENED" not in logs and "refused /dev/kfd" in logs, logs
            assert "mknod Permission denied" in logs, logs
            await lc.client.create(pod("gpu-unset", True, unset + f"exec {BIN}/rocm-vector-add --print-uuid"))
            p = await wait_pod(lc.client, "default", "gpu-unset", ("Succeeded", "Failed"), 120)
            logs = await lc.client.logs("default", "gpu-unset")
            assert p["status"]["phase"] == "Succeeded" and "Test PASSED" in logs, (p["status"], logs)
            [did] = p["spec"]["extendedResources"][0]["assigned"]
            assert f"uuid={lc.plugin.by_id[did]['hip_uuid']}" in logs, logs
            print("device guard:", lc.shim.isolation, lc.shim.isolation_probe)
    run(go(), 300)


def test_02d_rootfs_image_pod_on_mi355x(tmp_path):
    """A real image: a docker archive built here from rocm-vector-add plus its shared-library
    closure (everything but /opt/rocm, which comes from a hostPath volume and the rocm
    handler), pulled from file://, runs as a GPU pod from the image's own loader and libc."""
    import subprocess as sp
    from amdkube.runtime.oci import write_docker_archive
    vadd = os.path.join(BIN, "rocm-vector-add")
    files = {vadd: "usr/local/bin/rocm-vector-add"}
    for line in sp.run(["ldd", vadd], capture_output=True, text=True, check=True).stdout.splitlines():
        for tok in line.split():
            if tok.startswith("/") and os.path.exists(tok) and not tok.startswith("/opt/rocm"):
                files[tok] = tok.lstrip("/")
    entries, dirs = [], set()
    for src, rel in sorted(files.items(), key=lambda kv: kv[1]):
        d = os.path.dirname(rel)
        while d and d not in dirs:
            dirs.add(d)
            d = os.path.dirname(d)
        with open(os.path.realpath(src), "rb") as f:
            entries.append((rel, f.read(), 0o755, None))
    layer = [(d, None, 0o755, None) for d in sorted(dirs)] + entries
    if os.environ.get("_AMDKUBE_RETURN_LAYER"):
        return layer
    arch = str(tmp_path / "vadd-image.tar")
    write_docker_archive(arch, [layer], {"Entrypoint": ["/usr/local/bin/rocm-vector-add"], "Cmd": ["--print-uuid"],
                                         "Env": ["PATH=/usr/local/bin:/usr/bin:/bin"], "WorkingDir": "/"},
                         ["amdkube/vadd-rootfs:r3"])

    async def go():
        async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False) as lc:
            await lc.wait_gpus(1, 60)
            pod = vadd_pod("image-pod")
            c = pod["spec"]["containers"][0]
            c["image"], c["imagePullPolicy"], c["args"] = f"file://{arch}", "IfNotPresent", []
            c["volumeMounts"] = [{"name": "rocm", "mountPath": "/opt/rocm", "readOnly": True}]
            pod["spec"]["volumes"] = [{"name": "rocm", "hostPath": {"path": "/opt/rocm"}}]
            await lc.client.create(pod)
            p = await wait_pod(lc.client, "default", "image-pod", ("Succeeded", "Failed"), 120)
            logs = await lc.client.logs("default", "image-pod")
            assert p["status"]["phase"] == "Succeeded" and "Test PASSED" in logs, (p["status"], logs)
            [ct] = [x for x in lc.shim.containers.values() if x.name == "vadd"]
            assert ct.resources.get("rootfs"), ct.resources      # ran from the unpacked image
            [(name, spec)] = [(n, s) for n, s in lc.shim.images.images.items() if n.startswith("amdkube/vadd-rootfs")]
            assert len(spec["layers"]) == 1 and spec["size"] > 0
            print("rootfs image pod:", lc.shim.isolation, logs.strip().splitlines()[0])
    run(go(), 300)


def test_02e_registry_pulled_image_pod_on_mi355x(tmp_path, monkeypatch):
    """The same vector-add image served by an in-test Docker Registry v2 on localhost behind
    token auth: the pod's imagePullSecrets authenticate the pull, the layers are digest-checked
    and unpacked, and the image runs as a GPU pod on MI355X (round-3 review, registry pull)."""
    import base64
    from tests.fake_registry import FakeRegistry
    monkeypatch.setenv("_AMDKUBE_RETURN_LAYER", "1")
    layer = test_02d_rootfs_image_pod_on_mi355x(tmp_path)
    monkeypatch.delenv("_AMDKUBE_RETURN_LAYER")

    async def go():
        with FakeRegistry(users={"ci": "s3cret"}) as reg:
            reg.push("rocm/vadd", "r4", [layer], {"Entrypoint": ["/usr/local/bin/rocm-vector-add"], "Cmd": ["--print-uuid"],
                                                  "Env": ["PATH=/usr/local/bin:/usr/bin:/bin"], "WorkingDir": "/"})
            async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False) as lc:
                await lc.wait_gpus(1, 60)
                cfg = {"auths": {reg.host: {"auth": base64.b64encode(b"ci:s3cret").decode()}}}
                await lc.client.create({"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "regcred"},
                                        "type": "kubernetes.io/dockerconfigjson",
                                        "data": {".dockerconfigjson": base64.b64encode(json.dumps(cfg).encode()).decode()}},
                                       "default")
                pod = vadd_pod("registry-pod")
                c = pod["spec"]["containers"][0]
                c["image"], c["args"] = f"{reg.host}/rocm/vadd:r4", []
                c["volumeMounts"] = [{"name": "rocm", "mountPath": "/opt/rocm", "readOnly": True}]
                pod["spec"]["volumes"] = [{"name": "rocm", "hostPath": {"path": "/opt/rocm"}}]
                pod["spec"]["imagePullSecrets"] = [{"name": "regcred"}]
                await lc.client.create(pod)
                p = await wait_pod(lc.client, "default", "registry-pod", ("Succeeded", "Failed"), 180)
                logs = await lc.client.logs("default", "registry-pod")
                assert p["status"]["phase"] == "Succeeded" and "Test PASSED" in logs, (p["status"], logs)
                assert any(path.startswith("/token?") for _, path, _ in reg.log)
                print("registry image pod:", logs.strip().splitlines()[0])
    run(go(), 300)


def test_02b_legacy_accelerators_pod_on_real_gpu():
    """Accelerators gate (F22): alpha.kubernetes.io/amd-gpu from the real render nodes; the pod
    gets /dev/kfd + its render node + ROCR_VISIBLE_DEVICES and vector-add passes."""
    from amdkube.kubelet.gpu_legacy import ANNOTATION, RESOURCE

    async def go():
        async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False,
                                kubelet_kw={"feature_gates": "Accelerators=true"}) as lc:
            node = await lc.wait_gpus(1, 60)
            for _ in range(100):
                node = await lc.client.get("nodes", lc.node_name)
                if int(node["status"]["allocatable"].get(RESOURCE, "0")) >= 1:
                    break
                await asyncio.sleep(0.1)
            assert int(node["status"]["capacity"][RESOURCE]) >= 1
            pod = vadd_pod("legacy")
            pod["spec"]["containers"][0]["resources"] = {"limits": {RESOURCE: "1"}}
            await lc.client.create(pod)
            p = await wait_pod(lc.client, "default", "legacy", ("Succeeded", "Failed"), 120)
            logs = await lc.client.logs("default", "legacy")
            assert p["status"]["phase"] == "Succeeded" and "Test PASSED" in logs, (p["status"], logs)
            [ct] = [c for c in lc.shim.containers.values() if c.annotations.get(ANNOTATION)]
            assert any(d["host_path"].endswith("/kfd") for d in ct.devices)
            assert ct.env.get("ROCR_VISIBLE_DEVICES")
    run(go(), 300)


def test_03_plugin_hbm_health_probe_marks_healthy():
    async def go():
        async with LocalCluster(gpus="amdsmi", n_gpus=1, with_controllers=False, health_probe="hbm") as lc:
            node = await lc.wait_gpus(1, 120)
            devs = node["status"]["extendedResources"]["amd.com/gpu"]["resources"]
            assert all(d["health"] == "Healthy" for d in devs.values()), lc.plugin.reasons
    run(go(), 300)


def test_05_cpu_manager_exclusive_cpus_near_the_gpu():
    """Static CPU manager on the real node: a Guaranteed GPU pod gets exclusive CPUs, taken
    from its GPU's NUMA node (amd.com/numa-node from amd-smi) when that node has room, and the
    running workload is pinned to exactly them."""
    from amdkube.kubelet.cpumanager import CPUTopology, parse_cpuset
    topo = CPUTopology.discover()
    if topo.num_cpus < 4:
        pytest.skip("needs ≥ 4 allowed CPUs")

    async def go():
        async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False,
                                kubelet_kw={"cpu_manager_policy": "static", "kube_reserved": "cpu=1"}) as lc:
            node = await lc.wait_gpus(1, 60)
            [dev] = node["status"]["extendedResources"]["amd.com/gpu"]["resources"].values()
            numa = int(dev["attributes"].get("amd.com/numa-node", "-1"))
            pod = vadd_pod("pinned", args=("--print-uuid",))
            ct = pod["spec"]["containers"][0]
            ct["image"], ct["command"] = "busybox", ["sh", "-c", f"grep Cpus_allowed_list /proc/self/status && exec {BIN}/rocm-vector-add"]
            ct["args"] = []
            ct["resources"] = {"limits": {"amd.com/gpu": "1", "cpu": "2", "memory": "512Mi"}}
            await lc.client.create(pod)
            p = await wait_pod(lc.client, "default", "pinned", ("Succeeded", "Failed"), 120)
            logs = await lc.client.logs("default", "pinned")
            assert p["status"]["phase"] == "Succeeded" and "Test PASSED" in logs, (p["status"], logs)
            allowed = parse_cpuset(logs.split("Cpus_allowed_list:")[1].split()[0])
            assert len(allowed) == 2 and not allowed & lc.kubelet.cpu_manager.reserved, allowed
            local = {cpu for cpu, info in topo.cpus.items() if info.numa == numa} - lc.kubelet.cpu_manager.reserved
            if numa >= 0 and len(local) >= 2:
                assert allowed <= local, (allowed, numa)
    run(go(), 300)


def test_06_accelerator_stats_of_a_running_gpu_pod():
    """cAdvisor accelerator path on the real MI355X (F24, U18/U19): while a gpu-burn pod runs,
    /stats/summary attributes the busy GPU to its container (memory in use, duty cycle) and
    /metrics/cadvisor exports container_accelerator_* for it; the node lists the GPU too."""
    async def go():
        async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False) as lc:
            node = await lc.wait_gpus(1, 60)
            [did] = list(node["status"]["extendedResources"]["amd.com/gpu"]["resources"])
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "burn", "namespace": "default"},
                   "spec": {"restartPolicy": "Never", "containers": [{
                       "name": "burn", "image": "amdkube/gpu-burn", "args": ["--ms", "6000"],
                       "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
            await lc.client.create(pod)
            await wait_pod(lc.client, "default", "burn", ("Running",), 60)
            best, seen, text = {}, False, ""
            loop = asyncio.get_running_loop()
            end = loop.time() + 8
            while loop.time() < end:
                summ = await lc.kubelet.stats.summary()
                for ps in summ["pods"]:
                    if ps["podRef"]["name"] != "burn":
                        continue
                    for cs in ps["containers"]:
                        for acc in cs.get("accelerators") or []:
                            seen = True
                            assert acc["id"] == did and acc["make"] == "amd", acc
                            assert acc["memoryTotal"] >= 250 * 2 ** 30, acc
                            for k in ("memoryUsed", "dutyCycle"):
                                best[k] = max(best.get(k, 0), acc[k])
                if best.get("dutyCycle", 0) > 0 and best.get("memoryUsed", 0) > 0:
                    text = await lc.kubelet.stats.render_cadvisor()
                    break
                await asyncio.sleep(0.25)
            assert seen and best.get("dutyCycle", 0) > 0 and best.get("memoryUsed", 0) > 0, best
            assert f'container_accelerator_duty_cycle{{container_name="burn",pod_name="burn",namespace="default"' in text
            assert any(a["id"] == did for a in summ["node"]["accelerators"])
            p = await wait_pod(lc.client, "default", "burn", ("Succeeded", "Failed"), 60)
            assert p["status"]["phase"] == "Succeeded", p["status"]
    run(go(), 300)


def test_06b_hpa_scales_on_mi355x_activity(tmp_path):
    """The GPU autoscaling path on real hardware: amd-smi duty cycle of a gpu-burn pod →
    kubelet summary → metrics-server custom.metrics.k8s.io (behind the aggregator) → an
    autoscaling/v2beta1 HPA with a Pods metric on gpu_utilization scales its Deployment."""
    from amdkube.metrics import MetricsServer
    from tests.test_metrics_server import _ca, _leaf
    d = str(tmp_path)
    _ca(d, "serving-ca")
    scert, skey = _leaf(d, "serving-ca", "metrics", "metrics-server", server=True)

    async def go():
        kw = {"hpa_sync_period": 0.5, "hpa_upscale_delay": 0.0, "hpa_downscale_delay": 600.0}
        async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, controllers_kw=kw) as lc:
            c = lc.client
            await lc.wait_gpus(1, 60)
            ms = await MetricsServer(c, resolution=0.5, tls_cert=scert, tls_key=skey, authorize=False).start()
            try:
                await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "metrics-server", "namespace": "kube-system"},
                                "spec": {"ports": [{"port": 443, "targetPort": ms.port}]}})
                await c.create({"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "metrics-server", "namespace": "kube-system"},
                                "subsets": [{"addresses": [{"ip": "127.0.0.1"}], "ports": [{"port": ms.port}]}]})
                await c.create({"apiVersion": "apiregistration.k8s.io/v1beta1", "kind": "APIService",
                                "metadata": {"name": "v1beta1.custom.metrics.k8s.io"},
                                "spec": {"group": "custom.metrics.k8s.io", "version": "v1beta1", "groupPriorityMinimum": 100,
                                         "versionPriority": 100, "insecureSkipTLSVerify": True,
                                         "service": {"namespace": "kube-system", "name": "metrics-server"}}})
                tpl = {"metadata": {"labels": {"app": "burn"}}, "spec": {"containers": [{
                    "name": "burn", "image": "amdkube/gpu-burn", "args": ["--ms", "30000"],
                    "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
                await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "burn"},
                                "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "burn"}}, "template": tpl}}, "default")
                await c.request("POST", "/apis/autoscaling/v2beta1/namespaces/default/horizontalpodautoscalers", body={
                    "apiVersion": "autoscaling/v2beta1", "kind": "HorizontalPodAutoscaler", "metadata": {"name": "burn"},
                    "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": "burn"},
                             "minReplicas": 1, "maxReplicas": 2,
                             "metrics": [{"type": "Pods", "pods": {"metricName": "gpu_utilization", "targetAverageValue": "10"}}]}})
                loop = asyncio.get_running_loop()
                end, h, util = loop.time() + 90, None, None
                while loop.time() < end:
                    dep = await c.get("deployments", "burn", "default")
                    h = await c.request("GET", "/apis/autoscaling/v2beta1/namespaces/default/horizontalpodautoscalers/burn")
                    cur = (h.get("status") or {}).get("currentMetrics") or []
                    util = cur[0]["pods"]["currentAverageValue"] if cur else util
                    if dep["spec"]["replicas"] == 2:
                        break
                    await asyncio.sleep(0.5)
                print("hpa status:", json.dumps(h.get("status")))
                assert dep["spec"]["replicas"] == 2, (h.get("status"), util)
                assert float(util.rstrip("m")) / (1000 if util.endswith("m") else 1) > 10, util
                conds = {x["type"]: x for x in h["status"]["conditions"]}
                assert conds["ScalingActive"]["reason"] == "ValidMetricFound"
            finally:
                await ms.stop()
    run(go(), 200)


def test_07_native_activity_sampler_averages_a_burn():
    """The shim's background sampler (native/sampler_core.h via _amdsmi.start_sampler) on the
    real MI355X: while gpu-burn keeps the MFMA pipes busy for 2 s, the windowed mean over
    its samples is busy, and an idle window after it reads lower (gonvml AverageGPUUtilization)."""
    import time
    from amdkube.smi import AmdSmiBackend
    b = AmdSmiBackend()
    try:
        assert b.start_sampling(20.0)
        b.lib.start_sampler(20.0, 1024)   # restart at 20 ms even if an earlier test left one at 100 ms
        time.sleep(0.3)
        p = subprocess.run([os.path.join(BIN, "gpu-burn"), "--ms", "2000"], capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr
        busy = b.average_activity(0, 2.5)
        st = b.lib.sampler_state()
        assert st["running"] and st["ticks"] >= 50, st
        assert busy and busy["samples"] >= 50 and busy["span_s"] > 1.5, busy
        assert busy["gfx_activity"] > 20, busy
        time.sleep(1.5)
        idle = b.average_activity(0, 1.0)
        assert idle and idle["gfx_activity"] < busy["gfx_activity"], (idle, busy)
    finally:
        b.close()
    assert not b.lib.sampler_state()["running"]


def test_08_restart_continuity_and_exporter_scrape():
    """test/e2e_node/gpu_device_plugin.go:45-143 on MI355X: a running gpu-burn pod keeps its
    device across a kubelet restart and while the device plugin is down (capacity 0), capacity
    returns without flapping when the plugin comes back, a second 1-GPU pod waits until the
    first one ends; the amd-smi exporter attributes the busy GPU's series to the pod."""
    import aiohttp
    from amdkube.client import Client
    from amdkube.deviceplugin.amd import make_plugins
    from amdkube.kubelet.kubelet import Kubelet
    from amdkube.monitoring.exporter import Exporter

    def burn(name, ms):
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
                "spec": {"restartPolicy": "Never", "containers": [{
                    "name": "burn", "image": "amdkube/gpu-burn", "args": ["--ms", str(ms)],
                    "resources": {"limits": {"amd.com/gpu": "1"}}}]}}

    async def capacity(lc):
        node = await lc.client.get("nodes", lc.node_name)
        return (node["status"].get("capacity") or {}).get("amd.com/gpu", "0")

    async def go():
        async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, node_status_update_frequency=0.5,
                                with_controllers=False) as lc:
            await lc.wait_gpus(1, 60)
            await lc.client.create(burn("burn", 25000))
            p = await wait_pod(lc.client, "default", "burn", ("Running",), 60)
            assigned = p["spec"]["extendedResources"][0]["assigned"]
            cid = p["status"]["containerStatuses"][0]["containerID"]
            # exporter scrape while the burn runs: series attributed to the pod
            ex = await Exporter(lc.backend, node=lc.node_name,
                                kubelet_url=f"http://127.0.0.1:{lc.kubelet.server.port}").start("127.0.0.1", 0)
            try:
                await asyncio.sleep(1.0)
                async with aiohttp.ClientSession() as s:
                    async with s.get(f"http://127.0.0.1:{ex.port}/metrics") as r:
                        text = await r.text()
            finally:
                await ex.stop()
            for series in ("amd_gpu_utilization_percent", "amd_gpu_vram_used_bytes", "amd_gpu_power_watts",
                           "amd_gpu_temperature_celsius", "amd_gpu_ecc_uncorrectable_total"):
                lines = [ln for ln in text.splitlines() if ln.startswith(series + "{")]
                assert lines and all('pod="burn"' in ln and 'namespace="default"' in ln for ln in lines), (series, lines)
            # kubelet restart: same container, same GPU
            cfg = lc.kubelet.cfg
            await lc.kubelet.stop()
            lc.kubelet = await Kubelet(Client(lc.api.url, token=lc.api.loopback_token), cfg, smi_backend=lc.backend).start()
            await asyncio.sleep(1.5)
            p = await lc.client.get("pods", "burn", "default")
            assert p["status"]["phase"] == "Running" and p["status"]["containerStatuses"][0]["containerID"] == cid, p["status"]
            assert p["spec"]["extendedResources"][0]["assigned"] == assigned
            # a second 1-GPU pod waits: the node's only GPU is taken
            await lc.client.create(burn("second", 500))
            # plugin down: capacity → 0, the burn keeps running
            for pl in lc.plugins:
                await pl.stop()
            for _ in range(100):
                if await capacity(lc) == "0":
                    break
                await asyncio.sleep(0.1)
            assert await capacity(lc) == "0"
            p = await lc.client.get("pods", "burn", "default")
            assert p["status"]["phase"] == "Running" and p["status"]["containerStatuses"][0]["containerID"] == cid
            # plugin back: capacity returns and stays (no flap)
            lc.plugins = make_plugins(lc.backend, lc.resource_naming, plugins_dir=os.path.join(lc.base, "plugins"),
                                      health_interval=5.0, health_probe="none")
            for pl in lc.plugins:
                await pl.start()
            lc.plugin = lc.plugins[0]
            for _ in range(100):
                if await capacity(lc) == "1":
                    break
                await asyncio.sleep(0.1)
            seen = []
            for _ in range(20):
                seen.append(await capacity(lc))
                await asyncio.sleep(0.1)
            assert set(seen) == {"1"}, seen
            p2 = await lc.client.get("pods", "second", "default")
            assert p2["status"]["phase"] == "Pending" and not p2["spec"].get("nodeName"), p2["status"]
            # the first ends → the second runs on the freed GPU
            p = await wait_pod(lc.client, "default", "burn", ("Succeeded", "Failed"), 60)
            assert p["status"]["phase"] == "Succeeded", p["status"]
            p2 = await wait_pod(lc.client, "default", "second", ("Succeeded", "Failed"), 90)
            assert p2["status"]["phase"] == "Succeeded" and p2["spec"]["extendedResources"][0]["assigned"] == assigned
    run(go(), 240)


def test_09_gpu_pods_over_a_raft_store_with_protobuf_and_spdy_exec(tmp_path):
    """The control plane's HA store on the MI355X node: the apiserver keeps its objects in a
    3-member `amdkube etcd` raft group in the reference's protobuf storage format; a kubectl-style
    SPDY exec runs vector-add INSIDE a running GPU pod's container (its device guard) and
    passes, the same exec in a GPU-less pod finds no GPU; the store's leader is killed and
    the next GPU pod still schedules and runs."""
    import grpc
    from amdkube.api import protobuf as pb
    from amdkube.client.stream import exec_stream
    from amdkube.grpcdesc.etcd import ETCD as E
    from amdkube.store.etcd3 import Etcd3Store
    from tests.test_raft import Cluster

    def burn(name, ms, gpu=True):
        c = {"name": "burn", "image": "amdkube/gpu-burn", "args": ["--ms", str(ms)]}
        if gpu:
            c["resources"] = {"limits": {"amd.com/gpu": "1"}}
        else:
            c = {"name": "plain", "image": "busybox", "command": ["sleep", str(ms // 1000)]}
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
                "spec": {"restartPolicy": "Never", "containers": [c]}}

    async def go():
        cl = Cluster(tmp_path)
        for nm in cl.names:
            cl.start(nm)
        store = None
        try:
            leader = await asyncio.to_thread(cl.leader)
            store = await asyncio.to_thread(Etcd3Store, list(cl.client.values()))
            async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False,
                                    api_kw={"store": store, "options": {"storage_media_type": pb.MEDIA_TYPE}}) as lc:
                await lc.wait_gpus(1, 60)
                c = lc.client
                await c.create(burn("burner", 20000))
                await c.create(burn("plain", 120000, gpu=False))      # outlives both execs
                t0 = time.monotonic()
                await wait_pod(c, "default", "burner", ("Running",), 60)
                await wait_pod(c, "default", "plain", ("Running",), 60)
                print(f"test_09: both pods running after {time.monotonic() - t0:.2f}s", flush=True)
                # the object as the store holds it: protobuf, replicated to every member
                for nm in cl.names:
                    with grpc.insecure_channel(cl.client[nm]) as ch:
                        r = E.KV.stub(ch).Range(E.RangeRequest(key=b"/registry/pods/default/burner", serializable=True),
                                                timeout=5)
                    assert r.kvs and r.kvs[0].value[:4] == b"k8s\x00", nm
                vadd = os.path.join(BIN, "rocm-vector-add")
                out, err = bytearray(), bytearray()
                rc = await exec_stream(c, "default", "burner", [vadd], on_stdout=out.extend, on_stderr=err.extend,
                                       transport="spdy")
                assert rc == 0 and b"Test PASSED" in out, (rc, bytes(out[-400:]), bytes(err[-400:]))
                print(f"test_09: exec in the GPU pod done at {time.monotonic() - t0:.2f}s", flush=True)
                out, err = bytearray(), bytearray()
                rc = await exec_stream(c, "default", "plain", [vadd], on_stdout=out.extend, on_stderr=err.extend,
                                       transport="spdy")
                assert rc != 0 and b"Test PASSED" not in out, (rc, bytes(out[-400:]))
                p = await wait_pod(c, "default", "burner", ("Succeeded", "Failed"), 90)
                assert p["status"]["phase"] == "Succeeded", p["status"]
                # lose the store's leader: a new one is elected and the node keeps working
                cl.kill(leader)
                await asyncio.to_thread(cl.leader, [n for n in cl.names if n != leader])
                await c.create(vadd_pod("after-failover"))
                p = await wait_pod(c, "default", "after-failover", ("Succeeded", "Failed"), 120)
                assert p["status"]["phase"] == "Succeeded", p["status"]
                assert "Test PASSED" in await c.logs("default", "after-failover")
        finally:
            if store is not None:
                store.close()
            cl.stop()
    run(go(), 400)


def test_04a_xgmi_probe_gang_pod_runs_rccl_on_exactly_its_gpus():
    """BASELINE config 4 / SURVEY §7.7: the RCCL probe runs as a pod on the GPUs the scheduler
    bound. A gang of min(4, node GPUs) is requested; inside the pod RCCL opens exactly that many
    ranks, its all-reduce sums are right, and the PCI buses of the GPUs the communicator opened
    are exactly the amd.com/pci-bus attributes of spec.extendedResources[].assigned (the device
    list the container was given, docker_container.go:155-172)."""
    from amdkube.smi import AmdSmiBackend
    b = AmdSmiBackend()
    n_node = len(b.gpus())
    b.close()
    k = min(4, n_node)

    async def go():
        async with LocalCluster(gpus="amdsmi", relist_period=0.5, with_controllers=False) as lc:
            node = await lc.wait_gpus(k, 60)
            await lc.client.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "xgmi", "namespace": "default"},
                                    "spec": {"restartPolicy": "Never", "containers": [{
                                        "name": "probe", "image": "amdkube/xgmi-probe:latest",
                                        "args": ["--max-mib", "16", "--iters", "2"],
                                        "resources": {"limits": {"amd.com/gpu": str(k)}}}]}})
            pod = await wait_pod(lc.client, "default", "xgmi", ("Succeeded", "Failed"), 180)
            logs = await lc.client.logs("default", "xgmi")
            assert pod["status"]["phase"] == "Succeeded", (pod["status"], logs[-2000:])
            x = json.loads(logs[logs.index("{\"gpus\""):logs.rindex("}") + 1])
            assigned = [d for er in pod["spec"]["extendedResources"] for d in er["assigned"]]
            assert len(assigned) == k and x["gpus"] == k and x["verify"]["ranks"] == k and x["verify"]["wrong"] == 0, x
            attrs = node["status"]["extendedResources"]["amd.com/gpu"]["resources"]
            want = sorted(attrs[d]["attributes"]["amd.com/pci-bus"].replace("-", ":").lower() for d in assigned)
            got = sorted(d["bus"].lower() for d in x["devices"])
            assert got == want, (got, want, assigned)
            print("xgmi-probe pod:", k, "rank(s) on", got, "busbw", [r["busbw_gbps"] for r in x["allreduce"]])
    run(go(), 400)


def _xgmi_pod(name, k, sizes_mib=256):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {"restartPolicy": "Never", "containers": [{
                "name": "probe", "image": "amdkube/xgmi-probe:latest",
                "args": ["--max-mib", str(sizes_mib), "--iters", "5"],
                "resources": {"limits": {"amd.com/gpu": str(k)}}}]}}


def _per_link_gbps(b, idx: list[int]) -> float | None:
    """The xGMI per-link bandwidth amd-smi reports between the given GPUs (the driver's max of
    amdsmi_get_minmax_bandwidth_between_processors, MB/s; else link_metrics max_bandwidth)."""
    topo = b.topology()
    vals = [topo[i][j].get("max_bw_mbps") for i in idx for j in idx if i != j]
    vals = [v / 1000.0 for v in vals if v]
    if vals:
        return min(vals)
    for i in idx:
        lm = [x.get("max_bandwidth_gbps") for x in b.link_metrics(i) if x.get("max_bandwidth_gbps")]
        if lm:
            return float(min(lm))
    return None


def test_04c_xgmi_allreduce_bandwidth_at_expectation():
    """BASELINE config 4: an xgmi-probe pod on min(4, n) GPUs measures the RCCL all-reduce at
    256 MiB; its bus bandwidth must reach at least half the per-link xGMI bandwidth amd-smi
    reports (a PCIe fallback would not). With n >= 8, two 4-GPU probe pods run at once on
    disjoint sets that each sit in one NUMA domain. On a 1-GPU node there is no link: the
    bandwidth assertion is skipped with the reason, the pod must still run and verify."""
    from amdkube.smi import AmdSmiBackend
    b = AmdSmiBackend()
    n_node = len(b.gpus())
    k = min(4, n_node)

    async def go():
        async with LocalCluster(gpus="amdsmi", relist_period=0.5, with_controllers=False) as lc:
            node = await lc.wait_gpus(k, 60)
            attrs = node["status"]["extendedResources"]["amd.com/gpu"]["resources"]
            names = ["bw-a", "bw-b"] if n_node >= 8 else ["bw-a"]
            for nm in names:
                await lc.client.create(_xgmi_pod(nm, k))
            out = {}
            for nm in names:
                pod = await wait_pod(lc.client, "default", nm, ("Succeeded", "Failed"), 240)
                logs = await lc.client.logs("default", nm)
                assert pod["status"]["phase"] == "Succeeded", (pod["status"], logs[-2000:])
                x = json.loads(logs[logs.index("{\"gpus\""):logs.rindex("}") + 1])
                assert x["verify"]["wrong"] == 0 and x["gpus"] == k, x
                out[nm] = (pod, x)
            if len(names) == 2:
                sets = [set(d for er in out[nm][0]["spec"]["extendedResources"] for d in er["assigned"]) for nm in names]
                assert not (sets[0] & sets[1]), sets
                for s_ in sets:
                    numa = {attrs[d]["attributes"].get("amd.com/numa-node") for d in s_}
                    assert len(numa) == 1, (s_, numa)
            if k < 2:
                print("xgmi bandwidth assertion skipped: 1 GPU on this node, no xGMI link to measure")
                return
            for nm in names:
                pod, x = out[nm]
                assigned = [d for er in pod["spec"]["extendedResources"] for d in er["assigned"]]
                idx = [int(attrs[d]["attributes"]["amd.com/index"]) for d in assigned]
                link = _per_link_gbps(b, idx)
                big = max(x["allreduce"], key=lambda r: r["bytes"])
                assert big["bytes"] >= 256 << 20, x["allreduce"]
                if link is None:
                    pytest.skip("amd-smi reports no xGMI link bandwidth on this node")
                assert big["busbw_gbps"] >= 0.5 * link, (nm, big, link)
                print(f"{nm}: all-reduce busbw {big['busbw_gbps']:.1f} GB/s >= 0.5 x {link:.1f} GB/s per link")
    try:
        run(go(), 600)
    finally:
        b.close()


def test_03b_gpu_selector_pods_on_real_attributes():
    """BASELINE config 3: a pod asking for min(4, n) GPUs with `amd.com/gpu-type In [MI355X]`
    and `amd.com/gpu-memory Gt 262143` (MiB) runs to Succeeded on the assigned GPUs of the real
    amd-smi backend; one asking for `gpu-memory Gt 1000000` stays Pending with a
    FailedScheduling event."""
    from amdkube.smi import AmdSmiBackend
    b = AmdSmiBackend()
    k = min(4, len(b.gpus()))
    b.close()

    def sel_pod(name, mem_gt):
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
                "spec": {"restartPolicy": "Never",
                         "extendedResources": [{"name": "gpus", "resources": {"limits": {"amd.com/gpu": str(k)}},
                                                "affinity": {"required": [
                                                    {"key": "amd.com/gpu-type", "operator": "In", "values": ["MI355X"]},
                                                    {"key": "amd.com/gpu-memory", "operator": "Gt", "values": [str(mem_gt)]}]}}],
                         "containers": [{"name": "vadd", "image": "rocm/vector-add", "args": ["--print-uuid"],
                                         "extendedResourceRequests": ["gpus"]}]}}

    async def go():
        async with LocalCluster(gpus="amdsmi", relist_period=0.5, with_controllers=False) as lc:
            node = await lc.wait_gpus(k, 60)
            attrs = node["status"]["extendedResources"]["amd.com/gpu"]["resources"]
            await lc.client.create(sel_pod("fits", 262143))
            p = await wait_pod(lc.client, "default", "fits", ("Succeeded", "Failed"), 180)
            logs = await lc.client.logs("default", "fits")
            assert p["status"]["phase"] == "Succeeded" and "Test PASSED" in logs, (p["status"], logs[-1500:])
            assigned = p["spec"]["extendedResources"][0]["assigned"]
            assert len(assigned) == k
            for d in assigned:
                assert attrs[d]["attributes"]["amd.com/gpu-type"] == "MI355X"
                assert int(attrs[d]["attributes"]["amd.com/gpu-memory"]) > 262143
            await lc.client.create(sel_pod("too-big", 1000000))
            deadline = time.time() + 30
            why = None
            while time.time() < deadline and why is None:
                evs, _ = await lc.client.list("events", "default")
                why = next((e for e in evs if (e.get("involvedObject") or {}).get("name") == "too-big"
                            and e.get("reason") == "FailedScheduling"), None)
                await asyncio.sleep(0.3)
            assert why is not None, "no FailedScheduling event"
            p = await lc.client.get("pods", "too-big", "default")
            assert p["status"]["phase"] == "Pending" and not p["spec"].get("nodeName")
            print("selector pod ran on", assigned, "| unsatisfiable one:", why.get("message"))
    run(go(), 300)


def test_04_probe_binaries():
    r = subprocess.run([os.path.join(BIN, "hbm-probe"), "--mib", "1024", "--iters", "3"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["errors"] == 0 and d["copy_gbps"] > 2000, d
    r = subprocess.run([os.path.join(BIN, "xgmi-probe"), "--max-mib", "16", "--iters", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    try:
        x = json.loads(r.stdout[r.stdout.index("{"):r.stdout.rindex("}") + 1])
    except ValueError as e:
        raise AssertionError(f"xgmi-probe output is not JSON ({e}): {r.stdout[:800]!r}")
    # rank-dependent inputs, every element of the sum checked on every rank (right at any N)
    assert x["verify"]["wrong"] == 0 and x["verify"]["ranks"] == x["gpus"] >= 1 and x["verify"]["elements"] > 0, x
    r = subprocess.run([os.path.join(BIN, "gpu-burn"), "--ms", "100"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and json.loads(r.stdout)["bf16_tflops"] > 500, r.stdout


def test_04b_hsa_vector_add_matches_the_hip_build():
    """The pod workload on the bare ROCr runtime (AQL dispatch of the embedded gfx950 code
    object): every element checked on the host for ragged sizes, and the same device identity
    (UUID, PCI bus, ISA) as the HIP build reports."""
    def run_one(binary, *args):
        r = subprocess.run([os.path.join(BIN, binary), "--json", *args], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0 and "Test PASSED" in r.stdout, (binary, args, r.stdout, r.stderr)
        return json.loads(next(x for x in r.stdout.splitlines() if x.startswith("{")))
    hip_id = run_one("rocm-vector-add")
    for n in ("50000", "50001", "7", "1", "1048579"):
        d = run_one("hsa-vector-add", "-n", n)
        assert d["ok"] and d["runtime"] == "hsa" and d["n"] == int(n)
        assert (d["uuid"], d["bus"], d["arch"]) == (hip_id["uuid"], hip_id["bus"], hip_id["arch"]), (d, hip_id)
    r = subprocess.run([os.path.join(BIN, "hsa-vector-add"), "--expect-devices", "2"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and "expected 2 visible GPU(s), found 1" in r.stderr


# --- in-process HIP from here on (no process spawning after this point) -------------------
def test_90_hip_vector_add_matches_fp32_reference():
    from amdkube.ops import hip
    for n in (1, 3, 50000, 1 << 22, (1 << 22) + 7):
        r = hip.vector_add(n, 0)
        assert r["ok"] and r["mismatches"] == 0, (n, r)


def test_91_hip_hbm_probe_pattern_and_bandwidth():
    from amdkube.ops import hip
    r = hip.hbm_probe(1024, 3, 0)
    assert r["errors"] == 0
    assert r["read_gbps"] > 3000 and r["copy_gbps"] > 2000, r


def test_93_mfma_tile_matches_torch_fp32():
    """One wave's 32x32x16 bf16 MFMA chain on Python-supplied A/B vs torch's fp32 matmul of the
    same bf16 values: a wrong operand or accumulator layout fails this, whatever the burn rate."""
    import torch
    from amdkube.ops import hip
    g = torch.Generator().manual_seed(7)
    for k in (16, 64, 256):
        a = torch.randn(32, k, generator=g)
        b = torch.randn(k, 32, generator=g)
        c = hip.mfma_tile(a, b)
        ref = a.to(torch.bfloat16).float() @ b.to(torch.bfloat16).float()
        err = (c - ref).abs().max().item()
        assert err <= 1e-4 * max(1.0, ref.abs().max().item()) * (k / 16), (k, err)
    # structure, not just magnitude: a one-hot A picks out rows of B exactly
    a = torch.zeros(32, 16)
    a[torch.arange(32), torch.arange(32) % 16] = 1.0
    b = torch.arange(16 * 32, dtype=torch.float32).reshape(16, 32) / 64
    assert torch.equal(hip.mfma_tile(a, b), b.to(torch.bfloat16).float()[torch.arange(32) % 16])


def test_94_vector_add_on_torch_inputs():
    import torch
    from amdkube.ops import hip
    g = torch.Generator().manual_seed(3)
    for n in (1, 7, 50000, (1 << 20) + 3):
        a, b = torch.randn(n, generator=g), torch.randn(n, generator=g)
        assert torch.equal(hip.vector_add_tensors(a, b), a + b), n     # fp32 add: bit-exact


def test_95_hbm_pattern_verify_copy_against_host_reference():
    import numpy as np
    import torch
    from amdkube.ops import hip
    n16, seed = (1 << 16) + 5, 0x5EED
    got = hip.hbm_pattern(n16, seed)
    # re-derive the probe's address hash on the host (uint32 arithmetic)
    i = np.arange(n16, dtype=np.uint64)
    base = ((i * 4) & 0xFFFFFFFF) ^ seed ^ ((i >> 30) & 0xFFFFFFFF)

    def mix32(x):
        x = x & 0xFFFFFFFF
        x ^= x >> 16
        x = (x * 0x7FEB352D) & 0xFFFFFFFF
        x ^= x >> 15
        x = (x * 0x846CA68B) & 0xFFFFFFFF
        x ^= x >> 16
        return x
    want = np.stack([mix32(base + j) for j in range(4)], axis=1).ravel().astype(np.uint32)
    assert np.array_equal(got, want)
    assert hip.hbm_verify(got, seed) == 0
    bad = got.copy()
    flip = np.random.default_rng(1).choice(bad.size, 37, replace=False)
    bad[flip] ^= 0x10
    assert hip.hbm_verify(bad, seed) == 37                          # every corrupted word is counted
    t = torch.randint(0, 2**31 - 1, (4 * 4099,), dtype=torch.int64).to(torch.int32)
    assert np.array_equal(hip.hbm_copy(t.numpy().view(np.uint32)), t.numpy().view(np.uint32))


def test_92_hip_mfma_burn():
    from amdkube.ops import hip
    info = hip.device_info(0)
    assert info["arch"].startswith("gfx950")
    r = hip.mfma_burn(50.0, 0)
    assert r["bf16_tflops"] > 500, r
