"""kubectl against a live apiserver (background thread), the amd-smi exporter, hollow-node
density with simulated GPUs, leader election failover and chaos (fault-injected) clients."""
import asyncio
import io
import json
import threading
import time
from contextlib import redirect_stdout

import pytest

from amdkube.apiserver import APIServer
from amdkube.client import ChaosError, Client, Informer, LeaderElector
from amdkube.hollow.hollow_node import HollowNode
from amdkube.kubectl.main import main as kubectl
from amdkube.monitoring.exporter import Exporter
from amdkube.scheduler import Scheduler
from amdkube.smi import FakeBackend
from tests.conftest import run


@pytest.fixture(scope="module")
def server():
    loop = asyncio.new_event_loop()
    box = {}
    ready = threading.Event()

    def serve():
        asyncio.set_event_loop(loop)
        box["srv"] = loop.run_until_complete(APIServer().start())
        ready.set()
        loop.run_forever()
    t = threading.Thread(target=serve, daemon=True)
    t.start()
    ready.wait(10)
    yield box["srv"].url
    asyncio.run_coroutine_threadsafe(box["srv"].stop(), loop).result(30)
    loop.call_soon_threadsafe(loop.stop)
    t.join(10)
    loop.close()


def k(url, *args):
    buf = io.StringIO()
    with redirect_stdout(buf):
        rc = kubectl(["--server", url, *args])
    return rc, buf.getvalue()


def test_kubectl_create_get_describe_label_delete(server, tmp_path):
    f = tmp_path / "p.yaml"
    f.write_text("apiVersion: v1\nkind: Pod\nmetadata: {name: kp}\nspec:\n  containers:\n  - name: c\n    image: rocm/vector-add\n"
                 "    resources: {limits: {amd.com/gpu: 2}}\n")
    rc, out = k(server, "create", "-f", str(f))
    assert rc == 0 and "pod/kp created" in out
    rc, out = k(server, "get", "pods")
    assert "GPUS" in out.splitlines()[0] and "kp" in out and " 2 " in out
    rc, out = k(server, "get", "pod", "kp", "-o", "jsonpath={.spec.extendedResources[0].resources.limits}")
    assert out == "map[amd.com/gpu:2]"      # fmt's %v of a map, as the reference prints it
    rc, out = k(server, "describe", "pod", "kp")
    assert "Extended Resources:" in out and "amd.com/gpu=2" in out and "<not yet scheduled>" in out
    rc, out = k(server, "label", "pod", "kp", "tier=gpu")
    rc, out = k(server, "get", "pods", "-l", "tier=gpu", "-o", "name")
    assert out.strip() == "pod/kp"
    f.write_text(f.read_text().replace("metadata: {name: kp}", "metadata: {name: kp, labels: {v: '2'}}"))
    rc, out = k(server, "apply", "-f", str(f))
    assert "configured" in out
    rc, out = k(server, "get", "pod", "kp", "-o", "json")
    assert json.loads(out)["metadata"]["labels"]["v"] == "2"
    rc, out = k(server, "delete", "pod", "kp")
    assert 'pod "kp" deleted' in out
    rc, out = k(server, "api-resources")
    assert "daemonsets" in out and "ds" in out


def test_kubectl_nodes_gpu_columns(server):
    async def mk():
        c = Client(server)
        from amdkube.benchmark.schedperf import fake_node
        await c.create(fake_node(7, 8, FakeBackend()))
        await c.close()
    asyncio.run(mk())
    rc, out = k(server, "get", "nodes")
    head, row = out.splitlines()[0], [line for line in out.splitlines() if "node-0007" in line][0]
    assert "GPU-HEALTHY" in head and "MI355X" in row and row.split()[5] == "8"
    rc, out = k(server, "describe", "node", "node-0007")
    assert "type=MI355X mem=294912MiB numa=0" in out


def test_exporter_metrics_and_attribution():
    async def go():
        fb = FakeBackend(n=2)
        fb.set_sample(1, gfx_activity=87, vram_used_bytes=123)
        fb.inject_ecc(1)                        # historical error on GPU 1: not a new fault
        ex = Exporter(fb, node="n1")
        ex.collect({})                          # baseline
        fb.inject_ecc(0)                        # a NEW uncorrectable error on GPU 0
        from amdkube.smi import device_id
        text = ex.collect({device_id(fb.gpus()[1]): ("ml", "trainer", "c")})
        assert 'amd_gpu_health{gpu="0"' in text and text.count("amd_gpu_health{") == 2
        assert [l for l in text.splitlines() if l.startswith('amd_gpu_health{gpu="0"')][0].endswith(" 0")
        assert [l for l in text.splitlines() if l.startswith('amd_gpu_health{gpu="1"')][0].endswith(" 1")
        assert 'amd_gpu_xgmi_error_status{gpu="0"' in text and 'amd_gpu_bad_pages{gpu="0"' in text
        assert 'amd_gpu_utilization_percent{gpu="1",uuid="GPU-5b4a01c0d1e2f3a1",node="n1",model="AMD Instinct MI355X",namespace="ml",pod="trainer",container="c"} 87' in text
        assert 'container_accelerator_duty_cycle{container_name="c",pod_name="trainer",namespace="ml"' in text
        assert "amd_gpu_xgmi_link_write_bytes_total" in text
        await ex.start("127.0.0.1", 0)
        import aiohttp
        async with aiohttp.ClientSession() as s:
            body = await (await s.get(f"http://127.0.0.1:{ex.port}/metrics")).text()
        assert "amd_gpu_exporter_scrape_duration_seconds" in body
        await ex.stop()
    run(go())


def test_duty_cycle_is_the_10s_average(monkeypatch):
    """cAdvisor DutyCycle = NVML average over 10 s (accelerators/nvidia.go:216-252): the
    collector and the exporter read the backend's sampler window, not one instant."""
    import time as _t
    from amdkube.monitoring.collector import AcceleratorCollector
    from amdkube.smi import device_id
    fb = FakeBackend(n=2)
    col = AcceleratorCollector(fb, "n1")          # starts sampling
    assert fb.sampling
    for v in (100, 100, 40, 0):                   # samples inside the window
        fb.set_sample(1, gfx_activity=v, umc_activity=v // 2)
    did = device_id(fb.gpus()[1])
    st = col.accelerator_stats([did])[0]
    assert st["dutyCycle"] == round((0 + 100 + 100 + 40 + 0) / 5)   # start_sampling recorded the initial 0
    ex = Exporter(fb, node="n1")
    text = ex.collect({did: ("ml", "trainer", "c")})
    line = [l for l in text.splitlines() if l.startswith('amd_gpu_utilization_avg10s_percent{gpu="1"')][0]
    assert float(line.split()[-1]) == 48.0
    assert 'amd_gpu_utilization_percent{gpu="1"' in text and text.count("amd_gpu_memory_utilization_avg10s_percent{") == 2
    # samples older than the window no longer count: only the instantaneous value remains
    real = _t.monotonic
    monkeypatch.setattr("amdkube.smi.backend.time.monotonic", lambda: real() + 11)
    assert fb.average_activity(1, 10.0) is None
    assert col.accelerator_stats([did])[0]["dutyCycle"] == 0


def test_hollow_nodes_gpu_density():
    """kubemark-style: 4 hollow nodes × 8 simulated MI355X, 32 GPU pods, no double assignment."""
    async def go():
        srv = await APIServer().start()
        sched = await Scheduler(Client(srv.url)).start()
        nodes = [await HollowNode(srv.url, f"h{i}", gpus=8).start() for i in range(4)]
        c = Client(srv.url)
        try:
            for _ in range(100):
                ns, _ = await c.list("nodes")
                if len(ns) == 4 and all((n["status"].get("allocatable") or {}).get("amd.com/gpu") == "8" for n in ns):
                    break
                await asyncio.sleep(0.1)
            t0 = time.time()
            for i in range(32):
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"d{i}", "namespace": "default"},
                                "spec": {"containers": [{"name": "c", "image": "rocm/vector-add",
                                                         "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
            for _ in range(300):
                pods, _ = await c.list("pods", "default")
                if sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Running") == 32:
                    break
                await asyncio.sleep(0.05)
            running = [p for p in pods if p["status"].get("phase") == "Running"]
            assert len(running) == 32, time.time() - t0
            ids = [(p["spec"]["nodeName"], d) for p in running for d in p["spec"]["extendedResources"][0]["assigned"]]
            assert len(set(ids)) == 32
            # the kubelet learns each fresh pod's state from the runtime's full-state events:
            # no per-pod status RPCs (only the startup snapshot and periodic relists list)
            for n in nodes:
                calls = n.runtime.calls
                assert calls.get("RunPodSandbox", 0) == calls.get("CreateContainer", 0) >= 1, calls
                assert calls.get("PodSandboxStatus", 0) == 0 and calls.get("ContainerStatus", 0) == 0, calls
        finally:
            for n in nodes:
                await n.stop()
            await sched.stop()
            await c.close()
            await srv.stop()
            await srv.stop()
    run(go(), 120)


def test_leader_election_failover():
    async def go():
        srv = await APIServer().start()
        c1, c2 = Client(srv.url), Client(srv.url)
        try:
            e1 = LeaderElector(c1, "lock", "a", lease_duration=0.6, renew_deadline=0.4, retry_period=0.1)
            e2 = LeaderElector(c2, "lock", "b", lease_duration=0.6, renew_deadline=0.4, retry_period=0.1)
            started = []
            work1 = asyncio.Event()

            async def lead(name, ev=None):
                started.append(name)
                await (ev.wait() if ev else asyncio.Event().wait())
            t1 = asyncio.create_task(e1.run(lambda: lead("a", work1)))
            await asyncio.sleep(0.3)
            t2 = asyncio.create_task(e2.run(lambda: lead("b")))
            await asyncio.sleep(0.5)
            assert started == ["a"] and e1.is_leader and not e2.is_leader
            t1.cancel()  # leader dies without releasing
            for _ in range(50):
                if e2.is_leader:
                    break
                await asyncio.sleep(0.1)
            assert e2.is_leader and started == ["a", "b"]
            t2.cancel()
        finally:
            await c1.close()
            await c2.close()
            await srv.stop()
    run(go(), 30)


def test_chaos_client_and_informer_recovery():
    """--chaos-chance: the client randomly fails requests; informers/controllers must converge."""
    async def go():
        srv = await APIServer().start()
        chaotic = Client(srv.url, chaos=0.3)
        good = Client(srv.url)
        try:
            fails = 0
            for i in range(40):
                try:
                    await chaotic.get("namespaces", "default")
                except ChaosError:
                    fails += 1
            assert 2 < fails < 30
            inf = Informer(chaotic, "configmaps", "default").start()
            for i in range(20):
                await good.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": f"c{i}", "namespace": "default"}})
            for _ in range(200):
                if inf.has_synced() and len(inf.list()) == 20:
                    break
                await asyncio.sleep(0.05)
            assert len(inf.list()) == 20
            await inf.stop()
        finally:
            await chaotic.close()
            await good.close()
            await srv.stop()
    run(go(), 60)


def test_store_conflict_injection_exercises_retry_loops():
    """--store-conflict-chance: half the conditional writes lose a simulated race; updates,
    patches, status writes, bindings and deletes still succeed through the apiserver's
    GuaranteedUpdate retries, and a precondition that really is stale is still a 409."""
    from amdkube.api import meta as m
    from amdkube.store import MVCCStore
    store = MVCCStore()
    store.conflict_chance = 0.5

    async def go():
        srv = await APIServer(store).start()
        c = Client(srv.url, token=srv.loopback_token)
        try:
            cm = await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x", "namespace": "default"},
                                 "data": {"n": "0"}}, "default")
            for i in range(1, 21):
                cm["data"]["n"] = str(i)
                cm = await c.update(cm)
                await c.patch("configmaps", "x", {"metadata": {"labels": {"i": str(i)}}}, "default")
                cm = await c.get("configmaps", "x", "default")
            assert cm["data"]["n"] == "20" and cm["metadata"]["labels"]["i"] == "20"
            stale = dict(cm, metadata=dict(cm["metadata"], resourceVersion="1"))
            with pytest.raises(m.StatusError) as ei:
                await c.update(stale)
            assert ei.value.code == 409
            await c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n1"},
                            "status": {"capacity": {"cpu": "4", "memory": "4Gi", "pods": "10"}}})
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default"},
                            "spec": {"containers": [{"name": "c", "image": "busybox"}]}}, "default")
            await c.bind("default", "p", "n1")
            assert (await c.get("pods", "p", "default"))["spec"]["nodeName"] == "n1"
            await c.delete("configmaps", "x", "default")
            assert await c.get_or_none("configmaps", "x", "default") is None
            assert store.injected_conflicts >= 10
        finally:
            await c.close()
            await srv.stop()
    run(go(), 60)
