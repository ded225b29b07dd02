"""Kubelet command-line surface beyond the GPU path (cmd/kubelet/app/options/options.go):
read-only and healthz listeners, debugging handlers, the HTTP static-pod source
(config/http.go), registration options, canRunPod (--allow-privileged, --host-*-sources),
--pods-per-core, the event spam filter (events_cache.go) and the process setup helpers."""
import asyncio
import json
import socket

import aiohttp
import pytest
from aiohttp import web

from amdkube.api import meta as m
from amdkube.client.record import EventRecorder
from amdkube.kubelet import node_setup
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_listeners_registration_and_http_manifests():
    ro, hz = _port(), _port()
    manifests = {"apiVersion": "v1", "kind": "PodList", "items": [
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "from-url"},
         "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}]}
    seen_headers = []

    async def serve(req):
        seen_headers.append(req.headers.get("X-Node"))
        return web.json_response(manifests)

    async def go():
        app = web.Application()
        app.router.add_get("/pods", serve)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        url = f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}/pods"
        try:
            async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False, kubelet_kw={
                    "read_only_port": ro, "healthz_port": hz, "enable_debugging_handlers": False,
                    "manifest_url": url, "manifest_url_header": {"X-Node": "mi355x"}, "http_check_frequency": 0.5,
                    "register_schedulable": False, "pod_cidr": "10.244.7.0/24", "provider_id": "baremetal://rack1/n0",
                    "pods_per_core": 1, "cpu_capacity": 4}) as lc:
                for _ in range(100):     # with a static-pod source the kubelet registers in the background
                    node = await lc.client.get_or_none("nodes", lc.node_name)
                    if node is not None and node["status"].get("capacity"):
                        break
                    await asyncio.sleep(0.1)
                assert node["spec"]["unschedulable"] is True
                assert node["spec"]["podCIDR"] == "10.244.7.0/24" and node["spec"]["providerID"] == "baremetal://rack1/n0"
                assert node["status"]["capacity"]["pods"] == "4"       # min(110, 4 cores × 1)
                # the HTTP source: pod <name>-<node>, source http, mirrored into the API
                p = await wait_pod(lc.client, "default", f"from-url-{lc.node_name}", ("Running",), 30)
                assert m.annotations_of(p)["kubernetes.io/config.source"] == "http"
                assert seen_headers and seen_headers[0] == "mi355x"
                async with aiohttp.ClientSession() as s:
                    async with s.get(f"http://127.0.0.1:{ro}/pods") as r:       # read-only: no authentication
                        assert r.status == 200
                        names = {x["metadata"]["name"] for x in (await r.json())["items"]}
                        assert f"from-url-{lc.node_name}" in names
                    async with s.get(f"http://127.0.0.1:{ro}/stats/summary") as r:
                        assert r.status == 200 and (await r.json())["node"]["nodeName"] == lc.node_name
                    async with s.post(f"http://127.0.0.1:{ro}/run/default/x/c") as r:
                        assert r.status in (404, 405)                          # never debugging handlers
                    async with s.get(f"http://127.0.0.1:{hz}/healthz") as r:
                        assert r.status == 200 and await r.text() == "ok"
                    async with s.get(f"http://127.0.0.1:{hz}/pods") as r:
                        assert r.status == 404
                    port = lc.kubelet.server.port
                    async with s.get(f"http://127.0.0.1:{port}/containerLogs/default/x/c") as r:
                        assert r.status == 404                                # --enable-debugging-handlers=false
                    async with s.get(f"http://127.0.0.1:{port}/healthz") as r:
                        assert r.status == 200
                # the URL's list changes: the pod goes, and so does its mirror
                manifests["items"] = []
                for _ in range(100):
                    if await lc.client.get_or_none("pods", f"from-url-{lc.node_name}", "default") is None:
                        break
                    await asyncio.sleep(0.1)
                assert await lc.client.get_or_none("pods", f"from-url-{lc.node_name}", "default") is None
        finally:
            await runner.cleanup()
    run(go(), 90)


def test_can_run_pod_privileged_and_host_namespace_sources():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False, kubelet_kw={
                "allow_privileged": False, "host_network_sources": ["file"]}) as lc:
            c = lc.client
            ctr = {"name": "c", "image": "busybox", "command": ["sleep", "60"]}
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "priv"},
                            "spec": {"nodeName": lc.node_name,
                                     "containers": [dict(ctr, securityContext={"privileged": True})]}}, "default")
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "hostnet"},
                            "spec": {"nodeName": lc.node_name, "hostNetwork": True, "containers": [ctr]}}, "default")
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "plain"},
                            "spec": {"nodeName": lc.node_name, "containers": [ctr]}}, "default")
            p = await wait_pod(c, "default", "priv", ("Failed",), 20)
            assert p["status"]["reason"] == "Forbidden" and "privileged container" in p["status"]["message"]
            p = await wait_pod(c, "default", "hostnet", ("Failed",), 20)
            assert "hostNetwork, but is disallowed for source api" in p["status"]["message"]
            await wait_pod(c, "default", "plain", ("Running",), 20)
    run(go(), 60)


def test_event_spam_filter_and_rate_limit():
    class Sink:
        def __init__(self):
            self.created, self.patched = [], 0

        async def create(self, ev, ns):
            self.created.append(ev)
            return ev

        async def patch(self, *a, **k):
            self.patched += 1
            return {}

    async def go():
        sink = Sink()
        rec = EventRecorder(sink, "kubelet", "n0", qps=1000, burst=1000).start()
        pod = {"kind": "Pod", "metadata": {"name": "p", "namespace": "default", "uid": "u1"}}
        other = {"kind": "Pod", "metadata": {"name": "q", "namespace": "default", "uid": "u2"}}
        for i in range(40):
            rec.event(pod, "Warning", "BackOff", f"restart {i}")
        rec.event(other, "Normal", "Started", "ok")
        for _ in range(100):
            if rec.queue.empty():
                break
            await asyncio.sleep(0.01)
        await asyncio.sleep(0.05)
        await rec.stop()
        mine = [e for e in sink.created if e["involvedObject"]["name"] == "p"]
        # the spam filter passes 25 of the 40: nine distinct messages, then (from the tenth) one
        # "(combined from similar events)" event created once and patched for the rest
        assert len(mine) == 10 and sink.patched == 15
        assert mine[-1]["message"].startswith("(combined from similar events): ")
        assert any(e["involvedObject"]["name"] == "q" for e in sink.created)
        # --event-qps: 3 writes at 20/s with burst 1 take ≥ 0.1 s
        sink2 = Sink()
        rec2 = EventRecorder(sink2, "kubelet", "n0", qps=20, burst=1).start()
        t0 = asyncio.get_running_loop().time()
        for i in range(3):
            rec2.event({"kind": "Pod", "metadata": {"name": f"x{i}", "uid": str(i)}}, "Normal", "R", "m")
        while len(sink2.created) < 3:
            await asyncio.sleep(0.01)
        assert asyncio.get_running_loop().time() - t0 >= 0.09
        await rec2.stop()
    run(go(), 30)


def test_process_setup_helpers(tmp_path):
    swaps = tmp_path / "swaps"
    swaps.write_text("Filename\tType\tSize\tUsed\tPriority\n")
    node_setup.check_swap(str(swaps))
    swaps.write_text("Filename\tType\tSize\tUsed\tPriority\n/swapfile file 1024 0 -2\n")
    with pytest.raises(SystemExit, match="swap"):
        node_setup.check_swap(str(swaps))
    root = tmp_path / "sys"
    for k, v in (("vm/overcommit_memory", 0), ("vm/panic_on_oom", 0), ("kernel/panic", 0), ("kernel/panic_on_oops", 1)):
        (root / k).parent.mkdir(parents=True, exist_ok=True)
        (root / k).write_text(f"{v}\n")
    with pytest.raises(SystemExit, match="vm.overcommit_memory"):
        node_setup.kernel_tunables(True, str(root))
    assert node_setup.kernel_tunables(False, str(root)) == []       # fixed in place
    assert (root / "vm/overcommit_memory").read_text() == "1" and (root / "kernel/panic").read_text() == "10"
    node_setup.kernel_tunables(True, str(root))
    lock = tmp_path / "kubelet.lock"
    held = node_setup.acquire_lock(str(lock))
    with pytest.raises(SystemExit, match="held by another process"):
        node_setup.acquire_lock(str(lock), exit_on_contention=True)
    held.close()
    assert node_setup.raise_nofile(1024) >= 1
    assert isinstance(node_setup.apply_oom_score_adj(0), bool)
    # a kubeconfig that exists is never re-bootstrapped
    kc = tmp_path / "kubeconfig"
    kc.write_text(json.dumps({"apiVersion": "v1"}))
    assert node_setup.bootstrap_client_cert(str(kc), "/nonexistent", str(tmp_path / "pki"), "n0") is False
