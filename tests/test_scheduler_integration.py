"""Scheduler integration: real apiserver + scheduler over HTTP with API-only nodes, the
reference's test/integration/scheduler harness shape (framework.RunAMasterUsingServer + fake
Node objects):

  extender_test.go        -> test_extender_filter_prioritize_bind (HTTP extender incl. bindVerb,
                             which also receives the chosen device IDs)
  predicates_test.go      -> test_interpod_affinity_and_anti_affinity
  taint_test.go           -> test_extended_resource_taint_toleration (ExtendedResourceToleration)
  preemption_test.go      -> test_priority_preemption_frees_devices
"""
import asyncio

import pytest
from aiohttp import web

from amdkube.apiserver import APIServer
from amdkube.benchmark.schedperf import fake_node
from amdkube.client import Client
from amdkube.scheduler import Scheduler
from amdkube.smi import FakeBackend
from tests.conftest import run


PRIORITIES = (0, 1, 1000)


async def _cluster(n_nodes=3, gpus=0, **kw):
    api = await APIServer().start()
    c = Client(api.url)
    fb = FakeBackend()
    for i in range(n_nodes):
        await c.create(fake_node(i, gpus, fb))
    for prio in PRIORITIES:       # the Priority admission plugin resolves priorityClassName
        await c.create({"apiVersion": "scheduling.k8s.io/v1alpha1", "kind": "PriorityClass",
                        "metadata": {"name": f"prio-{prio}"}, "value": prio})
    s = await Scheduler(Client(api.url), **kw).start()
    return api, c, s


async def _stop(api, c, s):
    await s.stop()
    await s.client.close()
    await c.close()
    await api.stop()


def _pod(name, labels=None, gpus=0, prio=None, affinity=None, cpu="100m"):
    c = {"name": "c", "image": "busybox", "resources": {"requests": {"cpu": cpu}, "limits": {"cpu": cpu}}}
    if gpus:
        c["resources"]["limits"]["amd.com/gpu"] = str(gpus)
    spec = {"containers": [c]}
    if prio is not None:
        spec["priorityClassName"] = f"prio-{prio}"
    if affinity:
        spec["affinity"] = affinity
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "labels": labels or {}},
            "spec": spec}


async def _node_of(c, name, timeout=10.0):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        p = await c.get("pods", name, "default")
        if (p.get("spec") or {}).get("nodeName"):
            return p["spec"]["nodeName"]
        await asyncio.sleep(0.02)
    raise AssertionError(f"{name} never scheduled")


async def _condition(c, name, timeout=10.0):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        p = await c.get("pods", name, "default")
        for cond in (p.get("status") or {}).get("conditions") or []:
            if cond.get("type") == "PodScheduled" and cond.get("status") == "False":
                return cond
        await asyncio.sleep(0.02)
    raise AssertionError(f"{name} never marked unschedulable")


def test_extender_filter_prioritize_bind():
    async def go():
        seen = {"filter": 0, "prioritize": 0, "bind": []}
        api_holder = {}

        async def filt(r):
            body = await r.json()
            seen["filter"] += 1
            items = [n for n in body["nodes"]["items"] if n["metadata"]["name"] != "node-0002"]
            return web.json_response({"nodes": {"items": items}, "failedNodes": {"node-0002": "extender says no"}})

        async def prio(r):
            body = await r.json()
            seen["prioritize"] += 1
            return web.json_response([{"host": n["metadata"]["name"], "score": 10 if n["metadata"]["name"] == "node-0001" else 0}
                                      for n in body["nodes"]["items"]])

        async def bind(r):
            body = await r.json()
            seen["bind"].append(body)
            # ExtenderBindingArgs carries Go's field names (no json tags in the reference)
            await api_holder["c"].bind(body["PodNamespace"], body["PodName"], body["Node"], body.get("extendedResourceBinding"))
            return web.json_response({})

        app = web.Application()
        app.router.add_post("/ext/filter", filt)
        app.router.add_post("/ext/prioritize", prio)
        app.router.add_post("/ext/bind", bind)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        policy = {"kind": "Policy", "extenders": [{"urlPrefix": f"http://127.0.0.1:{port}/ext", "filterVerb": "filter",
                                                   "prioritizeVerb": "prioritize", "bindVerb": "bind", "weight": 100}]}
        api, c, s = await _cluster(3, gpus=8, policy=policy)
        api_holder["c"] = c
        try:
            await c.create(_pod("e1", gpus=2))
            assert await _node_of(c, "e1") == "node-0001"
            p = await c.get("pods", "e1", "default")
            assert len(p["spec"]["extendedResources"][0]["assigned"]) == 2
            assert seen["filter"] >= 1 and seen["prioritize"] >= 1 and len(seen["bind"]) == 1
            assert list(seen["bind"][0]["extendedResourceBinding"].values())[0]["resources"] == \
                p["spec"]["extendedResources"][0]["assigned"]
        finally:
            await _stop(api, c, s)
            await runner.cleanup()
    run(go())


def test_interpod_affinity_and_anti_affinity():
    anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": "kubernetes.io/hostname"}]}}
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": "kubernetes.io/hostname"}]}}

    async def go():
        api, c, s = await _cluster(2)
        try:
            await c.create(_pod("db-0", {"app": "db"}, affinity=anti))
            n0 = await _node_of(c, "db-0")
            await c.create(_pod("db-1", {"app": "db"}, affinity=anti))
            n1 = await _node_of(c, "db-1")
            assert {n0, n1} == {"node-0000", "node-0001"}
            await c.create(_pod("db-2", {"app": "db"}, affinity=anti))
            cond = await _condition(c, "db-2")
            assert "0/2 nodes are available" in cond["message"]
            await c.create(_pod("web", {"app": "web"}, affinity=aff))
            assert await _node_of(c, "web") in (n0, n1)
        finally:
            await _stop(api, c, s)
    run(go())


def test_extended_resource_taint_toleration():
    async def go():
        api, c, s = await _cluster(0)
        fb = FakeBackend()
        gpu = fake_node(0, 8, fb)
        gpu["spec"] = {"taints": [{"key": "amd.com/gpu", "value": "present", "effect": "NoSchedule"}]}
        await c.create(gpu)
        await c.create(fake_node(1, 0, fb))
        try:
            # the CPU pod must avoid the tainted GPU node; the GPU pod is admitted with a
            # toleration for the amd.com/gpu taint by ExtendedResourceToleration
            for i in range(4):
                await c.create(_pod(f"cpu-{i}"))
            await c.create(_pod("gpu", gpus=1))
            for i in range(4):
                assert await _node_of(c, f"cpu-{i}") == "node-0001"
            assert await _node_of(c, "gpu") == "node-0000"
            p = await c.get("pods", "gpu", "default")
            assert any(t.get("key") == "amd.com/gpu" and t.get("operator") == "Exists" for t in p["spec"]["tolerations"])
        finally:
            await _stop(api, c, s)
    run(go())


def test_priority_preemption_frees_devices():
    async def go():
        api, c, s = await _cluster(1, gpus=2)
        try:
            for i in range(2):
                await c.create(_pod(f"low-{i}", gpus=1, prio=1))
                await _node_of(c, f"low-{i}")
            await c.create(_pod("high", gpus=2, prio=1000))
            loop = asyncio.get_running_loop()
            end = loop.time() + 10
            while loop.time() < end:
                h = await c.get("pods", "high", "default")
                if ((h.get("metadata") or {}).get("annotations") or {}).get("NominatedNodeName"):
                    break
                await asyncio.sleep(0.02)
            assert h["metadata"]["annotations"]["NominatedNodeName"] == "node-0000"
            # both 1-GPU victims are gone (or terminating); once removed, the 2-GPU pod binds
            for i in range(2):
                v = await c.get_or_none("pods", f"low-{i}", "default")
                assert v is None or (v.get("metadata") or {}).get("deletionTimestamp")
                if v is not None:
                    await c.delete("pods", f"low-{i}", "default", grace=0)
            assert await _node_of(c, "high", timeout=15) == "node-0000"
            h = await c.get("pods", "high", "default")
            assert len(h["spec"]["extendedResources"][0]["assigned"]) == 2
        finally:
            await _stop(api, c, s)
    run(go())


def test_nominated_preemptor_is_not_overtaken_by_a_lower_priority_pod():
    """Priority inversion (scheduling_queue.go nominatedPods + addNominatedPods): a priority-1000
    8-GPU pod preempts eight priority-0 1-GPU pods; a priority-0 1-GPU pod created while the
    victims terminate must not take a freed GPU before the preemptor binds."""
    async def go():
        api, c, s = await _cluster(1, gpus=8)
        try:
            for i in range(8):
                await c.create(_pod(f"low-{i}", gpus=1, prio=0))
            for i in range(8):
                await _node_of(c, f"low-{i}")
            await c.create(_pod("big", gpus=8, prio=1000))
            loop = asyncio.get_running_loop()
            end = loop.time() + 10
            while loop.time() < end:
                h = await c.get("pods", "big", "default")
                if ((h.get("metadata") or {}).get("annotations") or {}).get("NominatedNodeName"):
                    break
                await asyncio.sleep(0.02)
            assert h["metadata"]["annotations"]["NominatedNodeName"] == "node-0000"
            await c.create(_pod("sneak", gpus=1, prio=0))
            await _condition(c, "sneak")
            # the victims go one at a time; after each, the sneak pod is retried and must wait
            for i in range(8):
                if await c.get_or_none("pods", f"low-{i}", "default") is not None:
                    await c.delete("pods", f"low-{i}", "default", grace=0)
                await asyncio.sleep(0.05)
                if i < 7:
                    assert not (await c.get("pods", "sneak", "default"))["spec"].get("nodeName")
            assert await _node_of(c, "big", timeout=15) == "node-0000"
            sneak = await c.get("pods", "sneak", "default")
            assert not sneak["spec"].get("nodeName")
            assert len((await c.get("pods", "big", "default"))["spec"]["extendedResources"][0]["assigned"]) == 8
        finally:
            await _stop(api, c, s)
    run(go(), 60)


def test_extender_over_tls_with_client_certificate_and_node_cache(tmp_path):
    """extender.go makeTransport + nodeCacheCapable: an HTTPS extender that demands a client
    certificate gets `nodenames` (not full Node objects) for filter and prioritize, answers with
    `nodenames`, and the pod lands where it says; httpTimeout is a Duration in nanoseconds."""
    import ssl
    from amdkube.kubeadm import new_ca, new_cert
    d = str(tmp_path)
    new_ca(d)
    new_cert(d, "ext", "extender", sans=["IP:127.0.0.1", "DNS:localhost"], server=True)
    new_cert(d, "sched", "system:kube-scheduler")

    async def go():
        seen = {"filter": [], "prioritize": [], "peer": []}

        async def filt(r):
            body = await r.json()
            seen["filter"].append(body)
            seen["peer"].append(r.transport.get_extra_info("peercert"))
            keep = [n for n in body["nodenames"] if n != "node-0000"]
            return web.json_response({"nodenames": keep, "failedNodes": {"node-0000": "cached: no"}})

        async def prio(r):
            body = await r.json()
            seen["prioritize"].append(body)
            return web.json_response([{"host": n, "score": 10 if n == "node-0002" else 1} for n in body["nodenames"]])

        app = web.Application()
        app.router.add_post("/ext/filter", filt)
        app.router.add_post("/ext/prioritize", prio)
        sctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        sctx.load_cert_chain(f"{d}/ext.crt", f"{d}/ext.key")
        sctx.load_verify_locations(f"{d}/ca.crt")
        sctx.verify_mode = ssl.CERT_REQUIRED
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0, ssl_context=sctx)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        policy = {"kind": "Policy", "extenders": [{
            "urlPrefix": f"https://127.0.0.1:{port}/ext", "filterVerb": "filter", "prioritizeVerb": "prioritize",
            "weight": 5, "enableHttps": True, "nodeCacheCapable": True, "httpTimeout": 3_000_000_000,
            "tlsConfig": {"CAFile": f"{d}/ca.crt", "CertFile": f"{d}/sched.crt", "KeyFile": f"{d}/sched.key"}}]}
        api, c, s = await _cluster(3, policy=policy)
        try:
            ext = s.extenders[0]
            assert ext.timeout == 3.0 and ext.node_cache_capable
            await c.create(_pod("t1"))
            assert await _node_of(c, "t1") == "node-0002"
            assert seen["filter"] and all("nodes" not in b and set(b["nodenames"]) <= {"node-0000", "node-0001", "node-0002"}
                                          for b in seen["filter"])
            assert seen["prioritize"] and "node-0000" not in seen["prioritize"][0]["nodenames"]
            assert seen["peer"][0] and dict(x[0] for x in seen["peer"][0]["subject"])["commonName"] == "system:kube-scheduler"
            # without the client certificate the extender refuses the handshake: scheduling fails
            from amdkube.scheduler.extender import HTTPExtender
            bare = HTTPExtender({**policy["extenders"][0], "tlsConfig": {"CAFile": f"{d}/ca.crt"}})
            try:
                with pytest.raises(Exception):
                    await bare.filter({"metadata": {"name": "x"}}, [{"metadata": {"name": "node-0001"}}])
            finally:
                await bare.close()
        finally:
            await _stop(api, c, s)
            await runner.cleanup()
    run(go(), 60)


def test_extender_config_keys_and_errors():
    """Go's case-insensitive decoding (BindVerb has no json tag), Duration nanoseconds, the 5 s
    default, enableHttps without a CA → insecure, and the send() error text on a non-200 answer."""
    import ssl
    from amdkube.scheduler.extender import HTTPExtender, tls_context

    e = HTTPExtender({"urlPrefix": "http://x/", "BindVerb": "bind", "FilterVerb": "f", "httpTimeout": 0})
    assert e.bind_verb == "bind" and e.filter_verb == "f" and e.timeout == 5.0 and e.ssl is None
    assert HTTPExtender({"urlPrefix": "http://x", "httpTimeout": 250_000_000}).timeout == 0.25
    ctx = tls_context(True, None)
    assert ctx is not None and ctx.verify_mode == ssl.CERT_NONE

    async def go():
        app = web.Application()
        app.router.add_post("/e/filter", lambda r: web.Response(status=500))
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        ext = HTTPExtender({"urlPrefix": f"http://127.0.0.1:{port}/e", "filterVerb": "filter", "prioritizeVerb": "filter"})
        try:
            with pytest.raises(RuntimeError, match=f"Failed filter with extender at URL http://127.0.0.1:{port}/e, code 500"):
                await ext.filter({"metadata": {"name": "p"}}, [{"metadata": {"name": "n"}}])
            assert await ext.prioritize({"metadata": {"name": "p"}}, [{"metadata": {"name": "n"}}]) == {}
        finally:
            await ext.close()
            await runner.cleanup()
    run(go())
