"""kube-aggregator in the apiserver (staging/src/k8s.io/kube-aggregator handler_proxy_test.go,
available_controller_test.go, handler_apis_test.go): an APIService backed by a Service is
discovered under /apis, proxied over TLS with the caller's identity in X-Remote-* headers and
without its credentials, and its Available condition follows the backend."""
import asyncio
import os
import ssl
import subprocess

from aiohttp import web

from amdkube.api import meta as m
from amdkube.localcluster import LocalCluster
from tests.conftest import run


def _self_signed(d):
    crt, key = os.path.join(d, "tls.crt"), os.path.join(d, "tls.key")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", crt, "-days", "1",
                    "-subj", "/CN=api.example.svc"], check=True, capture_output=True)
    return crt, key


def test_apiservice_discovery_proxy_and_availability(tmp_path):
    async def go():
        seen = []

        async def discovery(request):
            return web.json_response({"kind": "APIResourceList", "groupVersion": "metrics.example.com/v1alpha1",
                                      "resources": [{"name": "widgets", "namespaced": True, "kind": "Widget"}]})

        async def widgets(request):
            seen.append({k: v for k, v in request.headers.items()} | {"_groups": request.headers.getall("X-Remote-Group", [])})
            return web.json_response({"kind": "WidgetList", "apiVersion": "metrics.example.com/v1alpha1", "items": [
                {"metadata": {"name": "w1"}}]})
        app = web.Application()
        app.router.add_get("/apis/metrics.example.com/v1alpha1", discovery)
        app.router.add_get("/apis/metrics.example.com/v1alpha1/namespaces/default/widgets", widgets)
        crt, key = _self_signed(str(tmp_path))
        sctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        sctx.load_cert_chain(crt, key)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0, ssl_context=sctx)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]

        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False,
                                api_kw={"token_auth": {"tok-bob": {"name": "bob", "uid": "1", "groups": ["devs"]}}}) as lc:
            c = lc.client
            agg = lc.api.aggregator
            assert (await c.get("apiservices", "v1.apps"))["spec"]["groupPriorityMinimum"] == 17800   # autoregistered
            await c.create({"apiVersion": "apiregistration.k8s.io/v1beta1", "kind": "APIService",
                            "metadata": {"name": "v1alpha1.metrics.example.com"},
                            "spec": {"group": "metrics.example.com", "version": "v1alpha1", "groupPriorityMinimum": 100,
                                     "versionPriority": 10, "insecureSkipTLSVerify": True,
                                     "service": {"namespace": "default", "name": "metrics"}}})

            async def available():
                for _ in range(100):
                    a = await c.get("apiservices", "v1alpha1.metrics.example.com")
                    conds = {x["type"]: x for x in (a.get("status") or {}).get("conditions") or []}
                    if "Available" in conds:
                        return conds["Available"]
                    await asyncio.sleep(0.05)
            cond = await available()
            assert cond["status"] == "False" and cond["reason"] == "ServiceNotFound"
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "metrics", "namespace": "default"},
                            "spec": {"ports": [{"port": 443, "targetPort": port}]}})
            await c.create({"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "metrics", "namespace": "default"},
                            "subsets": [{"addresses": [{"ip": "127.0.0.1"}], "ports": [{"port": port}]}]})
            for _ in range(100):
                cond = await available()
                if cond["status"] == "True":
                    break
                await asyncio.sleep(0.05)
            assert cond["reason"] == "Passed", cond
            groups = [g["name"] for g in (await c.request("GET", "/apis"))["groups"]]
            assert "metrics.example.com" in groups
            grp = await c.request("GET", "/apis/metrics.example.com")
            assert grp["preferredVersion"]["version"] == "v1alpha1"
            import aiohttp
            async with aiohttp.ClientSession() as s:
                async with s.get(lc.api.url + "/apis/metrics.example.com/v1alpha1/namespaces/default/widgets",
                                 headers={"Authorization": "Bearer tok-bob", "X-Remote-User": "mallory"}) as r:
                    assert r.status == 200
                    body = await r.json()
            assert body["items"][0]["metadata"]["name"] == "w1"
            h = seen[-1]
            assert h["X-Remote-User"] == "bob" and h["_groups"][:1] == ["devs"] and "Authorization" not in h
            # backend gone → unavailable → 503
            await runner.cleanup()
            for _ in range(200):
                cond = await available()
                if cond["status"] == "False":
                    break
                agg._dirty.set()
                await asyncio.sleep(0.05)
            assert cond["reason"] == "FailedDiscoveryCheck"
            try:
                await c.request("GET", "/apis/metrics.example.com/v1alpha1/namespaces/default/widgets")
                raise AssertionError("expected 503")
            except m.StatusError as e:
                assert e.code == 503
    run(go(), 60)
