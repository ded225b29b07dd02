"""Resource metrics pipeline: kubelet summary (usageNanoCores) → metrics-server → aggregator →
`kubectl top` (staging/src/k8s.io/metrics types, kube-aggregator handler_proxy front-proxy
identity, authentication/request/headerrequest requestheader_test.go, kubectl top_node/top_pod
tests). The metrics-server authenticates the aggregator by its front-proxy client certificate and
authorizes the asserted user with a SubjectAccessReview against the main apiserver's RBAC."""
import asyncio
import io
import os
import ssl
import subprocess
from contextlib import redirect_stdout

import aiohttp

from amdkube.apiserver.auth import Authenticator
from amdkube.kubectl.main import parser
from amdkube.kubectl.top import cmd_top
from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.metrics import MetricsServer
from tests.conftest import run


def _ca(d, name="ca"):
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/{name}.key", "-out",
                    f"{d}/{name}.crt", "-days", "2", "-subj", f"/CN={name}"], check=True, capture_output=True)
    return f"{d}/{name}.crt", f"{d}/{name}.key"


def _leaf(d, ca, name, cn, server=False):
    subprocess.run(["openssl", "req", "-new", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/{name}.key", "-out",
                    f"{d}/{name}.csr", "-subj", f"/CN={cn}"], check=True, capture_output=True)
    open(f"{d}/{name}.ext", "w").write("subjectAltName=IP:127.0.0.1\nextendedKeyUsage=serverAuth\n" if server else
                                       "extendedKeyUsage=clientAuth\n")
    subprocess.run(["openssl", "x509", "-req", "-in", f"{d}/{name}.csr", "-CA", f"{d}/{ca}.crt", "-CAkey", f"{d}/{ca}.key",
                    "-CAcreateserial", "-out", f"{d}/{name}.crt", "-days", "1", "-extfile", f"{d}/{name}.ext"],
                   check=True, capture_output=True)
    return f"{d}/{name}.crt", f"{d}/{name}.key"


def _der(path):
    from amdkube.utils.crypto import x509_pem_to_der
    return x509_pem_to_der(open(path, "rb").read())[0]


def test_requestheader_authenticator(tmp_path):
    d = str(tmp_path)
    ca, _ = _ca(d, "front-proxy-ca")
    other, _ = _ca(d, "client-ca")
    leaf, _ = _leaf(d, "front-proxy-ca", "fp", "front-proxy-client")
    issuer = ssl._ssl._test_decode_cert(ca)["subject"]
    a = Authenticator(None, {}, None, True)
    a.configure_requestheader(ca, ["front-proxy-client"])
    from multidict import CIMultiDict
    hdr = CIMultiDict([("X-Remote-User", "bob"), ("X-Remote-Group", "devs"), ("X-Remote-Group", "ops"),
                       ("X-Remote-Extra-Scopes", "view")])
    pc = {"issuer": issuer, "subject": ((("commonName", "front-proxy-client"),),)}
    u = a.authenticate(hdr, pc, _der(leaf))
    assert u["name"] == "bob" and u["groups"] == ["devs", "ops", "system:authenticated"] and u["extra"] == {"scopes": ["view"]}
    # a CN outside --requestheader-allowed-names, or another issuer, cannot assert identities
    bad_cn = {"issuer": issuer, "subject": ((("commonName", "mallory"),),)}
    assert a.authenticate(hdr, bad_cn, _der(leaf))["name"] == "system:anonymous"
    other_issuer = {"issuer": ssl._ssl._test_decode_cert(other)["subject"], "subject": pc["subject"]}
    assert a.authenticate(hdr, other_issuer)["name"] == "front-proxy-client"    # plain x509 identity, headers ignored
    # a client CA with the SAME subject as the front-proxy CA issues a certificate
    # whose issuer name matches; only the signature check tells them apart
    os.makedirs(f"{d}/imp")
    _ca(f"{d}/imp", "front-proxy-ca")
    fake, _ = _leaf(f"{d}/imp", "front-proxy-ca", "fp", "front-proxy-client")
    assert ssl._ssl._test_decode_cert(fake)["issuer"] == issuer
    assert a.authenticate(hdr, pc, _der(fake))["name"] == "system:anonymous"    # X-Remote-User ignored
    assert a.authenticate(hdr, pc)["name"] == "system:anonymous"                # no DER: never trusted


def test_metrics_api_through_aggregator_and_kubectl_top(tmp_path):
    d = str(tmp_path)
    ca, _ = _ca(d, "front-proxy-ca")
    pcert, pkey = _leaf(d, "front-proxy-ca", "proxy", "front-proxy-client")
    _ca(d, "serving-ca")
    scert, skey = _leaf(d, "serving-ca", "metrics", "metrics-server", server=True)
    toks = {"tok-bob": {"name": "bob", "uid": "1", "groups": ["devs"]}, "tok-eve": {"name": "eve", "uid": "2", "groups": []}}

    async def go():
        async with LocalCluster(gpus="none", with_controllers=False, relist_period=0.2,
                                api_kw={"token_auth": toks, "authorization_mode": "RBAC",
                                        "proxy_client_cert_file": pcert, "proxy_client_key_file": pkey}) as lc:
            c = lc.client
            await c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                            "metadata": {"name": "metrics-reader"},
                            "rules": [{"apiGroups": ["metrics.k8s.io"], "resources": ["pods", "nodes"], "verbs": ["get", "list"]}]})
            await c.create({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                            "metadata": {"name": "devs-read-metrics"},
                            "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "metrics-reader"},
                            "subjects": [{"kind": "Group", "name": "devs", "apiGroup": "rbac.authorization.k8s.io"}]})
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "busy", "labels": {"app": "busy"}},
                            "spec": {"containers": [{"name": "spin", "image": "busybox",
                                                     "command": ["sh", "-c", "while :; do :; done"]}]}}, "default")
            await wait_pod(c, "default", "busy", timeout=30)
            ms = await MetricsServer(c, resolution=0.3, requestheader_ca=ca, allowed_names=["front-proxy-client"],
                                     tls_cert=scert, tls_key=skey).start()
            try:
                await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "metrics-server", "namespace": "kube-system"},
                                "spec": {"ports": [{"port": 443, "targetPort": ms.port}]}})
                await c.create({"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "metrics-server", "namespace": "kube-system"},
                                "subsets": [{"addresses": [{"ip": "127.0.0.1"}], "ports": [{"port": ms.port}]}]})
                await c.create({"apiVersion": "apiregistration.k8s.io/v1beta1", "kind": "APIService",
                                "metadata": {"name": "v1beta1.metrics.k8s.io"},
                                "spec": {"group": "metrics.k8s.io", "version": "v1beta1", "groupPriorityMinimum": 100,
                                         "versionPriority": 100, "insecureSkipTLSVerify": True,
                                         "service": {"namespace": "kube-system", "name": "metrics-server"}}})
                # without the front-proxy certificate the X-Remote-User header is worthless
                async with aiohttp.ClientSession() as s:
                    async with s.get(f"https://127.0.0.1:{ms.port}/apis/metrics.k8s.io/v1beta1/pods",
                                     headers={"X-Remote-User": "system:admin"}, ssl=False) as r:
                        assert r.status == 401
                url = lc.api.url + "/apis/metrics.k8s.io/v1beta1"
                body = None
                async with aiohttp.ClientSession() as s:
                    for _ in range(150):
                        async with s.get(url + "/namespaces/default/pods?labelSelector=app%3Dbusy",
                                         headers={"Authorization": "Bearer tok-bob"}) as r:
                            if r.status == 200:
                                body = await r.json()
                                items = body["items"]
                                if items and items[0]["containers"][0]["usage"]["cpu"] not in ("0m", "0n"):
                                    break
                        await asyncio.sleep(0.1)
                    assert body is not None and body["kind"] == "PodMetricsList", body
                    pm = body["items"][0]
                    assert pm["metadata"]["name"] == "busy" and pm["containers"][0]["name"] == "spin"
                    assert pm["containers"][0]["usage"]["cpu"] not in ("0m", "0n")     # the spinning container
                    async with s.get(url + "/nodes", headers={"Authorization": "Bearer tok-bob"}) as r:
                        assert r.status == 200
                        nodes = (await r.json())["items"]
                    assert [n["metadata"]["name"] for n in nodes] == [lc.node_name] and nodes[0]["usage"]["memory"].endswith("Ki")
                    # eve authenticates but RBAC (asked through SubjectAccessReview) says no
                    async with s.get(url + "/nodes", headers={"Authorization": "Bearer tok-eve"}) as r:
                        assert r.status == 403, r.status
                    async with s.get(url + "/namespaces/default/pods/nope", headers={"Authorization": "Bearer tok-bob"}) as r:
                        assert r.status == 404
                # kubectl top goes through the metrics API
                out = io.StringIO()
                with redirect_stdout(out):
                    await cmd_top(c, parser().parse_args(["top", "pod", "--containers"]))
                lines = out.getvalue().splitlines()
                assert lines[0].split() == ["POD", "NAME", "CPU(cores)", "MEMORY(bytes)"] and lines[1].split()[:2] == ["busy", "spin"]
                out = io.StringIO()
                with redirect_stdout(out):
                    await cmd_top(c, parser().parse_args(["top", "node"]))
                lines = out.getvalue().splitlines()
                assert lines[0].split() == ["NAME", "CPU(cores)", "CPU%", "MEMORY(bytes)", "MEMORY%"]
                assert lines[1].split()[0] == lc.node_name and lines[1].split()[2].endswith("%")
                # the pod goes away → its metrics go away
                await c.delete("pods", "busy", "default", grace=0)
                for _ in range(100):
                    if ("default", "busy") not in ms.pods:
                        break
                    await asyncio.sleep(0.1)
                assert ("default", "busy") not in ms.pods
            finally:
                await ms.stop()
    run(go(), 90)


def test_kubectl_top_falls_back_to_kubelet_summary():
    async def go():
        async with LocalCluster(gpus="fake", with_controllers=False, relist_period=0.2) as lc:
            out = io.StringIO()
            with redirect_stdout(out):
                await cmd_top(lc.client, parser().parse_args(["top", "node"]))
            lines = out.getvalue().splitlines()
            assert lines[1].split()[0] == lc.node_name
            out = io.StringIO()
            with redirect_stdout(out):
                await cmd_top(lc.client, parser().parse_args(["top", "gpu"]))
            lines = out.getvalue().splitlines()
            assert lines[0].split()[:3] == ["NODE", "GPU", "MODEL"] and len(lines) > 1
    run(go(), 60)


def test_hpa_reads_resource_metrics_api_and_falls_back():
    from amdkube.controllers.autoscaling import ResourceMetricsAPI

    class FakeClient:
        served = True

        async def request(self, method, path, **kw):
            if path == "/apis":
                return {"groups": [{"name": "metrics.k8s.io"}] if self.served else []}
            assert path == "/apis/metrics.k8s.io/v1beta1/namespaces/ns/pods"
            return {"items": [{"metadata": {"name": "a", "annotations": {"amd.com/gpu-duty-cycle": "87"}},
                               "containers": [{"usage": {"cpu": "250m"}}, {"usage": {"cpu": "500000n"}}]}]}

    class Fallback:
        async def pod_metrics(self, ns):
            return {"fb": {"cpu_milli": 1.0}}

        async def close(self):
            pass

    async def go():
        fc = FakeClient()
        src = ResourceMetricsAPI(fc, Fallback())
        got = await src.pod_metrics("ns")
        assert got == {"a": {"cpu_milli": 250.5, "gpu_util": 87.0}}
        fc.served = False
        assert await src.pod_metrics("ns") == {"fb": {"cpu_milli": 1.0}}
    run(go(), 10)
