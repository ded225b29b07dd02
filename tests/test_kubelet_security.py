"""Kubelet API security and certificate rotation (pkg/kubelet/server/auth_test.go,
pkg/kubelet/certificate/manager_test.go): TokenReview/SubjectAccessReview delegation, x509
client certificates over the kubelet's TLS listener, rotated client/server certificates
issued through CertificateSigningRequests, the apiserver reaching kubelets over HTTPS."""
import asyncio
import os
import ssl
import subprocess

import aiohttp
import pytest

from amdkube.api import meta as m
from amdkube.kubelet.certificate import CertManager, cert_validity, split_pem
from amdkube.localcluster import LocalCluster
from tests.conftest import run


def _ca(d):
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/ca.key", "-out", f"{d}/ca.crt",
                    "-days", "2", "-subj", "/CN=test-ca"], check=True, capture_output=True)
    return f"{d}/ca.crt", f"{d}/ca.key"


def _leaf(d, name, cn, orgs=(), server=False):
    subj = "".join(f"/O={o}" for o in orgs) + f"/CN={cn}"
    subprocess.run(["openssl", "req", "-new", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/{name}.key", "-out",
                    f"{d}/{name}.csr", "-subj", subj], check=True, capture_output=True)
    ext = f"{d}/{name}.ext"
    open(ext, "w").write("subjectAltName=IP:127.0.0.1\nextendedKeyUsage=serverAuth\n" if server else
                         "extendedKeyUsage=clientAuth\n")
    subprocess.run(["openssl", "x509", "-req", "-in", f"{d}/{name}.csr", "-CA", f"{d}/ca.crt", "-CAkey", f"{d}/ca.key",
                    "-CAcreateserial", "-out", f"{d}/{name}.crt", "-days", "1", "-extfile", ext], check=True, capture_output=True)
    return f"{d}/{name}.crt", f"{d}/{name}.key"


def test_kubelet_webhook_authn_authz_and_x509_over_tls(tmp_path):
    d = str(tmp_path)
    ca, _ = _ca(d)
    srv_crt, srv_key = _leaf(d, "kubelet", "kubelet-serving", server=True)
    adm_crt, adm_key = _leaf(d, "apiclient", "kube-apiserver-kubelet-client", orgs=("system:masters",))

    async def go():
        tokens = {"tok-admin": {"name": "admin", "uid": "1", "groups": ["system:masters"]},
                  "tok-bob": {"name": "bob", "uid": "2", "groups": []}}
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                api_kw={"token_auth": tokens, "authorization_mode": "RBAC", "kubelet_https": True,
                                        "kubelet_client_certificate": adm_crt, "kubelet_client_key": adm_key,
                                        "kubelet_certificate_authority": ca},
                                kubelet_kw={"tls_cert_file": srv_crt, "tls_private_key_file": srv_key, "client_ca_file": ca,
                                            "anonymous_auth": False, "authentication_token_webhook": True,
                                            "authorization_mode": "Webhook"}) as lc:
            url = f"https://127.0.0.1:{lc.kubelet.server.port}"
            verify = ssl.create_default_context(cafile=ca)
            verify.check_hostname = False
            async with aiohttp.ClientSession() as s:
                async with s.get(url + "/pods", ssl=verify) as r:
                    assert r.status == 401                                  # anonymous disabled
                async with s.get(url + "/pods", ssl=verify, headers={"Authorization": "Bearer tok-bob"}) as r:
                    assert r.status == 403                                  # SubjectAccessReview: no nodes/proxy
                async with s.get(url + "/pods", ssl=verify, headers={"Authorization": "Bearer nope"}) as r:
                    assert r.status == 401
                async with s.get(url + "/stats/summary", ssl=verify, headers={"Authorization": "Bearer tok-admin"}) as r:
                    assert r.status == 200
                cctx = ssl.create_default_context(cafile=ca)
                cctx.check_hostname = False
                cctx.load_cert_chain(adm_crt, adm_key)
                async with s.get(url + "/pods", ssl=cctx) as r:             # x509: CN/O from the client certificate
                    assert r.status == 200
            # the apiserver talks HTTPS to the kubelet with its client certificate
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "hello"},
                            "spec": {"restartPolicy": "Never",
                                     "containers": [{"name": "c", "image": "busybox", "command": ["echo", "hi-from-tls"]}]}},
                           "default")
            for _ in range(100):
                p = await c.get("pods", "hello", "default")
                if p["status"].get("phase") == "Succeeded":
                    break
                await asyncio.sleep(0.1)
            assert "hi-from-tls" in await c.logs("default", "hello")
    run(go(), 60)


def test_certificate_manager_rotates_through_csr(tmp_path):
    d = str(tmp_path)
    ca, ca_key = _ca(d)

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False,
                                controllers_kw={"cluster_signing_cert_file": ca, "cluster_signing_key_file": ca_key}) as lc:
            c = lc.client

            async def approver():    # server certificates need a human (or a policy) to approve them
                while True:
                    for csr in (await c.list("certificatesigningrequests"))[0]:
                        if not (csr.get("status") or {}).get("conditions"):
                            csr["status"] = {"conditions": [{"type": "Approved", "reason": "Test", "message": "ok"}]}
                            await c.request("PUT", f"/apis/certificates.k8s.io/v1beta1/certificatesigningrequests/"
                                                   f"{m.name_of(csr)}/approval", body=csr)
                    await asyncio.sleep(0.1)
            task = asyncio.create_task(approver())
            try:
                clock = [1e10]
                mgr = CertManager(c, os.path.join(d, "pki"), "node-a", "server", addresses=["10.0.0.7", "node-a"],
                                  clock=lambda: clock[0], rng=lambda: 0.5)
                seen = []
                mgr.listeners.append(seen.append)
                assert mgr.current() is None and mgr.deadline() == clock[0]      # nothing yet: rotate now
                path = await asyncio.wait_for(mgr.rotate(), 30)
                assert seen == [mgr.current_path] and os.path.islink(mgr.current_path)
                cert, key = split_pem(mgr.current())
                text = subprocess.run(["openssl", "x509", "-noout", "-text"], input=cert, capture_output=True).stdout.decode()
                assert "CN = system:node:node-a" in text and "IP Address:10.0.0.7" in text and "TLS Web Server Authentication" in text
                nb, na = cert_validity(cert)
                clock[0] = nb
                assert abs(mgr.deadline() - (nb + 0.8 * (na - nb))) < 1.0        # 70 % + 0.5 × 20 % of the lifetime
                path2 = await asyncio.wait_for(mgr.rotate(), 30)
                assert path2 != path and os.readlink(mgr.current_path) == os.path.basename(path2)
            finally:
                task.cancel()
    run(go(), 60)
