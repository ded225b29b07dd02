"""gke-certificates-controller (cmd/gke-certificates-controller/app gke_signer_test.go): approved
CSRs are POSTed to the signing webhook named by a kubeconfig, retried with backoff on 5xx, and
the answer's status.certificate lands in the CSR; a rejection is a SigningError event. With
--insecure-experimental-approve-all-kubelet-csrs-for-group, node client CSRs from that group are
approved without a SubjectAccessReview."""
import base64
import subprocess

from aiohttp import web

from amdkube.client import Client
from amdkube.controllers import ControllerManager, Options
from amdkube.localcluster import LocalCluster
from tests.test_controllers_ext import until


def _csr(path, name):
    subprocess.run(["openssl", "req", "-new", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{path}.key", "-out", f"{path}.csr",
                    "-subj", name], check=True, capture_output=True)
    return base64.b64encode(open(f"{path}.csr", "rb").read()).decode()


async def test_webhook_signer_and_group_approver(tmp_path):
    d = str(tmp_path)
    node_req = _csr(f"{d}/n", "/O=system:nodes/CN=system:node:mi355x-7")
    user_req = _csr(f"{d}/u", "/CN=alice")
    calls = []

    async def sign(request):
        csr = await request.json()
        calls.append(csr["metadata"]["name"])
        if csr["metadata"]["name"] == "reject-me":
            return web.json_response({"kind": "Status", "apiVersion": "v1", "status": "Failure", "code": 400,
                                      "reason": "BadRequest", "message": "policy forbids this subject"}, status=400)
        if calls.count(csr["metadata"]["name"]) == 1:
            return web.json_response({"error": {"code": 503, "message": "try again"}}, status=503)
        assert csr["apiVersion"] == "certificates.k8s.io/v1beta1" and csr["spec"]["request"]
        return web.json_response({**csr, "status": {"certificate": base64.b64encode(b"SIGNED-" + csr["metadata"]["name"].encode()).decode()}})

    app = web.Application()
    app.router.add_post("/sign", sign)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    port = site._server.sockets[0].getsockname()[1]
    kc = tmp_path / "signer.kubeconfig"
    kc.write_text(f"apiVersion: v1\nkind: Config\nclusters:\n- name: gke\n  cluster:\n    server: http://127.0.0.1:{port}/sign\n"
                  "contexts:\n- name: gke\n  context:\n    cluster: gke\n    user: signer\ncurrent-context: gke\n"
                  "users:\n- name: signer\n  user:\n    token: s3cr3t\n")
    users = {"kubelet-token": {"name": "kubelet-bootstrap", "groups": ["system:bootstrappers:mi355x"]},
             "alice-token": {"name": "alice", "groups": []}}
    try:
        async with LocalCluster(gpus="none", with_controllers=False, with_kubelet=False, api_kw={"token_auth": users}) as lc:
            c = lc.client
            cmc = Client(lc.api.url, token=lc.api.loopback_token)
            opts = Options(extra={"signing_kubeconfig": str(kc), "signing_retry_backoff": 0.05,
                                  "approve_group": "system:bootstrappers:mi355x"})
            cm = await ControllerManager(cmc, ["csrsigning-webhook", "csrapproving-group"], options=opts).start()
            try:
                for token, name, req in (("kubelet-token", "node-csr", node_req), ("alice-token", "alice-csr", user_req)):
                    uc = Client(lc.api.url, token=token)
                    try:
                        await uc.create({"apiVersion": "certificates.k8s.io/v1beta1", "kind": "CertificateSigningRequest",
                                         "metadata": {"name": name}, "spec": {"request": req, "usages": [
                                             "digital signature", "key encipherment", "client auth"]}})
                    finally:
                        await uc.close()

                async def signed():
                    o = await c.get("certificatesigningrequests", "node-csr")
                    return (o.get("status") or {}).get("certificate")
                assert base64.b64decode(await until(signed, 20)) == b"SIGNED-node-csr"
                o = await c.get("certificatesigningrequests", "node-csr")
                assert o["status"]["conditions"][0]["reason"] == "AutoApproved"
                assert calls.count("node-csr") == 2                       # one 503, then signed
                a = await c.get("certificatesigningrequests", "alice-csr")
                assert not (a.get("status") or {}).get("conditions")     # not in the group: left alone
                # an approved CSR the signer rejects: no certificate, a SigningError event
                await c.create({"apiVersion": "certificates.k8s.io/v1beta1", "kind": "CertificateSigningRequest",
                                "metadata": {"name": "reject-me"}, "spec": {"request": user_req, "usages": ["client auth"]}})
                r = await c.get("certificatesigningrequests", "reject-me")
                r["status"] = {"conditions": [{"type": "Approved", "reason": "Manual", "message": "ok"}]}
                await c.update(r, sub="approval")

                async def warned():
                    evs, _ = await c.list("events", "default")
                    return [e for e in evs if e.get("reason") == "SigningError"]
                ev = (await until(warned, 20))[0]
                assert "policy forbids this subject" in ev["message"]
                assert not ((await c.get("certificatesigningrequests", "reject-me")).get("status") or {}).get("certificate")
            finally:
                await cm.stop()
                await cmc.close()
    finally:
        await runner.cleanup()
