"""kube-apiserver authentication/authorization modes and server options beyond tokens and RBAC
(plugin/pkg/auth/authenticator/{password/passwordfile,token/webhook,token/oidc},
plugin/pkg/auth/authorizer/webhook, pkg/auth/authorizer/abac, storage/value/encrypt/aes,
plugin/pkg/audit/webhook, --runtime-config, --allow-privileged, --cors-allowed-origins,
--insecure-port next to --secure-port, /logs/)."""
import base64
import json
import os
import subprocess
import time

import aiohttp
import pytest
from aiohttp import web

from amdkube.apiserver import APIServer
from amdkube.apiserver.encryption import load as load_encryption
from amdkube.store import MVCCStore
from tests.conftest import run


async def _serve(routes):
    app = web.Application()
    for method, path, fn in routes:
        app.router.add_route(method, path, fn)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    return runner, f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"


def _kubeconfig(path, server):
    path.write_text(json.dumps({"apiVersion": "v1", "kind": "Config", "current-context": "c",
                                "clusters": [{"name": "w", "cluster": {"server": server}}],
                                "users": [{"name": "u", "user": {}}],
                                "contexts": [{"name": "c", "context": {"cluster": "w", "user": "u"}}]}))
    return str(path)


async def _get(url, headers=None, method="GET", body=None):
    async with aiohttp.ClientSession() as s:
        async with s.request(method, url, headers=headers or {}, json=body) as r:
            return r.status, (await r.read()).decode(errors="replace"), dict(r.headers)


def test_encryption_at_rest_and_key_rotation(tmp_path):
    k1, k2 = base64.b64encode(os.urandom(32)).decode(), base64.b64encode(os.urandom(32)).decode()
    cfg = tmp_path / "enc.yaml"
    cfg.write_text(f"kind: EncryptionConfig\napiVersion: v1\nresources:\n- resources: [secrets]\n  providers:\n"
                   f"  - aescbc: {{keys: [{{name: key1, secret: {k1}}}]}}\n  - identity: {{}}\n")
    data_dir = str(tmp_path / "data")
    secret = base64.b64encode(b"mi355x-hbm-password").decode()

    async def go(store, create=True):
        srv = await APIServer(store).start()
        try:
            c = {"Authorization": f"Bearer {srv.loopback_token}"}
            if create:
                st, _, _ = await _get(f"{srv.url}/api/v1/namespaces/default/secrets", c, "POST",
                                      {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "s"}, "data": {"pw": secret}})
                assert st == 201
                st, _, _ = await _get(f"{srv.url}/api/v1/namespaces/default/configmaps", c, "POST",
                                      {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "plain"},
                                       "data": {"k": "visible-value"}})
                assert st == 201
            st, body, _ = await _get(f"{srv.url}/api/v1/namespaces/default/secrets/s", c)
            assert st == 200 and json.loads(body)["data"]["pw"] == secret
        finally:
            await srv.stop()
    store = MVCCStore(data_dir, transformer=load_encryption(str(cfg)))
    run(go(store), 30)
    wal = open(os.path.join(data_dir, "wal.log"), "rb").read()
    assert secret.encode() not in wal and b"mi355x-hbm-password" not in wal and b"visible-value" in wal
    assert _disk_value(wal, "/registry/secrets/default/s").startswith(b"k8s:enc:aescbc:v1:key1:")
    store.close()
    # restart: recovery decrypts
    store = MVCCStore(data_dir, transformer=load_encryption(str(cfg)))
    run(go(store, create=False), 30)
    # a store without the key cannot read it
    store.close()
    with pytest.raises(ValueError):
        MVCCStore(data_dir, transformer=load_encryption(_write(
            tmp_path / "id.yaml", "kind: EncryptionConfig\nresources:\n- resources: [secrets]\n  providers:\n  - identity: {}\n")))
    # rotation: the new key first, the old one still readable; a snapshot rewrites with key2 (GCM)
    cfg.write_text(f"kind: EncryptionConfig\nresources:\n- resources: [secrets]\n  providers:\n"
                   f"  - aesgcm: {{keys: [{{name: key2, secret: {k2}}}]}}\n"
                   f"  - aescbc: {{keys: [{{name: key1, secret: {k1}}}]}}\n")
    store = MVCCStore(data_dir, transformer=load_encryption(str(cfg)))
    store.snapshot()
    snap = json.load(open(os.path.join(data_dir, "snapshot.json")))
    from amdkube.store.mvcc import _unb
    stored = {k: _unb(v) for k, v, *_ in snap["kv"]}
    assert stored["/registry/secrets/default/s"].startswith(b"k8s:enc:aesgcm:v1:key2:")
    assert b"visible-value" in stored["/registry/configmaps/default/plain"]
    store.close()
    store = MVCCStore(data_dir, transformer=load_encryption(str(cfg)))
    run(go(store, create=False), 30)
    store.close()
    with pytest.raises(ValueError, match="secretbox"):
        load_encryption(_write(tmp_path / "sb.yaml", "kind: EncryptionConfig\nresources:\n- resources: [secrets]\n"
                                                       "  providers:\n  - secretbox: {keys: [{name: a, secret: eA==}]}\n"))


def _disk_value(wal: bytes, key: str) -> bytes:
    from amdkube.store.mvcc import _unb
    for line in wal.splitlines():
        rec = json.loads(line)
        if rec["k"] == key and rec["o"] == "p":
            return _unb(rec["v"])
    raise KeyError(key)


def _write(p, text):
    p.write_text(text)
    return str(p)


def test_basic_auth_webhooks_abac_and_server_options(tmp_path):
    calls = {"tokenreview": 0, "sar": 0, "audit": []}

    async def tokenreview(req):
        calls["tokenreview"] += 1
        body = await req.json()
        ok = body["spec"]["token"] == "good-token"
        st = {"authenticated": ok}
        if ok:
            st["user"] = {"username": "alice", "uid": "42", "groups": ["gpu-devs"]}
        return web.json_response(dict(body, status=st))

    async def sar(req):
        calls["sar"] += 1
        body = await req.json()
        ra = body["spec"].get("resourceAttributes") or {}
        ok = body["spec"]["user"] == "alice" and ra.get("resource") == "pods" and ra.get("namespace") == "default"
        return web.json_response(dict(body, status={"allowed": ok, "reason": "gpu-devs may read pods" if ok else ""}))

    async def audit(req):
        calls["audit"] += (await req.json())["items"]
        return web.json_response({})

    async def go():
        runner, hook = await _serve([("POST", "/authn", tokenreview), ("POST", "/authz", sar), ("POST", "/audit", audit)])
        basic = tmp_path / "basic.csv"
        basic.write_text('hunter2,bob,7,"ops,readers"\n')
        abac = tmp_path / "abac.jsonl"
        abac.write_text(json.dumps({"apiVersion": "abac.authorization.kubernetes.io/v1beta1", "kind": "Policy",
                                    "spec": {"user": "bob", "namespace": "*", "resource": "*", "apiGroup": "*",
                                             "readonly": True}}) + "\n")
        logs = tmp_path / "logs"
        logs.mkdir()
        (logs / "kubelet.log").write_text("node log line\n")
        opts = {"basic_auth_file": str(basic),
                "authentication_token_webhook_config_file": _kubeconfig(tmp_path / "authn.kc", hook + "/authn"),
                "authorization_webhook_config_file": _kubeconfig(tmp_path / "authz.kc", hook + "/authz"),
                "authorization_policy_file": str(abac), "runtime_config": "batch/v1beta1=false,batch/v2alpha1=false",
                "allow_privileged": False, "cors_allowed_origins": [r"//dashboard\.example$"], "logs_dir": str(logs),
                "audit_webhook_config_file": _kubeconfig(tmp_path / "audit.kc", hook + "/audit"),
                "audit_webhook_batch_max_wait": 0.2}
        srv = await APIServer(authorization_mode="ABAC,Webhook", anonymous_auth=False, audit_log_path=str(tmp_path / "audit.log"),
                              options=opts).start()
        try:
            u = srv.url
            good = {"Authorization": "Bearer good-token"}
            # webhook token authentication + webhook authorization (cached: one review per token)
            assert (await _get(f"{u}/api/v1/namespaces/default/pods", good))[0] == 200
            assert (await _get(f"{u}/api/v1/namespaces/default/pods", good))[0] == 200
            assert calls["tokenreview"] == 1 and calls["sar"] == 1
            st, body, _ = await _get(f"{u}/api/v1/nodes", good)
            assert st == 403 and 'User "alice" cannot list nodes' in json.loads(body)["message"]
            assert (await _get(f"{u}/api/v1/namespaces/default/pods", {"Authorization": "Bearer nope"}))[0] == 401
            # TokenReview through the apiserver consults the webhook too
            loop = {"Authorization": f"Bearer {srv.loopback_token}"}
            st, body, _ = await _get(f"{u}/apis/authentication.k8s.io/v1/tokenreviews", loop, "POST",
                                     {"apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview", "spec": {"token": "good-token"}})
            assert json.loads(body)["status"]["user"]["username"] == "alice"
            # basic auth + ABAC read-only policy
            bob = {"Authorization": "Basic " + base64.b64encode(b"bob:hunter2").decode()}
            assert (await _get(f"{u}/api/v1/nodes", bob))[0] == 200
            st, body, _ = await _get(f"{u}/api/v1/namespaces/default/configmaps", bob, "POST",
                                     {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}})
            assert st == 403
            bad = {"Authorization": "Basic " + base64.b64encode(b"bob:wrong").decode()}
            assert (await _get(f"{u}/api/v1/nodes", bad))[0] == 401
            # --runtime-config: batch/v1beta1 is off (requests and discovery), batch/v1 stays
            assert (await _get(f"{u}/apis/batch/v1beta1/namespaces/default/cronjobs", loop))[0] == 404
            st, body, _ = await _get(f"{u}/apis", loop)
            batch = next(g for g in json.loads(body)["groups"] if g["name"] == "batch")
            assert [v["version"] for v in batch["versions"]] == ["v1"]
            # --allow-privileged=false
            st, body, _ = await _get(f"{u}/api/v1/namespaces/default/pods", loop, "POST", {
                "apiVersion": "v1", "kind": "Pod", "metadata": {"name": "priv"},
                "spec": {"containers": [{"name": "c", "image": "busybox", "securityContext": {"privileged": True}}]}})
            assert st == 422 and "disallowed by cluster policy" in body
            # CORS
            _, _, hdr = await _get(f"{u}/api/v1/namespaces", dict(loop, Origin="https://dashboard.example"))
            assert hdr.get("Access-Control-Allow-Origin") == "https://dashboard.example"
            _, _, hdr = await _get(f"{u}/api/v1/namespaces", dict(loop, Origin="https://evil.example"))
            assert "Access-Control-Allow-Origin" not in hdr
            # /logs/ for admins only, no escaping the directory
            st, body, _ = await _get(f"{u}/logs/kubelet.log", loop)
            assert st == 200 and body == "node log line\n"
            assert (await _get(f"{u}/logs/kubelet.log", good))[0] == 403
            assert (await _get(f"{u}/logs/..%2F..%2Fetc%2Fpasswd", loop))[0] == 404
            # audit events reach the webhook in batches
            for _ in range(50):
                if calls["audit"]:
                    break
                await asyncio_sleep(0.1)
            assert any(e.get("user", {}).get("username") == "alice" for e in calls["audit"])
        finally:
            await srv.stop()
            await runner.cleanup()
    run(go(), 60)


async def asyncio_sleep(t):
    import asyncio
    await asyncio.sleep(t)


def _b64u(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def test_oidc_id_tokens(tmp_path):
    key = tmp_path / "k.pem"
    subprocess.run(["openssl", "genrsa", "-out", str(key), "2048"], check=True, capture_output=True)
    mod = subprocess.run(["openssl", "rsa", "-in", str(key), "-noout", "-modulus"], capture_output=True, text=True,
                         check=True).stdout.strip().split("=")[1]
    n = int(mod, 16)
    jwk = {"kty": "RSA", "kid": "k1", "alg": "RS256", "n": _b64u(n.to_bytes((n.bit_length() + 7) // 8, "big")),
           "e": _b64u((65537).to_bytes(3, "big"))}

    def sign(claims, kid="k1"):
        h = _b64u(json.dumps({"alg": "RS256", "kid": kid}).encode())
        p = _b64u(json.dumps(claims).encode())
        (tmp_path / "d").write_bytes(f"{h}.{p}".encode())
        subprocess.run(["openssl", "dgst", "-sha256", "-sign", str(key), "-out", str(tmp_path / "s"), str(tmp_path / "d")],
                       check=True, capture_output=True)
        return f"{h}.{p}.{_b64u((tmp_path / 's').read_bytes())}"

    async def go():
        state = {}

        async def disc(req):
            return web.json_response({"issuer": state["iss"], "jwks_uri": state["iss"] + "/keys"})

        async def keys(req):
            return web.json_response({"keys": [jwk]})
        runner, iss = await _serve([("GET", "/.well-known/openid-configuration", disc), ("GET", "/keys", keys)])
        state["iss"] = iss
        srv = await APIServer(authorization_mode="RBAC", anonymous_auth=False, options={
            "oidc_issuer_url": iss, "oidc_client_id": "amdkube", "oidc_groups_claim": "groups",
            "oidc_groups_prefix": "oidc:"}).start()
        try:
            loop = {"Authorization": f"Bearer {srv.loopback_token}"}
            now = int(time.time())
            tok = sign({"iss": iss, "aud": "amdkube", "sub": "1234", "exp": now + 600, "groups": ["mlops"]})
            st, body, _ = await _get(f"{srv.url}/apis/authentication.k8s.io/v1/tokenreviews", loop, "POST",
                                     {"apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview", "spec": {"token": tok}})
            u = json.loads(body)["status"]
            assert u["authenticated"] and u["user"]["username"] == f"{iss}#1234" and "oidc:mlops" in u["user"]["groups"]
            # an RBAC binding for the OIDC group lets the token read pods
            for obj, path in (({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                                "metadata": {"name": "mlops-view"}, "roleRef": {"apiGroup": "rbac.authorization.k8s.io",
                                                                              "kind": "ClusterRole", "name": "view"},
                                "subjects": [{"kind": "Group", "name": "oidc:mlops", "apiGroup": "rbac.authorization.k8s.io"}]},
                               "/apis/rbac.authorization.k8s.io/v1/clusterrolebindings"),):
                assert (await _get(srv.url + path, loop, "POST", obj))[0] == 201
            assert (await _get(f"{srv.url}/api/v1/namespaces/default/pods", {"Authorization": f"Bearer {tok}"}))[0] == 200
            for bad in (sign({"iss": iss, "aud": "other", "sub": "1", "exp": now + 600}),
                        sign({"iss": iss, "aud": "amdkube", "sub": "1", "exp": now - 10}),
                        tok[:-4] + ("AAAA" if not tok.endswith("AAAA") else "BBBB")):
                assert (await _get(f"{srv.url}/api/v1/namespaces/default/pods", {"Authorization": f"Bearer {bad}"}))[0] == 401
        finally:
            await srv.stop()
            await runner.cleanup()
    run(go(), 60)


def test_secure_and_insecure_listeners(tmp_path):
    d = str(tmp_path)
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/s.key", "-out", f"{d}/s.crt",
                    "-days", "1", "-subj", "/CN=localhost", "-addext", "subjectAltName=IP:127.0.0.1"], check=True, capture_output=True)

    async def go():
        srv = await APIServer(anonymous_auth=False, tls_cert_file=f"{d}/s.crt", tls_key_file=f"{d}/s.key",
                              token_auth={"t0k": {"name": "carol", "groups": []}},
                              options={"insecure_port": 0 or _free(), "insecure_bind_address": "127.0.0.1"}).start()
        try:
            import ssl
            ctx = ssl.create_default_context(cafile=f"{d}/s.crt")
            async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(ssl=ctx)) as s:
                async with s.get(f"{srv.url}/api/v1/namespaces") as r:
                    assert r.status == 401          # the secure port authenticates
                async with s.get(f"{srv.url}/api/v1/namespaces", headers={"Authorization": "Bearer t0k"}) as r:
                    assert r.status == 200
            st, body, _ = await _get(f"http://127.0.0.1:{srv.insecure_port}/api/v1/namespaces")
            assert st == 200 and "default" in body      # the local insecure port is unauthenticated
        finally:
            await srv.stop()
    run(go(), 60)


def _free():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
