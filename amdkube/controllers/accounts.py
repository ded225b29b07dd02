"""Service accounts, their tokens, certificate signing requests and bootstrap tokens.

Reference:
  * pkg/controller/serviceaccount/serviceaccounts_controller.go — every active namespace
    gets the `default` ServiceAccount.
  * pkg/controller/serviceaccount/tokens_controller.go — each ServiceAccount gets a secret
    `<sa>-token-<suffix>` of type kubernetes.io/service-account-token holding `token`
    (JWT, see apiserver/auth.py), `namespace` and `ca.crt`, referenced from sa.secrets; a
    token secret whose account is gone is deleted; a deleted secret is unreferenced.
  * pkg/controller/certificates/{approver/sarapprove.go, signer/cfssl_signer.go,
    cleaner/cleaner.go} — a CSR for a node client certificate (CN system:node:<name>,
    O system:nodes, usages within digital signature / key encipherment / client auth) is
    approved when a SubjectAccessReview lets its requester create
    certificatesigningrequests/nodeclient (or /selfnodeclient for its own node); approved
    CSRs are signed by the cluster CA (--cluster-signing-{cert,key}-file, openssl here);
    issued or denied CSRs are removed after 1 h, pending ones after 24 h.
  * pkg/controller/bootstrap/{bootstrapsigner.go, tokencleaner.go} — kube-public/cluster-info
    carries a detached JWS `jws-kubeconfig-<token-id>` of its kubeconfig for every bootstrap
    token allowed to sign (HS256 keyed by the full token); expired bootstrap-token secrets
    are deleted.
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import hmac
import json
import os
import secrets as pysecrets
import subprocess
import tempfile
import time

from ..api import meta as m
from ..apiserver.auth import service_account_token
from .base import Controller, split_key

SA_TOKEN_TYPE = "kubernetes.io/service-account-token"
BOOTSTRAP_TYPE = "bootstrap.kubernetes.io/token"
A_SA_NAME = "kubernetes.io/service-account.name"
A_SA_UID = "kubernetes.io/service-account.uid"


def _b64(s: str | bytes) -> str:
    return base64.b64encode(s.encode() if isinstance(s, str) else s).decode()


class ServiceAccountsController(Controller):
    name = "serviceaccount"
    workers = 1
    accounts = ("default",)

    def setup(self):
        f = self.mgr.factory
        self.ns_inf = f.informer("namespaces")
        self.sa_inf = f.informer("serviceaccounts")
        self.ns_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))
        self.sa_inf.add_handler(on_delete=lambda sa: self.enqueue(m.namespace_of(sa)))

    async def sync(self, key):
        _, ns = split_key(key)
        nsobj = self.ns_inf.get(ns)
        if nsobj is None or (nsobj.get("status") or {}).get("phase") == "Terminating":
            return
        for name in self.accounts:
            if self.sa_inf.get(f"{ns}/{name}") is None:
                try:
                    await self.client.create({"apiVersion": "v1", "kind": "ServiceAccount",
                                              "metadata": {"name": name, "namespace": ns}}, ns)
                except m.StatusError as e:
                    if not m.is_already_exists(e):
                        raise


class TokensController(Controller):
    name = "serviceaccount-token"
    workers = 1

    def __init__(self, mgr, key: bytes | None = None, root_ca: bytes = b""):
        super().__init__(mgr)
        self.key = key
        self.root_ca = root_ca

    def setup(self):
        f = self.mgr.factory
        self.sa_inf = f.informer("serviceaccounts")
        self.sec_inf = f.informer("secrets")
        self.sa_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n),
                                on_delete=lambda sa: self.enqueue("delete:" + m.key_of(sa)))
        self.sec_inf.add_handler(on_delete=self._secret_deleted)

    def _secret_deleted(self, s):
        if s.get("type") == SA_TOKEN_TYPE:
            name = m.annotations_of(s).get(A_SA_NAME)
            if name:
                self.enqueue(f"{m.namespace_of(s)}/{name}")

    def _tokens_of(self, ns, sa_name, sa_uid=None):
        return [s for s in self.sec_inf.list() if m.namespace_of(s) == ns and s.get("type") == SA_TOKEN_TYPE
                and m.annotations_of(s).get(A_SA_NAME) == sa_name
                and (sa_uid is None or m.annotations_of(s).get(A_SA_UID) == sa_uid)]

    async def sync(self, key):
        if self.key is None:
            return
        if key.startswith("delete:"):
            ns, name = split_key(key[len("delete:"):])
            for s in self._tokens_of(ns, name):
                try:
                    await self.client.delete("secrets", m.name_of(s), ns)
                except m.StatusError:
                    pass
            return
        sa = self.sa_inf.get(key)
        if sa is None:
            return
        ns, name = split_key(key)
        live = {m.name_of(s) for s in self._tokens_of(ns, name, m.uid_of(sa))}
        refs = [r for r in sa.get("secrets") or [] if r.get("name") in live or not r.get("name", "").startswith(f"{name}-token-")]
        if not any(r.get("name") in live for r in refs):
            sname = f"{name}-token-{pysecrets.token_hex(3)[:5]}"
            tok = service_account_token(self.key, ns, name, m.uid_of(sa), sname)
            data = {"token": _b64(tok), "namespace": _b64(ns)}
            if self.root_ca:
                data["ca.crt"] = _b64(self.root_ca)
            await self.client.create({"apiVersion": "v1", "kind": "Secret", "type": SA_TOKEN_TYPE,
                                      "metadata": {"name": sname, "namespace": ns,
                                                   "annotations": {A_SA_NAME: name, A_SA_UID: m.uid_of(sa)}},
                                      "data": data}, ns)
            refs.append({"name": sname})
        if refs != (sa.get("secrets") or []):
            await self.client.patch("serviceaccounts", name, {"secrets": refs}, ns)


# --------------------------------------------------------------------------- CSRs
def csr_subject(pem: bytes) -> dict:
    """CN / O of a PEM CSR (openssl req -subject)."""
    r = subprocess.run(["openssl", "req", "-noout", "-subject", "-nameopt", "sep_multiline,utf8"], input=pem,
                       capture_output=True, timeout=10)
    if r.returncode != 0:
        raise ValueError("unparseable certificate request: " + r.stderr.decode()[-200:])
    out: dict[str, list] = {}
    for line in r.stdout.decode().splitlines()[1:]:
        k, _, v = line.strip().partition("=")
        out.setdefault(k.strip(), []).append(v.strip())
    return out


NODE_CLIENT_USAGES = {"key encipherment", "digital signature", "client auth"}


def _condition(csr, t):
    return any(c.get("type") == t for c in (csr.get("status") or {}).get("conditions") or [])


class CSRApprovingController(Controller):
    name = "csrapproving"
    workers = 1

    def setup(self):
        self.csr_inf = self.mgr.factory.informer("certificatesigningrequests")
        self.csr_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))

    async def _allowed(self, spec, subresource) -> bool:
        sar = {"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
               "spec": {"user": spec.get("username", ""), "groups": spec.get("groups") or [], "uid": spec.get("uid", ""),
                        "resourceAttributes": {"group": "certificates.k8s.io", "resource": "certificatesigningrequests",
                                               "subresource": subresource, "verb": "create"}}}
        r = await self.client.create(sar)
        return bool((r.get("status") or {}).get("allowed"))

    async def sync(self, key):
        _, name = split_key(key)
        csr = self.csr_inf.get(name)
        if csr is None or _condition(csr, "Approved") or _condition(csr, "Denied"):
            return
        spec = csr.get("spec") or {}
        try:
            subj = await asyncio.get_running_loop().run_in_executor(None, csr_subject, base64.b64decode(spec.get("request", "")))
        except (ValueError, subprocess.SubprocessError):
            return
        cn = (subj.get("CN") or [""])[0]
        if not cn.startswith("system:node:") or subj.get("O") != ["system:nodes"]:
            return  # not a node client certificate: left for a human (kubectl certificate approve)
        if not set(spec.get("usages") or []) <= NODE_CLIENT_USAGES:
            return
        sub = "selfnodeclient" if spec.get("username") == cn else "nodeclient"
        if not await self._allowed(spec, sub):
            return
        csr = dict(csr, status=dict(csr.get("status") or {}, conditions=[
            {"type": "Approved", "reason": "AutoApproved", "message": f"Auto approving {sub} certificate after SubjectAccessReview.",
             "lastUpdateTime": m.now_rfc3339()}]))
        await self.client.update(csr, sub="approval")


class CSRSigningController(Controller):
    name = "csrsigning"
    workers = 1

    def __init__(self, mgr, cert_file: str | None = None, key_file: str | None = None, days: int = 365):
        super().__init__(mgr)
        self.cert_file, self.key_file, self.days = cert_file, key_file, days

    def setup(self):
        self.csr_inf = self.mgr.factory.informer("certificatesigningrequests")
        self.csr_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))

    KEY_USAGES = {"digital signature": "digitalSignature", "key encipherment": "keyEncipherment",
                  "content commitment": "nonRepudiation", "data encipherment": "dataEncipherment",
                  "key agreement": "keyAgreement", "cert sign": "keyCertSign", "crl sign": "cRLSign"}
    EXT_USAGES = {"client auth": "clientAuth", "server auth": "serverAuth", "code signing": "codeSigning",
                  "email protection": "emailProtection", "timestamping": "timeStamping", "ocsp signing": "OCSPSigning"}

    def sign(self, pem: bytes, usages=()) -> bytes:
        """cfssl_signer.go: the CSR's subject and SANs, the requested key usages, the signing duration."""
        with tempfile.TemporaryDirectory() as d:
            req = os.path.join(d, "req.pem")
            with open(req, "wb") as f:
                f.write(pem)
            ku = [self.KEY_USAGES[u] for u in usages if u in self.KEY_USAGES]
            eku = [self.EXT_USAGES[u] for u in usages if u in self.EXT_USAGES]
            ext = os.path.join(d, "ext.cnf")
            with open(ext, "w") as f:
                f.write("basicConstraints=critical,CA:FALSE\n")
                if ku:
                    f.write(f"keyUsage=critical,{','.join(ku)}\n")
                if eku:
                    f.write(f"extendedKeyUsage={','.join(eku)}\n")
            r = subprocess.run(["openssl", "x509", "-req", "-in", req, "-CA", self.cert_file, "-CAkey", self.key_file,
                                "-CAcreateserial", "-CAserial", os.path.join(d, "ca.srl"), "-days", str(self.days),
                                "-sha256", "-extfile", ext, "-copy_extensions", "copy"], capture_output=True, timeout=20)
            if r.returncode != 0:
                raise RuntimeError("signing failed: " + r.stderr.decode()[-300:])
            return r.stdout

    async def sync(self, key):
        if not (self.cert_file and self.key_file):
            return
        _, name = split_key(key)
        csr = self.csr_inf.get(name)
        if csr is None or not _condition(csr, "Approved") or (csr.get("status") or {}).get("certificate"):
            return
        pem = base64.b64decode((csr.get("spec") or {}).get("request", ""))
        usages = (csr.get("spec") or {}).get("usages") or []
        cert = await asyncio.get_running_loop().run_in_executor(None, self.sign, pem, usages)
        csr = dict(csr, status=dict(csr.get("status") or {}, certificate=_b64(cert)))
        await self.client.update(csr, sub="status")


class WebhookSigningController(Controller):
    """cmd/gke-certificates-controller gke_signer.go: approved CSRs are POSTed (certificates.k8s.io/
    v1beta1 JSON) to the signing service a kubeconfig names; its answer's status.certificate is
    written back through the status subresource. Retries back off exponentially from
    --cluster-signing-gke-retry-backoff; a failure is a Warning SigningError event and a requeue."""
    name = "csrsigning-webhook"
    workers = 1

    def __init__(self, mgr, kubeconfig: str, retry_backoff: float = 0.5, attempts: int = 5):
        super().__init__(mgr)
        self.kubeconfig, self.retry_backoff, self.attempts = kubeconfig, retry_backoff, attempts
        self._hook = None

    def setup(self):
        self.csr_inf = self.mgr.factory.informer("certificatesigningrequests")
        self.csr_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n))

    async def stop(self):
        if self._hook is not None:
            await self._hook.close()
        await super().stop()

    async def _sign(self, csr: dict) -> str:
        from ..apiserver.authx import _webhook_client
        if self._hook is None:
            self._hook = _webhook_client(self.kubeconfig)
        body = {**csr, "apiVersion": "certificates.k8s.io/v1beta1", "kind": "CertificateSigningRequest"}
        delay, last = self.retry_backoff, None
        for attempt in range(self.attempts):
            try:
                out = await self._hook.request("POST", "", body=body)
                cert = ((out or {}).get("status") or {}).get("certificate")
                if not cert:
                    raise RuntimeError("the signing service answered without status.certificate")
                return cert
            except m.StatusError as e:
                last = RuntimeError(f"server responded with error: {e}")
                if e.code < 500 and e.code != 429:
                    break           # a rejection: retrying will not help
            except Exception as e:  # noqa: BLE001 — connection errors are retried
                last = e
            if attempt + 1 < self.attempts:
                await asyncio.sleep(delay)
                delay *= 2
        raise last

    async def sync(self, key):
        _, name = split_key(key)
        csr = self.csr_inf.get(name)
        if csr is None or not _condition(csr, "Approved") or (csr.get("status") or {}).get("certificate"):
            return
        try:
            cert = await self._sign(csr)
        except Exception as e:
            rec = getattr(self.mgr, "recorder", None)
            if rec is not None:
                rec.event(csr, "Warning", "SigningError", f"error while calling GKE: {e}")
            raise
        csr = dict(csr, status=dict(csr.get("status") or {}, certificate=cert))
        await self.client.update(csr, sub="status")


class GroupCSRApprovingController(CSRApprovingController):
    """--insecure-experimental-approve-all-kubelet-csrs-for-group: every kubelet client CSR from a
    member of the group is approved without a SubjectAccessReview (gke-certificates-controller)."""
    name = "csrapproving-group"

    def __init__(self, mgr, group: str):
        super().__init__(mgr)
        self.group = group

    async def _allowed(self, spec, subresource) -> bool:
        return self.group in (spec.get("groups") or [])


class CSRCleanerController(Controller):
    name = "csrcleaner"
    workers = 1
    period = 3600.0
    APPROVED_TTL, DENIED_TTL, PENDING_TTL = 3600.0, 3600.0, 24 * 3600.0

    def setup(self):
        self.csr_inf = self.mgr.factory.informer("certificatesigningrequests")
        self._poll = None

    async def start(self):
        await super().start()
        self._poll = asyncio.create_task(self._loop())

    async def stop(self):
        if self._poll:
            self._poll.cancel()
        await super().stop()

    async def _loop(self):
        while True:
            for c in self.csr_inf.list():
                self.enqueue(c)
            await asyncio.sleep(self.period)

    def expired(self, csr, now=None) -> bool:
        now = now or time.time()
        created = m.parse_time((csr.get("metadata") or {}).get("creationTimestamp")) or now
        if _condition(csr, "Denied"):
            return now - created > self.DENIED_TTL
        if _condition(csr, "Approved") and (csr.get("status") or {}).get("certificate"):
            return now - created > self.APPROVED_TTL
        return now - created > self.PENDING_TTL

    async def sync(self, key):
        _, name = split_key(key)
        csr = self.csr_inf.get(name)
        if csr is not None and self.expired(csr):
            await self.client.delete("certificatesigningrequests", name)


# --------------------------------------------------------------------- bootstrap tokens
def _b64url(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def detached_jws(payload: str, token_id: str, token_secret: str) -> str:
    head = _b64url(json.dumps({"alg": "HS256", "kid": token_id}, separators=(",", ":")).encode())
    body = _b64url(payload.encode())
    sig = hmac.new(f"{token_id}.{token_secret}".encode(), f"{head}.{body}".encode(), hashlib.sha256).digest()
    return f"{head}..{_b64url(sig)}"


def verify_detached_jws(jws: str, payload: str, token_id: str, token_secret: str) -> bool:
    return hmac.compare_digest(jws, detached_jws(payload, token_id, token_secret))


def _token_data(s) -> dict:
    return {k: base64.b64decode(v).decode() for k, v in (s.get("data") or {}).items()}


class BootstrapSignerController(Controller):
    name = "bootstrapsigner"
    workers = 1

    def setup(self):
        f = self.mgr.factory
        self.cm_inf = f.informer("configmaps")
        self.sec_inf = f.informer("secrets")
        self.cm_inf.add_handler(on_add=self._cm, on_update=lambda o, n: self._cm(n))
        self.sec_inf.add_handler(on_add=self._sec, on_update=lambda o, n: self._sec(n), on_delete=self._sec)

    def _cm(self, cm):
        if m.key_of(cm) == "kube-public/cluster-info":
            self.enqueue("kube-public/cluster-info")

    def _sec(self, s):
        if s.get("type") == BOOTSTRAP_TYPE:
            self.enqueue("kube-public/cluster-info")

    async def sync(self, key):
        cm = self.cm_inf.get("kube-public/cluster-info")
        if cm is None:
            return
        data = dict(cm.get("data") or {})
        payload = data.get("kubeconfig")
        if payload is None:
            return
        want = {k: v for k, v in data.items() if not k.startswith("jws-kubeconfig-")}
        now = time.time()
        for s in self.sec_inf.list():
            if m.namespace_of(s) != "kube-system" or s.get("type") != BOOTSTRAP_TYPE:
                continue
            d = _token_data(s)
            exp = m.parse_time(d.get("expiration"))
            if d.get("usage-bootstrap-signing") != "true" or (exp is not None and exp < now):
                continue
            if d.get("token-id") and d.get("token-secret"):
                want[f"jws-kubeconfig-{d['token-id']}"] = detached_jws(payload, d["token-id"], d["token-secret"])
        if want != data:
            cm = dict(cm, data=want)
            await self.client.update(cm)


class TokenCleanerController(Controller):
    name = "tokencleaner"
    workers = 1

    def setup(self):
        self.sec_inf = self.mgr.factory.informer("secrets")
        self.sec_inf.add_handler(on_add=self._sec, on_update=lambda o, n: self._sec(n))

    def _sec(self, s):
        if s.get("type") == BOOTSTRAP_TYPE and m.namespace_of(s) == "kube-system":
            exp = m.parse_time(_token_data(s).get("expiration"))
            if exp is not None:
                delay = max(0.0, exp - time.time())
                asyncio.get_running_loop().call_later(delay + 0.01, self.enqueue, m.key_of(s))

    async def sync(self, key):
        s = self.sec_inf.get(key)
        if s is None:
            return
        exp = m.parse_time(_token_data(s).get("expiration"))
        if exp is not None and exp <= time.time():
            ns, name = split_key(key)
            try:
                await self.client.delete("secrets", name, ns)
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise
