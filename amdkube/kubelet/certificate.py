"""Kubelet certificate rotation (pkg/kubelet/certificate: manager.go, kubelet.go,
transport.go; RotateKubeletClientCertificate beta / RotateKubeletServerCertificate alpha).

A CertManager owns one identity in --cert-dir: `kubelet-<kind>-current.pem` (a symlink to
`kubelet-<kind>-<timestamp>.pem`, certificate + key in one file). Its rotation deadline is a
random point between 70 % and 90 % of the certificate's validity (manager.go
nextRotationDeadline); at the deadline — or at once when there is no usable certificate — it
makes a new key, submits a CertificateSigningRequest (client: O=system:nodes,
CN=system:node:<name>, usages digital signature/key encipherment/client auth; server: the same
subject plus the node's addresses as SANs and server auth), waits for it to be approved and
issued, writes the new pair and tells its listeners (the API client re-dials with it, the
kubelet's TLS listener serves it to new connections).
"""
from __future__ import annotations

import asyncio
import base64
import datetime as _dt
import hashlib
import logging
import os
import random
import subprocess
import tempfile
import time

log = logging.getLogger("amdkube.kubelet.certificate")

USAGES = {"client": ["digital signature", "key encipherment", "client auth"],
          "server": ["digital signature", "key encipherment", "server auth"]}


def _openssl(*args, input=None) -> bytes:
    r = subprocess.run(["openssl", *args], capture_output=True, input=input, timeout=60)
    if r.returncode != 0:
        raise RuntimeError(f"openssl {args[0]} failed: {r.stderr.decode()[-300:]}")
    return r.stdout


def cert_validity(pem: bytes) -> tuple[float, float]:
    """(notBefore, notAfter) as epoch seconds."""
    out = _openssl("x509", "-noout", "-startdate", "-enddate", input=pem).decode()
    vals = {}
    for line in out.splitlines():
        k, _, v = line.partition("=")
        vals[k] = _dt.datetime.strptime(v.strip().replace("  ", " "), "%b %d %H:%M:%S %Y %Z").replace(
            tzinfo=_dt.timezone.utc).timestamp()
    return vals["notBefore"], vals["notAfter"]


def split_pem(blob: bytes) -> tuple[bytes, bytes]:
    """Certificate and key blocks of a combined PEM file."""
    cert, key, cur = [], [], None
    for line in blob.splitlines(keepends=True):
        if line.startswith(b"-----BEGIN"):
            cur = key if b"PRIVATE KEY" in line else cert
        if cur is not None:
            cur.append(line)
        if line.startswith(b"-----END"):
            cur = None
    return b"".join(cert), b"".join(key)


class CertManager:
    def __init__(self, client, cert_dir: str, node_name: str, kind: str = "client", addresses=(),
                 wait_timeout: float = 900.0, clock=time.time, rng=random.random):
        if kind not in USAGES:
            raise ValueError(kind)
        self.client, self.dir, self.node, self.kind = client, cert_dir, node_name, kind
        self.addresses = list(addresses)
        self.wait_timeout, self.clock, self.rng = wait_timeout, clock, rng
        self.listeners: list = []          # fn(cert_path) after every rotation
        os.makedirs(cert_dir, mode=0o700, exist_ok=True)
        self.rotations = 0

    @property
    def current_path(self) -> str:
        return os.path.join(self.dir, f"kubelet-{self.kind}-current.pem")

    def current(self) -> bytes | None:
        try:
            with open(self.current_path, "rb") as f:
                return f.read()
        except OSError:
            return None

    def deadline(self) -> float:
        """nextRotationDeadline: notBefore + U(0.7, 0.9) × lifetime; now if unusable."""
        pem = self.current()
        if not pem:
            return self.clock()
        try:
            nb, na = cert_validity(split_pem(pem)[0])
        except (RuntimeError, ValueError, KeyError):
            return self.clock()
        return nb + (na - nb) * (0.7 + 0.2 * self.rng())

    def install(self, cert_pem: bytes, key_pem: bytes) -> str:
        """Write `kubelet-<kind>-<ts>.pem` and repoint the -current symlink atomically."""
        ts = _dt.datetime.utcfromtimestamp(self.clock()).strftime("%Y-%m-%d-%H-%M-%S")
        path = os.path.join(self.dir, f"kubelet-{self.kind}-{ts}-{self.rotations}.pem")
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "wb") as f:
            f.write(cert_pem + (b"" if cert_pem.endswith(b"\n") else b"\n") + key_pem)
        tmp = self.current_path + ".tmp"
        if os.path.lexists(tmp):
            os.unlink(tmp)
        os.symlink(os.path.basename(path), tmp)
        os.replace(tmp, self.current_path)
        self.rotations += 1
        for cb in list(self.listeners):
            cb(self.current_path)
        return path

    def _key_and_csr(self) -> tuple[bytes, bytes]:
        with tempfile.TemporaryDirectory() as td:
            cfg = os.path.join(td, "csr.cnf")
            sans = []
            for a in self.addresses:
                sans.append(("IP:" if a.replace(".", "").isdigit() or ":" in a else "DNS:") + a)
            with open(cfg, "w") as f:
                f.write("[req]\ndistinguished_name=dn\nprompt=no\n" + ("req_extensions=ext\n" if sans else "") +
                        f"[dn]\nO=system:nodes\nCN=system:node:{self.node}\n" +
                        (f"[ext]\nsubjectAltName={','.join(sans)}\n" if sans else ""))
            key, csr = os.path.join(td, "k.pem"), os.path.join(td, "r.pem")
            _openssl("req", "-new", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes",
                     "-keyout", key, "-out", csr, "-config", cfg)
            return open(key, "rb").read(), open(csr, "rb").read()

    async def rotate(self) -> str:
        key, csr = await asyncio.to_thread(self._key_and_csr)
        name = f"csr-{self.kind}-{hashlib.sha256(csr).hexdigest()[:16]}"
        await self.client.create({"apiVersion": "certificates.k8s.io/v1beta1", "kind": "CertificateSigningRequest",
                                  "metadata": {"name": name},
                                  "spec": {"request": base64.b64encode(csr).decode(), "usages": USAGES[self.kind]}})
        end = time.monotonic() + self.wait_timeout
        while time.monotonic() < end:
            o = await self.client.get("certificatesigningrequests", name)
            st = o.get("status") or {}
            if any(x.get("type") == "Denied" for x in st.get("conditions") or []):
                raise RuntimeError(f"certificate signing request {name} was denied")
            if st.get("certificate"):
                path = self.install(base64.b64decode(st["certificate"]), key)
                log.info("rotated the kubelet %s certificate (%s)", self.kind, os.path.basename(path))
                return path
            await asyncio.sleep(0.2)
        raise TimeoutError(f"timed out waiting for the certificate of {name}")

    async def run(self):
        backoff = 1.0
        while True:
            wait = self.deadline() - self.clock()
            if wait > 0:
                await asyncio.sleep(min(wait, 3600.0))
                continue
            try:
                await self.rotate()
                backoff = 1.0
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.warning("kubelet %s certificate rotation failed: %r; retrying in %.0fs", self.kind, e, backoff)
                await asyncio.sleep(backoff)
                backoff = min(128.0, backoff * 2)
