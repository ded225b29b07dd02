"""Docker Registry HTTP API v2 client: the pull half of rocshim's ImageService.

Reference: the kubelet asks the runtime to pull (kubeGenericRuntimeManager.PullImage,
pkg/kubelet/kuberuntime/kuberuntime_image.go:31, behind imageManager.EnsureImageExists,
pkg/kubelet/images/image_manager.go:86) with the CRI AuthConfig it derived from the pod's
imagePullSecrets / the node's docker config; dockershim hands it to dockerd
(dockerService.PullImage, pkg/kubelet/dockershim/docker_image.go:73), which speaks this
protocol (docker/distribution "Registry HTTP API V2").

What is implemented:
  * `GET /v2/` probe; `WWW-Authenticate: Bearer realm=…,service=…[,scope=…]` → token from the
    realm with `scope=repository:<repo>:pull` (Basic-authenticated with the AuthConfig when
    given; `token` or `access_token` in the reply); `WWW-Authenticate: Basic` → Basic on every
    request. A 401 after authenticating is "unauthorized: authentication required".
  * `GET /v2/<repo>/manifests/<tag|digest>` accepting Docker schema2 and OCI image manifests
    and manifest lists / OCI indexes; a list resolves to its linux/amd64 entry, fetched by
    digest. A manifest fetched by digest must hash to that digest.
  * `GET /v2/<repo>/blobs/<digest>` for the config and every layer, streamed to disk and
    verified against its digest (a tampered blob is refused); registry redirects are followed
    without forwarding the Authorization header.
  * Scheme: https (optionally with a CA bundle); plain http for hosts listed as insecure and
    for loopback registries (dockerd's default for 127.0.0.0/8 and localhost).

The result feeds oci.import_layers, the same unpacker as docker-archive / OCI-layout imports.
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import re
import shutil
import ssl
import urllib.error
import urllib.parse
import urllib.request

from .oci import ImageFormatError

MT_MANIFEST_V2 = "application/vnd.docker.distribution.manifest.v2+json"
MT_MANIFEST_LIST = "application/vnd.docker.distribution.manifest.list.v2+json"
MT_OCI_MANIFEST = "application/vnd.oci.image.manifest.v1+json"
MT_OCI_INDEX = "application/vnd.oci.image.index.v1+json"
ACCEPT = ", ".join((MT_MANIFEST_V2, MT_MANIFEST_LIST, MT_OCI_MANIFEST, MT_OCI_INDEX))
DOCKER_HUB = "registry-1.docker.io"
_DIGEST = re.compile(r"^(sha256|sha512):[0-9a-f]+$")


class RegistryError(Exception):
    pass


class Unauthorized(PermissionError):
    pass


def parse_reference(ref: str) -> tuple[str, str, str]:
    """(registry host[:port], repository, tag or digest) of an image reference, as
    docker/distribution's reference.ParseNormalizedNamed reads it."""
    ref = ref.strip()
    name, digest = (ref.split("@", 1) + [""])[:2]
    first, _, rest = name.partition("/")
    if rest and ("." in first or ":" in first or first == "localhost"):
        host, path = first, rest
    else:
        host, path = DOCKER_HUB, name
    tag = ""
    last = path.rsplit("/", 1)[-1]
    if ":" in last:
        path, tag = path.rsplit(":", 1)
    if host == DOCKER_HUB and "/" not in path:
        path = "library/" + path
    return host, path, digest or tag or "latest"


def is_remote(ref: str) -> bool:
    """A reference naming a registry host (`host.domain/…`, `host:port/…`, `localhost/…`)."""
    if ref.startswith(("file://", "/")):
        return False
    first, _, rest = ref.split("@", 1)[0].partition("/")
    return bool(rest) and ("." in first or ":" in first or first == "localhost")


def _loopback(host: str) -> bool:
    h = host.rsplit(":", 1)[0] if not host.startswith("[") else host[1:host.index("]")]
    return h in ("localhost", "::1") or h.startswith("127.")


class _NoAuthRedirect(urllib.request.HTTPRedirectHandler):
    """Follow registry redirects (blob storage) without the registry's Authorization."""

    def redirect_request(self, req, fp, code, msg, headers, newurl):
        new = super().redirect_request(req, fp, code, msg, headers, newurl)
        if new is not None:
            new.headers.pop("Authorization", None)
            new.unredirected_hdrs.pop("Authorization", None)
        return new


class RegistryClient:
    def __init__(self, insecure: tuple[str, ...] | list[str] = (), ca_file: str | None = None, timeout: float = 60.0,
                 platform: tuple[str, str] = ("linux", "amd64")):
        self.insecure = set(insecure)
        self.timeout = timeout
        self.platform = platform
        ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()
        self._opener = urllib.request.build_opener(_NoAuthRedirect(), urllib.request.HTTPSHandler(context=ctx))
        self._auth: dict[tuple, str] = {}     # (host, repo, credentials) -> Authorization header value

    # ------------------------------------------------------------------ transport
    def _base(self, host: str) -> str:
        return ("http://" if host in self.insecure or _loopback(host) else "https://") + host

    def _open(self, url: str, headers: dict | None = None):
        req = urllib.request.Request(url)
        for k, v in (headers or {}).items():
            if k == "Authorization":
                req.add_unredirected_header(k, v)
            else:
                req.add_header(k, v)
        return self._opener.open(req, timeout=self.timeout)

    @staticmethod
    def _basic(creds: dict | None) -> str | None:
        if not creds:
            return None
        user, pw = creds.get("username") or "", creds.get("password") or ""
        if not user and creds.get("auth"):
            try:
                user, _, pw = base64.b64decode(creds["auth"]).decode().partition(":")
            except ValueError:
                return None
        if not user:
            return None
        return "Basic " + base64.b64encode(f"{user}:{pw}".encode()).decode()

    @staticmethod
    def _challenge(header: str) -> tuple[str, dict]:
        scheme, _, rest = header.strip().partition(" ")
        params = dict(re.findall(r'(\w+)="([^"]*)"', rest))
        return scheme.lower(), params

    def _authorize(self, host: str, repo: str, challenge: str, creds: dict | None) -> str:
        scheme, p = self._challenge(challenge)
        if scheme == "basic":
            basic = self._basic(creds)
            if basic is None:
                raise Unauthorized(f"pull access denied for {host}/{repo}: unauthorized: authentication required")
            return basic
        if scheme != "bearer" or "realm" not in p:
            raise RegistryError(f"{host}: unsupported authentication challenge {challenge!r}")
        q = {"scope": f"repository:{repo}:pull"}
        if p.get("service"):
            q["service"] = p["service"]
        url = p["realm"] + ("&" if "?" in p["realm"] else "?") + urllib.parse.urlencode(q)
        hdr = {}
        basic = self._basic(creds)
        if basic:
            hdr["Authorization"] = basic
        try:
            with self._open(url, hdr) as r:
                body = json.loads(r.read() or b"{}")
        except urllib.error.HTTPError as e:
            if e.code in (401, 403):
                raise Unauthorized(f"pull access denied for {host}/{repo}: unauthorized: incorrect username or password") from None
            raise RegistryError(f"{host}: token endpoint answered {e.code}") from None
        token = body.get("token") or body.get("access_token")
        if not token:
            raise RegistryError(f"{host}: token endpoint returned no token")
        return "Bearer " + token

    def _get(self, host: str, repo: str, path: str, creds: dict | None, accept: str | None = None):
        """GET with the registry's auth dance; returns the open response."""
        url = self._base(host) + path
        key = (host, repo, self._basic(creds) or "")     # a token is only reused for the same credentials
        for attempt in range(2):
            hdr = {"Accept": accept} if accept else {}
            if key in self._auth:
                hdr["Authorization"] = self._auth[key]
            try:
                return self._open(url, hdr)
            except urllib.error.HTTPError as e:
                if e.code == 401 and attempt == 0:
                    ch = e.headers.get("WWW-Authenticate")
                    if not ch:
                        raise Unauthorized(f"pull access denied for {host}/{repo}: unauthorized") from None
                    self._auth[key] = self._authorize(host, repo, ch, creds)
                    continue
                if e.code in (401, 403):
                    raise Unauthorized(f"pull access denied for {host}/{repo}: unauthorized: authentication required") from None
                if e.code == 404:
                    raise KeyError(f"{host}/{repo}: {path.rsplit('/', 1)[-1]} not found") from None
                raise RegistryError(f"{host}/{repo}: GET {path}: HTTP {e.code}") from None
            except urllib.error.URLError as e:
                raise RegistryError(f"{host}: {e.reason}") from None
        raise Unauthorized(f"pull access denied for {host}/{repo}")

    # ------------------------------------------------------------------ protocol
    def manifest(self, host: str, repo: str, ref: str, creds: dict | None = None) -> tuple[dict, str]:
        """The image manifest (a list/index resolved to this platform) and its digest."""
        for _ in range(2):
            with self._get(host, repo, f"/v2/{repo}/manifests/{ref}", creds, ACCEPT) as r:
                body = r.read()
                ctype = (r.headers.get("Content-Type") or "").split(";")[0].strip()
                hdr_digest = r.headers.get("Docker-Content-Digest")
            digest = "sha256:" + hashlib.sha256(body).hexdigest()
            if _DIGEST.match(ref) and not self._matches(body, ref):
                raise ImageFormatError(f"{host}/{repo}: manifest does not match its digest {ref}")
            if hdr_digest and hdr_digest.startswith("sha256:") and hdr_digest != digest:
                raise ImageFormatError(f"{host}/{repo}: manifest digest {digest} differs from Docker-Content-Digest {hdr_digest}")
            try:
                m = json.loads(body)
            except ValueError:
                raise ImageFormatError(f"{host}/{repo}: manifest is not JSON") from None
            mt = m.get("mediaType") or ctype
            if mt in (MT_MANIFEST_LIST, MT_OCI_INDEX) or (m.get("manifests") and not m.get("layers")):
                ref = self._pick(host, repo, m)
                continue
            if m.get("schemaVersion") != 2 or "config" not in m:
                raise ImageFormatError(f"{host}/{repo}: unsupported manifest (schemaVersion {m.get('schemaVersion')}, "
                                       f"{mt or 'no media type'})")
            return m, digest
        raise ImageFormatError(f"{host}/{repo}: manifest list nested in a manifest list")

    def _pick(self, host: str, repo: str, index: dict) -> str:
        os_, arch = self.platform
        for d in index.get("manifests") or []:
            p = d.get("platform") or {}
            if p.get("os") == os_ and p.get("architecture") == arch:
                return d["digest"]
        raise KeyError(f"{host}/{repo}: no manifest for platform {os_}/{arch}")

    @staticmethod
    def _matches(data: bytes, digest: str) -> bool:
        algo, _, hexd = digest.partition(":")
        return hashlib.new(algo, data).hexdigest() == hexd

    def blob(self, host: str, repo: str, digest: str, dest: str, creds: dict | None = None) -> str:
        """Stream blob `digest` to `dest`, verified against the digest."""
        if not _DIGEST.match(digest or ""):
            raise ImageFormatError(f"{host}/{repo}: malformed digest {digest!r}")
        algo, _, hexd = digest.partition(":")
        h = hashlib.new(algo)
        with self._get(host, repo, f"/v2/{repo}/blobs/{digest}", creds) as r, open(dest, "wb") as f:
            while True:
                chunk = r.read(1 << 20)
                if not chunk:
                    break
                h.update(chunk)
                f.write(chunk)
        if h.hexdigest() != hexd:
            os.unlink(dest)
            raise ImageFormatError(f"{host}/{repo}: blob {digest} does not match its digest")
        return dest

    def pull(self, ref: str, work: str, creds: dict | None = None) -> tuple[dict, list[str], str]:
        """(image config, [layer files in order], manifest digest) of `ref`, blobs under `work`."""
        host, repo, tag = parse_reference(ref)
        m, digest = self.manifest(host, repo, tag, creds)
        os.makedirs(work, exist_ok=True)
        cfg_path = self.blob(host, repo, m["config"]["digest"], os.path.join(work, "config.json"), creds)
        with open(cfg_path) as f:
            cfg = json.load(f)
        layers = []
        for i, layer in enumerate(m.get("layers") or []):
            mt = layer.get("mediaType") or ""
            if "foreign" in mt or layer.get("urls"):
                raise ImageFormatError(f"{host}/{repo}: layer {i} is a foreign layer ({mt})")
            layers.append(self.blob(host, repo, layer["digest"], os.path.join(work, f"layer{i}.tar"), creds))
        return cfg, layers, digest


def pull_image(ref: str, store_root: str, creds: dict | None = None, client: RegistryClient | None = None) -> dict:
    """Pull `ref` and unpack it into the image store (oci.import_layers); returns the record."""
    from .oci import import_layers
    client = client or RegistryClient()
    import tempfile
    os.makedirs(store_root, exist_ok=True)
    work = tempfile.mkdtemp(dir=store_root, prefix=".pull-")
    try:
        cfg, layers, digest = client.pull(ref, work, creds)
        rec = import_layers(cfg, layers, [ref], store_root)
        host, repo, _ = parse_reference(ref)
        rec["repo_digests"] = [f"{host}/{repo}@{digest}"]
        return rec
    finally:
        shutil.rmtree(work, ignore_errors=True)
