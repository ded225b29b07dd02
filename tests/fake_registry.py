"""An in-process Docker Registry HTTP API v2 server for tests (like the fake clouds): /v2/,
a Bearer token service (realm /token, Basic-authenticated), manifests by tag or digest
(schema2, OCI, manifest lists), blobs (optionally via a redirect to an unauthenticated blob
store, as registries hand blobs to object storage), and hooks to tamper with a blob."""
from __future__ import annotations

import base64
import gzip
import hashlib
import json
import secrets
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from amdkube.runtime.oci import _tar_bytes
from amdkube.runtime.registry import MT_MANIFEST_LIST, MT_MANIFEST_V2

MT_LAYER = "application/vnd.docker.image.rootfs.diff.tar.gzip"
MT_CONFIG = "application/vnd.docker.container.image.v1+json"


class FakeRegistry:
    def __init__(self, users: dict[str, str] | None = None, auth: str = "bearer", redirect_blobs: bool = False):
        self.users = users or {}          # empty: public
        self.auth = auth                  # "bearer" | "basic"
        self.redirect_blobs = redirect_blobs
        self.blobs: dict[str, bytes] = {}
        self.manifests: dict[tuple[str, str], tuple[str, bytes]] = {}   # (repo, tag|digest) -> (media type, body)
        self.tokens: dict[str, str] = {}  # token -> scope
        self.log: list[tuple[str, str, str | None]] = []               # (method, path, Authorization)
        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self.host = f"127.0.0.1:{self.srv.server_address[1]}"
        self._t = threading.Thread(target=self.srv.serve_forever, daemon=True)

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *exc):
        self.srv.shutdown()
        self.srv.server_close()

    # ------------------------------------------------------------------ content
    def put_blob(self, data: bytes) -> str:
        d = "sha256:" + hashlib.sha256(data).hexdigest()
        self.blobs[d] = data
        return d

    def push(self, repo: str, tag: str, layers: list[list[tuple]], config: dict, arch: str = "amd64") -> str:
        """Push an image of in-memory layers (oci._tar_bytes entries); returns its manifest digest."""
        descs, diffs = [], []
        for entries in layers:
            raw = _tar_bytes(entries)
            diffs.append("sha256:" + hashlib.sha256(raw).hexdigest())
            gz = gzip.compress(raw)
            descs.append({"mediaType": MT_LAYER, "size": len(gz), "digest": self.put_blob(gz)})
        cfg = json.dumps({"architecture": arch, "os": "linux", "config": config,
                          "rootfs": {"type": "layers", "diff_ids": diffs}}).encode()
        man = json.dumps({"schemaVersion": 2, "mediaType": MT_MANIFEST_V2,
                          "config": {"mediaType": MT_CONFIG, "size": len(cfg), "digest": self.put_blob(cfg)},
                          "layers": descs}).encode()
        d = "sha256:" + hashlib.sha256(man).hexdigest()
        self.manifests[(repo, tag)] = self.manifests[(repo, d)] = (MT_MANIFEST_V2, man)
        return d

    def push_list(self, repo: str, tag: str, entries: dict[str, str]) -> str:
        """A manifest list over {arch: manifest digest}."""
        lst = json.dumps({"schemaVersion": 2, "mediaType": MT_MANIFEST_LIST, "manifests": [
            {"mediaType": MT_MANIFEST_V2, "digest": d, "size": len(self.manifests[(repo, d)][1]),
             "platform": {"architecture": a, "os": "linux"}} for a, d in entries.items()]}).encode()
        d = "sha256:" + hashlib.sha256(lst).hexdigest()
        self.manifests[(repo, tag)] = self.manifests[(repo, d)] = (MT_MANIFEST_LIST, lst)
        return d

    def tamper(self, digest: str):
        self.blobs[digest] = gzip.compress(b"tampered")

    # ------------------------------------------------------------------ HTTP
    def _authorized(self, header: str | None, repo: str) -> bool:
        if not self.users:
            return True
        if not header:
            return False
        if self.auth == "basic":
            return header.startswith("Basic ") and self._basic_ok(header)
        return header.startswith("Bearer ") and self.tokens.get(header[7:]) in (f"repository:{repo}:pull", "*")

    def _basic_ok(self, header: str) -> bool:
        try:
            user, _, pw = base64.b64decode(header[6:]).decode().partition(":")
        except ValueError:
            return False
        return self.users.get(user) == pw

    def _handler(self):
        reg = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body=b"", headers=None):
                self.send_response(code)
                for k, v in (headers or {}).items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _challenge(self, repo):
                if reg.auth == "basic":
                    return {"WWW-Authenticate": 'Basic realm="fake-registry"'}
                scope = f',scope="repository:{repo}:pull"' if repo else ""
                return {"WWW-Authenticate": f'Bearer realm="http://{reg.host}/token",service="fake-registry"{scope}'}

            def do_GET(self):
                auth = self.headers.get("Authorization")
                reg.log.append(("GET", self.path, auth))
                path = self.path.split("?", 1)[0]
                if path == "/token":
                    from urllib.parse import parse_qs, urlparse
                    q = parse_qs(urlparse(self.path).query)
                    if reg.users and not (auth and auth.startswith("Basic ") and reg._basic_ok(auth)):
                        return self._send(401, b'{"errors":[{"code":"UNAUTHORIZED"}]}')
                    tok = secrets.token_hex(16)
                    reg.tokens[tok] = (q.get("scope") or ["*"])[0]
                    return self._send(200, json.dumps({"token": tok, "expires_in": 300}).encode(),
                                      {"Content-Type": "application/json"})
                if path.startswith("/blobstore/"):       # the redirect target: no auth here
                    data = reg.blobs.get(path.rsplit("/", 1)[1])
                    return self._send(200, data) if data is not None else self._send(404)
                if path == "/v2/" or path == "/v2":
                    if not reg._authorized(auth, ""):
                        if reg.auth == "bearer" and auth and auth.startswith("Bearer ") and auth[7:] in reg.tokens:
                            return self._send(200, b"{}")
                        return self._send(401, b"{}", self._challenge(""))
                    return self._send(200, b"{}")
                if not path.startswith("/v2/"):
                    return self._send(404)
                rest = path[4:]
                for kind in ("/manifests/", "/blobs/"):
                    if kind in rest:
                        repo, ref = rest.split(kind, 1)
                        break
                else:
                    return self._send(404)
                if not reg._authorized(auth, repo):
                    return self._send(401, b'{"errors":[{"code":"UNAUTHORIZED"}]}', self._challenge(repo))
                if kind == "/manifests/":
                    m = reg.manifests.get((repo, ref))
                    if m is None:
                        return self._send(404, b'{"errors":[{"code":"MANIFEST_UNKNOWN"}]}')
                    mt, body = m
                    return self._send(200, body, {"Content-Type": mt,
                                                  "Docker-Content-Digest": "sha256:" + hashlib.sha256(body).hexdigest()})
                data = reg.blobs.get(ref)
                if data is None:
                    return self._send(404, b'{"errors":[{"code":"BLOB_UNKNOWN"}]}')
                if reg.redirect_blobs:
                    return self._send(307, b"", {"Location": f"http://{reg.host}/blobstore/{ref}"})
                return self._send(200, data, {"Content-Type": "application/octet-stream"})

        return H
