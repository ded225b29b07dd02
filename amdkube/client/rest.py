"""Async REST client (client-go rest + typed clientset equivalent).

Reference: staging/src/k8s.io/client-go/rest (request building, errors → StatusError,
QPS/burst token-bucket throttling), watch decoding (rest/watch + streamwatcher), and the
fork's Binding with extendedResourceBinding (plugin/pkg/scheduler/scheduler.go:483-491).
Fault injection: `chaos` = probability of a simulated "connection reset by peer" before
a request is sent (pkg/client/chaosclient/chaosclient.go:37-110, kubelet --chaos-chance).
"""
from __future__ import annotations

import asyncio
import os
import json
import random
import time
from urllib.parse import quote

import aiohttp

from ..api import meta as m
from ..api.scheme import SCHEME, ResourceInfo


class ChaosError(ConnectionResetError):
    pass


IN_CLUSTER_TOKEN_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class ConfigError(RuntimeError):
    pass


class TokenBucket:
    def __init__(self, qps: float, burst: int):
        self.qps, self.burst = qps, max(1, burst)
        self.tokens = float(self.burst)
        self.t = time.monotonic()

    async def wait(self):
        while True:
            now = time.monotonic()
            self.tokens = min(self.burst, self.tokens + (now - self.t) * self.qps)
            self.t = now
            if self.tokens >= 1:
                self.tokens -= 1
                return
            await asyncio.sleep((1 - self.tokens) / self.qps)


def _ssl_context(ca_file=None, ca_data=None, cert_file=None, key_file=None, insecure=False):
    import ssl
    ctx = ssl.create_default_context(ssl.Purpose.SERVER_AUTH)
    if insecure:
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    elif ca_file or ca_data:
        ctx.load_verify_locations(cafile=ca_file, cadata=ca_data)
        ctx.check_hostname = False   # certificates name the cluster IPs / node names, not always the dial address
    if cert_file:
        ctx.load_cert_chain(cert_file, key_file)
    return ctx


def load_kubeconfig(path: str | None = None, context: str | None = None) -> dict:
    """clientcmd: KUBECONFIG / ~/.kube/config YAML (clusters, users, contexts, current-context) →
    {"server", "token", "ca_data", "cert_file"/"key_file" (data is spilled to a private temp dir)}."""
    import base64
    import tempfile
    import yaml
    path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    ctx_name = context or cfg.get("current-context")
    ctxs = {c["name"]: c.get("context") or {} for c in cfg.get("contexts") or []}
    ctx = ctxs.get(ctx_name) or (next(iter(ctxs.values())) if ctxs else {})
    cluster = next((c.get("cluster") or {} for c in cfg.get("clusters") or [] if c["name"] == ctx.get("cluster")),
                   (cfg.get("clusters") or [{}])[0].get("cluster") or {})
    user = next((u.get("user") or {} for u in cfg.get("users") or [] if u["name"] == ctx.get("user")), {})
    out = {"server": cluster.get("server", "http://127.0.0.1:8080"), "token": user.get("token"),
           "insecure": bool(cluster.get("insecure-skip-tls-verify"))}
    base = os.path.dirname(os.path.abspath(path))
    rel = lambda p: p if os.path.isabs(p) else os.path.join(base, p)  # noqa: E731
    if cluster.get("certificate-authority-data"):
        out["ca_data"] = base64.b64decode(cluster["certificate-authority-data"]).decode()
    elif cluster.get("certificate-authority"):
        out["ca_file"] = rel(cluster["certificate-authority"])
    if user.get("client-certificate-data"):
        d = tempfile.mkdtemp(prefix="amdkube-kc-")
        os.chmod(d, 0o700)
        out["cert_file"], out["key_file"] = os.path.join(d, "c.crt"), os.path.join(d, "c.key")
        open(out["cert_file"], "wb").write(base64.b64decode(user["client-certificate-data"]))
        open(out["key_file"], "wb").write(base64.b64decode(user["client-key-data"]))
    elif user.get("client-certificate"):
        out["cert_file"], out["key_file"] = rel(user["client-certificate"]), rel(user.get("client-key", ""))
    return out


class Client:
    def __init__(self, server: str, token: str | None = None, qps: float = 0, burst: int = 0,
                 chaos: float = 0.0, user_agent: str = "amdkube", timeout: float = 60.0, pool: int = 64,
                 ca_file: str | None = None, ca_data: str | None = None, cert_file: str | None = None,
                 key_file: str | None = None, insecure: bool = False, content_type: str = "application/json"):
        self.server = server.rstrip("/")
        self.ssl = _ssl_context(ca_file, ca_data, cert_file, key_file, insecure) if self.server.startswith("https") else None
        # --kube-api-content-type: application/vnd.kubernetes.protobuf asks for the protobuf
        # encoding (JSON stays acceptable for kinds without a protobuf schema)
        self.proto = content_type == "application/vnd.kubernetes.protobuf"
        accept = "application/vnd.kubernetes.protobuf, application/json" if self.proto else "application/json"
        self.headers = {"User-Agent": user_agent, "Accept": accept}
        if token:
            self.headers["Authorization"] = f"Bearer {token}"
        self.limiter = TokenBucket(qps, burst or int(qps * 2) or 1) if qps else None
        self.chaos = chaos
        self.timeout = timeout
        self.pool = pool
        self._session: aiohttp.ClientSession | None = None
        self._loop = None

    def set_client_cert(self, cert_file: str, key_file: str):
        """Certificate rotation (kubelet/certificate/transport.go): new connections present the
        new client certificate; the pooled ones are closed so none keeps the old identity."""
        if self.ssl is None:
            return
        self.ssl.load_cert_chain(cert_file, key_file)
        sess, self._session = self._session, None
        if sess is not None and not sess.closed:
            import asyncio as _asyncio
            try:
                _asyncio.get_running_loop().create_task(sess.close())
            except RuntimeError:
                pass

    # ---------------------------------------------------------------- session
    @property
    def session(self) -> aiohttp.ClientSession:
        loop = asyncio.get_running_loop()
        if self._session is None or self._session.closed or self._loop is not loop:
            conn = aiohttp.TCPConnector(limit=self.pool, keepalive_timeout=60, ttl_dns_cache=None,
                                        ssl=self.ssl if self.ssl is not None else None)
            self._session = aiohttp.ClientSession(connector=conn, headers=self.headers,
                                                  timeout=aiohttp.ClientTimeout(total=None, sock_connect=10))
            self._loop = loop
        return self._session

    async def close(self):
        if self._session is not None and not self._session.closed:
            await self._session.close()
        self._session = None

    @classmethod
    def from_kubeconfig(cls, path: str | None = None, context: str | None = None, **kw) -> "Client":
        c = load_kubeconfig(path, context)
        return cls(c["server"], token=c.get("token"), ca_file=c.get("ca_file"), ca_data=c.get("ca_data"),
                   cert_file=c.get("cert_file"), key_file=c.get("key_file"), insecure=c.get("insecure", False), **kw)

    @classmethod
    def in_cluster(cls, **kw) -> "Client":
        """rest.InClusterConfig (staging/src/k8s.io/client-go/rest/config.go): the apiserver from
        KUBERNETES_SERVICE_HOST/PORT, the pod's ServiceAccount token and the cluster CA from the
        token volume the ServiceAccount admission plugin mounts. A container without a mount
        namespace finds the volume under $AMDKUBE_ROOTFS. ConfigError when not in a pod."""
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if not host or not port:
            raise ConfigError("unable to load in-cluster configuration, KUBERNETES_SERVICE_HOST and "
                              "KUBERNETES_SERVICE_PORT must be defined")
        base = IN_CLUSTER_TOKEN_DIR
        if not os.path.exists(os.path.join(base, "token")) and os.environ.get("AMDKUBE_ROOTFS"):
            base = os.path.join(os.environ["AMDKUBE_ROOTFS"], base.lstrip("/"))
        try:
            with open(os.path.join(base, "token")) as f:
                token = f.read().strip()
        except OSError as e:
            raise ConfigError(f"no in-cluster ServiceAccount token: {e}") from None
        ca = os.path.join(base, "ca.crt")
        h = f"[{host}]" if ":" in host else host
        return cls(f"https://{h}:{port}", token=token, ca_file=ca if os.path.exists(ca) else None, **kw)

    async def discover(self) -> int:
        """Learn resources the local scheme does not know (custom resources) from the server's
        discovery documents (/apis → /apis/<group>/<version>), as kubectl's discovery client
        does. Returns how many were added."""
        from ..api.scheme import SCHEME, ResourceInfo
        added = 0
        groups = (await self.request("GET", "/apis")).get("groups") or []
        for g in groups:
            for v in g.get("versions") or []:
                gv = v["groupVersion"]
                group, _, version = gv.partition("/")
                try:
                    rl = await self.request("GET", f"/apis/{gv}")
                except m.StatusError:
                    continue
                for r in rl.get("resources") or []:
                    if "/" in r["name"] or SCHEME.for_plural(group, r["name"]) is not None:
                        continue
                    subs = tuple(x["name"].split("/", 1)[1] for x in rl["resources"] if x["name"].startswith(r["name"] + "/"))
                    SCHEME.add(ResourceInfo(group, version, r["kind"], r["name"], bool(r.get("namespaced")),
                                            tuple(r.get("shortNames") or ()), subs))
                    added += 1
        return added

    # ---------------------------------------------------------------- paths
    @staticmethod
    def resource_info(resource: str) -> ResourceInfo:
        ri = SCHEME.resolve(resource)
        if ri is None:
            raise KeyError(f"unknown resource {resource!r}")
        return ri

    def path(self, ri: ResourceInfo, ns: str = "", name: str | None = None, sub: str = "") -> str:
        p = ri.api_prefix()
        if ri.namespaced and ns:
            p += f"/namespaces/{quote(ns)}"
        p += f"/{ri.plural}"
        if name:
            p += f"/{quote(name)}"
        if sub:
            p += f"/{sub}"
        return p

    # -------------------------------------------------------------- request
    async def request(self, method: str, path: str, params=None, body=None, content_type="application/json",
                      raw=False, timeout=None):
        if self.limiter:
            await self.limiter.wait()
        if self.chaos and random.random() < self.chaos:
            raise ChaosError("connection reset by peer (chaos)")
        data = None
        headers = None
        if body is not None:
            data = body if isinstance(body, (bytes, str)) else json.dumps(body, separators=(",", ":"))
            headers = {"Content-Type": content_type}
        to = aiohttp.ClientTimeout(total=timeout or self.timeout)
        async with self.session.request(method, self.server + path, params=params, data=data, headers=headers,
                                        timeout=to) as r:
            payload = await r.read()
            if payload[:4] == b"k8s\x00":
                from ..api import protobuf as pb
                obj = pb.decode(payload)
                if r.status >= 400:
                    raise m.StatusError.from_status(obj)
                return payload if raw else obj
            if r.status >= 400:
                try:
                    st = json.loads(payload)
                    if isinstance(st, dict) and st.get("kind") == "Status":
                        raise m.StatusError.from_status(st)
                except ValueError:
                    pass
                raise m.StatusError(r.status, "Unknown", payload.decode(errors="replace")[:500])
            if raw:
                return payload
            return json.loads(payload) if payload else None

    # ------------------------------------------------------------ typed verbs
    async def get(self, resource: str, name: str, ns: str = "") -> dict:
        ri = self.resource_info(resource)
        return await self.request("GET", self.path(ri, ns, name))

    async def get_or_none(self, resource: str, name: str, ns: str = "") -> dict | None:
        try:
            return await self.get(resource, name, ns)
        except m.StatusError as e:
            if m.is_not_found(e):
                return None
            raise

    async def list(self, resource: str, ns: str = "", label_selector=None, field_selector=None, limit=0):
        """Returns (items, resourceVersion)."""
        ri = self.resource_info(resource)
        params = {}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        items, cont = [], None
        while True:
            if limit:
                params["limit"] = str(limit)
            if cont:
                params["continue"] = cont
            d = await self.request("GET", self.path(ri, ns), params=params)
            items.extend(d.get("items") or [])
            cont = (d.get("metadata") or {}).get("continue")
            if not cont:
                return items, (d.get("metadata") or {}).get("resourceVersion", "")

    async def create(self, obj: dict, ns: str | None = None) -> dict:
        ri = SCHEME.for_object(obj)
        if ri is None:
            raise KeyError(f"unknown kind {obj.get('apiVersion')}/{obj.get('kind')}")
        ns = ns if ns is not None else (m.namespace_of(obj) or ("default" if ri.namespaced else ""))
        return await self.request("POST", self.path(ri, ns), body=obj)

    async def update(self, obj: dict, sub: str = "") -> dict:
        ri = SCHEME.for_object(obj)
        return await self.request("PUT", self.path(ri, m.namespace_of(obj), m.name_of(obj), sub), body=obj)

    async def update_status(self, obj: dict) -> dict:
        return await self.update(obj, "status")

    async def patch(self, resource: str, name: str, patch, ns: str = "", sub: str = "",
                    patch_type: str = "application/merge-patch+json") -> dict:
        ri = self.resource_info(resource)
        return await self.request("PATCH", self.path(ri, ns, name, sub), body=patch, content_type=patch_type)

    async def delete(self, resource: str, name: str, ns: str = "", grace: int | None = None,
                     uid: str | None = None, propagation: str | None = None):
        ri = self.resource_info(resource)
        opts = {"kind": "DeleteOptions", "apiVersion": "v1"}
        if grace is not None:
            opts["gracePeriodSeconds"] = grace
        if uid:
            opts["preconditions"] = {"uid": uid}
        if propagation:
            opts["propagationPolicy"] = propagation
        return await self.request("DELETE", self.path(ri, ns, name), body=opts)

    async def delete_collection(self, resource: str, ns: str = "", label_selector=None, grace=None):
        ri = self.resource_info(resource)
        params = {"labelSelector": label_selector} if label_selector else None
        body = {"gracePeriodSeconds": grace} if grace is not None else None
        return await self.request("DELETE", self.path(ri, ns), params=params, body=body)

    async def bind(self, ns: str, name: str, node: str, ext_binding: dict | None = None, uid: str | None = None):
        b = {"apiVersion": "v1", "kind": "Binding", "metadata": {"name": name, "namespace": ns},
             "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        if uid:
            b["metadata"]["uid"] = uid
        if ext_binding:
            b["target"]["extendedResourceBinding"] = ext_binding
        ri = self.resource_info("pods")
        return await self.request("POST", self.path(ri, ns, name, "binding"), body=b)

    async def evict(self, ns: str, name: str):
        ri = self.resource_info("pods")
        body = {"apiVersion": "policy/v1beta1", "kind": "Eviction", "metadata": {"name": name, "namespace": ns}}
        return await self.request("POST", self.path(ri, ns, name, "eviction"), body=body)

    @staticmethod
    def _log_params(container=None, tail=None, previous=False, since_seconds=None, since_time=None, timestamps=False,
                    limit_bytes=None, follow=False) -> dict:
        """PodLogOptions as query parameters."""
        params = {}
        if container:
            params["container"] = container
        if tail is not None:
            params["tailLines"] = str(tail)
        if previous:
            params["previous"] = "true"
        if since_seconds is not None:
            params["sinceSeconds"] = str(since_seconds)
        if since_time:
            params["sinceTime"] = since_time
        if timestamps:
            params["timestamps"] = "true"
        if limit_bytes is not None:
            params["limitBytes"] = str(limit_bytes)
        if follow:
            params["follow"] = "true"
        return params

    async def logs(self, ns: str, name: str, container: str | None = None, tail: int | None = None, **opts) -> str:
        """GET pods/{name}/log; `opts`: previous, since_seconds, since_time, timestamps, limit_bytes."""
        ri = self.resource_info("pods")
        params = self._log_params(container, tail, **opts)
        return (await self.request("GET", self.path(ri, ns, name, "log"), params=params, raw=True)).decode(errors="replace")

    async def stream_logs(self, ns: str, name: str, container: str | None = None, tail: int | None = None, **opts):
        """Async iterator over the chunks of a (followed) pod log."""
        ri = self.resource_info("pods")
        params = self._log_params(container, tail, follow=opts.pop("follow", True), **opts)
        async with self.session.get(self.server + self.path(ri, ns, name, "log"), params=params,
                                    timeout=aiohttp.ClientTimeout(total=None, sock_read=None)) as r:
            if r.status >= 400:
                payload = await r.read()
                try:
                    st = json.loads(payload)
                except ValueError:
                    st = None
                if isinstance(st, dict) and st.get("kind") == "Status":
                    raise m.StatusError.from_status(st)
                raise m.StatusError(r.status, "Unknown", payload.decode(errors="replace")[:500])
            async for chunk in r.content.iter_any():
                yield chunk

    async def watch(self, resource: str, ns: str = "", resource_version: str = "", label_selector=None,
                    field_selector=None, timeout_seconds: int | None = None):
        """Async generator of (type, obj). Raises StatusError(410) on ERROR/Expired frames."""
        ri = self.resource_info(resource)
        params = {"watch": "true", "resourceVersion": resource_version or ""}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        if timeout_seconds:
            params["timeoutSeconds"] = str(timeout_seconds)
        if self.limiter:
            await self.limiter.wait()
        if self.chaos and random.random() < self.chaos:
            raise ChaosError("connection reset by peer (chaos)")
        async with self.session.get(self.server + self.path(ri, ns), params=params,
                                    timeout=aiohttp.ClientTimeout(total=None, sock_read=None)) as r:
            if r.status >= 400:
                payload = await r.read()
                try:
                    raise m.StatusError.from_status(json.loads(payload))
                except ValueError:
                    raise m.StatusError(r.status, "Unknown", payload.decode(errors="replace"))
            buf = b""
            if "protobuf" in r.headers.get("Content-Type", ""):
                from ..api import protobuf as pb
                async for chunk in r.content.iter_any():
                    buf += chunk
                    events, buf = pb.decode_watch_frames(buf)
                    for typ, obj in events:
                        if typ == "ERROR":
                            raise m.StatusError.from_status(obj)
                        yield typ, obj
                return
            async for chunk in r.content.iter_any():
                buf += chunk
                while True:
                    i = buf.find(b"\n")
                    if i < 0:
                        break
                    line, buf = buf[:i], buf[i + 1:]
                    if not line.strip():
                        continue
                    ev = json.loads(line)
                    if ev.get("type") == "ERROR":
                        raise m.StatusError.from_status(ev.get("object") or {})
                    yield ev["type"], ev["object"]
