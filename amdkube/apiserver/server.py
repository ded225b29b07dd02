"""kube-apiserver equivalent: REST + chunked watch over aiohttp on the embedded MVCC store.

Reference: handler chain and verbs — staging/src/k8s.io/apiserver/pkg/endpoints/handlers/
{create.go:37-170, get.go, update.go, patch.go, delete.go, watch.go}; filters
(authn/authz/max-in-flight) staging/.../server/filters; discovery /api, /apis; request
metrics staging/.../endpoints/metrics/metrics.go:41-93; profiling routes/profiling.go.

Fast paths (all single-threaded on the event loop, no locks):
  * GET/LIST stream stored JSON bytes straight from the store (resourceVersion was
    embedded at commit) — no decode/encode unless a selector must be evaluated;
  * watch frames are `{"type":T,"object":<stored bytes>}` lines, one decode per event
    shared by every filtered watcher (storage.event_object cache).
"""
from __future__ import annotations

import asyncio
import collections
import json
import logging
import random
import time

from aiohttp import ClientSession, ClientTimeout, web

from .. import GIT_VERSION
from ..api import meta as m
from ..api.scheme import SCHEME
from ..store import MVCCStore, PUT
from ..utils import greenbridge, profiling
from ..utils.metrics import CONTENT_TYPE, Counter, Histogram, new_registry, render
from ..utils.quantiles import QuantileSummary
from ..store.storage import kv_json, kv_proto
from . import admission as adm
from .registry import Registry
from .service import ServiceAllocator, parse_port_range
from .auth import Attributes, Authenticator, UnionAuthorizer, ensure_bootstrap_policy

log = logging.getLogger("amdkube.apiserver")

_JSON = "application/json"


_STREAMING_SUBS = {"exec", "attach", "portforward", "proxy"}


def _to_scale(obj: dict) -> dict:
    """autoscaling/v1 Scale view of a scalable object (registry/*/storage ScaleREST)."""
    from ..api.labels import selector_from_label_selector, selector_from_set
    md, spec = obj.get("metadata") or {}, obj.get("spec") or {}
    sel = spec.get("selector") or {}
    sel_str = str(selector_from_label_selector(sel) if "matchLabels" in sel or "matchExpressions" in sel
                  else selector_from_set(sel))
    return {"kind": "Scale", "apiVersion": "autoscaling/v1",
            "metadata": {k: md[k] for k in ("name", "namespace", "uid", "resourceVersion", "creationTimestamp") if k in md},
            "spec": {"replicas": int(spec.get("replicas", 1))},
            "status": {"replicas": int((obj.get("status") or {}).get("replicas", 0)), "selector": sel_str}}


_USER_KEY = web.RequestKey("amdkube_user", dict) if hasattr(web, "RequestKey") else "amdkube_user"


def _uninitialized(obj) -> bool:
    ini = ((obj or {}).get("metadata") or {}).get("initializers")
    return bool(ini) and bool(ini.get("pending"))


def _convert_out(obj, storage_ri, served):
    """Storage-version object (or list) → the served version the client asked for."""
    if isinstance(obj, dict):
        if obj.get("apiVersion") == storage_ri.api_version and obj.get("kind") == storage_ri.kind:
            obj["apiVersion"], obj["kind"] = served.api_version, served.kind
            if served.from_storage is not None:
                served.from_storage(obj)
        elif obj.get("kind") == storage_ri.list_kind:
            obj["apiVersion"], obj["kind"] = served.api_version, served.list_kind
            for it in obj.get("items") or []:
                _convert_out(it, storage_ri, served)
    return obj


def _convert_frame(data: bytes, storage_ri, served) -> bytes:
    ev = json.loads(data)
    _convert_out(ev.get("object"), storage_ri, served)
    return json.dumps(ev, separators=(",", ":")).encode() + b"\n"


def _wants_protobuf(request) -> bool:
    """Accept lists application/vnd.kubernetes.protobuf before any JSON type (or without one)."""
    acc = request.headers.get("Accept", "")
    if "protobuf" not in acc:
        return False
    for part in acc.split(","):
        mt = part.split(";", 1)[0].strip().lower()
        if mt.startswith("application/vnd.kubernetes.protobuf"):
            return True
        if mt in ("application/json", "*/*", "application/*"):
            return False
    return False


def _resp(obj, status=200) -> web.Response:
    body = obj if isinstance(obj, (bytes, bytearray)) else json.dumps(obj, separators=(",", ":")).encode()
    return web.Response(body=body, status=status, content_type=_JSON)


def _err(e: m.StatusError) -> web.Response:
    return _resp(e.status(), e.code)


_METRIC_VERBS = {"create": "POST", "update": "PUT", "patch": "PATCH", "delete": "DELETE",
                 "deletecollection": "DELETECOLLECTION", "get": "GET", "list": "LIST", "watch": "WATCH"}



def _subresource_doc(ri, sub: str) -> dict:
    """A subresource's APIResource entry as the reference's discovery serves it: its own kind
    (Binding, Eviction in policy/v1beta1, Scale) and the verbs it accepts."""
    doc = {"name": f"{ri.plural}/{sub}", "singularName": "", "namespaced": ri.namespaced, "kind": ri.kind,
           "verbs": ["get", "patch", "update"]}
    if sub == "binding":
        doc.update(kind="Binding", verbs=["create"])
    elif sub == "eviction":
        doc.update(group="policy", version="v1beta1", kind="Eviction", verbs=["create"])
    elif sub == "scale":
        doc["kind"] = "Scale"
        if not ri.group:
            doc.update(group="autoscaling", version="v1")
    elif sub == "log":
        doc["verbs"] = ["get"]
    elif sub in ("exec", "attach", "portforward"):
        doc["verbs"] = ["create", "get"]
    elif sub == "proxy":
        doc["verbs"] = ["create", "delete", "get", "patch", "update"]
    return doc

class APIServer:
    def __init__(self, store: MVCCStore | None = None, admission_plugins=adm.DEFAULT_CHAIN, admission_config=None,
                 token_auth: dict | None = None, authorization_mode: str = "AlwaysAllow",
                 max_in_flight: int = 400, max_mutating_in_flight: int = 200, event_ttl: float = 3600.0,
                 anonymous_auth: bool = True, service_cidr: str = "10.0.0.0/24", node_port_range: str = "30000-32767",
                 service_account_key: bytes | None = None, tls_cert_file: str | None = None, tls_key_file: str | None = None,
                 client_ca_file: str | None = None, audit_log_path: str | None = None, audit_policy_file: str | None = None,
                 audit_log_maxsize: int = 0, audit_log_maxbackup: int = 0, kubelet_https: bool = False,
                 kubelet_client_certificate: str | None = None, kubelet_client_key: str | None = None,
                 kubelet_certificate_authority: str | None = None, requestheader_client_ca_file: str | None = None,
                 requestheader_allowed_names=(), proxy_client_cert_file: str | None = None,
                 proxy_client_key_file: str | None = None, options: dict | None = None):
        """`options`: the rest of kube-apiserver's flags (see _apply_options)."""
        self.store = store or MVCCStore()
        self._bridged = bool(getattr(self.store, "async_writes", False))
        self.opts = dict(options or {})
        # --kubelet-https / --kubelet-client-certificate / --kubelet-client-key /
        # --kubelet-certificate-authority: how the apiserver reaches kubelets (logs, exec, proxy)
        self.kubelet_scheme = "https" if kubelet_https else "http"
        self.kubelet_ssl = None
        if kubelet_https:
            import ssl
            ctx = ssl.create_default_context(ssl.Purpose.SERVER_AUTH, cafile=kubelet_certificate_authority)
            ctx.check_hostname = False
            if not kubelet_certificate_authority:
                ctx.verify_mode = ssl.CERT_NONE
            if kubelet_client_certificate:
                ctx.load_cert_chain(kubelet_client_certificate, kubelet_client_key)
            self.kubelet_ssl = ctx
        self.admission = adm.Chain(admission_plugins, admission_config)
        smt = self.opts.get("storage_media_type") or "application/json"
        if smt not in ("application/json", "application/vnd.kubernetes.protobuf"):
            raise ValueError(f"--storage-media-type {smt!r}: application/json or application/vnd.kubernetes.protobuf")
        self.registry = Registry(self.store, self.admission, ServiceAllocator(service_cidr, parse_port_range(node_port_range)),
                                 media_type=smt)
        from .crd import CRDManager
        from .webhook import WebhookDispatcher
        self.crds = CRDManager(self.registry)
        self.webhooks = WebhookDispatcher(self.registry)
        self.auditor = None
        o = self.opts
        if audit_log_path or o.get("audit_webhook_config_file"):
            from .audit import Auditor, LogBackend, MultiBackend, WebhookBackend, load_policy
            backends = []
            if audit_log_path:
                backends.append(LogBackend(audit_log_path, audit_log_maxsize, audit_log_maxbackup,
                                           o.get("audit_log_format") or "json", int(o.get("audit_log_maxage") or 0)))
            if o.get("audit_webhook_config_file"):
                backends.append(WebhookBackend(o["audit_webhook_config_file"], o.get("audit_webhook_mode") or "batch",
                                               int(o.get("audit_webhook_batch_buffer_size") or 10000),
                                               int(o.get("audit_webhook_batch_max_size") or 400),
                                               float(o.get("audit_webhook_batch_max_wait") or 30.0),
                                               float(o.get("audit_webhook_batch_throttle_qps") or 10.0),
                                               int(o.get("audit_webhook_batch_throttle_burst") or 15)))
            self.auditor = Auditor(load_policy(audit_policy_file), backends[0] if len(backends) == 1 else MultiBackend(backends))
        self.tokens = dict(token_auth or {})
        # genericapiserver loopback client: the apiserver's own (and in-process components')
        # credential, a random bearer token for system:apiserver in system:masters
        self.loopback_token = m.new_uid()
        self.tokens[self.loopback_token] = {"name": "system:apiserver", "uid": "", "groups": ["system:masters"]}
        self.anonymous = anonymous_auth
        self.authz_mode = authorization_mode
        self.sa_key = service_account_key
        self.tls = (tls_cert_file, tls_key_file, client_ca_file) if tls_cert_file else None
        self.authn = Authenticator(self.registry, self.tokens, service_account_key, anonymous_auth)
        self.authn.user_tokens = len(token_auth or {})
        self.requestheader_ca = requestheader_client_ca_file
        if requestheader_client_ca_file:
            o = self.opts
            self.authn.configure_requestheader(
                requestheader_client_ca_file, requestheader_allowed_names,
                tuple(o.get("requestheader_username_headers") or ("X-Remote-User",)),
                tuple(o.get("requestheader_group_headers") or ("X-Remote-Group",)),
                tuple(o.get("requestheader_extra_headers_prefix") or ("X-Remote-Extra-",)))
            if client_ca_file:
                import ssl
                self.authn.requestheader["client_ca_same"] = \
                    ssl._ssl._test_decode_cert(client_ca_file).get("subject") == self.authn.requestheader["issuer"]
        # the aggregator's identity towards extension API servers (--proxy-client-cert-file)
        self.proxy_client_cert = (proxy_client_cert_file, proxy_client_key_file) if proxy_client_cert_file else None
        self.authz = UnionAuthorizer(authorization_mode, self.registry, self.opts.get("authorization_policy_file"),
                                     self.opts.get("authorization_webhook_config_file"),
                                     self.opts.get("authorization_webhook_cache_authorized_ttl", 300.0),
                                     self.opts.get("authorization_webhook_cache_unauthorized_ttl", 30.0))
        self.registry.authorizer = self.authz
        self._apply_options()
        from .aggregator import Aggregator
        self.aggregator = Aggregator(self)
        self._ro = asyncio.Semaphore(max_in_flight) if max_in_flight else None
        self._rw = asyncio.Semaphore(max_mutating_in_flight) if max_mutating_in_flight else None
        self.event_ttl = event_ttl
        self.metrics = new_registry()
        # endpoints/metrics/metrics.go:37-70: the request counter, the latency histogram
        # (ExponentialBuckets(125000, 2, 7)) and the latency Summary (quantiles 0.5/0.9/0.99 over
        # 5 h) that the e2e API-responsiveness check reads (metrics_util.go:264-350)
        self.m_count = Counter("apiserver_request_count", "Counter of apiserver requests broken out for each verb, API resource, client, and HTTP response contentType and code.",
                               ["verb", "resource", "subresource", "scope", "client", "contentType", "code"], registry=self.metrics)
        self.m_lat = Histogram("apiserver_request_latencies", "Response latency distribution in microseconds for each verb, resource and subresource.",
                               ["verb", "resource", "subresource", "scope"], buckets=tuple(125000 * 2 ** i for i in range(7)),
                               registry=self.metrics)
        self.m_lat_summary = QuantileSummary("apiserver_request_latencies_summary", "Response latency summary in microseconds for each verb, resource and subresource.",
                                             ["verb", "resource", "subresource", "scope"], registry=self.metrics, max_age=5 * 3600.0)
        # exact per-request latencies for the SLO report (metrics_util.go HighLatencyRequests
        # reads the apiserver's latency summary quantiles; this keeps the raw samples instead)
        self.lat_samples: collections.deque = collections.deque(maxlen=200_000)
        self.watch_count = 0
        self.app = web.Application(client_max_size=64 * 1024 * 1024,
                                   middlewares=([self._cors_middleware] if self.opts.get("cors_allowed_origins") else []) +
                                   [self._protobuf_middleware])
        self.app.router.add_get("/healthz", self.healthz)
        self.app.router.add_get("/healthz/{check}", self.healthz)
        self.app.router.add_get("/version", self.version)
        self.app.router.add_get("/metrics", self.metrics_handler)
        self.app.router.add_delete("/metrics", self.metrics_reset)
        self.app.router.add_get("/openapi/v2", self.openapi)
        self.app.router.add_get("/swagger.json", self.openapi)
        self.app.router.add_get("/api", self.api_versions)
        self.app.router.add_get("/apis", self.api_groups)
        if self.opts.get("profiling", True):
            profiling.add_routes(self.app)
        if self.opts.get("enable_logs_handler", True):
            self.app.router.add_get("/logs", self.logs_handler)
            self.app.router.add_get("/logs/{path:.*}", self.logs_handler)
        self.app.router.add_route("*", "/api/{tail:.*}", self.dispatch)
        self.app.router.add_route("*", "/apis/{tail:.*}", self.dispatch)
        self._runner = None
        self._site = None
        self._bg: list[asyncio.Task] = []
        self.port = None
        self._http: ClientSession | None = None
        self._bootstrap()

    def _bootstrap(self):
        for ns in ("default", "kube-system", "kube-public"):
            if self.registry.get_namespace(ns) is None:
                self.registry.create_namespace(ns)
        if "RBAC" in self.authz.modes:
            ensure_bootstrap_policy(self.registry)
        self.aggregator.autoregister()

    def _apply_options(self):
        """Authenticators and policies from the remaining flags: --basic-auth-file, --oidc-*,
        --authentication-token-webhook-config-file, --allow-privileged, --runtime-config,
        --cors-allowed-origins, --min-request-timeout, --advertise-address,
        --kubernetes-service-node-port, --insecure-port/--insecure-bind-address, --tls-sni-cert-key."""
        import re as _re
        o = self.opts
        if o.get("basic_auth_file"):
            from .authx import BasicAuthenticator
            self.authn.basic = BasicAuthenticator(o["basic_auth_file"])
        if o.get("oidc_issuer_url"):
            from .authx import OIDCAuthenticator
            if not o.get("oidc_client_id"):
                raise ValueError("--oidc-issuer-url needs --oidc-client-id")
            self.authn.oidc = OIDCAuthenticator(o["oidc_issuer_url"], o["oidc_client_id"], o.get("oidc_ca_file"),
                                                o.get("oidc_username_claim") or "sub", o.get("oidc_username_prefix"),
                                                o.get("oidc_groups_claim"), o.get("oidc_groups_prefix") or "")
        if o.get("authentication_token_webhook_config_file"):
            from .authx import WebhookTokenAuthenticator
            self.authn.webhook = WebhookTokenAuthenticator(o["authentication_token_webhook_config_file"],
                                                           o.get("authentication_token_webhook_cache_ttl", 120.0))
        from ..api import validation as _val
        _val.CAPABILITIES["allow_privileged"] = bool(o.get("allow_privileged", True))
        # --runtime-config: group/version=true|false, api/all, api/legacy
        self.disabled_gv: set[tuple[str, str]] = set()
        gvs = {(ri.group, ri.version) for ri in SCHEME.by_kind.values()}
        for item in [x.strip() for x in (o.get("runtime_config") or "").split(",") if x.strip()]:
            key, _, val = item.partition("=")
            on = val.lower() != "false"
            if key == "api/all":
                self.disabled_gv = set() if on else set(gvs)
                continue
            if key in ("api/legacy", "api/v1", "v1"):
                target = {("", "v1")}
            else:
                g, _, v = key.partition("/")
                target = {(g, v)} if v else {x for x in gvs if x[0] == g}
            self.disabled_gv = (self.disabled_gv - target) if on else (self.disabled_gv | target)
        self._cors = [_re.compile(x) for x in o.get("cors_allowed_origins") or []]
        self.min_request_timeout = float(o.get("min_request_timeout", 1800))

    @web.middleware
    async def _cors_middleware(self, request, handler):
        """--cors-allowed-origins (filters/cors.go): origins matching one of the regexps."""
        origin = request.headers.get("Origin")
        allowed = origin and any(r.search(origin) for r in self._cors)
        if request.method == "OPTIONS" and allowed:
            resp = web.Response(status=204)
        else:
            resp = await handler(request)
        if allowed:
            resp.headers.update({"Access-Control-Allow-Origin": origin, "Access-Control-Allow-Credentials": "true",
                                 "Access-Control-Allow-Methods": "POST, GET, OPTIONS, PUT, DELETE, PATCH",
                                 "Access-Control-Allow-Headers": "Content-Type, Content-Length, Accept-Encoding, "
                                                                 "X-CSRF-Token, Authorization, X-Requested-With, If-Modified-Since",
                                 "Access-Control-Expose-Headers": "Date"})
        return resp

    async def logs_handler(self, request):
        """/logs/ (routes/logs.go): the node's /var/log for cluster admins (--enable-logs-handler)."""
        import os as _os
        user = await self._authenticate_async(request)
        ok, _ = await self.authz.authorize_async(Attributes(user, "get", path=request.path, resource_request=False))
        if not ok:
            return _err(m.forbidden(f'User "{user.get("name")}" cannot get path "{request.path}"'))
        root = _os.path.realpath(self.opts.get("logs_dir") or "/var/log")
        rel = request.match_info.get("path", "")
        target = _os.path.realpath(_os.path.join(root, rel))
        if target != root and not target.startswith(root + _os.sep):
            return web.Response(status=404)
        if _os.path.isdir(target):
            names = sorted(_os.listdir(target))
            return web.Response(text="".join(f'<a href="{n}">{n}</a>\n' for n in names), content_type="text/html")
        if not _os.path.isfile(target):
            return web.Response(status=404)
        return web.FileResponse(target)

    def _sni_context(self, base_ctx):
        """--tls-sni-cert-key cert,key[:name1,name2]: a serving certificate per requested server name."""
        import ssl
        entries = self.opts.get("tls_sni_cert_key") or []
        if not entries:
            return
        by_name = {}
        for cert, key, names in entries:
            ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
            ctx.load_cert_chain(cert, key)
            if not names:
                info = ssl._ssl._test_decode_cert(cert)
                names = [v for t, v in info.get("subjectAltName", ()) if t == "DNS"]
            for n in names:
                by_name[n.lower()] = ctx

        def pick(sock, server_name, _ctx):
            if server_name:
                name = server_name.lower()
                ctx = by_name.get(name) or by_name.get("*." + name.split(".", 1)[-1])
                if ctx is not None:
                    sock.context = ctx
        base_ctx.sni_callback = pick

    # ---------------------------------------------------------------- lifecycle
    async def start(self, host="127.0.0.1", port=0):
        self._runner = web.AppRunner(self.app, access_log=None, handler_cancellation=True)
        await self._runner.setup()
        ctx = None
        if self.tls:
            import ssl
            cert, key, ca = self.tls
            ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
            ctx.load_cert_chain(cert, key)
            if ca:   # --client-ca-file: request (not require) client certificates
                ctx.load_verify_locations(ca)
                ctx.verify_mode = ssl.CERT_OPTIONAL
            if self.requestheader_ca:   # front-proxy certificates are checked against their own CA
                ctx.load_verify_locations(self.requestheader_ca)
                ctx.verify_mode = ssl.CERT_OPTIONAL
        if ctx is not None:
            self._sni_context(ctx)
        self._site = web.TCPSite(self._runner, host, port, backlog=1024, reuse_address=True, ssl_context=ctx)
        await self._site.start()
        self.port = self._site._server.sockets[0].getsockname()[1]
        self.host = host
        # --insecure-port next to the secure one: no authentication, no authorization (the
        # reference's localhost port), for local tooling only
        self.insecure_port = None
        if ctx is not None and self.opts.get("insecure_port"):
            ins = web.TCPSite(self._runner, self.opts.get("insecure_bind_address") or "127.0.0.1", self.opts["insecure_port"],
                              reuse_address=True)
            await ins.start()
            self.insecure_port = ins._server.sockets[0].getsockname()[1]
        if hasattr(self.store, "start"):           # an etcd-backed replica applies its watch on this loop
            self.store.start(asyncio.get_running_loop())
        self._bg.append(asyncio.create_task(self._event_gc()))
        self._bg.append(asyncio.create_task(self.aggregator.run_availability(), name="apiservice-availability"))
        self.crds.start()
        self._bg.append(self.crds._task)
        self._reconcile_master_service()
        if self.opts.get("endpoint_reconciler_type") == "lease":
            self._bg.append(asyncio.create_task(self._lease_endpoints_loop(), name="master-leases"))
        log.info("apiserver serving on http://%s:%d", host, self.port)
        return self

    # pkg/master/reconcilers/lease.go: every apiserver keeps a lease on its address under
    # /masterleases/ (TTL 15 s, renewed every 10 s: EndpointInterval, MasterEndpointReconcileTTL);
    # the kubernetes endpoints list exactly the addresses with a live lease
    LEASE_PREFIX = "/registry/masterleases/"
    LEASE_TTL, LEASE_INTERVAL = 15.0, 10.0

    def _advertise_ip(self) -> str:
        return self.opts.get("advertise_address") or (self.host if self.host not in ("0.0.0.0", "", "::") else "127.0.0.1")

    async def _lease_endpoints_loop(self):
        while True:
            try:
                await self._w(self.reconcile_lease_endpoints)
            except Exception as e:       # noqa: BLE001 — retried next interval
                log.warning("master lease reconcile failed: %r", e)
            await asyncio.sleep(self.LEASE_INTERVAL)

    def reconcile_lease_endpoints(self, now: float | None = None, remove: bool = False):
        """Renew (or, on shutdown, drop) this apiserver's lease, expire stale ones, and set the
        kubernetes endpoints to every address that still holds one (lease.go ReconcileEndpoints)."""
        now = time.time() if now is None else now
        ip = self._advertise_ip()
        key = self.LEASE_PREFIX + ip
        if remove:
            try:
                self.store.delete(key)
            except Exception:       # noqa: BLE001 — already gone
                pass
        else:
            self.store.put(key, json.dumps({"ip": ip, "port": self.port, "expires": now + self.LEASE_TTL}).encode())
        kvs, _, _ = self.store.range(self.LEASE_PREFIX)
        live = []
        for kv in kvs:
            try:
                d = json.loads(kv.value)
            except ValueError:
                continue
            if float(d.get("expires", 0)) > now:
                live.append(d["ip"])
            else:
                try:
                    self.store.delete(kv.key, expect_mod_rev=kv.mod_rev)
                except Exception:   # noqa: BLE001 — renewed or removed meanwhile
                    pass
        subsets = [{"addresses": [{"ip": a} for a in sorted(set(live))],
                    "ports": [{"name": "https", "port": self.port, "protocol": "TCP"}]}] if live else []
        ers = self.registry.rs("endpoints")

        def upd(cur):      # read-modify-CAS: another apiserver may have written it meanwhile
            if (cur.get("subsets") or []) == subsets:
                return None
            new = m.deepcopy(cur)
            new["subsets"] = subsets
            return new
        try:
            ers.storage.guaranteed_update(ers.key("default", "kubernetes"), upd)
        except m.StatusError as e:
            if e.code != 404:
                raise
            ers.create("default", {"apiVersion": "v1", "kind": "Endpoints",
                                   "metadata": {"name": "kubernetes", "namespace": "default"}, "subsets": subsets})
        return sorted(set(live))

    def _reconcile_master_service(self):
        """pkg/master/controller.go: the `kubernetes` service (first IP of the service range, port
        443 "https") and its endpoints pointing at this apiserver."""
        alloc = self.registry.services
        first = str(next(alloc.net.hosts())) if alloc.net.num_addresses > 2 else str(alloc.net.network_address)
        svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "kubernetes", "namespace": "default",
                                                                    "labels": {"component": "apiserver", "provider": "kubernetes"}},
               "spec": {"clusterIP": first, "ports": [{"name": "https", "port": 443, "protocol": "TCP", "targetPort": self.port}],
                        "sessionAffinity": "ClientIP"}}
        if self.opts.get("kubernetes_service_node_port"):    # --kubernetes-service-node-port
            svc["spec"]["type"] = "NodePort"
            svc["spec"]["ports"][0]["nodePort"] = int(self.opts["kubernetes_service_node_port"])
        rs = self.registry.rs("services")
        try:
            if rs.storage.get(rs.key("default", "kubernetes"), ignore_not_found=True) is None:
                rs.create("default", svc)
        except m.StatusError as e:
            log.warning("cannot create the kubernetes service: %s", e)
        mode = self.opts.get("endpoint_reconciler_type") or "master-count"
        if mode == "none":
            return
        if mode == "lease":
            self.reconcile_lease_endpoints()
            return
        ip = self._advertise_ip()
        ep = {"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "kubernetes", "namespace": "default"},
              "subsets": [{"addresses": [{"ip": ip}], "ports": [{"name": "https", "port": self.port, "protocol": "TCP"}]}]}
        ers = self.registry.rs("endpoints")
        cur = ers.storage.get(ers.key("default", "kubernetes"), ignore_not_found=True)
        if cur is not None and int(self.opts.get("apiserver_count") or 1) > 1:
            # --apiserver-count > 1 (the master-count reconciler): keep the other apiservers' addresses
            mine = ep["subsets"][0]
            merged = [s for s in cur.get("subsets") or [] if s != mine]
            ep["subsets"] = sorted(merged + [mine], key=lambda s: json.dumps(s, sort_keys=True))
        if cur is None:
            try:
                ers.create("default", ep)
            except m.StatusError as e:          # another apiserver created it first
                if e.code != 409:
                    raise
        elif cur.get("subsets") != ep["subsets"]:
            ep["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            ers.update("default", "kubernetes", ep)

    @property
    def url(self):
        return f"{'https' if self.tls else 'http'}://{self.host}:{self.port}"

    async def stop(self):
        from ..utils import cancel_and_wait
        await cancel_and_wait(self._bg)
        if self.opts.get("endpoint_reconciler_type") == "lease":
            try:        # hand the address back at once instead of waiting out the TTL
                await self._w(self.reconcile_lease_endpoints, remove=True)
            except Exception as e:      # noqa: BLE001
                log.debug("dropping the master lease failed: %r", e)
        await self.aggregator.close()
        await self.crds.stop()
        await self.webhooks.close()
        for w in self.store.all_watchers():
            w.close()
        if self._http:
            await self._http.close()
        if self._runner:
            await self._runner.cleanup()

    async def _event_gc(self):
        rs = self.registry.rs("events")
        while True:
            await asyncio.sleep(min(60.0, self.event_ttl / 2))
            cutoff = time.time() - self.event_ttl
            for ev in rs.list()[0]:
                ts = m.parse_time(ev.get("lastTimestamp") or (ev.get("metadata") or {}).get("creationTimestamp"))
                if ts is not None and ts < cutoff:
                    try:
                        rs.storage.delete(rs.key(m.namespace_of(ev), m.name_of(ev)))
                    except m.StatusError:
                        pass

    # ----------------------------------------------------------- misc handlers
    async def healthz(self, request):
        return web.Response(text="ok")

    async def version(self, request):
        return _resp({"major": "1", "minor": "9", "gitVersion": GIT_VERSION, "platform": "linux/amd64",
                      "compiler": "cpython", "goVersion": "n/a"})

    async def openapi(self, request):
        """/openapi/v2 and /swagger.json (routes/openapi.go): the Swagger 2.0 document, ETag-cached."""
        import hashlib
        from ..api.openapi import document_bytes
        body = await asyncio.to_thread(document_bytes, GIT_VERSION)
        etag = '"' + hashlib.sha1(body).hexdigest() + '"'
        if request.headers.get("If-None-Match") == etag:
            return web.Response(status=304, headers={"ETag": etag})
        return web.Response(body=body, headers={"Content-Type": "application/json", "ETag": etag})

    async def metrics_handler(self, request):
        return web.Response(body=render(self.metrics), headers={"Content-Type": CONTENT_TYPE})

    async def metrics_reset(self, request):
        """DELETE /metrics (routes/metrics.go MetricsWithReset → metrics.Reset): the e2e framework
        resets the request metrics before a measured phase (metrics_util.go ResetMetrics)."""
        try:
            user = await self._authenticate_async(request)
            await self._authorize_nonresource(user, "delete", "/metrics")
        except m.StatusError as e:
            return _err(e)
        for metric in (self.m_count, self.m_lat, self.m_lat_summary):
            metric.clear()
        return web.Response(text="metrics reset\n")

    async def api_versions(self, request):
        return _resp({"kind": "APIVersions", "versions": ["v1"],
                      "serverAddressByClientCIDRs": [{"clientCIDR": "0.0.0.0/0", "serverAddress": request.host}]})

    @staticmethod
    def _group_doc(g: str, disabled=()) -> dict:
        from ..api.scheme import _version_sort
        vs = _version_sort(ri.version for ri in SCHEME.by_kind.values() if ri.group == g and (g, ri.version) not in disabled)
        pv = SCHEME.preferred_version(g)
        if vs and pv not in vs:
            pv = vs[0]
        return {"name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v} for v in vs],
                "preferredVersion": {"groupVersion": f"{g}/{pv}", "version": pv}}

    async def api_groups(self, request):
        groups = sorted({ri.group for ri in SCHEME.by_kind.values() if ri.group})
        docs = [d for d in (self._group_doc(g, self.disabled_gv) for g in groups) if d["versions"]] + \
            self.aggregator.group_docs(set(groups))
        return _resp({"kind": "APIGroupList", "apiVersion": "v1", "groups": docs})

    def _resource_list(self, group, version):  # noqa: C901
        res = []
        for ri in SCHEME.by_kind.values():
            if ri.group == group and ri.version == version:
                res.append({"name": ri.plural, "singularName": ri.kind.lower(), "namespaced": ri.namespaced,
                            "kind": ri.kind, "verbs": list(ri.verbs), "shortNames": list(ri.short_names)})
                for sub in ri.subresources:
                    res.append(_subresource_doc(ri, sub))
        return {"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": f"{group}/{version}" if group else version,
                "resources": res}

    # ------------------------------------------------------------------ auth
    @staticmethod
    def _peer_der(tr) -> bytes | None:
        so = tr.get_extra_info("ssl_object") if tr is not None else None
        try:
            return so.getpeercert(binary_form=True) if so is not None else None
        except (ValueError, AttributeError):
            return None

    def _authenticate(self, request):
        tr = request.transport
        pc = tr.get_extra_info("peercert") if self.tls and tr is not None else None
        return self.authn.authenticate(request.headers, pc, self._peer_der(tr) if pc else None)

    UNSECURED = {"name": "system:unsecured", "uid": "", "groups": ["system:masters", "system:authenticated"]}

    async def _authenticate_async(self, request):
        tr = request.transport
        if getattr(self, "insecure_port", None) and tr is not None and \
                (tr.get_extra_info("sockname") or (None, None))[1] == self.insecure_port:
            return self.UNSECURED
        pc = tr.get_extra_info("peercert") if self.tls and tr is not None else None
        return await self.authn.authenticate_async(request.headers, pc, self._peer_der(tr) if pc else None)

    async def _authorize(self, user, verb, resource, group="", ns="", name="", sub=""):
        ok, _ = await self.authz.authorize_async(Attributes(user, verb, group, resource, sub, ns, name))
        if not ok:
            what = f"{resource}/{sub}" if sub else resource
            where = f' in the namespace "{ns}"' if ns else " at the cluster scope"
            raise m.forbidden(f'User "{user.get("name")}" cannot {verb} {what}{" " + repr(name) if name else ""}'
                              f'{" in API group " + repr(group) if group else ""}{where}')

    async def _authorize_nonresource(self, user, verb, path):
        ok, _ = await self.authz.authorize_async(Attributes(user, verb, path=path, resource_request=False))
        if not ok:
            raise m.forbidden(f'User "{user.get("name")}" cannot {verb} path "{path}"')

    def _set_scale(self, rs, ns, name, scale: dict, user) -> dict:
        """PUT/PATCH .../scale: only spec.replicas changes; a resourceVersion in the Scale is a
        precondition, as for the parent object."""
        n = (scale.get("spec") or {}).get("replicas")
        if not isinstance(n, int) or n < 0:
            raise m.invalid("Scale", name, ["spec.replicas: Invalid value: must be a non-negative integer"])
        rv = (scale.get("metadata") or {}).get("resourceVersion")
        if rv:
            cur = rs.get(ns, name)
            if (cur.get("metadata") or {}).get("resourceVersion") != rv:
                raise m.conflict(rs.ri.group_resource, name, "the object has been modified; please apply your changes to the latest version and try again")
        obj, _ = rs.update(ns, name, None, user=user, patch=json.dumps({"spec": {"replicas": n}}).encode(),
                           content_type="application/merge-patch+json")
        return _to_scale(obj)

    async def _review(self, plural, body, requester=None, ns=""):
        """SubjectAccessReview / TokenReview (authorization.k8s.io, authentication.k8s.io): computed, not stored."""
        spec = body.get("spec") or {}
        if plural == "tokenreviews":
            u = await self.authn.authenticate_token_async(spec.get("token", "")) if spec.get("token") else None
            st = {"authenticated": u is not None}
            if u is not None:
                st["user"] = {"username": u.get("name"), "uid": u.get("uid", ""), "groups": u.get("groups") or []}
        else:
            if plural == "selfsubjectaccessreviews":   # the requester asks about itself
                user = {"name": (requester or {}).get("name", ""), "groups": (requester or {}).get("groups") or []}
            else:
                user = {"name": spec.get("user", ""), "groups": spec.get("groups") or []}
            ra, nra = spec.get("resourceAttributes"), spec.get("nonResourceAttributes")
            if plural == "localsubjectaccessreviews" and ra is not None:
                ra = dict(ra, namespace=ns)   # pinned to the URL's namespace
            if ra:
                a = Attributes(user, ra.get("verb", ""), ra.get("group", ""), ra.get("resource", ""), ra.get("subresource", ""),
                               ra.get("namespace", ""), ra.get("name", ""))
            else:
                a = Attributes(user, (nra or {}).get("verb", ""), path=(nra or {}).get("path", ""), resource_request=False)
            ok, why = await self.authz.authorize_async(a)
            st = {"allowed": ok, "reason": why}
        return dict(body, status=st)

    # -------------------------------------------------------------- dispatch
    def _parse(self, path: str):
        parts = [p for p in path.split("/") if p]
        if parts[0] == "api":
            if len(parts) < 2:
                raise m.not_found("path", path)
            group, version, rest = "", parts[1], parts[2:]
        else:
            if len(parts) < 3:
                if len(parts) == 2:
                    return parts[1], None, None, None, None, None, False
                raise m.not_found("path", path)
            group, version, rest = parts[1], parts[2], parts[3:]
        watch = False
        if rest and rest[0] == "watch":
            watch, rest = True, rest[1:]
        ns = ""
        # /namespaces/<ns>/<resource>... vs the namespace object's own subresources
        # (/namespaces/<name>/status, /namespaces/<name>/finalize)
        if len(rest) >= 3 and rest[0] == "namespaces" and not (len(rest) == 3 and rest[2] in ("status", "finalize")):
            ns, rest = rest[1], rest[2:]
        resource = rest[0] if rest else None
        name = rest[1] if len(rest) > 1 else None
        sub = "/".join(rest[2:]) if len(rest) > 2 else ""
        if resource == "namespaces" and name and not ns:
            pass
        return group, version, resource, ns, name, sub, watch

    async def dispatch(self, request: web.Request):
        t0 = time.perf_counter()
        verb, resource, sub, code = request.method, "", "", 500
        scope = ""
        sem = actx = resp = None
        try:
            user = await self._authenticate_async(request)
            group, version, resource, ns, name, sub, watch = self._parse(request.path)
            if (group, version) in self.disabled_gv:       # --runtime-config turned this group/version off
                raise m.not_found("path", request.path)
            target = self.aggregator.route(group, version) if request.path.startswith("/apis/") else None
            if target is not None:      # an extension API server's group/version (kube-aggregator proxy)
                resource = resource or ""
                resp = await self.aggregator.proxy(request, target, user)
                code = resp.status
                return resp
            if resource is None:
                if version is None:  # /apis/<group>
                    if not any(ri.group == group for ri in SCHEME.by_kind.values()):
                        agg = [d for d in self.aggregator.group_docs(set()) if d["name"] == group]
                        if agg:
                            code = 200
                            return _resp({"kind": "APIGroup", "apiVersion": "v1", **agg[0]})
                        raise m.not_found("group", group)
                    code = 200
                    return _resp({"kind": "APIGroup", "apiVersion": "v1", **self._group_doc(group, self.disabled_gv)})
                code = 200
                return _resp(self._resource_list(group, version))
            served = SCHEME.served(group, version, resource)
            rs = self.registry.resources.get(served.storage or (served.group, served.plural)) if served is not None else None
            if rs is None:
                raise m.not_found("resource", f"{group}/{version}/{resource}")
            conv = served if served.api_version != rs.ri.api_version else None
            # metrics.go cleanScope
            scope = "namespace" if ns else ("resource" if name else "cluster")
            q = request.query
            is_watch = watch or q.get("watch") in ("true", "1")
            kverb = {"GET": "watch" if is_watch else ("get" if name else "list"), "POST": "create", "PUT": "update",
                     "PATCH": "patch", "DELETE": "delete" if name else "deletecollection"}.get(verb, verb.lower())
            top_sub = sub.split("/")[0] if sub else ""
            if name and top_sub in _STREAMING_SUBS:
                kverb = "create"   # exec/attach/portforward/proxy always need create on the subresource
            # the verb label the reference's metrics carry (installer.go actions + cleanVerb)
            verb = "CONNECT" if name and top_sub in _STREAMING_SUBS else _METRIC_VERBS.get(kverb, kverb.upper())
            if self.auditor is not None:
                actx = self.auditor.begin(request, user, kverb, group, version, resource, sub, ns, name or "")
            await self._authorize(user, kverb, resource, group, "" if not rs.ri.namespaced else ns, name or "", top_sub)
            if is_watch:
                code = 200
                if actx is not None:
                    self.auditor.stage(actx, "ResponseStarted", 200)
                return await self._watch(request, rs, ns, name, q, conv)
            if name and top_sub in _STREAMING_SUBS:   # long-running: exempt from max-in-flight, like watches
                request[_USER_KEY] = user
                if actx is not None:
                    self.auditor.stage(actx, "ResponseStarted", 101)
                resp = await self._stream(request, rs, ns, name, sub, q)
                code = resp.status
                return resp
            sem = self._rw if request.method in ("POST", "PUT", "PATCH", "DELETE") else self._ro
            if sem is not None:
                if sem.locked():
                    raise m.too_many_requests()
                await sem.acquire()
            resp = await self._handle(request, rs, ns, name, sub, user, q, as_stored=conv is None, served=conv)
            if conv is not None and resp.body:
                resp = _resp(_convert_out(json.loads(resp.body), rs.ri, conv), resp.status)
            code = resp.status
            return resp
        except m.StatusError as e:
            code = e.code
            resp = _err(e)
            return resp
        except (ValueError, KeyError, TypeError) as e:
            code = 400
            log.debug("bad request %s %s: %r", request.method, request.path, e)
            return _err(m.bad_request(f"{type(e).__name__}: {e}"))
        finally:
            if sem is not None:
                sem.release()
            if actx is not None:
                self.auditor.stage(actx, "ResponseComplete", code, getattr(request, "_read_bytes", None), resp)
            client = request.headers.get("User-Agent", "")
            client = "Browser" if client.startswith("Mozilla/") else client
            ctype = (resp.headers.get("Content-Type", "") if resp is not None else "").split(";")[0]
            self.m_count.labels(verb, resource or "", sub or "", scope, client, ctype, str(code)).inc()
            if verb != "WATCH":
                dt = time.perf_counter() - t0
                us = float(int(dt * 1e6))          # elapsed / time.Microsecond
                self.m_lat.labels(verb, resource or "", sub or "", scope).observe(us)
                self.m_lat_summary.labels(verb, resource or "", sub or "", scope).observe(us)
                self.lat_samples.append((verb, resource or "", sub or "", dt))

    def latency_summary(self, since: int = 0) -> dict:
        """API call latency percentiles over the samples from index `since` on, as the
        reference's density SLO reads them (test/e2e/framework/metrics_util.go:52-59): the worst
        (verb, resource, subresource) p99 of non-LIST calls (limit 1 s) and of LISTs (5 s)."""
        groups: dict[tuple, list] = {}
        for verb, res, sub, dt in list(self.lat_samples)[since:]:
            if verb in ("WATCH", "CONNECT"):
                continue
            groups.setdefault((verb, res, sub), []).append(dt)

        def p(xs, q):
            xs = sorted(xs)
            return xs[min(len(xs) - 1, int(q / 100.0 * len(xs)))]
        rows = [{"verb": v, "resource": r, "subresource": s, "count": len(xs), "p50_ms": round(p(xs, 50) * 1e3, 3),
                 "p90_ms": round(p(xs, 90) * 1e3, 3), "p99_ms": round(p(xs, 99) * 1e3, 3)} for (v, r, s), xs in groups.items()]
        rows.sort(key=lambda x: -x["p99_ms"])
        nonlist = [x for x in rows if x["verb"] != "LIST"]
        lists = [x for x in rows if x["verb"] == "LIST"]
        return {"api_p99_ms": nonlist[0]["p99_ms"] if nonlist else None,
                "api_list_p99_ms": lists[0]["p99_ms"] if lists else None,
                "calls": sum(x["count"] for x in rows), "worst": rows[:5]}

    async def _body(self, request):
        data = await request.read()
        if not data:
            raise m.bad_request("empty request body")
        ct = request.headers.get("Content-Type", _JSON)
        if "yaml" in ct:
            import yaml
            return yaml.safe_load(data)
        if data.startswith(b"k8s\x00") or "protobuf" in ct:
            from ..api import protobuf as pb
            try:
                return pb.decode(data)
            except (pb.ProtoError, ValueError) as e:
                raise m.bad_request(f"protobuf body: {e}")
        return json.loads(data)

    @web.middleware
    async def _protobuf_middleware(self, request, handler):
        """Content negotiation (apiserver/pkg/endpoints/handlers/negotiation): a client whose
        Accept prefers application/vnd.kubernetes.protobuf gets the `k8s\x00` envelope for every
        kind with a protobuf schema (errors included: meta/v1 Status); other kinds stay JSON."""
        resp = await handler(request)
        if not _wants_protobuf(request) or not isinstance(resp, web.Response) or resp.content_type != _JSON:
            return resp
        body = resp.body
        if not isinstance(body, (bytes, bytearray)) or not body[:1] == b"{":
            return resp
        from ..api import protobuf as pb
        try:
            obj = json.loads(body)
            if not (isinstance(obj, dict) and pb.supports(obj)):
                return resp
            data = pb.encode(obj)
        except (ValueError, pb.ProtoError):
            return resp
        out = web.Response(body=data, status=resp.status, content_type=pb.MEDIA_TYPE)
        for k, v in resp.headers.items():
            if k.lower() not in ("content-type", "content-length"):
                out.headers[k] = v
        return out

    async def _w(self, fn, *args, **kwargs):
        """A registry write. Over a remote store it runs bridged (utils/greenbridge.py): where
        the store would wait on etcd, this request yields the loop to the others, and writes
        issued meanwhile are committed together."""
        if self._bridged:
            return await greenbridge.run_sync(fn, *args, **kwargs)
        return fn(*args, **kwargs)

    async def _handle(self, request, rs, ns, name, sub, user, q, as_stored=False, served=None):
        meth = request.method
        ri = rs.ri
        if ri.namespaced is False:
            ns = ""
        if meth == "GET":
            if name and sub == "log" and ri.plural == "pods":
                return await self._pod_log(request, ns, name, q)
            if name:
                if sub and sub not in ("status", "scale"):
                    raise m.not_found("subresource", sub)
                if sub == "scale":
                    return _resp(_to_scale(rs.get(ns, name)))
                if as_stored and _wants_protobuf(request):
                    kv = rs.storage.store.get(rs.key(ns, name))
                    body = kv_proto(kv) if kv is not None else None
                    if body is not None:
                        # protobuf client, same version: the stored bytes (or their cached transcode)
                        return web.Response(body=body, content_type="application/vnd.kubernetes.protobuf")
                raw = rs.storage.get_raw(rs.key(ns, name))
                if raw is None:
                    raise m.not_found(ri.group_resource, name)
                return _resp(raw)
            if as_stored and _wants_protobuf(request) \
                    and not any(q.get(k) for k in ("labelSelector", "fieldSelector", "limit", "continue")) \
                    and not self._hide_uninitialized(q):
                from ..api import protobuf as pb
                kvs, rev, _ = rs.storage.store.range(rs.prefix(ns))
                vals = [kv_proto(kv) for kv in kvs]
                body = None if None in vals else pb.list_from_stored(ri.api_version, ri.list_kind, str(rev), vals)
                if body is not None:
                    return web.Response(body=body, content_type=pb.MEDIA_TYPE)
            return self._list(rs, ns, q)
        if meth == "POST":
            body = await self._body(request)
            if name and sub == "binding" and ri.plural == "pods":
                body.setdefault("metadata", {}).setdefault("name", name)
                return _resp(await self._w(self.registry.bind, ns, body, user), 201)
            if name and sub == "eviction" and ri.plural == "pods":
                await self._w(self.registry.evict, ns, name, body, user)
                return _resp(m.success_status(), 201)
            if name and sub == "rollback" and ri.plural == "deployments":
                # extensions/v1beta1 DeploymentRollback (registry/extensions/deployment/storage:
                # RollbackREST): record spec.rollbackTo for the deployment controller
                patch = {"spec": {"rollbackTo": body.get("rollbackTo") or {"revision": 0}}}
                if body.get("updatedAnnotations"):
                    patch["metadata"] = {"annotations": body["updatedAnnotations"]}
                await self._w(rs.update, ns, name, None, user=user, patch=json.dumps(patch).encode(),
                              content_type="application/merge-patch+json")
                return _resp(m.success_status({"name": name, "kind": "deployments"}), 201)
            if ri.plural in ("subjectaccessreviews", "selfsubjectaccessreviews", "localsubjectaccessreviews", "tokenreviews"):
                return _resp(await self._review(ri.plural, body, user, ns), 201)
            if ri.plural == "pods" and sub == "" and name is None and body.get("kind") == "Binding":
                return _resp(await self._w(self.registry.bind, ns, body, user), 201)
            if name:
                raise m.method_not_allowed("POST on a named resource")
            dry = q.get("dryRun") == "All"
            await self.admission.admit_async(adm.Attributes(adm.CREATE, ri.plural, sub, ns, m.name_of(body), body, None, user,
                                                            ri.kind), self.registry)
            mut, val = self.webhooks.active("CREATE", ri, sub, ns)
            if mut:
                body = await self.webhooks.mutate(mut, "CREATE", ri, sub, ns, None, body, None, user)
            if val:
                final = rs.create(ns, json.loads(json.dumps(body)), user, dry_run=True)
                await self.webhooks.validate(val, "CREATE", ri, sub, ns, None, final, None, user)
            obj = await self._w(rs.create, ns, body, user, dry_run=dry)
            if not dry and q.get("includeUninitialized") not in ("true", "1") and _uninitialized(obj):
                obj = await self._wait_initialized(rs, ns, m.name_of(obj))
            return _resp(obj, 201)
        if meth == "PUT":
            if not name:
                raise m.method_not_allowed("PUT on a collection")
            body = await self._body(request)
            if sub == "scale":
                return _resp(await self._w(self._set_scale, rs, ns, name, body, user))
            subr = "status" if sub in ("status", "approval") else ""
            if sub == "finalize" and ri.plural == "namespaces":
                subr = "finalize"
            if not sub and self.admission.has("ImagePolicyWebhook"):
                await self.admission.admit_async(adm.Attributes(adm.UPDATE, ri.plural, sub, ns, name, body, rs.get(ns, name),
                                                                user, ri.kind), self.registry)
            mut, val = self.webhooks.active("UPDATE", ri, sub, ns)
            if mut or val:
                old = rs.get(ns, name)
                if mut:
                    body = await self.webhooks.mutate(mut, "UPDATE", ri, sub, ns, name, body, old, user)
                if val:
                    await self.webhooks.validate(val, "UPDATE", ri, sub, ns, name, body, old, user)
            obj, created = await self._w(rs.update, ns, name, body, subresource=subr, user=user)
            return _resp(obj, 201 if created else 200)
        if meth == "PATCH":
            if not name:
                raise m.method_not_allowed("PATCH on a collection")
            data = await request.read()
            ct = request.headers.get("Content-Type", "application/merge-patch+json")
            if sub == "scale":
                from .registry import apply_patch
                cur = _to_scale(rs.get(ns, name))
                return _resp(await self._w(self._set_scale, rs, ns, name, apply_patch(cur, data, ct), user))
            mut, val = self.webhooks.active("UPDATE", ri, sub, ns)
            if mut or val:
                # webhooks see the patched object; it is then written as an update conditioned on the
                # resourceVersion it was computed from (a concurrent writer gets a 409 to retry)
                from .registry import apply_patch
                old = rs.get(ns, name)
                new = apply_patch(old, data, ct)
                if mut:
                    new = await self.webhooks.mutate(mut, "UPDATE", ri, sub, ns, name, new, old, user)
                if val:
                    await self.webhooks.validate(val, "UPDATE", ri, sub, ns, name, new, old, user)
                new.setdefault("metadata", {})["resourceVersion"] = (old.get("metadata") or {}).get("resourceVersion")
                obj, _ = await self._w(rs.update, ns, name, new, subresource=sub if sub == "status" else "", user=user)
                return _resp(obj)
            obj, _ = await self._w(rs.update, ns, name, None, subresource=sub if sub == "status" else "", user=user,
                                   patch=data, content_type=ct, served=served)
            return _resp(obj)
        if meth == "DELETE":
            opts = {}
            data = await request.read()
            if data:
                try:
                    opts = json.loads(data)
                except ValueError:
                    raise m.bad_request("invalid DeleteOptions")
            grace = opts.get("gracePeriodSeconds")
            if "gracePeriodSeconds" in q:
                grace = int(q["gracePeriodSeconds"])
            prop = opts.get("propagationPolicy") or q.get("propagationPolicy")
            if opts.get("orphanDependents") is True:
                prop = "Orphan"
            uid = (opts.get("preconditions") or {}).get("uid")
            _, val = self.webhooks.active("DELETE", ri, sub, ns)
            if val and name:
                await self.webhooks.validate(val, "DELETE", ri, sub, ns, name, None, rs.get(ns, name), user)
            if name:
                obj, now = await self._w(rs.delete, ns, name, grace=grace, precond_uid=uid, user=user, propagation=prop)
                return _resp(obj if not now or ri.plural == "pods" else m.success_status(
                    {"name": name, "kind": ri.plural, "uid": m.uid_of(obj)}))
            items, _, _ = rs.list(ns, q.get("labelSelector"), q.get("fieldSelector"))
            for it in items:
                try:
                    await self._w(rs.delete, m.namespace_of(it), m.name_of(it), grace=grace, user=user, propagation=prop)
                except m.StatusError as e:
                    if not m.is_not_found(e):
                        raise
            return _resp({"kind": ri.list_kind, "apiVersion": ri.api_version, "metadata": {}, "items": items})
        raise m.method_not_allowed(meth)

    def _hide_uninitialized(self, q) -> bool:
        return self.admission.has("Initializers") and q.get("includeUninitialized") not in ("true", "1")

    async def _wait_initialized(self, rs, ns, name, timeout=30.0):
        """initialization: a create returns once every initializer has run (pending empty);
        a failed initialization (result set) deleted the object; past the timeout: 504."""
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while loop.time() < end:
            cur = rs.storage.get(rs.key(ns, name), ignore_not_found=True)
            if cur is None:
                raise m.StatusError(500, "InternalError", f"object {name} was deleted during initialization")
            ini = (cur.get("metadata") or {}).get("initializers") or {}
            if ini.get("result"):
                st = ini["result"]
                raise m.StatusError(int(st.get("code") or 500), st.get("reason") or "InternalError", st.get("message", ""))
            if not _uninitialized(cur):
                return cur
            await asyncio.sleep(0.05)
        raise m.StatusError(504, "Timeout", f"timed out waiting for the initialization of {name}")

    def _list(self, rs, ns, q):
        ri = rs.ri
        limit = int(q.get("limit", "0") or 0)
        cont = q.get("continue") or None
        ls, fs = q.get("labelSelector"), q.get("fieldSelector")
        if self._hide_uninitialized(q):
            items, rev, nxt = rs.list(ns, ls, fs, limit, cont)
            md = {"resourceVersion": str(rev), **({"continue": nxt} if nxt else {})}
            return _resp({"kind": ri.list_kind, "apiVersion": ri.api_version, "metadata": md,
                          "items": [o for o in items if not _uninitialized(o)]})
        if not ls and not fs and not limit and not cont:
            raws, rev = rs.storage.list_raw(rs.prefix(ns))
            body = (b'{"kind":"' + ri.list_kind.encode() + b'","apiVersion":"' + ri.api_version.encode() +
                    b'","metadata":{"resourceVersion":"' + str(rev).encode() + b'"},"items":[' + b",".join(raws) + b"]}")
            return _resp(body)
        items, rev, nxt = rs.list(ns, ls, fs, limit, cont)
        md = {"resourceVersion": str(rev)}
        if nxt:
            md["continue"] = nxt
        return _resp({"kind": ri.list_kind, "apiVersion": ri.api_version, "metadata": md, "items": items})

    async def _watch(self, request, rs, ns, name, q, conv=None):
        ri = rs.ri
        if not ri.namespaced:
            ns = ""
        rv = q.get("resourceVersion", "")
        ls, fs = q.get("labelSelector"), q.get("fieldSelector")
        if name:
            fs = f"metadata.name={name}" + (f",{fs}" if fs else "")
        mrt = getattr(self, "min_request_timeout", 1800.0)     # --min-request-timeout: watches end in [min, 2·min)
        timeout = float(q.get("timeoutSeconds") or (mrt + random.random() * mrt))
        initial = []
        if rv in ("", "0"):
            items, list_rev, _ = rs.list(ns, ls, fs)
            initial = items
            w = rs.watch(ns, str(list_rev), ls, fs)
        else:
            w = rs.watch(ns, rv, ls, fs)
        proto = _wants_protobuf(request)
        ctype = "application/vnd.kubernetes.protobuf;stream=watch" if proto else _JSON
        resp = web.StreamResponse(status=200, headers={"Content-Type": ctype, "Transfer-Encoding": "chunked"})
        resp.enable_chunked_encoding()
        await resp.prepare(request)
        self.watch_count += 1
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        try:
            frame = self._frame if conv is None else (lambda t: _convert_frame(self._frame(t), ri, conv))
            if proto:
                # length-delimited meta/v1 WatchEvent frames, objects enveloped (framer.go)
                from ..api import protobuf as pb
                json_frame = frame

                def frame(t, _jf=json_frame):
                    if conv is None and t[2].type == PUT:    # the object's (cached) protobuf form
                        raw = kv_proto(t[2].kv)
                        if raw is not None:
                            return pb.watch_frame(t[0], raw)
                    ev = json.loads(_jf(t))
                    return pb.encode_watch_event(ev["type"], ev["object"])
            if self._hide_uninitialized(q):
                initial = [o for o in initial if not _uninitialized(o)]
                inner = frame

                def frame(t):   # uninitialized objects are invisible; they appear once initialized
                    return b"" if t[1] is not None and _uninitialized(t[1]) else inner(t)
            if initial:
                buf = bytearray()
                for o in initial:
                    if conv is not None:
                        o = _convert_out(o, ri, conv)
                    if proto:
                        buf += pb.encode_watch_event("ADDED", o)
                    else:
                        buf += b'{"type":"ADDED","object":' + json.dumps(o, separators=(",", ":")).encode() + b"}\n"
                await resp.write(bytes(buf))
            while True:
                rem = deadline - loop.time()
                if rem <= 0:
                    break
                ev = await w.next(rem)
                if ev is None:
                    if w.closed:
                        if getattr(w.w, "err", None):
                            st = m.gone(f"watch closed: {w.w.err}").status()
                            await resp.write(pb.encode_watch_event("ERROR", st) if proto else
                                             b'{"type":"ERROR","object":' + json.dumps(st).encode() + b"}\n")
                        break
                    continue
                buf = bytearray(frame(ev))
                # drain whatever else is already queued into the same chunk (batching)
                while not w.w.queue.empty():
                    nxt = w.w.queue.get_nowait()
                    if nxt is None:
                        break
                    buf += frame(nxt)
                await resp.write(bytes(buf))
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            w.close()
            self.watch_count -= 1
        try:
            await resp.write_eof()
        except Exception:
            pass
        return resp

    @staticmethod
    def _frame(t) -> bytes:
        typ, obj, ev = t
        if ev.type == PUT:
            data = kv_json(ev.kv)
        else:
            data = json.dumps(obj, separators=(",", ":")).encode()
        return b'{"type":"' + typ.encode() + b'","object":' + data + b"}\n"

    def _kubelet_addr(self, node_name: str) -> tuple[str, int]:
        node = self.registry.rs("nodes").get("", node_name)
        st = node.get("status") or {}
        port = (((st.get("daemonEndpoints") or {}).get("kubeletEndpoint")) or {}).get("Port")
        addr = next((a["address"] for a in st.get("addresses") or [] if a.get("type") == "InternalIP"), None) or \
            next((a["address"] for a in st.get("addresses") or [] if a.get("type") == "Hostname"), "127.0.0.1")
        if not port:
            raise m.bad_request(f"node {node_name} has no kubelet endpoint")
        return addr, int(port)

    async def _stream(self, request, rs, ns, name, sub, q):
        """pods/{name}/exec|attach|portforward (WebSocket relayed to the node's kubelet, SPDY/3.1
        spliced through to it,
        registry/core/pod/rest/subresources.go) and pods|services|nodes/{name}/proxy/{path}
        (HTTP proxy to the pod IP, a service endpoint or the kubelet)."""
        from ..runtime import spdy
        from ..runtime.streaming import CHANNEL_PROTOCOLS, PORTFORWARD_PROTOCOLS, bridge
        plural = rs.ri.plural
        top, _, rest = sub.partition("/")
        if top == "proxy":
            return await self._proxy(request, plural, ns, name, rest, q)
        if plural != "pods":
            raise m.not_found("subresource", sub)
        pod = rs.get(ns, name)
        user = request.get(_USER_KEY)
        attrs = adm.Attributes(adm.CONNECT, "pods", top, ns, name, None, pod, user, "Pod")
        self.admission.admit(attrs, self.registry)      # DenyEscalatingExec / DenyExecOnPrivileged
        self.admission.validate(attrs, self.registry)
        node_name = (pod.get("spec") or {}).get("nodeName")
        if not node_name:
            raise m.bad_request(f'pod "{name}" is not scheduled yet')
        addr, port = self._kubelet_addr(node_name)
        qs = request.query_string
        if top == "portforward":
            url, protos = f"{self.kubelet_scheme}://{addr}:{port}/portForward/{ns}/{name}?{qs}", PORTFORWARD_PROTOCOLS
        else:
            container = q.get("container") or ((pod.get("spec") or {}).get("containers") or [{}])[0].get("name", "")
            url, protos = f"{self.kubelet_scheme}://{addr}:{port}/{top}/{ns}/{name}/{container}?{qs}", CHANNEL_PROTOCOLS
        if spdy.is_upgrade(request):
            return await spdy.upgrade_proxy(request, url, ssl=self.kubelet_ssl)
        ws = web.WebSocketResponse(protocols=protos, max_msg_size=0)
        if not ws.can_prepare(request).ok:
            raise m.bad_request(f"{top} needs a WebSocket upgrade (protocols {', '.join(protos)})")
        await ws.prepare(request)
        return await bridge(ws, url, [ws.ws_protocol or protos[0]], ssl=self.kubelet_ssl)

    async def _proxy(self, request, plural, ns, name, path, q):
        if self._http is None:
            self._http = ClientSession(timeout=ClientTimeout(total=None))
        if plural == "nodes":
            addr, port = self._kubelet_addr(name)
            target = f"{self.kubelet_scheme}://{addr}:{port}"
        elif plural == "pods":
            pod_name, _, pport = name.partition(":")
            pod = self.registry.rs("pods").get(ns, pod_name)
            ip = (pod.get("status") or {}).get("podIP")
            if not ip:
                raise m.bad_request(f'pod "{pod_name}" has no IP')
            if not pport:
                ports = [p for c in (pod.get("spec") or {}).get("containers") or [] for p in c.get("ports") or []]
                pport = str(ports[0]["containerPort"]) if ports else "80"
            target = f"http://{ip}:{pport}"
        elif plural == "services":
            svc_name, _, sport = name.partition(":")
            ep = self.registry.rs("endpoints").get(ns, svc_name)
            for subset in ep.get("subsets") or []:
                addrs = subset.get("addresses") or []
                ports = subset.get("ports") or []
                if not addrs or not ports:
                    continue
                p = next((x for x in ports if not sport or x.get("name") == sport or str(x.get("port")) == sport), None)
                if p is not None:
                    target = f"http://{addrs[0]['ip']}:{p['port']}"
                    break
            else:
                raise m.StatusError(503, "ServiceUnavailable", f'no endpoints available for service "{svc_name}"')
        else:
            raise m.not_found("subresource", "proxy")
        body = await request.read()
        hdrs = {k: v for k, v in request.headers.items() if k.lower() not in ("host", "authorization", "content-length")}
        async with self._http.request(request.method, f"{target}/{path}", params=q, data=body or None, headers=hdrs,
                                      ssl=self.kubelet_ssl if plural == "nodes" else None) as r:
            data = await r.read()
            return web.Response(status=r.status, body=data,
                                headers={k: v for k, v in r.headers.items() if k.lower() in ("content-type", "cache-control")})

    async def _pod_log(self, request, ns, name, q):
        """pods/log (registry/core/pod/rest/log.go + strategy.go LogLocation): the options are
        validated (ValidatePodLogOptions → 422), the container defaults to the pod's only one
        (else BadRequest naming the choices), an unscheduled pod has no log yet (empty body), and
        the node's kubelet answers /containerLogs with the options passed through."""
        from ..kubelet import logs as L
        try:
            opts = L.decode_log_query(q)
        except ValueError as e:
            raise m.bad_request(f"invalid log options: {e}") from None
        errs = L.validate_pod_log_options(opts)
        if errs:
            raise m.invalid("PodLogOptions", name, [str(e) for e in errs])
        pod = self.registry.rs("pods").get(ns, name)
        try:
            container = L.log_location_container(pod, name, opts.get("container"))
        except ValueError as e:
            raise m.bad_request(str(e)) from None
        node_name = (pod.get("spec") or {}).get("nodeName")
        if not node_name:
            return web.Response(body=b"", content_type="text/plain")
        node = self.registry.rs("nodes").get("", node_name)
        st = node.get("status") or {}
        port = (((st.get("daemonEndpoints") or {}).get("kubeletEndpoint")) or {}).get("Port")
        addr = next((a["address"] for a in st.get("addresses") or [] if a.get("type") == "InternalIP"), None) or \
            next((a["address"] for a in st.get("addresses") or [] if a.get("type") == "Hostname"), "127.0.0.1")
        if not port:
            raise m.bad_request(f"node {node_name} has no kubelet endpoint")
        params = {}
        for k in ("follow", "previous", "timestamps"):
            if opts.get(k):
                params[k] = "true"
        for k in ("sinceSeconds", "tailLines", "limitBytes"):
            if opts.get(k) is not None:
                params[k] = str(opts[k])
        if opts.get("sinceTime"):
            params["sinceTime"] = L.format_rfc3339nano(L.parse_rfc3339(opts["sinceTime"]) // 10**9 * 10**9)
        if self._http is None:
            self._http = ClientSession(timeout=ClientTimeout(total=None))
        url = f"{self.kubelet_scheme}://{addr}:{port}/containerLogs/{ns}/{name}/{container}"
        async with self._http.get(url, params=params, ssl=self.kubelet_ssl) as r:
            if r.status != 200:
                # GenericHttpResponseChecker: the kubelet's answer becomes the status message
                reason = {400: "BadRequest", 404: "NotFound", 422: "Invalid", 403: "Forbidden"}.get(r.status, "InternalError")
                raise m.StatusError(r.status, reason, (await r.text()).strip()[:1024])
            out = web.StreamResponse(status=200, headers={"Content-Type": "text/plain"})
            await out.prepare(request)
            async for chunk in r.content.iter_any():
                await out.write(chunk)
            await out.write_eof()
            return out
