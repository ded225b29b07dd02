"""metrics-server: the resource metrics API (metrics.k8s.io/v1beta1) as an aggregated API server.

Reference surface: staging/src/k8s.io/metrics (NodeMetrics / PodMetrics types of the
metrics.k8s.io group served through kube-aggregator; `kubectl top` and the HPA read it) and the
metrics-server that serves it (the reference release's Heapster successor). It scrapes every
node's kubelet /stats/summary each --metric-resolution (usageNanoCores, workingSetBytes — plus
the MI355X accelerator stats the amdkube kubelet reports), keeps the latest window per node
and pod, and serves

  /apis/metrics.k8s.io/v1beta1/nodes[/NAME]
  /apis/metrics.k8s.io/v1beta1/pods, /namespaces/NS/pods[/NAME]   (labelSelector supported)

and the custom metrics API (custom.metrics.k8s.io/v1beta1, staging/src/k8s.io/metrics/pkg/apis/
custom_metrics: MetricValueList of MetricValue{describedObject, metricName, timestamp, window,
value}) with the MI355X series autoscalers want — per pod `gpu_utilization` (duty cycle, %, the
busiest of the pod's GPUs), `gpu_memory_used_bytes` (its containers' VRAM), `gpu_count`; per
node the same over all its GPUs —

  /apis/custom.metrics.k8s.io/v1beta1/namespaces/NS/pods/{NAME|*}/METRIC   (labelSelector for *)
  /apis/custom.metrics.k8s.io/v1beta1/nodes/{NAME|*}/METRIC

all behind front-proxy authentication (the aggregator's client certificate, verified against
--requestheader-client-ca-file, asserting X-Remote-User/Group) or a bearer token checked by
TokenReview, and authorization delegated to the main apiserver (SubjectAccessReview, verbs
get/list on nodes.metrics.k8s.io / pods.metrics.k8s.io).
"""
from __future__ import annotations

import asyncio
import logging
import ssl

from aiohttp import ClientSession, ClientTimeout, web

from ..api import meta as m
from ..api.labels import parse_selector

log = logging.getLogger("amdkube.metrics")
GV = "metrics.k8s.io/v1beta1"
CGV = "custom.metrics.k8s.io/v1beta1"
POD_METRICS = ("gpu_utilization", "gpu_memory_used_bytes", "gpu_count")


def _cpu(nano: int) -> str:
    nano = max(0, int(nano))
    return f"{nano}n" if nano % 1_000_000 else f"{nano // 1_000_000}m"


def _mem(b: int) -> str:
    return f"{int(b) // 1024}Ki" if b % 1024 == 0 else str(int(b))


class MetricsServer:
    def __init__(self, client, resolution: float = 60.0, requestheader_ca: str | None = None, allowed_names=(),
                 tls_cert: str | None = None, tls_key: str | None = None, kubelet_scheme: str = "http",
                 kubelet_ssl=None, authorize: bool = True):
        self.client, self.resolution = client, resolution
        self.requestheader_ca, self.allowed = requestheader_ca, set(allowed_names or ())
        self.tls = (tls_cert, tls_key)
        self.kubelet_scheme, self.kubelet_ssl, self.authorize_requests = kubelet_scheme, kubelet_ssl, authorize
        self.nodes: dict[str, dict] = {}
        self.pods: dict[tuple[str, str], dict] = {}
        self.labels: dict[tuple[str, str], dict] = {}
        self._issuer = None
        self._http: ClientSession | None = None
        self._task = None
        self.runner = None
        self.port = None
        self.scrapes = 0
        app = self.app = web.Application(middlewares=[self._auth])
        app.router.add_get("/apis/metrics.k8s.io", self.group)
        app.router.add_get("/apis/metrics.k8s.io/v1beta1", self.resources)
        app.router.add_get("/apis/metrics.k8s.io/v1beta1/nodes", self.list_nodes)
        app.router.add_get("/apis/metrics.k8s.io/v1beta1/nodes/{name}", self.get_node)
        app.router.add_get("/apis/metrics.k8s.io/v1beta1/pods", self.list_pods)
        app.router.add_get("/apis/metrics.k8s.io/v1beta1/namespaces/{ns}/pods", self.list_pods)
        app.router.add_get("/apis/metrics.k8s.io/v1beta1/namespaces/{ns}/pods/{name}", self.get_pod)
        app.router.add_get("/apis/custom.metrics.k8s.io", self.custom_group)
        app.router.add_get("/apis/custom.metrics.k8s.io/v1beta1", self.custom_resources)
        app.router.add_get("/apis/custom.metrics.k8s.io/v1beta1/namespaces/{ns}/pods/{name}/{metric}", self.custom_pods)
        app.router.add_get("/apis/custom.metrics.k8s.io/v1beta1/nodes/{name}/{metric}", self.custom_nodes)
        app.router.add_get("/healthz", lambda r: web.Response(text="ok"))
        self.custom: dict[tuple, dict] = {}        # ("pod", ns, name) | ("node", "", name) -> {metric: value}
        self.node_labels: dict[str, dict] = {}
        self.stamp = ""

    # ------------------------------------------------------------------ scraping
    async def scrape_once(self):
        if self._http is None:
            self._http = ClientSession(timeout=ClientTimeout(total=10))
        nodes, _ = await self.client.list("nodes")
        pods, _ = await self.client.list("pods")
        self.labels = {(m.namespace_of(p), m.name_of(p)): m.labels_of(p) for p in pods}

        async def one(n):
            st = n.get("status") or {}
            port = ((st.get("daemonEndpoints") or {}).get("kubeletEndpoint") or {}).get("Port")
            addr = next((a["address"] for a in st.get("addresses") or [] if a.get("type") == "InternalIP"), None)
            if not port or not addr:
                return None
            try:
                async with self._http.get(f"{self.kubelet_scheme}://{addr}:{port}/stats/summary", ssl=self.kubelet_ssl) as r:
                    return n, await r.json()
            except Exception as e:    # noqa: BLE001 — an unreachable kubelet just has no fresh metrics
                log.debug("scrape of %s failed: %r", m.name_of(n), e)
                return None
        now = m.now_rfc3339()
        window = f"{int(self.resolution)}s"
        custom: dict[tuple, dict] = {}
        for res in await asyncio.gather(*(one(n) for n in nodes)):
            if res is None:
                continue
            n, summ = res
            node = summ.get("node") or {}
            nacc = node.get("accelerators") or []
            custom[("node", "", m.name_of(n))] = {
                "gpu_utilization": str(max((a.get("dutyCycle", 0) for a in nacc), default=0)),
                "gpu_memory_used_bytes": str(sum(a.get("memoryUsed", 0) for a in nacc)), "gpu_count": str(len(nacc))}
            self.nodes[m.name_of(n)] = {"kind": "NodeMetrics", "apiVersion": GV,
                                        "metadata": {"name": m.name_of(n), "creationTimestamp": now,
                                                     "labels": m.labels_of(n)},
                                        "timestamp": now, "window": window,
                                        "usage": {"cpu": _cpu((node.get("cpu") or {}).get("usageNanoCores", 0)),
                                                  "memory": _mem((node.get("memory") or {}).get("workingSetBytes", 0))}}
            for p in summ.get("pods") or []:
                ref = p.get("podRef") or {}
                key = (ref.get("namespace", ""), ref.get("name", ""))
                cs = [{"name": ct["name"], "usage": {"cpu": _cpu((ct.get("cpu") or {}).get("usageNanoCores", 0)),
                                                     "memory": _mem((ct.get("memory") or {}).get("workingSetBytes", 0))}}
                      for ct in p.get("containers") or []]
                accel = [a for ct in p.get("containers") or [] for a in ct.get("accelerators") or []]
                obj = {"kind": "PodMetrics", "apiVersion": GV,
                       "metadata": {"name": key[1], "namespace": key[0], "creationTimestamp": now,
                                    "labels": self.labels.get(key, {})},
                       "timestamp": now, "window": window, "containers": cs}
                custom[("pod", key[0], key[1])] = {
                    "gpu_utilization": str(max((a.get("dutyCycle", 0) for a in accel), default=0)),
                    "gpu_memory_used_bytes": str(sum(a.get("memoryUsed", 0) for a in accel)),
                    "gpu_count": str(len({a.get("id") for a in accel}))}
                if accel:   # amdkube: the pod's MI355X duty cycle and VRAM next to CPU/memory
                    obj["metadata"]["annotations"] = {"amd.com/gpu-duty-cycle": str(max(a.get("dutyCycle", 0) for a in accel)),
                                                      "amd.com/gpu-memory-used": str(sum(a.get("memoryUsed", 0) for a in accel))}
                self.pods[key] = obj
        live = {(m.namespace_of(p), m.name_of(p)) for p in pods}
        for k in [k for k in self.pods if k not in live]:
            del self.pods[k]
        self.custom, self.stamp = custom, now
        self.node_labels = {m.name_of(n): m.labels_of(n) for n in nodes}
        self.scrapes += 1

    async def _loop(self):
        while True:
            try:
                await self.scrape_once()
            except Exception as e:
                log.warning("metrics scrape failed: %r", e)
            await asyncio.sleep(self.resolution)

    # ------------------------------------------------------------ authn / authz
    def _user(self, request) -> dict | None:
        pc = request.transport.get_extra_info("peercert") if request.transport else None
        if pc and self._issuer is not None and pc.get("issuer") == self._issuer:
            cn = next((v for rdn in pc.get("subject") or () for k, v in rdn if k == "commonName"), "")
            if (not self.allowed or cn in self.allowed) and request.headers.get("X-Remote-User"):
                return {"name": request.headers["X-Remote-User"], "groups": request.headers.getall("X-Remote-Group", [])}
        return None

    @web.middleware
    async def _auth(self, request, handler):
        if request.path == "/healthz" or not self.authorize_requests:
            return await handler(request)
        user = self._user(request)
        if user is None and request.headers.get("Authorization", "").startswith("Bearer "):
            tr = await self.client.create({"apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview",
                                           "spec": {"token": request.headers["Authorization"][7:]}})
            st = tr.get("status") or {}
            if st.get("authenticated"):
                user = {"name": (st.get("user") or {}).get("username", ""), "groups": (st.get("user") or {}).get("groups") or []}
        if user is None:
            raise web.HTTPUnauthorized(text="Unauthorized")
        parts = request.path.split("/")
        if len(parts) > 4:
            group = "custom.metrics.k8s.io" if parts[2] == "custom.metrics.k8s.io" else "metrics.k8s.io"
            res = "nodes" if "nodes" in parts else "pods"
            if group == "custom.metrics.k8s.io" and request.match_info.get("metric"):
                res = f"{res}/{request.match_info['metric']}"     # custom metrics authorize per metric
            ns = request.match_info.get("ns", "")
            nm = request.match_info.get("name", "")
            verb = "get" if nm and nm != "*" else "list"
            sar = await self.client.create({"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview", "spec": {
                "user": user["name"], "groups": user.get("groups") or [],
                "resourceAttributes": {"verb": verb, "group": group, "resource": res.split("/")[0],
                                       "subresource": res.split("/")[1] if "/" in res else "", "namespace": ns,
                                       "name": "" if nm == "*" else nm}}})
            if not (sar.get("status") or {}).get("allowed"):
                raise web.HTTPForbidden(text=f'User "{user["name"]}" cannot {verb} {res}.{group}')
        return await handler(request)

    # ---------------------------------------------------------------- handlers
    async def group(self, r):
        return web.json_response({"kind": "APIGroup", "apiVersion": "v1", "name": "metrics.k8s.io",
                                  "versions": [{"groupVersion": GV, "version": "v1beta1"}],
                                  "preferredVersion": {"groupVersion": GV, "version": "v1beta1"}})

    async def resources(self, r):
        return web.json_response({"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": GV, "resources": [
            {"name": "nodes", "singularName": "", "namespaced": False, "kind": "NodeMetrics", "verbs": ["get", "list"]},
            {"name": "pods", "singularName": "", "namespaced": True, "kind": "PodMetrics", "verbs": ["get", "list"]}]})

    @staticmethod
    def _select(objs, q):
        sel = parse_selector(q["labelSelector"]) if q.get("labelSelector") else None
        return [o for o in objs if sel is None or sel.matches((o.get("metadata") or {}).get("labels") or {})]

    async def list_nodes(self, r):
        return web.json_response({"kind": "NodeMetricsList", "apiVersion": GV, "metadata": {},
                                  "items": self._select(sorted(self.nodes.values(), key=m.name_of), r.query)})

    async def get_node(self, r):
        o = self.nodes.get(r.match_info["name"])
        if o is None:
            raise web.HTTPNotFound(text=f'nodemetrics "{r.match_info["name"]}" not found')
        return web.json_response(o)

    async def list_pods(self, r):
        ns = r.match_info.get("ns")
        items = [o for (pns, _n), o in sorted(self.pods.items()) if ns is None or pns == ns]
        return web.json_response({"kind": "PodMetricsList", "apiVersion": GV, "metadata": {}, "items": self._select(items, r.query)})

    async def get_pod(self, r):
        o = self.pods.get((r.match_info["ns"], r.match_info["name"]))
        if o is None:
            raise web.HTTPNotFound(text=f'podmetrics "{r.match_info["name"]}" not found')
        return web.json_response(o)

    # ------------------------------------------------------------ custom metrics
    async def custom_group(self, r):
        return web.json_response({"kind": "APIGroup", "apiVersion": "v1", "name": "custom.metrics.k8s.io",
                                  "versions": [{"groupVersion": CGV, "version": "v1beta1"}],
                                  "preferredVersion": {"groupVersion": CGV, "version": "v1beta1"}})

    async def custom_resources(self, r):
        res = [{"name": f"pods/{mt}", "singularName": "", "namespaced": True, "kind": "MetricValueList", "verbs": ["get"]}
               for mt in POD_METRICS]
        res += [{"name": f"nodes/{mt}", "singularName": "", "namespaced": False, "kind": "MetricValueList", "verbs": ["get"]}
                for mt in POD_METRICS]
        return web.json_response({"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": CGV, "resources": res})

    def _values(self, kind, ns, name, metric, labels_of, q):
        if metric not in POD_METRICS:
            raise web.HTTPNotFound(text=f'the server could not find the metric {metric} for {kind.lower()}s')
        sel = parse_selector(q["labelSelector"]) if q.get("labelSelector") else None
        items = []
        scope = "pod" if kind == "Pod" else "node"
        for (sc, ons, oname), vals in sorted(self.custom.items()):
            if sc != scope or ons != ns or (name != "*" and oname != name):
                continue
            if sel is not None and not sel.matches(labels_of(ons, oname)):
                continue
            ref = {"kind": kind, "name": oname, "apiVersion": "/v1"}
            if ns:
                ref["namespace"] = ons
            items.append({"describedObject": ref, "metricName": metric, "timestamp": self.stamp,
                          "window": int(self.resolution), "value": vals[metric]})
        if name != "*" and not items:
            raise web.HTTPNotFound(text=f'the server could not find the metric {metric} for {kind.lower()}s {name}')
        return web.json_response({"kind": "MetricValueList", "apiVersion": CGV, "metadata": {"selfLink": ""}, "items": items})

    async def custom_pods(self, r):
        return self._values("Pod", r.match_info["ns"], r.match_info["name"], r.match_info["metric"],
                            lambda ns, n: self.labels.get((ns, n), {}), r.query)

    async def custom_nodes(self, r):
        return self._values("Node", "", r.match_info["name"], r.match_info["metric"],
                            lambda ns, n: self.node_labels.get(n, {}), r.query)

    # --------------------------------------------------------------- lifecycle
    async def start(self, host="127.0.0.1", port=0):
        ctx = None
        if self.tls[0]:
            ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
            ctx.load_cert_chain(*self.tls)
            if self.requestheader_ca:
                ctx.load_verify_locations(self.requestheader_ca)
                ctx.verify_mode = ssl.CERT_OPTIONAL
                self._issuer = ssl._ssl._test_decode_cert(self.requestheader_ca).get("subject")
        self.runner = web.AppRunner(self.app, access_log=None)
        await self.runner.setup()
        site = web.TCPSite(self.runner, host, port, ssl_context=ctx)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        self._task = asyncio.create_task(self._loop(), name="metrics-scrape")
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()
        if self._http:
            await self._http.close()
        if self.runner:
            await self.runner.cleanup()
