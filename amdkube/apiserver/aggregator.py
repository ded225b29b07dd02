"""API aggregation (kube-aggregator, run in-process as kube-apiserver does).

Reference staging/src/k8s.io/kube-aggregator:
  * apiregistration.k8s.io/v1beta1 APIService: `<version>.<group>` served either locally
    (spec.service unset) or by an extension API server behind a Service;
  * pkg/apiserver/handler_proxy.go: /apis/<group>/<version>/... of a non-local APIService is
    proxied to the service (https, caBundle or insecureSkipTLSVerify) with the caller's identity
    in X-Remote-User / X-Remote-Group / X-Remote-Extra-* (the request-header authentication the
    extension server trusts) and without the caller's credentials; an unavailable service → 503;
  * pkg/apiserver/handler_apis.go: /apis and /apis/<group> list the aggregated groups too,
    ordered by groupPriorityMinimum, versions by versionPriority;
  * pkg/controllers/status/available_controller.go: Available condition — Local, or
    ServiceNotFound / ServicePortError / MissingEndpoints / FailedDiscoveryCheck / Passed;
  * pkg/controllers/autoregister + cmd/kube-apiserver/app/aggregator.go: a local APIService for
    every built-in group/version with the reference's priorities.

Endpoints are resolved directly (the reference's --enable-aggregator-routing) so aggregation
works without a service proxy on the control-plane host.
"""
from __future__ import annotations

import asyncio
import logging
import ssl

from aiohttp import ClientSession, ClientTimeout, web

from ..api import meta as m
from ..api.scheme import SCHEME
from ..utils import wait_event

log = logging.getLogger("amdkube.aggregator")
GROUP = "apiregistration.k8s.io"

# cmd/kube-apiserver/app/aggregator.go apiVersionPriorities
PRIORITIES = {
    ("", "v1"): (18000, 1), ("extensions", "v1beta1"): (17900, 1),
    ("apps", "v1beta1"): (17800, 1), ("apps", "v1beta2"): (17800, 9), ("apps", "v1"): (17800, 15),
    ("events.k8s.io", "v1beta1"): (17750, 5),
    ("authentication.k8s.io", "v1"): (17700, 15), ("authentication.k8s.io", "v1beta1"): (17700, 9),
    ("authorization.k8s.io", "v1"): (17600, 15), ("authorization.k8s.io", "v1beta1"): (17600, 9),
    ("autoscaling", "v1"): (17500, 15), ("autoscaling", "v2beta1"): (17500, 9),
    ("batch", "v1"): (17400, 15), ("batch", "v1beta1"): (17400, 9), ("batch", "v2alpha1"): (17400, 9),
    ("certificates.k8s.io", "v1beta1"): (17300, 9), ("networking.k8s.io", "v1"): (17200, 15),
    ("policy", "v1beta1"): (17100, 9),
    ("rbac.authorization.k8s.io", "v1"): (17000, 15), ("rbac.authorization.k8s.io", "v1beta1"): (17000, 12),
    ("rbac.authorization.k8s.io", "v1alpha1"): (17000, 9), ("settings.k8s.io", "v1alpha1"): (16900, 9),
    ("storage.k8s.io", "v1"): (16800, 15), ("storage.k8s.io", "v1beta1"): (16800, 9),
    ("storage.k8s.io", "v1alpha1"): (16800, 1), ("apiextensions.k8s.io", "v1beta1"): (16700, 9),
    ("admissionregistration.k8s.io", "v1beta1"): (16700, 12), ("admissionregistration.k8s.io", "v1alpha1"): (16700, 9),
    ("scheduling.k8s.io", "v1alpha1"): (16600, 9),
}
HOP_HEADERS = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te", "trailers",
               "transfer-encoding", "upgrade", "authorization", "content-length", "host"}


def apiservice_name(group: str, version: str) -> str:
    return f"{version}.{group}" if group else f"{version}."


class Aggregator:
    def __init__(self, server):
        self.server = server
        self.registry = server.registry
        self.index: dict[tuple[str, str], dict] = {}     # (group, version) -> APIService
        self._http: ClientSession | None = None
        self._dirty = asyncio.Event()
        self.registry.store.commit_hooks.append(self._on_commit)
        self._rebuild()

    # ------------------------------------------------------------------ index
    def _rebuild(self):
        self.index = {}
        for a in self.registry.rs("apiservices", GROUP).list("")[0]:
            sp = a.get("spec") or {}
            self.index[(sp.get("group", ""), sp.get("version", ""))] = a

    def _on_commit(self, ev):
        k = ev.kv.key
        if k.startswith("/registry/apiservices/"):
            self._rebuild()
            self._dirty.set()
        elif k.startswith(("/registry/services/", "/registry/endpoints/")):
            self._dirty.set()

    def route(self, group: str, version: str | None) -> dict | None:
        """The non-local APIService that owns /apis/<group>/<version>, if any."""
        if version is None:
            return None
        a = self.index.get((group, version))
        return a if a is not None and (a.get("spec") or {}).get("service") else None

    def group_docs(self, local_groups: set[str]) -> list[dict]:
        """APIGroup documents for groups served only by extension API servers."""
        by_group: dict[str, list[dict]] = {}
        for (g, _v), a in self.index.items():
            if g and g not in local_groups and (a.get("spec") or {}).get("service"):
                by_group.setdefault(g, []).append(a)
        out = []
        for g, lst in by_group.items():
            lst.sort(key=lambda a: (-(a["spec"].get("versionPriority") or 0), a["spec"]["version"]))
            vs = [a["spec"]["version"] for a in lst]
            out.append((max(a["spec"].get("groupPriorityMinimum") or 0 for a in lst), g, {
                "name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v} for v in vs],
                "preferredVersion": {"groupVersion": f"{g}/{vs[0]}", "version": vs[0]}}))
        return [d for _p, _g, d in sorted(out, key=lambda x: (-x[0], x[1]))]

    # ------------------------------------------------------------------ proxy
    def _endpoint(self, svc_ref: dict) -> tuple[str, int]:
        ns, name, port = svc_ref.get("namespace", ""), svc_ref.get("name", ""), svc_ref.get("port") or 443
        svc = self.registry.get_object("services", ns, name)
        if svc is None:
            raise m.StatusError(503, "ServiceUnavailable", f'service "{ns}/{name}" not found')
        sport = next((p for p in (svc.get("spec") or {}).get("ports") or [] if p.get("port") == port), None)
        if sport is None:
            raise m.StatusError(503, "ServiceUnavailable", f"service {ns}/{name} has no port {port}")
        ep = self.registry.get_object("endpoints", ns, name) or {}
        for ss in ep.get("subsets") or []:
            for p in ss.get("ports") or []:
                if p.get("name", "") == sport.get("name", "") or len(ss.get("ports") or []) == 1:
                    for addr in ss.get("addresses") or []:
                        return addr["ip"], int(p["port"])
        raise m.StatusError(503, "ServiceUnavailable", f'no endpoints available for service "{ns}/{name}"')

    def _ssl(self, spec: dict):
        ctx = ssl.create_default_context()
        pc = getattr(self.server, "proxy_client_cert", None)
        if pc:     # the front-proxy client certificate the extension server's requestheader CA trusts
            ctx.load_cert_chain(pc[0], pc[1])
        if spec.get("insecureSkipTLSVerify"):
            ctx.check_hostname, ctx.verify_mode = False, ssl.CERT_NONE
        elif spec.get("caBundle"):
            import base64
            ctx.load_verify_locations(cadata=base64.b64decode(spec["caBundle"]).decode())
            ctx.check_hostname = False       # the service DNS name, not the endpoint IP, is in the cert
        return ctx

    async def proxy(self, request: web.Request, apiservice: dict, user: dict) -> web.StreamResponse:
        cond = {c.get("type"): c for c in ((apiservice.get("status") or {}).get("conditions") or [])}
        spec = apiservice.get("spec") or {}
        if cond.get("Available", {}).get("status") == "False":
            raise m.StatusError(503, "ServiceUnavailable", f"service unavailable: {cond['Available'].get('message', '')}")
        host, port = self._endpoint(spec.get("service") or {})
        if self._http is None:
            self._http = ClientSession(timeout=ClientTimeout(total=None, sock_connect=5))
        headers = {k: v for k, v in request.headers.items() if k.lower() not in HOP_HEADERS
                   and not k.lower().startswith("x-remote-")}
        headers["X-Remote-User"] = user.get("name", "")
        hdrs = list(headers.items()) + [("X-Remote-Group", g) for g in user.get("groups") or []]
        for k, vals in (user.get("extra") or {}).items():
            hdrs += [(f"X-Remote-Extra-{k}", v) for v in vals]
        url = f"https://{host}:{port}{request.rel_url}"
        body = await request.read()
        async with self._http.request(request.method, url, headers=hdrs, data=body or None, ssl=self._ssl(spec),
                                      allow_redirects=False) as up:
            out = web.StreamResponse(status=up.status, headers={k: v for k, v in up.headers.items()
                                                                if k.lower() not in HOP_HEADERS})
            await out.prepare(request)
            async for chunk in up.content.iter_any():
                await out.write(chunk)
            await out.write_eof()
            return out

    # ---------------------------------------------------------------- controllers
    def autoregister(self):
        """autoregister: a local APIService for every built-in group/version."""
        rs = self.registry.rs("apiservices", GROUP)
        for ri in SCHEME.by_kind.values():
            name = apiservice_name(ri.group, ri.version)
            if rs.storage.get(rs.key("", name), ignore_not_found=True) is not None:
                continue
            gp, vp = PRIORITIES.get((ri.group, ri.version), (16500, 9))
            try:
                rs.create("", {"apiVersion": f"{GROUP}/v1beta1", "kind": "APIService",
                               "metadata": {"name": name, "labels": {"kube-aggregator.kubernetes.io/automanaged": "onstart"}},
                               "spec": {"group": ri.group, "version": ri.version, "groupPriorityMinimum": gp,
                                        "versionPriority": vp}})
            except m.StatusError as e:
                if not m.is_already_exists(e):
                    raise

    async def _check(self, a: dict) -> tuple[str, str, str]:
        spec = a.get("spec") or {}
        svc = spec.get("service")
        if not svc:
            return "True", "Local", "Local APIServices are always available"
        ns, name = svc.get("namespace", ""), svc.get("name", "")
        s = self.registry.get_object("services", ns, name)
        if s is None:
            return "False", "ServiceNotFound", f"service/{name} in \"{ns}\" is not present"
        try:
            host, port = self._endpoint(svc)
        except m.StatusError as e:
            reason = "MissingEndpoints" if "endpoints" in e.message else "ServicePortError"
            return "False", reason, e.message
        if self._http is None:
            self._http = ClientSession(timeout=ClientTimeout(total=None, sock_connect=5))
        try:
            url = f"https://{host}:{port}/apis/{spec.get('group')}/{spec.get('version')}"
            async with self._http.get(url, ssl=self._ssl(spec), timeout=ClientTimeout(total=5)) as r:
                if r.status >= 300 and r.status not in (401, 403):
                    return "False", "FailedDiscoveryCheck", f"no response from {url}: {r.status}"
        except Exception as e:
            return "False", "FailedDiscoveryCheck", f"no response from {url}: {e!r}"
        return "True", "Passed", "all checks passed"

    async def run_availability(self, period: float = 10.0):
        rs = self.registry.rs("apiservices", GROUP)
        while True:
            self._dirty.clear()
            for a in list(self.index.values()):
                try:
                    st, reason, msg = await self._check(a)
                    cur = rs.storage.get(rs.key("", m.name_of(a)), ignore_not_found=True)
                    if cur is None:
                        continue
                    conds = (cur.get("status") or {}).get("conditions") or []
                    old = next((c for c in conds if c.get("type") == "Available"), None)
                    if old and (old.get("status"), old.get("reason"), old.get("message")) == (st, reason, msg):
                        continue
                    new = {"type": "Available", "status": st, "reason": reason, "message": msg,
                           "lastTransitionTime": old["lastTransitionTime"] if old and old.get("status") == st else m.now_rfc3339()}
                    cur["status"] = {"conditions": [c for c in conds if c.get("type") != "Available"] + [new]}
                    rs.update("", m.name_of(cur), cur, subresource="status")
                except Exception as e:    # noqa: BLE001 — one bad APIService must not stop the loop
                    log.debug("availability check of %s failed: %r", m.name_of(a), e)
            await wait_event(self._dirty, period)

    async def close(self):
        if self._http is not None:
            await self._http.close()
