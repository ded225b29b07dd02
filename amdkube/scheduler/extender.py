"""HTTP scheduler extender.

Reference: plugin/pkg/scheduler/core/extender.go:40-252 (NewHTTPExtender, makeTransport,
Filter / Prioritize / Bind / send) and api/v1/types.go:121-190 (ExtenderConfig,
ExtenderArgs, ExtenderFilterResult, ExtenderBindingArgs/Result, HostPriority).

  * POST {urlPrefix}/{verb} with ExtenderArgs {pod, nodes: {items}} — or, for a
    `nodeCacheCapable` extender, {pod, nodenames: [...]}: it caches the nodes itself, and
    answers with ExtenderFilterResult.nodenames, which are resolved against the scheduler's
    own node cache;
  * `enableHttps` + `tlsConfig` (restclient.TLSClientConfig: Insecure, ServerName, CertFile /
    KeyFile / CAFile and their inline *Data forms): https with the CA, a client certificate,
    or no verification; enableHttps without a CA means an insecure transport, as makeTransport
    does;
  * `httpTimeout` is a Go time.Duration, integer nanoseconds in the policy JSON (default 5 s);
  * a non-200 answer is an error ("Failed <verb> with extender at URL <url>, code <n>");
    filter errors fail the pod's scheduling, prioritize errors are ignored (PrioritizeNodes);
  * ExtenderBindingArgs go out with Go's field names (PodName, PodNamespace, PodUID, Node).

Policy keys are matched case-insensitively, as Go's encoding/json does (BindVerb carries no
json tag in the reference, so both `bindVerb` and `BindVerb` appear in policies).

amdkube additions: `extendedResourceBinding` (the chosen device IDs) rides along with the bind
call, since an extender that binds would otherwise drop the pod's GPU assignment; `ignorable`
lets a filter outage pass the nodes through.
"""
from __future__ import annotations

import base64
import os
import ssl
import tempfile

import aiohttp

DEFAULT_EXTENDER_TIMEOUT = 5.0


def _ci(d: dict | None, key: str, default=None):
    """A key of a Go-decoded struct: exact match first, then case-insensitive."""
    if not d:
        return default
    if key in d:
        return d[key]
    low = key.lower()
    for k, v in d.items():
        if k.lower() == low:
            return v
    return default


def duration_seconds(v) -> float:
    """time.Duration from JSON: integer nanoseconds (Go's encoding); 0 or absent → the 5 s
    default. Values below a millisecond-in-nanoseconds are taken as seconds, as older amdkube
    policies wrote them."""
    if v in (None, 0, ""):
        return DEFAULT_EXTENDER_TIMEOUT
    if isinstance(v, str):
        from ..api.protobuf import parse_duration
        return parse_duration(v) / 1e9 or DEFAULT_EXTENDER_TIMEOUT
    v = float(v)
    return v / 1e9 if v >= 1e6 else v


def _pem(data) -> bytes:
    """[]byte fields arrive base64-encoded; a PEM string is accepted as is."""
    if isinstance(data, bytes):
        return data
    s = str(data)
    if "-----BEGIN" in s:
        return s.encode()
    return base64.b64decode(s)


def tls_context(enable_https: bool, tls: dict | None) -> ssl.SSLContext | None:
    """makeTransport + restclient.TLSConfigFor."""
    tls = tls or {}
    ca_file, ca_data = _ci(tls, "CAFile"), _ci(tls, "CAData")
    cert_file, key_file = _ci(tls, "CertFile"), _ci(tls, "KeyFile")
    cert_data, key_data = _ci(tls, "CertData"), _ci(tls, "KeyData")
    insecure = bool(_ci(tls, "Insecure", False))
    has_ca = bool(ca_file or ca_data)
    if enable_https and not has_ca:
        insecure = True
    has_cert = bool(cert_file or cert_data)
    if not (has_ca or has_cert or insecure or _ci(tls, "ServerName")):
        return None
    if insecure and has_ca:
        raise ValueError("specifying a root certificates file with the insecure flag is not allowed")
    ctx = ssl.create_default_context(purpose=ssl.Purpose.SERVER_AUTH)
    if insecure:
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    elif ca_file or ca_data:
        ctx.load_verify_locations(cafile=ca_file or None, cadata=_pem(ca_data).decode() if ca_data and not ca_file else None)
    if has_cert:
        if cert_file:
            ctx.load_cert_chain(cert_file, key_file)
        else:
            # the ssl module loads chains from files only: stage the inline PEMs privately
            with tempfile.TemporaryDirectory() as d:
                cf, kf = os.path.join(d, "cert.pem"), os.path.join(d, "key.pem")
                with open(os.open(cf, os.O_WRONLY | os.O_CREAT, 0o600), "wb") as f:
                    f.write(_pem(cert_data))
                with open(os.open(kf, os.O_WRONLY | os.O_CREAT, 0o600), "wb") as f:
                    f.write(_pem(key_data))
                ctx.load_cert_chain(cf, kf)
    return ctx


class ExtenderError(RuntimeError):
    pass


class HTTPExtender:
    def __init__(self, cfg: dict):
        self.url = str(_ci(cfg, "urlPrefix", "")).rstrip("/")
        self.filter_verb = _ci(cfg, "filterVerb", "") or ""
        self.prioritize_verb = _ci(cfg, "prioritizeVerb", "") or ""
        self.bind_verb = _ci(cfg, "bindVerb", "") or ""
        self.weight = int(_ci(cfg, "weight", 1) or 0)
        self.timeout = duration_seconds(_ci(cfg, "httpTimeout"))
        self.node_cache_capable = bool(_ci(cfg, "nodeCacheCapable", False))
        self.enable_https = bool(_ci(cfg, "enableHttps", False))
        tls = _ci(cfg, "tlsConfig")
        self.ssl = tls_context(self.enable_https, tls)
        self.server_name = _ci(tls, "ServerName") or None
        self.ignorable = bool(_ci(cfg, "ignorable", False))
        self.calls: dict[str, int] = {}
        self._s: aiohttp.ClientSession | None = None

    def _session(self):
        if self._s is None or self._s.closed:
            conn = aiohttp.TCPConnector(ssl=self.ssl if self.ssl is not None else None)
            self._s = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout), connector=conn)
        return self._s

    async def _post(self, verb, body):
        """send: a non-200 answer is an error."""
        self.calls[verb] = self.calls.get(verb, 0) + 1
        kw = {"server_hostname": self.server_name} if self.server_name else {}
        async with self._session().post(f"{self.url}/{verb}", json=body, **kw) as r:
            if r.status != 200:
                raise ExtenderError(f"Failed {verb} with extender at URL {self.url}, code {r.status}")
            return await r.json(content_type=None)

    def _args(self, pod, nodes) -> dict:
        if self.node_cache_capable:
            return {"pod": pod, "nodenames": [n["metadata"]["name"] for n in nodes]}
        return {"pod": pod, "nodes": {"items": nodes}}

    async def filter(self, pod, nodes):
        """(names of the nodes that pass, failedNodes). With nodeCacheCapable the answer's
        `nodenames` name nodes of the scheduler's cache."""
        if not self.filter_verb:
            return [n["metadata"]["name"] for n in nodes], {}
        try:
            res = await self._post(self.filter_verb, self._args(pod, nodes)) or {}
        except Exception as e:
            if self.ignorable:
                return [n["metadata"]["name"] for n in nodes], {}
            raise ExtenderError(f"extender filter failed: {e}") from None
        if res.get("error"):
            raise ExtenderError(res["error"])
        names = _ci(res, "nodenames")
        if self.node_cache_capable and names is not None:
            known = {n["metadata"]["name"] for n in nodes}
            names = [x for x in names if x in known]
        elif res.get("nodes") is not None:
            names = [n["metadata"]["name"] for n in ((res.get("nodes") or {}).get("items") or [])]
        else:
            names = list(names or [])
        return names, dict(res.get("failedNodes") or {})

    async def prioritize(self, pod, nodes):
        """host -> score; errors are ignored by PrioritizeNodes (empty result)."""
        if not self.prioritize_verb:
            return {n["metadata"]["name"]: 0 for n in nodes}
        try:
            res = await self._post(self.prioritize_verb, self._args(pod, nodes))
        except Exception:
            return {}
        return {e["host"]: int(e["score"]) for e in res or []}

    async def bind(self, pod, node, ext_binding: dict | None = None):
        md = pod["metadata"]
        body = {"PodName": md["name"], "PodNamespace": md.get("namespace", ""), "PodUID": md.get("uid", ""), "Node": node}
        if ext_binding:
            body["extendedResourceBinding"] = ext_binding
        res = await self._post(self.bind_verb, body)
        err = _ci(res or {}, "Error")
        if err:
            raise ExtenderError(err)

    def is_binder(self) -> bool:
        return bool(self.bind_verb)

    async def close(self):
        if self._s is not None:
            await self._s.close()
