"""Kubelet API authentication and authorization (pkg/kubelet/server/auth.go and
cmd/kubelet/app/auth.go; staging/.../apiserver/pkg/authentication/request/x509,
.../authentication/token/webhook via TokenReview, .../authorization/authorizerfactory webhook
via SubjectAccessReview).

Authenticators, in order: x509 client certificates signed by --client-ca-file (user = CN,
groups = O), bearer tokens checked with the apiserver's TokenReview (--authentication-token-
webhook, cached --authentication-token-webhook-cache-ttl, 2 m), then anonymous
(system:anonymous / system:unauthenticated) unless --anonymous-auth=false (→ 401).
Authorization (--authorization-mode): AlwaysAllow, or Webhook — a SubjectAccessReview for
{verb from the HTTP method, resource nodes, name = this node, subresource by path: stats,
metrics, log, spec, proxy}, cached 5 m when allowed and 30 s when denied (→ 403).
"""
from __future__ import annotations

import time

from aiohttp import web

VERBS = {"GET": "get", "HEAD": "get", "POST": "create", "PUT": "update", "PATCH": "patch", "DELETE": "delete"}


def subresource_for(path: str) -> str:
    """server.go GetRequestAttributes: the nodes subresource a kubelet path maps to."""
    if path.startswith("/stats"):
        return "stats"
    if path.startswith("/metrics"):
        return "metrics"
    if path.startswith("/logs") or path.startswith("/containerLogs"):
        return "log"
    if path.startswith("/spec"):
        return "spec"
    return "proxy"


def user_from_cert(pc: dict | None) -> dict | None:
    if not pc:
        return None
    cn, orgs = "", []
    for rdn in pc.get("subject") or ():
        for k, v in rdn:
            if k == "commonName":
                cn = v
            elif k == "organizationName":
                orgs.append(v)
    return {"name": cn, "groups": orgs} if cn else None


class KubeletAuth:
    def __init__(self, node_name: str, client=None, anonymous: bool = True, token_webhook: bool = False,
                 authz_mode: str = "AlwaysAllow", authn_ttl: float = 120.0, authz_allowed_ttl: float = 300.0,
                 authz_denied_ttl: float = 30.0):
        if authz_mode not in ("AlwaysAllow", "Webhook"):
            raise ValueError(f"unknown kubelet authorization mode {authz_mode!r}")
        if (token_webhook or authz_mode == "Webhook") and client is None:
            raise ValueError("webhook authentication/authorization needs an API client")
        self.node, self.client, self.anonymous, self.token_webhook = node_name, client, anonymous, token_webhook
        self.authz_mode, self.ttls = authz_mode, (authn_ttl, authz_allowed_ttl, authz_denied_ttl)
        self._tokens: dict[str, tuple[float, dict | None]] = {}
        self._sars: dict[tuple, tuple[float, bool]] = {}

    async def _token_user(self, token: str) -> dict | None:
        hit = self._tokens.get(token)
        if hit is not None and hit[0] > time.monotonic():
            return hit[1]
        tr = await self.client.create({"apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview", "spec": {"token": token}})
        st = tr.get("status") or {}
        user = None
        if st.get("authenticated"):
            u = st.get("user") or {}
            user = {"name": u.get("username", ""), "groups": u.get("groups") or [], "uid": u.get("uid", "")}
        self._tokens[token] = (time.monotonic() + self.ttls[0], user)
        return user

    async def authenticate(self, request: web.Request) -> dict:
        user = user_from_cert(request.transport.get_extra_info("peercert") if request.transport else None)
        if user is not None:
            return user
        auth = request.headers.get("Authorization", "")
        if auth.startswith("Bearer ") and self.token_webhook:
            user = await self._token_user(auth[7:].strip())
            if user is not None:
                return user
            raise web.HTTPUnauthorized(text="Unauthorized")
        if self.anonymous:
            return {"name": "system:anonymous", "groups": ["system:unauthenticated"]}
        raise web.HTTPUnauthorized(text="Unauthorized")

    async def authorize(self, user: dict, request: web.Request):
        if self.authz_mode == "AlwaysAllow":
            return
        verb = VERBS.get(request.method, request.method.lower())
        sub = subresource_for(request.path)
        key = (user.get("name"), tuple(user.get("groups") or ()), verb, sub)
        hit = self._sars.get(key)
        if hit is not None and hit[0] > time.monotonic():
            ok = hit[1]
        else:
            sar = await self.client.create({"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview", "spec": {
                "user": user.get("name", ""), "groups": user.get("groups") or [],
                "resourceAttributes": {"verb": verb, "resource": "nodes", "subresource": sub, "name": self.node}}})
            ok = bool((sar.get("status") or {}).get("allowed"))
            self._sars[key] = (time.monotonic() + (self.ttls[1] if ok else self.ttls[2]), ok)
        if not ok:
            raise web.HTTPForbidden(text=f"Forbidden (user={user.get('name')}, verb={verb}, resource=nodes, subresource={sub})")

    def middleware(self):
        @web.middleware
        async def mw(request, handler):
            user = await self.authenticate(request)
            await self.authorize(user, request)
            return await handler(request)
        return mw
