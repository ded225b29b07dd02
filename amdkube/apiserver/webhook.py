"""Dynamic admission webhooks (admissionregistration.k8s.io/v1beta1).

Reference: staging/src/k8s.io/apiserver/pkg/admission/plugin/webhook — mutating/
dispatcher.go (webhooks called in order; each JSONPatch response is applied before the next
call), validating/admission.go (called in parallel; any denial rejects), config/
(clientConfig: url or service{namespace,name,path} + caBundle), namespace/matcher.go
(namespaceSelector), rules/rules.go (operations × apiGroups × apiVersions × resources with
"*" and "resource/subresource"), failurePolicy Ignore (the v1beta1 default) or Fail, and the
admission.k8s.io/v1beta1 AdmissionReview request/response body.

The registry's admission chain is synchronous; webhooks are HTTP calls, so the apiserver runs
them on the request path around it (mutating before the built-in chain, validating on the
object the chain and defaulting produced).
"""
from __future__ import annotations

import asyncio
import base64
import json
import ssl
import tempfile
import uuid
from urllib.parse import urlparse

from aiohttp import ClientSession, ClientTimeout

from ..api import meta as m
from ..api.labels import selector_from_label_selector

MUTATING, VALIDATING = "mutatingwebhookconfigurations", "validatingwebhookconfigurations"
GROUP = "admissionregistration.k8s.io"
TIMEOUT = 30.0


def rule_matches(rule: dict, op: str, group: str, version: str, resource: str, sub: str) -> bool:
    ops = rule.get("operations") or []
    if "*" not in ops and op not in ops:
        return False
    if "*" not in (rule.get("apiGroups") or []) and group not in (rule.get("apiGroups") or []):
        return False
    if "*" not in (rule.get("apiVersions") or []) and version not in (rule.get("apiVersions") or []):
        return False
    want = f"{resource}/{sub}" if sub else resource
    for r in rule.get("resources") or []:
        if r == "*/*" or r == want or (r == "*" and not sub) or (r.endswith("/*") and r[:-2] == resource and sub) \
                or (r.startswith("*/") and sub and r[2:] == sub):
            return True
    return False


class WebhookDispatcher:
    def __init__(self, registry):
        self.registry = registry
        self._gen = 0
        self._cache: tuple[int, list, list] | None = None
        self._sessions: dict[str, ClientSession] = {}
        registry.store.commit_hooks.append(self._on_commit)

    def _on_commit(self, ev):
        if ev.kv.key.startswith(("/registry/" + MUTATING + "/", "/registry/" + VALIDATING + "/")):
            self._gen += 1

    def _configs(self):
        if self._cache is None or self._cache[0] != self._gen:
            mut = sorted(self.registry.rs(MUTATING, GROUP).list()[0], key=m.name_of)
            val = sorted(self.registry.rs(VALIDATING, GROUP).list()[0], key=m.name_of)
            self._cache = (self._gen, [w for c in mut for w in c.get("webhooks") or []],
                           [w for c in val for w in c.get("webhooks") or []])
        return self._cache[1], self._cache[2]

    def _matching(self, hooks, op, ri, sub, ns):
        out = []
        for w in hooks:
            if not any(rule_matches(r, op, ri.group, ri.version, ri.plural, sub) for r in w.get("rules") or []):
                continue
            sel = w.get("namespaceSelector")
            if sel and ri.namespaced and ns:
                try:
                    labels = m.labels_of(self.registry.rs("namespaces").get("", ns))
                except m.StatusError:
                    labels = {}
                if not selector_from_label_selector(sel).matches(labels):
                    continue
            out.append(w)
        return out

    def active(self, op, ri, sub, ns) -> tuple[list, list]:
        if ri.group == GROUP:
            return [], []   # never call webhooks about webhook configurations (reference: same rule)
        mut, val = self._configs()
        if not mut and not val:
            return [], []
        return self._matching(mut, op, ri, sub, ns), self._matching(val, op, ri, sub, ns)

    # -------------------------------------------------------------- calling
    def _endpoint(self, cc: dict) -> str:
        if cc.get("url"):
            return cc["url"]
        svc = cc.get("service") or {}
        ep = self.registry.rs("endpoints").get(svc.get("namespace", "default"), svc["name"])
        for sub in ep.get("subsets") or []:
            if sub.get("addresses") and sub.get("ports"):
                port = sub["ports"][0]["port"]
                return f"https://{sub['addresses'][0]['ip']}:{port}{svc.get('path') or '/'}"
        raise RuntimeError(f"no endpoints for webhook service {svc.get('namespace')}/{svc.get('name')}")

    def _ssl(self, cc: dict, url: str):
        if not url.startswith("https://"):
            host = urlparse(url).hostname
            if host not in ("127.0.0.1", "localhost", "::1"):
                raise RuntimeError("webhook URLs must use https (plain http is accepted on loopback only)")
            return None
        ca = cc.get("caBundle")
        ctx = ssl.create_default_context()
        if ca:
            pem = base64.b64decode(ca).decode()
            with tempfile.NamedTemporaryFile("w", suffix=".pem") as f:
                f.write(pem)
                f.flush()
                ctx.load_verify_locations(f.name)
        return ctx

    async def _call(self, w: dict, review: dict) -> dict:
        cc = w.get("clientConfig") or {}
        url = self._endpoint(cc)
        ctx = self._ssl(cc, url)
        s = self._sessions.get(w["name"])
        if s is None or s.closed:
            s = self._sessions[w["name"]] = ClientSession(timeout=ClientTimeout(total=TIMEOUT))
        async with s.post(url, json=review, ssl=ctx if ctx is not None else False) as r:
            if r.status != 200:
                raise RuntimeError(f"webhook returned HTTP {r.status}")
            out = await r.json(content_type=None)
        resp = out.get("response") or {}
        if resp.get("uid") not in (None, review["request"]["uid"]):
            raise RuntimeError("webhook response uid does not match the request")
        return resp

    def _review(self, op, ri, sub, ns, name, obj, old, user) -> dict:
        return {"apiVersion": "admission.k8s.io/v1beta1", "kind": "AdmissionReview",
                "request": {"uid": str(uuid.uuid4()),
                            "kind": {"group": ri.group, "version": ri.version, "kind": ri.kind},
                            "resource": {"group": ri.group, "version": ri.version, "resource": ri.plural},
                            "subResource": sub, "name": name or m.name_of(obj or old or {}), "namespace": ns,
                            "operation": op,
                            "userInfo": {"username": (user or {}).get("name", ""), "uid": (user or {}).get("uid", ""),
                                         "groups": (user or {}).get("groups") or []},
                            "object": obj, "oldObject": old}}

    def _fail(self, w, err):
        if (w.get("failurePolicy") or "Ignore") == "Fail":
            raise m.StatusError(500, "InternalError", f'failed calling admission webhook "{w["name"]}": {err}')

    async def mutate(self, hooks, op, ri, sub, ns, name, obj, old, user) -> dict:
        from .registry import apply_patch
        for w in hooks:
            try:
                resp = await self._call(w, self._review(op, ri, sub, ns, name, obj, old, user))
            except (OSError, RuntimeError, asyncio.TimeoutError, ValueError) as e:
                self._fail(w, e)
                continue
            if not resp.get("allowed"):
                _deny(w, resp)
            if resp.get("patch"):
                if resp.get("patchType", "JSONPatch") != "JSONPatch":
                    self._fail(w, "unsupported patchType")
                    continue
                obj = apply_patch(obj, base64.b64decode(resp["patch"]), "application/json-patch+json")
        return obj

    async def validate(self, hooks, op, ri, sub, ns, name, obj, old, user):
        async def one(w):
            try:
                resp = await self._call(w, self._review(op, ri, sub, ns, name, obj, old, user))
            except (OSError, RuntimeError, asyncio.TimeoutError, ValueError) as e:
                self._fail(w, e)
                return
            if not resp.get("allowed"):
                _deny(w, resp)
        await asyncio.gather(*(one(w) for w in hooks))

    async def close(self):
        for s in self._sessions.values():
            await s.close()


def _deny(w, resp):
    st = resp.get("status") or {}
    msg = st.get("message") or st.get("reason") or "denied"
    raise m.StatusError(int(st.get("code") or 403), st.get("reason") or "Forbidden",
                        f'admission webhook "{w["name"]}" denied the request: {msg}')


__all__ = ["WebhookDispatcher", "rule_matches", "json"]
