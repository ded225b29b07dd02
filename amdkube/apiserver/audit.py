"""Advanced auditing (AdvancedAuditing beta, on): policy + log backend.

Reference: staging/src/k8s.io/apiserver/pkg/audit — policy/checker.go (first matching rule
decides the level: None | Metadata | Request | RequestResponse; rule fields users, userGroups,
verbs, resources[{group, resources, resourceNames}] (with "resource/subresource"),
namespaces, nonResourceURLs (with trailing "*"), omitStages), request.go (Event fields:
auditID, stage, requestURI, verb, user, sourceIPs, objectRef, responseStatus, request/response
objects at Request/RequestResponse level, requestReceivedTimestamp/stageTimestamp),
plugin/pkg/audit/log (one JSON event per line, --audit-log-path; rotation by
--audit-log-maxsize MB keeping --audit-log-maxbackup files).

Stages recorded: RequestReceived and ResponseComplete (ResponseStarted is the long-running
stage; watches and streams log it when they start), Panic on handler crashes.
"""
from __future__ import annotations

import json
import os
import time
import uuid

from ..api import meta as m

LEVELS = ("None", "Metadata", "Request", "RequestResponse")


def load_policy(path: str | None) -> dict:
    if not path:
        return {"rules": [{"level": "Metadata"}]}
    import yaml
    with open(path) as f:
        doc = yaml.safe_load(f) or {}
    if doc.get("kind") not in (None, "Policy"):
        raise ValueError(f"audit policy {path}: kind must be Policy")
    for r in doc.get("rules") or []:
        if r.get("level") not in LEVELS:
            raise ValueError(f"audit policy {path}: unknown level {r.get('level')!r}")
    return doc


def _match_resource(rule_res: list, group: str, resource: str, sub: str, name: str) -> bool:
    for gr in rule_res:
        if gr.get("group", "") != group and gr.get("group") != "*":
            continue
        names = gr.get("resourceNames") or []
        if names and name not in names:
            continue
        rs = gr.get("resources") or []
        if not rs:
            return True
        full = f"{resource}/{sub}" if sub else resource
        for r in rs:
            if r in (full, "*", "*/*") or (r == f"{resource}/*" and sub) or (r == f"*/{sub}" and sub):
                return True
    return False


def level_for(policy: dict, user: dict, verb: str, group: str, resource: str, sub: str, ns: str, name: str,
              path: str) -> tuple[str, set]:
    groups = set(user.get("groups") or [])
    for r in policy.get("rules") or []:
        if r.get("users") and user.get("name") not in r["users"]:
            continue
        if r.get("userGroups") and not groups & set(r["userGroups"]):
            continue
        if r.get("verbs") and verb not in r["verbs"]:
            continue
        if resource:
            if r.get("nonResourceURLs"):
                continue
            if r.get("resources") and not _match_resource(r["resources"], group, resource, sub, name):
                continue
            if r.get("namespaces") and ns not in r["namespaces"]:
                continue
        else:
            urls = r.get("nonResourceURLs")
            if r.get("resources") or r.get("namespaces"):
                continue
            if urls and not any(path == u or (u.endswith("*") and path.startswith(u[:-1])) for u in urls):
                continue
        return r["level"], set(r.get("omitStages") or []) | set(policy.get("omitStages") or [])
    return "None", set()


def legacy_line(ev: dict) -> str:
    """--audit-log-format=legacy (plugin/pkg/audit/log/backend.go EventString)."""
    u = ev.get("user") or {}
    ref = ev.get("objectRef") or {}
    resp = ev.get("responseStatus") or {}
    return (f'{ev.get("stageTimestamp")} AUDIT: id="{ev.get("auditID")}" stage="{ev.get("stage")}" '
            f'ip="{",".join(ev.get("sourceIPs") or [])}" method="{ev.get("verb")}" user="{u.get("username", "")}" '
            f'groups="{",".join(u.get("groups") or [])}" as="<self>" asgroups="<lookup>" '
            f'namespace="{ref.get("namespace", "<none>")}" uri="{ev.get("requestURI")}"'
            + (f' response="{resp.get("code")}"' if resp else "") + "\n")


class LogBackend:
    def __init__(self, path: str, max_size_mb: int = 0, max_backup: int = 0, fmt: str = "json", max_age_days: int = 0):
        self.path, self.max_bytes, self.max_backup = path, max_size_mb * (1 << 20), max_backup
        self.fmt, self.max_age = fmt, max_age_days * 86400
        self.f = None if path == "-" else open(path, "a", buffering=1)
        self.events = 0

    def write(self, ev: dict):
        line = legacy_line(ev) if self.fmt == "legacy" else json.dumps(ev, separators=(",", ":")) + "\n"
        self.events += 1
        if self.f is None:
            import sys
            sys.stdout.write(line)
            return
        if self.max_bytes and self.f.tell() + len(line) > self.max_bytes:
            self._rotate()
        self.f.write(line)

    def _rotate(self):
        self.f.close()
        stamp = time.strftime("%Y-%m-%dT%H-%M-%S", time.gmtime())
        os.replace(self.path, f"{self.path}-{stamp}.{time.time_ns() % 1000000:06d}")
        base = os.path.basename(self.path) + "-"
        d = os.path.dirname(os.path.abspath(self.path))
        olds = sorted(f for f in os.listdir(d) if f.startswith(base))
        if self.max_backup:
            for f in olds[:-self.max_backup]:
                os.unlink(os.path.join(d, f))
        if self.max_age:            # --audit-log-maxage (days)
            for f in olds:
                fp = os.path.join(d, f)
                try:
                    if time.time() - os.path.getmtime(fp) > self.max_age:
                        os.unlink(fp)
                except OSError:
                    pass
        self.f = open(self.path, "a", buffering=1)

    def close(self):
        if self.f is not None:
            self.f.close()


class WebhookBackend:
    """--audit-webhook-config-file (plugin/pkg/audit/webhook): events POSTed as an
    audit.k8s.io EventList to the service a kubeconfig names. mode "batch" (default) buffers
    up to --audit-webhook-batch-max-size events or --audit-webhook-batch-max-wait seconds per
    request, dropping events beyond --audit-webhook-batch-buffer-size; "blocking" sends each
    event before the request continues (here: as soon as the event loop allows)."""

    def __init__(self, kubeconfig_path: str, mode: str = "batch", buffer_size: int = 10000, max_size: int = 400,
                 max_wait: float = 30.0, throttle_qps: float = 10.0, throttle_burst: int = 15):
        import asyncio
        from ..client import Client
        from ..client.rest import TokenBucket
        self.client = Client.from_kubeconfig(kubeconfig_path, timeout=30.0)
        self.mode, self.max_size, self.max_wait = mode, max_size, max_wait
        self.queue: asyncio.Queue = asyncio.Queue(maxsize=buffer_size)
        self.limiter = TokenBucket(throttle_qps, throttle_burst) if throttle_qps else None
        self.sent = self.dropped = 0
        self._task = None

    def write(self, ev: dict):
        import asyncio
        if self._task is None:
            self._task = asyncio.get_running_loop().create_task(self._run())
        try:
            self.queue.put_nowait(ev)
        except asyncio.QueueFull:
            self.dropped += 1

    async def _send(self, items):
        if self.limiter is not None:
            await self.limiter.wait()
        try:
            await self.client.request("POST", "", body={"kind": "EventList", "apiVersion": "audit.k8s.io/v1beta1",
                                                        "items": items})
            self.sent += len(items)
        except Exception:     # audit is best effort; a webhook outage must not stall the apiserver
            self.dropped += len(items)

    async def _run(self):
        import asyncio
        while True:
            items = [await self.queue.get()]
            if self.mode != "blocking":
                end = asyncio.get_running_loop().time() + self.max_wait
                while len(items) < self.max_size:
                    left = end - asyncio.get_running_loop().time()
                    if left <= 0:
                        break
                    try:
                        items.append(await asyncio.wait_for(self.queue.get(), left))
                    except asyncio.TimeoutError:
                        break
            await self._send(items)

    def close(self):
        if self._task is not None:
            self._task.cancel()


class MultiBackend:
    def __init__(self, backends):
        self.backends = backends

    def write(self, ev: dict):
        for b in self.backends:
            b.write(ev)

    def close(self):
        for b in self.backends:
            b.close()


class Auditor:
    def __init__(self, policy: dict, backend: LogBackend):
        self.policy, self.backend = policy, backend

    def begin(self, request, user, verb, group, version, resource, sub, ns, name):
        lvl, omit = level_for(self.policy, user or {}, verb, group, resource, sub, ns, name, request.path)
        if lvl == "None":
            return None
        ev = {"kind": "Event", "apiVersion": "audit.k8s.io/v1beta1", "level": lvl,
              "timestamp": m.now_rfc3339_micro(), "auditID": str(uuid.uuid4()), "stage": "RequestReceived",
              "requestURI": request.path_qs, "verb": verb,
              "user": {"username": (user or {}).get("name", ""), "groups": (user or {}).get("groups") or []},
              "sourceIPs": [request.remote or ""],
              "requestReceivedTimestamp": m.now_rfc3339_micro(), "stageTimestamp": m.now_rfc3339_micro()}
        if resource:
            ev["objectRef"] = {k: v for k, v in (("resource", resource), ("namespace", ns), ("name", name),
                                                  ("apiGroup", group), ("apiVersion", version),
                                                  ("subresource", sub)) if v}
        if "RequestReceived" not in omit:
            self.backend.write(dict(ev))
        return ev, omit

    def stage(self, ctx, stage: str, code: int, request_body: bytes | None = None, response=None):
        if ctx is None:
            return
        ev, omit = ctx
        if stage in omit:
            return
        out = dict(ev, stage=stage, stageTimestamp=m.now_rfc3339_micro(), responseStatus={"metadata": {}, "code": code})
        if ev["level"] in ("Request", "RequestResponse") and request_body:
            try:
                out["requestObject"] = json.loads(request_body)
            except ValueError:
                pass
        if ev["level"] == "RequestResponse" and response is not None and getattr(response, "body", None):
            try:
                out["responseObject"] = json.loads(response.body)
            except (ValueError, TypeError):
                pass
        self.backend.write(out)
