"""HTTP scheduler extender (reference plugin/pkg/scheduler/core/extender.go:40-252 and
algorithm/scheduler_interface.go:28-44): POST {urlPrefix}/{filterVerb|prioritizeVerb|bindVerb}
with ExtenderArgs {pod, nodes: {items}} → ExtenderFilterResult {nodes, failedNodes, error} /
HostPriorityList [{host, score}] / ExtenderBindingResult {error}."""
from __future__ import annotations

import aiohttp


class HTTPExtender:
    def __init__(self, cfg: dict):
        self.url = cfg["urlPrefix"].rstrip("/")
        self.filter_verb = cfg.get("filterVerb", "")
        self.prioritize_verb = cfg.get("prioritizeVerb", "")
        self.bind_verb = cfg.get("bindVerb", "")
        self.weight = int(cfg.get("weight", 1))
        self.timeout = float(cfg.get("httpTimeout", 5.0))
        self.ignorable = bool(cfg.get("ignorable", False))
        self._s: aiohttp.ClientSession | None = None

    def _session(self):
        if self._s is None or self._s.closed:
            self._s = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout))
        return self._s

    async def _post(self, verb, body):
        async with self._session().post(f"{self.url}/{verb}", json=body) as r:
            r.raise_for_status()
            return await r.json()

    async def filter(self, pod, nodes):
        try:
            res = await self._post(self.filter_verb, {"pod": pod, "nodes": {"items": nodes}})
        except Exception as e:
            if self.ignorable:
                return [n["metadata"]["name"] for n in nodes], {}
            raise RuntimeError(f"extender filter failed: {e}")
        if res.get("error"):
            raise RuntimeError(res["error"])
        names = [n["metadata"]["name"] for n in ((res.get("nodes") or {}).get("items") or [])]
        if res.get("nodeNames") is not None:
            names = res["nodeNames"]
        return names, dict(res.get("failedNodes") or {})

    async def prioritize(self, pod, nodes):
        try:
            res = await self._post(self.prioritize_verb, {"pod": pod, "nodes": {"items": nodes}})
        except Exception:
            return {}
        return {e["host"]: int(e["score"]) for e in res or []}

    async def bind(self, pod, node, ext_binding: dict | None = None):
        """ExtenderBindingArgs; `extendedResourceBinding` (the chosen device IDs) is an amdkube
        addition — without it an extender that binds would drop the pod's GPU assignment."""
        md = pod["metadata"]
        body = {"podName": md["name"], "podNamespace": md.get("namespace", ""), "podUID": md.get("uid", ""), "node": node}
        if ext_binding:
            body["extendedResourceBinding"] = ext_binding
        res = await self._post(self.bind_verb, body)
        if res and res.get("error"):
            raise RuntimeError(res["error"])

    async def close(self):
        if self._s is not None:
            await self._s.close()
