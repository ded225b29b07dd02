"""Cluster-lifecycle controllers: node lifecycle, namespace, garbage collector, pod GC.

Reference: pkg/controller/node/node_controller.go:619 (monitorNodeStatus: heartbeat older
than the grace period → Ready=Unknown, taint unreachable:NoExecute, evict pods after the
eviction timeout unless they tolerate it for longer), pkg/controller/namespace
(delete every namespaced object, then finalize), pkg/controller/garbagecollector
(ownerReferences: delete dependents of vanished owners; honour orphan / foregroundDeletion
finalizers), pkg/controller/podgc (terminated-pod threshold, orphaned pods on deleted nodes).
"""
from __future__ import annotations

import asyncio
import time

from ..api import meta as m
from ..api.helpers import get_condition, is_pod_terminal, tolerations_tolerate_taint
from ..api.scheme import SCHEME
from .base import Controller, split_key

UNREACHABLE_TAINT = {"key": "node.kubernetes.io/unreachable", "effect": "NoExecute"}


class NodeLifecycleController(Controller):
    name = "node-lifecycle"

    def __init__(self, mgr, grace: float = 40.0, eviction_timeout: float = 300.0, period: float = 5.0):
        super().__init__(mgr)
        self.grace, self.eviction_timeout, self.period = grace, eviction_timeout, period
        self.unknown_since: dict[str, float] = {}

    def setup(self):
        self.nodes = self.mgr.nodes
        self.pods = self.mgr.pods

    async def start(self):
        self.tasks.append(asyncio.create_task(self._monitor(), name="node-monitor"))

    async def _monitor(self):
        while True:
            await asyncio.sleep(self.period)
            try:
                await self.monitor_once()
            except Exception:
                pass

    async def monitor_once(self, now: float | None = None):
        now = now or time.time()
        for node in self.nodes.list():
            name = m.name_of(node)
            ready = get_condition(node, "Ready")
            hb = m.parse_time((ready or {}).get("lastHeartbeatTime")) if ready else None
            stale = hb is None or now - hb > self.grace
            if stale and (ready or {}).get("status") != "Unknown":
                conds = [dict(c, status="Unknown", reason="NodeStatusUnknown", message="Kubelet stopped posting node status.",
                              lastTransitionTime=m.now_rfc3339()) for c in (node.get("status") or {}).get("conditions") or []]
                if not conds:
                    conds = [{"type": "Ready", "status": "Unknown", "reason": "NodeStatusUnknown", "lastTransitionTime": m.now_rfc3339()}]
                await self.client.patch("nodes", name, {"status": {"conditions": conds}}, sub="status")
                taints = list((node.get("spec") or {}).get("taints") or [])
                if not any(t.get("key") == UNREACHABLE_TAINT["key"] for t in taints):
                    taints.append(dict(UNREACHABLE_TAINT, timeAdded=m.now_rfc3339()))
                    await self.client.patch("nodes", name, {"spec": {"taints": taints}})
                self.unknown_since[name] = now
            elif not stale and ready and ready.get("status") == "True":
                self.unknown_since.pop(name, None)
                taints = (node.get("spec") or {}).get("taints") or []
                if any(t.get("key") == UNREACHABLE_TAINT["key"] for t in taints):
                    await self.client.patch("nodes", name, {"spec": {"taints": [t for t in taints if t.get("key") != UNREACHABLE_TAINT["key"]]}})
            since = self.unknown_since.get(name)
            if since is not None:
                for p in self.pods.list():
                    if (p.get("spec") or {}).get("nodeName") != name or is_pod_terminal(p) or (p.get("metadata") or {}).get("deletionTimestamp"):
                        continue
                    tols = (p.get("spec") or {}).get("tolerations") or []
                    limit = self.eviction_timeout
                    for t in tols:
                        if tolerations_tolerate_taint([t], UNREACHABLE_TAINT):
                            limit = float("inf") if t.get("tolerationSeconds") is None else float(t["tolerationSeconds"])
                    if now - since >= limit:
                        try:
                            await self.client.delete("pods", m.name_of(p), m.namespace_of(p))
                        except m.StatusError:
                            pass

    async def sync(self, key):
        pass


class NamespaceController(Controller):
    name = "namespace"

    def setup(self):
        self.ns_inf = self.mgr.factory.informer("namespaces")
        self.ns_inf.add_handler(on_add=self._ns, on_update=lambda o, n: self._ns(n))

    def _ns(self, ns):
        if (ns.get("status") or {}).get("phase") == "Terminating":
            self.enqueue(m.name_of(ns))

    async def sync(self, key):
        ns = self.ns_inf.get(key)
        if ns is None:
            return
        remaining = 0
        if (ns.get("metadata") or {}).get("deletionTimestamp"):
            try:
                await self.client.discover()   # custom resources are namespace content too
            except Exception:
                pass
        for ri in list(SCHEME.by_kind.values()):
            if not ri.namespaced or ri.plural in ("bindings", "localsubjectaccessreviews") or "list" not in ri.verbs:
                continue
            try:
                items, _ = await self.client.list(ri.plural if not ri.group else f"{ri.plural}.{ri.group}", key)
            except m.StatusError:
                continue
            for it in items:
                remaining += 1
                if not (it.get("metadata") or {}).get("deletionTimestamp"):
                    try:
                        await self.client.delete(ri.plural if not ri.group else f"{ri.plural}.{ri.group}", m.name_of(it), key)
                    except m.StatusError:
                        pass
                elif ri.plural == "pods" and not (it.get("spec") or {}).get("nodeName"):
                    await self.client.delete("pods", m.name_of(it), key, grace=0)
        if remaining:
            self.queue.add_after(key, 0.5)
            return
        ns = await self.client.get_or_none("namespaces", key)
        if ns and (ns.get("spec") or {}).get("finalizers"):
            ns["spec"]["finalizers"] = []
            await self.client.request("PUT", f"/api/v1/namespaces/{key}/finalize", body=ns)


class GarbageCollector(Controller):
    name = "garbagecollector"
    OWNED = ("pods", "replicasets", "jobs", "daemonsets", "deployments", "replicationcontrollers", "statefulsets",
             "controllerrevisions", "cronjobs", "services", "endpoints", "configmaps", "secrets", "persistentvolumeclaims",
             "horizontalpodautoscalers", "poddisruptionbudgets", "serviceaccounts")

    def __init__(self, mgr, period: float = 2.0):
        super().__init__(mgr)
        self.period = period

    def setup(self):
        self.infs = {r: (self.mgr.pods if r == "pods" else self.mgr.factory.informer(r)) for r in self.OWNED}
        for r, inf in self.infs.items():
            inf.add_handler(on_delete=lambda o: self.queue.add("scan"),
                            on_update=lambda o, n: self.queue.add("scan") if (n.get("metadata") or {}).get("deletionTimestamp") else None)

    async def start(self):
        await super().start()
        self.tasks.append(asyncio.create_task(self._tick()))

    async def _tick(self):
        while True:
            await asyncio.sleep(self.period)
            self.queue.add("scan")

    async def sync(self, key):
        alive = {}
        for r, inf in self.infs.items():
            for o in inf.list():
                alive[m.uid_of(o)] = (r, o)
        for r, inf in self.infs.items():
            for o in inf.list():
                md = o.get("metadata") or {}
                fins = md.get("finalizers") or []
                if md.get("deletionTimestamp") and ("orphan" in fins or "foregroundDeletion" in fins):
                    await self._finalize(r, o, alive)
                    continue
                refs = md.get("ownerReferences") or []
                if refs and not any([await self._owner_alive(ref, o, alive) for ref in refs]):
                    try:
                        await self.client.delete(r, m.name_of(o), m.namespace_of(o), propagation="Background")
                    except m.StatusError:
                        pass

    async def _owner_alive(self, ref, dependent, alive) -> bool:
        """An owner of a watched kind is checked in the cache; any other kind with a GET
        (garbagecollector.go attemptToDeleteItem → isDangling), unknown kinds count as alive."""
        if ref.get("uid") in alive:
            return True
        from ..api.scheme import SCHEME
        ri = SCHEME.for_kind(ref.get("apiVersion", ""), ref.get("kind", ""))
        if ri is None:
            return True
        if ri.plural in self.infs:
            return False
        try:
            o = await self.client.get(ri.plural, ref.get("name", ""), m.namespace_of(dependent) if ri.namespaced else "")
        except m.StatusError as e:
            return not m.is_not_found(e)
        return m.uid_of(o) == ref.get("uid")

    async def _finalize(self, r, owner, alive):
        uid = m.uid_of(owner)
        md = owner["metadata"]
        deps = [(dr, d) for dr, d in alive.values() if any(ref.get("uid") == uid for ref in (d.get("metadata") or {}).get("ownerReferences") or [])]
        if "orphan" in md["finalizers"]:
            for dr, d in deps:
                refs = [x for x in d["metadata"]["ownerReferences"] if x.get("uid") != uid]
                await self.client.patch(dr, m.name_of(d), {"metadata": {"ownerReferences": refs or None}}, m.namespace_of(d))
            fins = [f for f in md["finalizers"] if f != "orphan"]
        else:
            if deps:
                for dr, d in deps:
                    if not (d.get("metadata") or {}).get("deletionTimestamp"):
                        await self.client.delete(dr, m.name_of(d), m.namespace_of(d))
                return
            fins = [f for f in md["finalizers"] if f != "foregroundDeletion"]
        await self.client.patch(r, m.name_of(owner), {"metadata": {"finalizers": fins or None}}, m.namespace_of(owner))


class PodGCController(Controller):
    name = "podgc"

    def __init__(self, mgr, threshold: int = 12500, period: float = 20.0):
        super().__init__(mgr)
        self.threshold, self.period = threshold, period

    def setup(self):
        self.pods = self.mgr.pods
        self.nodes = self.mgr.nodes

    async def start(self):
        self.tasks.append(asyncio.create_task(self._loop()))

    async def _loop(self):
        while True:
            await asyncio.sleep(self.period)
            try:
                await self.gc_once()
            except Exception:
                pass

    async def gc_once(self):
        pods = self.pods.list()
        term = sorted([p for p in pods if is_pod_terminal(p)], key=lambda p: (p.get("metadata") or {}).get("creationTimestamp", ""))
        for p in term[:max(0, len(term) - self.threshold)]:
            await self.client.delete("pods", m.name_of(p), m.namespace_of(p), grace=0)
        nodes = {m.name_of(n) for n in self.nodes.list()}
        if not self.nodes.has_synced():
            return
        for p in pods:
            nn = (p.get("spec") or {}).get("nodeName")
            if nn and nn not in nodes:
                try:
                    await self.client.delete("pods", m.name_of(p), m.namespace_of(p), grace=0)
                except m.StatusError:
                    pass

    async def sync(self, key):
        pass
