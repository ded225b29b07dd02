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
import logging
import time

from ..api import meta as m
from ..api.helpers import get_condition, is_pod_terminal, tolerations_tolerate_taint
from ..api.scheme import SCHEME
from .base import Controller

log = logging.getLogger("amdkube.controllers.lifecycle")

UNREACHABLE_TAINT = {"key": "node.kubernetes.io/unreachable", "effect": "NoExecute"}
NOT_READY_TAINT = {"key": "node.kubernetes.io/not-ready", "effect": "NoExecute"}
NODE_TAINT_KEYS = (UNREACHABLE_TAINT["key"], NOT_READY_TAINT["key"])
ZONE_LABELS = ("failure-domain.beta.kubernetes.io/region", "failure-domain.beta.kubernetes.io/zone")
NORMAL, PARTIAL, FULL = "Normal", "PartialDisruption", "FullDisruption"


def zone_of(node: dict) -> str:
    """utilnode.GetZoneKey: region + zone labels ("" without them)."""
    labels = m.labels_of(node)
    r, z = (labels.get(k, "") for k in ZONE_LABELS)
    return f"{r}:\x00:{z}" if r or z else ""


class _Limiter:
    """A non-blocking token bucket whose rate the zone state changes (RateLimitedTimedQueue)."""

    def __init__(self, qps: float):
        self.qps, self.tokens, self.t = qps, 1.0, None

    def set_rate(self, qps: float):
        self.qps = qps

    def take(self, now: float) -> bool:
        if self.t is not None:
            self.tokens = min(1.0, self.tokens + (now - self.t) * self.qps)
        self.t = now
        if self.qps > 0 and self.tokens >= 1.0:
            self.tokens -= 1.0
            return True
        return False


def zone_state(ready: int, not_ready: int, threshold: float) -> str:
    """node_controller.go ComputeZoneState."""
    if ready == 0 and not_ready > 0:
        return FULL
    if not_ready > 2 and not_ready / max(1, ready + not_ready) >= threshold:
        return PARTIAL
    return NORMAL


class NodeLifecycleController(Controller):
    """pkg/controller/node/node_controller.go (1.9): monitorNodeStatus every --node-monitor-period.

    * A node whose kubelet has not posted status for --node-monitor-grace-period (or, for a node
      that never posted, --node-startup-grace-period after creation) goes Ready=Unknown and its
      pods are marked NotReady.
    * Zones (failure-domain region/zone labels) are Normal, PartialDisruption (more than 2 and at
      least --unhealthy-zone-threshold of the nodes not ready) or FullDisruption (none ready).
      Per-zone work is rate limited: --node-eviction-rate in Normal and FullDisruption,
      --secondary-node-eviction-rate in PartialDisruption when the zone has more than
      --large-cluster-size-threshold nodes, otherwise nothing. When every zone is fully disrupted
      (the masters are probably the ones cut off) nothing is evicted and node taints are lifted.
    * TaintBasedEvictions (on here: DefaultTolerationSeconds admission gives every pod a 300 s
      toleration): a not-ready node is tainted node.kubernetes.io/not-ready:NoExecute, an
      unreachable one node.kubernetes.io/unreachable:NoExecute, one node per limiter token, and
      the NoExecute taint manager evicts by the pods' tolerations. With the gate off the legacy
      path deletes a node's pods (DaemonSet pods excepted) once it has been not ready for
      --pod-eviction-timeout, again one node per token.
    """
    name = "node-lifecycle"

    def __init__(self, mgr, grace: float = 40.0, eviction_timeout: float = 300.0, period: float = 5.0,
                 startup_grace: float = 60.0, eviction_rate: float = 0.1, secondary_eviction_rate: float = 0.01,
                 unhealthy_zone_threshold: float = 0.55, large_cluster_threshold: int = 50, enable_taint_manager: bool = True,
                 taint_based_evictions: bool = True):
        super().__init__(mgr)
        self.grace, self.eviction_timeout, self.period = grace, eviction_timeout, period
        self.startup_grace, self.eviction_rate, self.secondary_rate = startup_grace, eviction_rate, secondary_eviction_rate
        self.unhealthy_threshold, self.large_cluster = unhealthy_zone_threshold, large_cluster_threshold
        self.taint_based = taint_based_evictions
        self.unknown_since: dict[str, float] = {}
        self.evicted: set[str] = set()
        self.zone_states: dict[str, str] = {}
        self.limiters: dict[str, _Limiter] = {}
        self.master_disruption = False
        self.taint_manager = NoExecuteTaintManager(mgr) if enable_taint_manager else None

    def setup(self):
        self.nodes = self.mgr.nodes
        self.pods = self.mgr.pods
        if self.taint_manager is not None:
            self.taint_manager.setup()

    async def start(self):
        self.tasks.append(asyncio.create_task(self._monitor(), name="node-monitor"))
        if self.taint_manager is not None:
            await self.taint_manager.start()

    async def stop(self):
        if self.taint_manager is not None:
            await self.taint_manager.stop()
        await super().stop()

    async def _monitor(self):
        while True:
            await asyncio.sleep(self.period)
            try:
                await self.monitor_once()
            except Exception:
                pass

    async def _set_taints(self, node: dict, add: dict | None, remove: tuple = ()) -> bool:
        taints = list((node.get("spec") or {}).get("taints") or [])
        keep = [t for t in taints if t.get("key") not in remove or (add and t.get("key") == add["key"])]
        if add and not any(t.get("key") == add["key"] and t.get("effect") == add["effect"] for t in keep):
            keep.append(dict(add, timeAdded=m.now_rfc3339()))
        if keep != taints:
            await self.client.patch("nodes", m.name_of(node), {"spec": {"taints": keep}})
            return True
        return False

    async def _mark_pods_not_ready(self, name: str):
        """MarkAllPodsNotReady: the pods of an unreachable node stop counting as ready endpoints."""
        for p in self.pods.list():
            if (p.get("spec") or {}).get("nodeName") != name or is_pod_terminal(p):
                continue
            conds = [dict(c) for c in (p.get("status") or {}).get("conditions") or []]
            changed = False
            for c in conds:
                if c.get("type") == "Ready" and c.get("status") != "False":
                    c.update(status="False", lastTransitionTime=m.now_rfc3339())
                    changed = True
            if changed:
                try:
                    await self.client.patch("pods", m.name_of(p), {"status": {"conditions": conds}}, m.namespace_of(p), sub="status")
                except m.StatusError:
                    pass

    async def _delete_pods(self, name: str):
        """util.DeletePods: every pod of the node except DaemonSet pods (they would come back)."""
        for p in self.pods.list():
            if (p.get("spec") or {}).get("nodeName") != name or is_pod_terminal(p) or \
                    (p.get("metadata") or {}).get("deletionTimestamp"):
                continue
            if any(r.get("kind") == "DaemonSet" for r in (p.get("metadata") or {}).get("ownerReferences") or []):
                continue
            try:
                await self.client.delete("pods", m.name_of(p), m.namespace_of(p))
                self.mgr.recorder.event(p, "Normal", "NodeControllerEviction",
                                        f"Marking for deletion Pod {m.name_of(p)} from Node {name}")
            except m.StatusError:
                pass

    async def monitor_once(self, now: float | None = None):
        now = now or time.time()
        counts: dict[str, list[int]] = {}
        status_of: dict[str, str] = {}
        nodes = self.nodes.list()
        for node in nodes:
            name = m.name_of(node)
            ready = get_condition(node, "Ready")
            if ready is None:
                created = m.parse_time((node.get("metadata") or {}).get("creationTimestamp")) or now
                stale = now - created > self.startup_grace
            else:
                hb = m.parse_time(ready.get("lastHeartbeatTime"))
                stale = hb is None or now - hb > self.grace
            cur = "Unknown" if stale else (ready or {}).get("status", "Unknown")
            if stale and (ready or {}).get("status") != "Unknown":
                conds = [dict(c, status="Unknown", reason="NodeStatusUnknown", message="Kubelet stopped posting node status.",
                              lastTransitionTime=m.now_rfc3339()) for c in (node.get("status") or {}).get("conditions") or []]
                if not conds:
                    conds = [{"type": "Ready", "status": "Unknown", "reason": "NodeStatusNeverUpdated",
                              "message": "Kubelet never posted node status.", "lastTransitionTime": m.now_rfc3339()}]
                await self.client.patch("nodes", name, {"status": {"conditions": conds}}, sub="status")
                await self._mark_pods_not_ready(name)
            status_of[name] = cur
            counts.setdefault(zone_of(node), [0, 0])[0 if cur == "True" else 1] += 1
        states = {z: zone_state(r, nr, self.unhealthy_threshold) for z, (r, nr) in counts.items()}
        all_full = bool(states) and all(st == FULL for st in states.values())
        if all_full != self.master_disruption:
            self.master_disruption = all_full
            if not all_full:      # leaving master disruption: every outage clock restarts now
                for name in list(self.unknown_since):
                    self.unknown_since[name] = now
        for z, st in states.items():
            size = sum(counts[z])
            rate = self.eviction_rate if st in (NORMAL, FULL) else (self.secondary_rate if size > self.large_cluster else 0.0)
            self.limiters.setdefault(z, _Limiter(rate)).set_rate(rate)
        self.zone_states = states
        for node in nodes:
            name = m.name_of(node)
            cur = status_of[name]
            if cur == "True":
                self.unknown_since.pop(name, None)
                self.evicted.discard(name)
                await self._set_taints(node, None, NODE_TAINT_KEYS)
                continue
            self.unknown_since.setdefault(name, now)
            if self.master_disruption:
                await self._set_taints(node, None, NODE_TAINT_KEYS)
                continue
            limiter = self.limiters[zone_of(node)]
            if self.taint_based:
                want = UNREACHABLE_TAINT if cur == "Unknown" else NOT_READY_TAINT
                have = {t.get("key") for t in (node.get("spec") or {}).get("taints") or []}
                if want["key"] in have and not (have & set(NODE_TAINT_KEYS)) - {want["key"]}:
                    continue
                if want["key"] in have or limiter.take(now):     # swapping the kind of taint costs no token
                    await self._set_taints(node, want, NODE_TAINT_KEYS)
                continue
            if name in self.evicted or now - self.unknown_since[name] < self.eviction_timeout:
                continue
            if limiter.take(now):
                await self._delete_pods(name)
                self.evicted.add(name)
        if self.taint_manager is not None:
            await self.taint_manager.process_once(now)

    async def sync(self, key):
        pass


class NoExecuteTaintManager(Controller):
    """pkg/controller/node/scheduler/taint_controller.go: pods on a node with NoExecute taints
    they do not tolerate are deleted; pods that tolerate every such taint for a limited
    tolerationSeconds are deleted when the shortest of them has elapsed since the taint was
    added; removing the taint (or the node becoming ready) cancels it."""
    name = "taint-manager"

    def __init__(self, mgr, period: float = 1.0):
        super().__init__(mgr)
        self.period = period
        self.first_seen: dict[tuple, float] = {}

    def setup(self):
        self.nodes = self.mgr.nodes
        self.pods = self.mgr.pods

    async def start(self):
        self.tasks.append(asyncio.create_task(self._loop(), name="taint-manager"))

    async def _loop(self):
        while True:
            await asyncio.sleep(self.period)
            try:
                await self.process_once()
            except Exception:
                pass

    def _deadline(self, pod: dict, taints: list[dict], now: float) -> float | None:
        """None: never; otherwise the time the pod must go (now for an untolerated taint)."""
        tols = (pod.get("spec") or {}).get("tolerations") or []
        best = None
        for t in taints:
            matching = [x for x in tols if tolerations_tolerate_taint([x], t)]
            if not matching:
                return now
            secs = [float(x["tolerationSeconds"]) for x in matching if x.get("tolerationSeconds") is not None]
            if len(secs) < len(matching):
                continue          # some toleration holds forever
            added = m.parse_time(t.get("timeAdded")) or self.first_seen.setdefault(
                (m.uid_of(pod), t.get("key"), t.get("value")), now)
            d = added + max(0.0, min(secs))
            best = d if best is None else min(best, d)
        return best

    async def process_once(self, now: float | None = None):
        now = now or time.time()
        tainted = {}
        for n in self.nodes.list():
            ts = [t for t in (n.get("spec") or {}).get("taints") or [] if t.get("effect") == "NoExecute"]
            if ts:
                tainted[m.name_of(n)] = ts
        live = set()
        for p in self.pods.list():
            node = (p.get("spec") or {}).get("nodeName")
            if node not in tainted or is_pod_terminal(p) or (p.get("metadata") or {}).get("deletionTimestamp"):
                continue
            live.add(m.uid_of(p))
            d = self._deadline(p, tainted[node], now)
            if d is not None and now >= d:
                try:
                    await self.client.delete("pods", m.name_of(p), m.namespace_of(p))
                    self.mgr.recorder.event(p, "Normal", "TaintManagerEviction", f"Marking for deletion Pod {m.namespace_of(p)}/{m.name_of(p)}")
                except m.StatusError:
                    pass
        self.first_seen = {k: v for k, v in self.first_seen.items() if k[0] in live}

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


class PodGCController(Controller):
    """pkg/controller/podgc/gc_controller.go: every gcCheckPeriod (20 s) terminated pods beyond
    --terminated-pod-gc-threshold (oldest first; 0 disables this step), pods bound to nodes that
    no longer exist (checked against a fresh node list) and unscheduled pods that are being
    deleted are force-deleted."""
    name = "podgc"

    def __init__(self, mgr, threshold: int = 12500, period: float = 20.0):     # --terminated-pod-gc-threshold
        super().__init__(mgr)
        self.threshold, self.period = threshold, period

    def setup(self):
        self.pods = self.mgr.pods

    async def start(self):
        self.tasks.append(asyncio.create_task(self._loop()))

    async def _loop(self):
        while True:
            await asyncio.sleep(self.period)
            try:
                await self.gc()
            except Exception as e:
                log.debug("podgc: %r", e)

    async def delete_pod(self, ns: str, name: str):
        await self.client.delete("pods", name, ns, grace=0)

    async def _delete(self, p):
        try:
            await self.delete_pod(m.namespace_of(p), m.name_of(p))
        except m.StatusError as e:
            if not m.is_not_found(e):
                log.debug("podgc: deleting %s: %r", m.key_of(p), e)

    @staticmethod
    def is_pod_terminated(pod) -> bool:
        return (pod.get("status") or {}).get("phase", "") not in ("Pending", "Running", "Unknown")

    async def gc(self):
        pods = self.pods.list()
        if self.threshold > 0:
            await self.gc_terminated(pods)
        await self.gc_orphaned(pods)
        await self.gc_unscheduled_terminating(pods)


    async def gc_terminated(self, pods):
        term = [p for p in pods if self.is_pod_terminated(p)]
        term.sort(key=lambda p: (m.parse_time((p.get("metadata") or {}).get("creationTimestamp")) or 0.0, m.name_of(p)))
        n = len(term) - self.threshold
        if n > 0:
            await asyncio.gather(*(self._delete(p) for p in term[:n]))

    async def gc_orphaned(self, pods):
        try:
            nodes, _ = await self.client.list("nodes")
        except Exception as e:
            log.debug("podgc: listing nodes: %r", e)
            return
        names = {m.name_of(n) for n in nodes}
        for p in pods:
            nn = (p.get("spec") or {}).get("nodeName")
            if nn and nn not in names:
                await self._delete(p)

    async def gc_unscheduled_terminating(self, pods):
        for p in pods:
            if (p.get("metadata") or {}).get("deletionTimestamp") and not (p.get("spec") or {}).get("nodeName"):
                await self._delete(p)

    async def sync(self, key):
        pass
