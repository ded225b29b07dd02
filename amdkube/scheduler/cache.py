"""Scheduler cache: per-node aggregates + device-level (extended resource) accounting,
with optimistic assume / forget / finish-binding / TTL expiry.

Reference: plugin/pkg/scheduler/schedulercache/cache.go:118 (AssumePod), :139
(FinishBinding), :163 (ForgetPod), :223-285 (Add/Update/RemovePod, assumed-pod
confirmation), :431 (cleanup of expired assumed pods); node_info.go (requested /
nonzero-requested resources, used host ports); the fork's extended_resources.go:25-210
(allocatable/available/used device maps updated by SetNode/AddPod/RemovePod).

Deliberate fixes:
  #1 an assumed pod carries its chosen device IDs, so the cache reserves them at assume
     time — back-to-back pods can never be handed the same GPU;
  #2 availability is derived on demand as allocatable − ∪assigned(pods), so AddPod before
     SetNode (or any event order) yields the same answer;
  #6 Unhealthy devices are never allocatable.
"""
from __future__ import annotations

import json
import time

from ..api import meta as m
from ..api.helpers import (HEALTHY, node_allocatable, pod_assigned_devices, pod_host_ports, pod_requests)

DEFAULT_MILLI_CPU, DEFAULT_MEMORY = 100, 200 * 2 ** 20   # priorities' non-zero defaults (util/non_zero.go)
TOPOLOGY_ANNOTATION = "amd.com/gpu-topology"


class NodeInfo:
    __slots__ = ("node", "name", "pods", "requested", "nonzero", "ports", "allocatable", "devices", "device_owner",
                 "generation", "_topo_src", "_topo", "labels", "taints", "groups")

    def __init__(self, name: str):
        self.name = name
        self.node: dict | None = None
        self.pods: dict[str, dict] = {}
        self.requested: dict[str, int] = {}
        self.nonzero = [0, 0]
        self.ports: dict[tuple, int] = {}
        self.allocatable: dict[str, int] = {}
        self.devices: dict[str, dict[str, dict]] = {}       # rname -> id -> {id, health, attributes}
        self.device_owner: dict[str, dict[str, str]] = {}   # rname -> id -> pod key
        self.generation = 0
        self._topo_src = None
        self._topo = None
        self.labels: dict = {}
        self.taints: list = []
        # (namespace, sorted labels) -> live pods on this node with exactly those labels: the
        # selector-spreading count matches each distinct label set once, not each pod
        self.groups: dict[tuple, int] = {}

    # ------------------------------------------------------------------ node
    def set_node(self, node: dict):
        self.node = node
        self.allocatable = node_allocatable(node)
        self.labels = m.labels_of(node)
        self.taints = (node.get("spec") or {}).get("taints") or []
        ext = (node.get("status") or {}).get("extendedResources") or {}
        self.devices = {r: dict((d or {}).get("resources") or {}) for r, d in ext.items()}
        self.generation += 1

    # ------------------------------------------------------------------ pods
    def add_pod(self, key: str, pod: dict):
        if key in self.pods:
            self.remove_pod(key)
        self.pods[key] = pod
        for k, v in pod_requests(pod).items():
            self.requested[k] = self.requested.get(k, 0) + v
        cpu, mem = nonzero_requests(pod)
        self.nonzero[0] += cpu
        self.nonzero[1] += mem
        for p in pod_host_ports(pod):
            self.ports[p] = self.ports.get(p, 0) + 1
        g = _group(pod)
        if g is not None:
            self.groups[g] = self.groups.get(g, 0) + 1
        for rname, ids in pod_assigned_devices(pod).items():
            own = self.device_owner.setdefault(rname, {})
            for did in ids:
                own[did] = key
        self.generation += 1

    def remove_pod(self, key: str):
        pod = self.pods.pop(key, None)
        if pod is None:
            return
        for k, v in pod_requests(pod).items():
            self.requested[k] = self.requested.get(k, 0) - v
        cpu, mem = nonzero_requests(pod)
        self.nonzero[0] -= cpu
        self.nonzero[1] -= mem
        for p in pod_host_ports(pod):
            self.ports[p] -= 1
            if self.ports[p] <= 0:
                del self.ports[p]
        g = _group(pod)
        if g is not None:
            c = self.groups.get(g, 0) - 1
            if c > 0:
                self.groups[g] = c
            else:
                self.groups.pop(g, None)
        for rname, ids in pod_assigned_devices(pod).items():
            own = self.device_owner.get(rname, {})
            for did in ids:
                if own.get(did) == key:
                    del own[did]
        self.generation += 1

    # ---------------------------------------------------------------- devices
    def available_devices(self, rname: str) -> dict[str, dict]:
        """Healthy, unassigned devices of `rname` (derived on demand: fix #2/#6)."""
        devs = self.devices.get(rname)
        if not devs:
            return {}
        own = self.device_owner.get(rname, {})
        return {did: d for did, d in devs.items() if did not in own and (d.get("health") or HEALTHY) == HEALTHY}

    def all_device_ids(self, rname: str) -> list[str]:
        return list((self.devices.get(rname) or {}).keys())

    def topology(self):
        """(ids, index map, numa list, link matrix, parent list | None) from the node's
        gpu-topology annotation; `parent` groups the partitions of one physical GPU."""
        src = m.annotations_of(self.node or {}).get(TOPOLOGY_ANNOTATION)
        if src != self._topo_src:
            self._topo_src = src
            self._topo = None
            if src:
                try:
                    t = json.loads(src)
                    ids = t["ids"]
                    self._topo = (ids, {d: i for i, d in enumerate(ids)}, t["numa"], t["link"], t.get("parent"))
                except (ValueError, KeyError, TypeError):
                    self._topo = None
        return self._topo

    def clone(self) -> "NodeInfo":
        n = NodeInfo(self.name)
        n.node, n.allocatable, n.labels, n.taints = self.node, dict(self.allocatable), self.labels, self.taints
        n.pods = dict(self.pods)
        n.requested = dict(self.requested)
        n.nonzero = list(self.nonzero)
        n.ports = dict(self.ports)
        n.groups = dict(self.groups)
        n.devices = self.devices
        n.device_owner = {r: dict(o) for r, o in self.device_owner.items()}
        n._topo_src, n._topo = self._topo_src, self._topo
        n.generation = self.generation
        return n


def _group(pod: dict):
    """The spreading group of a pod: None for a pod being deleted (selector_spreading.go skips
    pods with a deletionTimestamp)."""
    md = pod.get("metadata") or {}
    if md.get("deletionTimestamp"):
        return None
    return md.get("namespace") or "", tuple(sorted((md.get("labels") or {}).items()))


def nonzero_requests(pod: dict) -> tuple[int, int]:
    cpu = mem = 0
    for c in (pod.get("spec") or {}).get("containers") or []:
        req = (c.get("resources") or {}).get("requests") or {}
        from ..api.quantity import Quantity
        cpu += Quantity(req["cpu"]).milli_value() if "cpu" in req else DEFAULT_MILLI_CPU
        mem += Quantity(req["memory"]).value() if "memory" in req else DEFAULT_MEMORY
    return cpu, mem


def _has_anti_affinity(pod) -> bool:
    return bool((((pod.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity") or {})
                .get("requiredDuringSchedulingIgnoredDuringExecution"))


def _has_affinity(pod) -> bool:
    return bool((((pod.get("spec") or {}).get("affinity") or {}).get("podAffinity") or {})
                .get("requiredDuringSchedulingIgnoredDuringExecution"))


def _has_pref_affinity(pod) -> bool:
    aff = (pod.get("spec") or {}).get("affinity") or {}
    return bool((aff.get("podAffinity") or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or
                (aff.get("podAntiAffinity") or {}).get("preferredDuringSchedulingIgnoredDuringExecution"))


class SchedulerCache:
    def __init__(self, ttl: float = 30.0):
        self.anti_affinity_pods = 0  # pods carrying required anti-affinity (MatchInterPodAffinity fast path)
        self.affinity_pods = 0       # pods carrying required affinity (hardPodAffinitySymmetricWeight)
        self.pref_affinity_pods = 0  # pods carrying preferred (anti-)affinity (InterPodAffinity symmetry)
        self.nodes: dict[str, NodeInfo] = {}
        self.pod_node: dict[str, str] = {}          # pod key -> node name
        self.pod_states: dict[str, dict] = {}       # pod key -> pod
        self.assumed: dict[str, float | None] = {}  # pod key -> deadline (None until binding finished)
        self.ttl = ttl
        # names of nodes whose NodeInfo changed, in order (log[i] has sequence log_base + i): the
        # scheduler's per-equivalence-class fit index replays it to re-check only those nodes
        self.log: list[str] = []
        self.log_base = 0
        self.prefer_no_schedule = 0  # ready nodes carrying a PreferNoSchedule taint

    def _touch(self, name: str):
        self.log.append(name)
        if len(self.log) > 200_000:         # indexes further behind than this rebuild
            cut = len(self.log) // 2
            del self.log[:cut]
            self.log_base += cut

    @property
    def seq(self) -> int:
        return self.log_base + len(self.log)

    @staticmethod
    def _pns(ni) -> bool:
        return ni.node is not None and any(t.get("effect") == "PreferNoSchedule" for t in ni.taints)

    def _track(self, pod, delta):
        if _has_anti_affinity(pod):
            self.anti_affinity_pods += delta
        if _has_affinity(pod):
            self.affinity_pods += delta
        if _has_pref_affinity(pod):
            self.pref_affinity_pods += delta

    def _ni(self, name) -> NodeInfo:
        ni = self.nodes.get(name)
        if ni is None:
            ni = self.nodes[name] = NodeInfo(name)
        return ni

    # ------------------------------------------------------------------ nodes
    def add_node(self, node: dict):
        ni = self._ni(m.name_of(node))
        self.prefer_no_schedule -= self._pns(ni)
        ni.set_node(node)
        self.prefer_no_schedule += self._pns(ni)
        self._touch(ni.name)

    update_node = add_node

    def remove_node(self, node: dict):
        name = m.name_of(node)
        ni = self.nodes.get(name)
        if ni is None:
            return
        self.prefer_no_schedule -= self._pns(ni)
        self._touch(name)
        if ni.pods:
            ni.node = None  # keep pods until they go away (cache.go RemoveNode)
            ni.allocatable = {}
            ni.devices = {}
        else:
            del self.nodes[name]

    def ready_nodes(self) -> list[NodeInfo]:
        return [ni for ni in self.nodes.values() if ni.node is not None]

    # ------------------------------------------------------------------- pods
    def assume_pod(self, pod: dict):
        key = m.key_of(pod)
        if key in self.pod_states:
            raise KeyError(f"pod {key} is in the cache, so can't be assumed")
        node = (pod.get("spec") or {}).get("nodeName")
        self._ni(node).add_pod(key, pod)
        self._touch(node)
        self.pod_node[key] = node
        self.pod_states[key] = pod
        self.assumed[key] = None
        self._track(pod, 1)

    def finish_binding(self, pod: dict):
        key = m.key_of(pod)
        if key in self.assumed:
            self.assumed[key] = time.monotonic() + self.ttl

    def forget_pod(self, pod: dict):
        key = m.key_of(pod)
        if key not in self.assumed:
            return
        node = self.pod_node.pop(key, None)
        if node and node in self.nodes:
            self.nodes[node].remove_pod(key)
            self._touch(node)
        old = self.pod_states.pop(key, None)
        if old is not None:
            self._track(old, -1)
        self.assumed.pop(key, None)

    def add_pod(self, pod: dict):
        """An assigned pod observed from the API (confirms an assumed pod)."""
        key = m.key_of(pod)
        node = (pod.get("spec") or {}).get("nodeName")
        if key in self.assumed:
            self.assumed.pop(key, None)
            old_node = self.pod_node.get(key)
            if old_node and old_node in self.nodes:
                self.nodes[old_node].remove_pod(key)
                self._touch(old_node)
            old = self.pod_states.get(key)
            if old is not None:
                self._track(old, -1)
        elif key in self.pod_states:
            self.remove_pod(self.pod_states[key])
        self._ni(node).add_pod(key, pod)
        self._touch(node)
        self.pod_node[key] = node
        self.pod_states[key] = pod
        self._track(pod, 1)

    def update_pod(self, old: dict, new: dict):
        self.add_pod(new)

    def remove_pod(self, pod: dict):
        key = m.key_of(pod)
        node = self.pod_node.pop(key, None)
        if node and node in self.nodes:
            ni = self.nodes[node]
            ni.remove_pod(key)
            self._touch(node)
            if ni.node is None and not ni.pods:
                del self.nodes[node]
        old = self.pod_states.pop(key, None)
        if old is not None:
            self._track(old, -1)
        self.assumed.pop(key, None)

    def is_assumed(self, pod) -> bool:
        return m.key_of(pod) in self.assumed

    def cleanup_expired(self):
        now = time.monotonic()
        for key, dl in list(self.assumed.items()):
            if dl is not None and dl < now:
                pod = self.pod_states.get(key)
                if pod is not None:
                    self.forget_pod(pod)
