"""Networking controllers: Endpoints and node IPAM (pod CIDR per node).

Reference:
  * pkg/controller/endpoint/endpoints_controller.go — syncService: for a service with a
    selector, every non-terminal, non-deleting pod with a podIP that matches the selector
    contributes one address per service port (targetPort resolved by number or by
    container-port name, podutil.FindPort); ready pods go to `addresses`, others to
    `notReadyAddresses` unless the service tolerates unready endpoints; subsets are
    repacked (endpoints.RepackSubsets) so addresses sharing one port set share a subset;
    the Endpoints object is written only when it changes, and deleted with its service.
  * pkg/controller/node/ipam/range_allocator.go — `--allocate-node-cidrs`: each node gets
    the next free `--node-cidr-mask-size` block of `--cluster-cidr` in spec.podCIDR; the
    in-use set is rebuilt from existing nodes, and a deleted node's CIDR is released.
"""
from __future__ import annotations

import ipaddress

from ..api import meta as m
from ..api.helpers import is_pod_ready, is_pod_terminal
from ..api.labels import selector_from_set
from .base import Controller, split_key

TOLERATE_UNREADY = "service.alpha.kubernetes.io/tolerate-unready-endpoints"


def find_port(pod: dict, svc_port: dict) -> int | None:
    """podutil.FindPort: int targetPort as is; a name matches a container port name+protocol."""
    tp = svc_port.get("targetPort", svc_port.get("port"))
    if isinstance(tp, int):
        return tp
    if isinstance(tp, str) and tp.isdigit():
        return int(tp)
    proto = svc_port.get("protocol", "TCP")
    for c in (pod.get("spec") or {}).get("containers") or []:
        for cp in c.get("ports") or []:
            if cp.get("name") == tp and cp.get("protocol", "TCP") == proto:
                return cp.get("containerPort")
    return None


def repack_subsets(entries) -> list[dict]:
    """entries: (address dict, ready, sorted tuple of port item-tuples) -> deterministic subsets."""
    by_ports: dict[tuple, dict] = {}
    for addr, ready, ports in entries:
        s = by_ports.setdefault(ports, {"addresses": {}, "notReadyAddresses": {}})
        s["addresses" if ready else "notReadyAddresses"][addr["ip"]] = addr
    out = []
    for ports in sorted(by_ports, key=repr):
        s = by_ports[ports]
        sub = {}
        if s["addresses"]:
            sub["addresses"] = [s["addresses"][ip] for ip in sorted(s["addresses"])]
        if s["notReadyAddresses"]:
            sub["notReadyAddresses"] = [s["notReadyAddresses"][ip] for ip in sorted(s["notReadyAddresses"])]
        sub["ports"] = [dict(p) for p in ports]
        out.append(sub)
    return out


class EndpointsController(Controller):
    name = "endpoint"
    workers = 4

    def setup(self):
        f = self.mgr.factory
        self.svc_inf = f.informer("services")
        self.ep_inf = f.informer("endpoints")
        self.pod_inf = self.mgr.pods
        self.svc_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.pod_inf.add_handler(on_add=self._pod, on_update=self._pod_update, on_delete=self._pod)

    def _services_for(self, pod):
        ns, labels = m.namespace_of(pod), m.labels_of(pod)
        for svc in self.svc_inf.list():
            if m.namespace_of(svc) != ns:
                continue
            sel = (svc.get("spec") or {}).get("selector")
            if sel and selector_from_set(sel).matches(labels):
                yield svc

    def _pod(self, pod):
        for svc in self._services_for(pod):
            self.enqueue(svc)

    def _pod_update(self, old, new):
        if m.labels_of(old) != m.labels_of(new):
            self._pod(old)
        self._pod(new)

    async def sync(self, key):
        ns, name = split_key(key)
        svc = self.svc_inf.get(key)
        if svc is None:
            try:
                await self.client.delete("endpoints", name, ns)
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise
            return
        spec = svc.get("spec") or {}
        if not spec.get("selector"):
            return  # selector-less services have user-managed endpoints
        sel = selector_from_set(spec["selector"])
        tolerate = m.annotations_of(svc).get(TOLERATE_UNREADY) == "true"
        entries = []
        for pod in self.pod_inf.list():
            if m.namespace_of(pod) != ns or not sel.matches(m.labels_of(pod)):
                continue
            pmd = pod.get("metadata") or {}
            ip = (pod.get("status") or {}).get("podIP")
            if not ip or pmd.get("deletionTimestamp") or is_pod_terminal(pod):
                continue
            addr = {"ip": ip, "nodeName": (pod.get("spec") or {}).get("nodeName", ""),
                    "targetRef": {"kind": "Pod", "namespace": ns, "name": m.name_of(pod), "uid": m.uid_of(pod),
                                  "resourceVersion": pmd.get("resourceVersion", "")}}
            pspec = pod.get("spec") or {}
            if pspec.get("hostname") and pspec.get("subdomain") == m.name_of(svc):
                addr["hostname"] = pspec["hostname"]   # endpoints_controller.go: per-pod DNS names
            ports = []
            for sp in spec.get("ports") or []:
                port = find_port(pod, sp)
                if port is None:
                    continue
                ports.append(tuple(sorted({"name": sp.get("name", ""), "port": port,
                                           "protocol": sp.get("protocol", "TCP")}.items())))
            if not ports and spec.get("ports"):
                continue
            ready = tolerate or is_pod_ready(pod)
            entries.append((addr, ready, tuple(sorted(ports))))
        subsets = repack_subsets(entries)
        cur = self.ep_inf.get(key)
        want_labels = m.labels_of(svc)
        if cur is not None and (cur.get("subsets") or []) == subsets and m.labels_of(cur) == want_labels:
            return
        body = {"apiVersion": "v1", "kind": "Endpoints",
                "metadata": {"name": name, "namespace": ns, "labels": want_labels}, "subsets": subsets}
        if cur is None:
            try:
                await self.client.create(body, ns)
                return
            except m.StatusError as e:
                if not m.is_already_exists(e):
                    raise
        await self.client.patch("endpoints", name, {"metadata": {"labels": want_labels}, "subsets": subsets}, ns)


class NodeIPAMController(Controller):
    """range_allocator.go: per-node pod CIDRs carved from the cluster CIDR."""
    name = "nodeipam"
    workers = 1

    def __init__(self, mgr, cluster_cidr: str = "10.244.0.0/16", node_mask: int = 24):
        super().__init__(mgr)
        self.cluster = ipaddress.ip_network(cluster_cidr, strict=False)
        if node_mask < self.cluster.prefixlen:
            raise ValueError("node CIDR mask must be longer than the cluster CIDR mask")
        self.node_mask = node_mask
        self.used: dict[str, str] = {}   # cidr -> node

    def setup(self):
        self.node_inf = self.mgr.nodes
        self.node_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self._deleted)

    def _deleted(self, node):
        cidr = (node.get("spec") or {}).get("podCIDR")
        if cidr and self.used.get(cidr) == m.name_of(node):
            del self.used[cidr]

    def _occupy(self):
        for n in self.node_inf.list():
            c = (n.get("spec") or {}).get("podCIDR")
            if c:
                self.used[c] = m.name_of(n)

    def next_cidr(self) -> str:
        for sub in self.cluster.subnets(new_prefix=self.node_mask):
            if str(sub) not in self.used:
                return str(sub)
        raise RuntimeError(f"CIDR allocation failed: {self.cluster} is exhausted")

    async def sync(self, key):
        _, name = split_key(key)
        node = self.node_inf.get(name)
        if node is None:
            return
        self._occupy()
        if (node.get("spec") or {}).get("podCIDR"):
            return
        cidr = self.next_cidr()
        self.used[cidr] = name
        try:
            await self.client.patch("nodes", name, {"spec": {"podCIDR": cidr}})
        except Exception:
            self.used.pop(cidr, None)
            raise
