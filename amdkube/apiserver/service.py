"""Service REST strategy: ClusterIP and NodePort allocation, validation, repair.

Reference: pkg/registry/core/service/rest.go (Create allocates spec.clusterIP from
--service-cluster-ip-range and every NodePort/LoadBalancer port's nodePort from
--service-node-port-range; Update keeps clusterIP immutable and allocates new node ports;
Delete releases both), ipallocator/allocator.go (bitmap over the CIDR, network and
broadcast addresses reserved), portallocator/allocator.go, and the repair controllers
(ipallocator/controller/repair.go, portallocator/controller/repair.go) that rebuild the
bitmaps from the stored services after a restart.

amdkube keeps no separate allocation record: the allocated sets are an index derived from the
store's commit stream (the same mechanism as the GPU device index), so "repair" is the
index rebuild at start-up and a deleted service releases its IP and ports by construction.
Allocation and the store write happen in one event-loop step, so two creates cannot race.
"""
from __future__ import annotations

import ipaddress
import random

from ..api import meta as m
from ..store.storage import decode_kv
from ..api.field import go_value

DEFAULT_SERVICE_CIDR = "10.0.0.0/24"          # kube-apiserver --service-cluster-ip-range default
DEFAULT_NODE_PORT_RANGE = (30000, 32767)      # --service-node-port-range default 30000-32767


def parse_port_range(s: str) -> tuple[int, int]:
    lo, _, hi = s.partition("-")
    lo, hi = int(lo), int(hi or lo)
    if not 0 < lo <= hi < 65536:
        raise ValueError(f"invalid port range {s!r}")
    return lo, hi


class ServiceAllocator:
    def __init__(self, cidr: str = DEFAULT_SERVICE_CIDR, node_ports: tuple[int, int] = DEFAULT_NODE_PORT_RANGE):
        self.net = ipaddress.ip_network(cidr, strict=False)
        self.node_ports = node_ports
        self.ips: dict[str, str] = {}          # ip -> service key
        self.ports: dict[tuple[str, int], str] = {}  # (proto, port) -> service key
        self._by_key: dict[str, tuple[list, list]] = {}
        # allocations handed to a write that has not committed yet: over a bridged store
        # (Etcd3Store group commit) other requests run while it is in flight, and must not be
        # given the same address or port. Released once the write settled (release_pending).
        self._pending: dict[str, set] = {}
        self._rng = random.Random()
        # the first usable address is reserved for the `kubernetes` service (master.go
        # ServiceIPRange: first IP of the range)
        hosts = self.net.num_addresses - (2 if self.net.version == 4 and self.net.prefixlen < 31 else 0)
        if hosts < 1:
            raise ValueError(f"service CIDR {cidr} has no usable addresses")

    # ---------------------------------------------------------------- index
    def index(self, key: str, svc: dict | None):
        ips, ports = self._by_key.pop(key, ([], []))
        for ip in ips:
            if self.ips.get(ip) == key:
                del self.ips[ip]
        for p in ports:
            if self.ports.get(p) == key:
                del self.ports[p]
        if svc is None:
            return
        spec = svc.get("spec") or {}
        ips, ports = [], []
        ip = spec.get("clusterIP")
        if ip and ip != "None":
            self.ips[ip] = key
            ips.append(ip)
        for p in spec.get("ports") or []:
            if p.get("nodePort"):
                k = (p.get("protocol", "TCP"), int(p["nodePort"]))
                self.ports[k] = key
                ports.append(k)
        if spec.get("healthCheckNodePort"):
            k = ("TCP", int(spec["healthCheckNodePort"]))
            self.ports[k] = key
            ports.append(k)
        self._by_key[key] = (ips, ports)

    def _reserve(self, key: str, kind: str, v):
        table = self.ips if kind == "ip" else self.ports
        if v not in table:
            table[v] = key
            self._pending.setdefault(key, set()).add((kind, v))

    def release_pending(self, key: str):
        """Drop `key`'s in-flight reservations that its committed object does not hold (the
        write failed, or allocated something it then did not keep)."""
        ips, ports = self._by_key.get(key, ([], []))
        for kind, v in self._pending.pop(key, ()):
            if kind == "ip" and v not in ips and self.ips.get(v) == key:
                del self.ips[v]
            elif kind == "port" and v not in ports and self.ports.get(v) == key:
                del self.ports[v]

    def rebuild(self, kvs):
        for kv in kvs:
            self.index(kv.key, decode_kv(kv.value))

    # ------------------------------------------------------------- allocate
    def _usable(self, ip) -> bool:
        if ip not in self.net:
            return False
        if self.net.version == 4 and self.net.prefixlen < 31 and ip in (self.net.network_address, self.net.broadcast_address):
            return False
        return True

    def allocate_ip(self, key: str, requested: str | None = None) -> str:
        if requested:
            try:
                ip = ipaddress.ip_address(requested)
            except ValueError:
                raise m.invalid("Service", key.rsplit("/", 1)[-1], [f"spec.clusterIP: Invalid value: {go_value(requested)}: must be a valid IP address"])
            if not self._usable(ip):
                raise m.invalid("Service", key.rsplit("/", 1)[-1], [f"spec.clusterIP: Invalid value: {go_value(requested)}: provided IP is not in the valid range. "
                                                 f"The range of valid IPs is {self.net}"])
            if str(ip) in self.ips and self.ips[str(ip)] != key:
                raise m.invalid("Service", key.rsplit("/", 1)[-1], [f"spec.clusterIP: Invalid value: {go_value(requested)}: provided IP is already allocated"])
            self._reserve(key, "ip", str(ip))
            return str(ip)
        first = int(self.net.network_address) + (1 if self.net.version == 4 and self.net.prefixlen < 31 else 0)
        last = int(self.net.broadcast_address) - (1 if self.net.version == 4 and self.net.prefixlen < 31 else 0)
        size = last - first + 1
        start = self._rng.randrange(size)  # allocator.go AllocateNext: random offset, linear probe
        for i in range(size):
            ip = str(ipaddress.ip_address(first + (start + i) % size))
            if ip not in self.ips:
                self._reserve(key, "ip", ip)
                return ip
        raise m.StatusError(500, "InternalError", "failed to allocate a serviceIP: range is full")

    def allocate_port(self, key: str, proto: str, requested: int | None, taken: set) -> int:
        lo, hi = self.node_ports
        if requested:
            if not lo <= requested <= hi:
                raise m.invalid("Service", key.rsplit("/", 1)[-1], [f"spec.ports[].nodePort: Invalid value: {requested}: provided port is not in the "
                                                 f"valid range. The range of valid ports is {lo}-{hi}"])
            owner = self.ports.get((proto, requested))
            if (owner and owner != key) or (proto, requested) in taken:
                raise m.invalid("Service", key.rsplit("/", 1)[-1], [f"spec.ports[].nodePort: Invalid value: {requested}: provided port is already allocated"])
            self._reserve(key, "port", (proto, requested))
            return requested
        size = hi - lo + 1
        start = self._rng.randrange(size)
        for i in range(size):
            p = lo + (start + i) % size
            if (proto, p) not in self.ports and (proto, p) not in taken:
                self._reserve(key, "port", (proto, p))
                return p
        raise m.StatusError(500, "InternalError", "failed to allocate a nodePort: range is full")

    # ------------------------------------------------------------- strategy
    def prepare_create(self, key: str, svc: dict):
        spec = svc.setdefault("spec", {})
        t = spec.setdefault("type", "ClusterIP")
        if t != "ExternalName":
            if spec.get("clusterIP") != "None":
                spec["clusterIP"] = self.allocate_ip(key, spec.get("clusterIP") or None)
        else:
            spec.pop("clusterIP", None)
        self._node_ports(key, spec, {})

    def prepare_update(self, key: str, new: dict, cur: dict):
        spec, cspec = new.setdefault("spec", {}), cur.get("spec") or {}
        spec.setdefault("type", cspec.get("type", "ClusterIP"))
        old_ip = cspec.get("clusterIP")
        if spec["type"] == "ExternalName":
            spec.pop("clusterIP", None)
        elif not spec.get("clusterIP"):
            # an update that omits clusterIP keeps it (a ClusterIP->ExternalName->ClusterIP flip allocates anew)
            spec["clusterIP"] = old_ip if old_ip else self.allocate_ip(key)
        elif old_ip and spec["clusterIP"] != old_ip:
            raise m.invalid("Service", m.name_of(new), ["spec.clusterIP: Invalid value: field is immutable"])
        elif not old_ip and spec["clusterIP"] != "None":
            spec["clusterIP"] = self.allocate_ip(key, spec["clusterIP"])
        old = {(p.get("protocol", "TCP"), p.get("port")): p.get("nodePort") for p in cspec.get("ports") or []}
        self._node_ports(key, spec, old, cspec.get("healthCheckNodePort"))

    def _node_ports(self, key, spec, old, old_hc=None):
        need = spec.get("type") in ("NodePort", "LoadBalancer")
        taken: set = set()
        if spec.get("healthCheckNodePort"):
            taken.add(("TCP", int(spec["healthCheckNodePort"])))
        for p in spec.get("ports") or []:
            proto = p.setdefault("protocol", "TCP")
            if not need:
                # a port carried over from a NodePort service is released; one the user set on a
                # ClusterIP service is left for validation to reject (rest.go / ValidateService)
                if p.get("nodePort") and old.get((proto, p.get("port"))) == p["nodePort"]:
                    p.pop("nodePort")
                continue
            req = p.get("nodePort") or old.get((proto, p.get("port")))
            p["nodePort"] = self.allocate_port(key, proto, int(req) if req else None, taken)
            taken.add((proto, p["nodePort"]))
        # rest.go: a LoadBalancer with externalTrafficPolicy=Local gets a health-check node port
        # (spec.healthCheckNodePort, kept across updates) that kube-proxy answers on every node
        if spec.get("type") == "LoadBalancer" and spec.get("externalTrafficPolicy") == "Local":
            req = spec.get("healthCheckNodePort") or old_hc
            if req:
                taken.discard(("TCP", int(req)))
            spec["healthCheckNodePort"] = self.allocate_port(key, "TCP", int(req) if req else None, taken)
        elif spec.get("healthCheckNodePort") and spec.get("healthCheckNodePort") == old_hc:
            spec.pop("healthCheckNodePort")     # released with the Local LoadBalancer it belonged to
