"""Service / endpoints change tracking shared by both proxy modes.

Reference: pkg/proxy/types.go (ServicePortName), pkg/proxy/iptables/proxier.go
(serviceInfo from a v1.ServicePort: clusterIP, port, protocol, nodePort,
sessionAffinity + ClientIP timeout, externalIPs, loadBalancer ingress; endpointsMap
holds only ready addresses, keyed by the endpoint port's *name* matching the service
port's name), pkg/proxy/config/config.go (ServiceConfig / EndpointsConfig handlers).
"""
from __future__ import annotations

from dataclasses import dataclass, field

from ..api import meta as m

DEFAULT_AFFINITY_TIMEOUT = 10800  # v1.DefaultClientIPServiceAffinitySeconds


@dataclass(frozen=True)
class ServicePortName:
    namespace: str
    name: str
    port: str = ""

    def __str__(self):
        return f"{self.namespace}/{self.name}" + (f":{self.port}" if self.port else "")


@dataclass
class ServiceInfo:
    cluster_ip: str
    port: int
    protocol: str
    node_port: int = 0
    session_affinity: str = "None"
    affinity_timeout: int = DEFAULT_AFFINITY_TIMEOUT
    external_ips: list = field(default_factory=list)
    lb_ingress: list = field(default_factory=list)
    only_local: bool = False        # externalTrafficPolicy: Local on a NodePort/LoadBalancer service
    source_ranges: list = field(default_factory=list)     # spec.loadBalancerSourceRanges
    health_check_node_port: int = 0


def service_infos(svc: dict) -> dict[ServicePortName, ServiceInfo]:
    spec = svc.get("spec") or {}
    ip = spec.get("clusterIP")
    if not ip or ip == "None" or spec.get("type") == "ExternalName":
        return {}
    out = {}
    timeout = (((spec.get("sessionAffinityConfig") or {}).get("clientIP") or {}).get("timeoutSeconds")
               or DEFAULT_AFFINITY_TIMEOUT)
    ingress = [i.get("ip") for i in (((svc.get("status") or {}).get("loadBalancer") or {}).get("ingress") or []) if i.get("ip")]
    # apiservice.RequestsOnlyLocalTraffic: Local only means something for NodePort/LoadBalancer
    local = spec.get("externalTrafficPolicy") == "Local" and spec.get("type") in ("NodePort", "LoadBalancer")
    ranges = [r.strip() for r in spec.get("loadBalancerSourceRanges") or [] if r.strip()]
    if not ranges:          # the legacy annotation (pkg/api/service/util.go GetLoadBalancerSourceRanges)
        ann = (m.annotations_of(svc) or {}).get("service.beta.kubernetes.io/load-balancer-source-ranges", "")
        ranges = [r.strip() for r in ann.split(",") if r.strip()]
    hc = int(spec.get("healthCheckNodePort") or 0) if local and spec.get("type") == "LoadBalancer" else 0
    for p in spec.get("ports") or []:
        spn = ServicePortName(m.namespace_of(svc), m.name_of(svc), p.get("name", ""))
        out[spn] = ServiceInfo(ip, int(p["port"]), p.get("protocol", "TCP"), int(p.get("nodePort") or 0),
                               spec.get("sessionAffinity", "None"), int(timeout), list(spec.get("externalIPs") or []),
                               ingress, local, ranges, hc)
    return out


def endpoints_map(ep: dict) -> dict[ServicePortName, list[tuple[str, int, str]]]:
    """ServicePortName -> [(ip, port, nodeName)] of READY addresses only."""
    out: dict[ServicePortName, list] = {}
    for ss in ep.get("subsets") or []:
        for p in ss.get("ports") or []:
            spn = ServicePortName(m.namespace_of(ep), m.name_of(ep), p.get("name", ""))
            lst = out.setdefault(spn, [])
            for a in ss.get("addresses") or []:
                lst.append((a["ip"], int(p["port"]), a.get("nodeName", "")))
    for v in out.values():
        v.sort()
    return out


class ChangeTracker:
    """Accumulates service/endpoints state from informer callbacks; `dirty` tells the proxier
    whether a sync is needed (the reference's serviceChanges / endpointsChanges)."""

    def __init__(self):
        self.services: dict[str, dict[ServicePortName, ServiceInfo]] = {}
        self.endpoints: dict[str, dict[ServicePortName, list]] = {}
        self.dirty = True

    def on_service(self, svc, deleted=False):
        key = m.key_of(svc)
        new = {} if deleted else service_infos(svc)
        if self.services.get(key) != new:
            if new:
                self.services[key] = new
            else:
                self.services.pop(key, None)
            self.dirty = True

    def on_endpoints(self, ep, deleted=False):
        key = m.key_of(ep)
        new = {} if deleted else endpoints_map(ep)
        if self.endpoints.get(key) != new:
            if new:
                self.endpoints[key] = new
            else:
                self.endpoints.pop(key, None)
            self.dirty = True

    def service_map(self) -> dict[ServicePortName, ServiceInfo]:
        out = {}
        for v in self.services.values():
            out.update(v)
        return out

    def endpoint_map(self) -> dict[ServicePortName, list]:
        out = {}
        for v in self.endpoints.values():
            out.update(v)
        return out
