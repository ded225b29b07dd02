"""Service validation and defaulting (reference pkg/apis/core/validation/validation.go
ValidateService, pkg/apis/core/v1/defaults.go SetDefaults_Service)."""
from __future__ import annotations

from .labels import is_dns1123_label
from .field import go_value

SERVICE_TYPES = ("ClusterIP", "NodePort", "LoadBalancer", "ExternalName")


def validate_service(svc: dict, old=None) -> list[str]:
    from .validation import validate_object_meta
    errs = validate_object_meta(svc, True, is_dns1123_label)
    spec = svc.get("spec") or {}
    t = spec.get("type", "ClusterIP")
    if t not in SERVICE_TYPES:
        errs.append(f"spec.type: Unsupported value: {go_value(t)}: supported values: {', '.join(SERVICE_TYPES)}")
    if t == "ExternalName":
        if not spec.get("externalName"):
            errs.append("spec.externalName: Required value")
        return errs
    ports = spec.get("ports") or []
    if not ports and spec.get("clusterIP") != "None":
        errs.append("spec.ports: Required value")
    seen_names, seen_ports = set(), set()
    for i, p in enumerate(ports):
        pref = f"spec.ports[{i}]"
        if len(ports) > 1 and not p.get("name"):
            errs.append(f"{pref}.name: Required value")
        if p.get("name"):
            if p["name"] in seen_names:
                errs.append(f"{pref}.name: Duplicate value: {go_value(p['name'])}")
            seen_names.add(p["name"])
        port = p.get("port")
        if not isinstance(port, int) or not 0 < port < 65536:
            errs.append(f"{pref}.port: Invalid value: {go_value(port)}: must be between 1 and 65535, inclusive")
        proto = p.get("protocol", "TCP")
        if proto not in ("TCP", "UDP"):
            errs.append(f"{pref}.protocol: Unsupported value: {go_value(proto)}: supported values: TCP, UDP")
        if (proto, port) in seen_ports:
            errs.append(f"{pref}: Duplicate value: {proto}/{port}")
        seen_ports.add((proto, port))
        tp = p.get("targetPort")
        if tp is not None and not ((isinstance(tp, int) and 0 < tp < 65536) or (isinstance(tp, str) and tp)):
            errs.append(f"{pref}.targetPort: Invalid value: {go_value(tp)}")
        if p.get("nodePort") and t == "ClusterIP":
            errs.append(f"{pref}.nodePort: Forbidden: may not be used when `type` is 'ClusterIP'")
    aff = spec.get("sessionAffinity", "None")
    if aff not in ("None", "ClientIP"):
        errs.append(f"spec.sessionAffinity: Unsupported value: {go_value(aff)}")
    sel = spec.get("selector") or {}
    if not isinstance(sel, dict):
        errs.append("spec.selector: Invalid value: must be a map")
    # validation.go validateServiceExternalTrafficFieldsValue / ValidateService (source ranges)
    etp = spec.get("externalTrafficPolicy")
    if etp:
        if t not in ("NodePort", "LoadBalancer"):
            errs.append(f"spec.externalTrafficPolicy: Invalid value: {go_value(etp)}: ExternalTrafficPolicy can only be set on "
                        "NodePort and LoadBalancer service")
        elif etp not in ("Cluster", "Local"):
            errs.append(f"spec.externalTrafficPolicy: Unsupported value: {go_value(etp)}: supported values: Cluster, Local")
    hc = spec.get("healthCheckNodePort")
    if hc:
        if not (t == "LoadBalancer" and etp == "Local"):
            errs.append(f"spec.healthCheckNodePort: Invalid value: {go_value(hc)}: HealthCheckNodePort can only be set on "
                        "LoadBalancer service with ExternalTrafficPolicy=Local")
        elif not isinstance(hc, int) or not 0 < hc < 65536:
            errs.append(f"spec.healthCheckNodePort: Invalid value: {go_value(hc)}: must be between 1 and 65535, inclusive")
    ranges = spec.get("loadBalancerSourceRanges") or []
    if ranges:
        import ipaddress
        if t != "LoadBalancer":
            errs.append("spec.loadBalancerSourceRanges: Forbidden: may only be used when `type` is 'LoadBalancer'")
        for i, r in enumerate(ranges):
            try:
                ipaddress.ip_network(str(r).strip(), strict=False)
            except ValueError:
                errs.append(f"spec.loadBalancerSourceRanges[{i}]: Invalid value: {go_value(r)}: must be a list of IP ranges. "
                            "For example, 10.240.0.0/24,10.250.0.0/24")
    return errs


def default_service(svc: dict):
    spec = svc.setdefault("spec", {})
    spec.setdefault("type", "ClusterIP")
    spec.setdefault("sessionAffinity", "None")
    if spec["type"] in ("NodePort", "LoadBalancer"):
        spec.setdefault("externalTrafficPolicy", "Cluster")     # SetDefaults_Service
    for p in spec.get("ports") or []:
        p.setdefault("protocol", "TCP")
        p.setdefault("targetPort", p.get("port"))
