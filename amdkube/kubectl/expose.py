"""kubectl expose and the service/v2 generator.

Reference: pkg/kubectl/cmd/expose.go RunExpose (:150-330) and pkg/kubectl/service.go —
  * exposable kinds: Pod, Service, ReplicationController, Deployment, ReplicaSet (CanBeExposed);
  * the selector: --selector, else the object's (MapBasedSelectorForObject: a pod's labels, a
    service's or RC's selector, a Deployment's/ReplicaSet's matchLabels — matchExpressions
    cannot be expressed);
  * the ports: --port, else every container port of the object (PortsForObject; a service's
    ports), several ports named port-1, port-2, ...; their protocols come from the object
    (ProtocolsForObject) unless --protocol; --target-port (or --container-port) for all ports,
    else each targets itself; no port is an error unless --cluster-ip=None (headless);
  * the labels: -l/--labels, else the object's own labels; the name: --name, else the object's
    (cut to 63 characters);
  * --type, --external-ip, --load-balancer-ip (LoadBalancer only), --session-affinity
    (None|ClientIP), --cluster-ip (None = headless), --overrides, --dry-run, -o;
  * `service "x" exposed`.
"""
from __future__ import annotations

import json
import sys

from ..api import meta as m
from ..api.scheme import SCHEME
from .drain import print_success
from .metacmds import UsageError, resource_arg
from .run import GenerateError, parse_labels_spec

EXPOSABLE = {"Pod", "Service", "ReplicationController", "Deployment", "ReplicaSet"}
PATCH_TYPES = ("strategic", "merge", "json")


def selector_for(obj: dict) -> str:
    """MapBasedSelectorForObject as `k=v,...`."""
    kind = obj.get("kind")
    spec = obj.get("spec") or {}
    if kind == "Pod":
        labels = m.labels_of(obj)
        if not labels:
            raise UsageError("the pod has no labels and cannot be exposed")
        sel = labels
    elif kind == "Service":
        sel = spec.get("selector") or {}
        if not sel:
            raise UsageError("the service has no pod selector set")
    elif kind == "ReplicationController":
        sel = spec.get("selector") or {}
    else:
        s = spec.get("selector") or {}
        if s.get("matchExpressions"):
            raise UsageError(f'couldn\'t convert expressions - "{s["matchExpressions"]}" to map-based selector format')
        sel = s.get("matchLabels") or {}
    return ",".join(f"{k}={v}" for k, v in sel.items())


def _containers(obj):
    spec = obj.get("spec") or {}
    if obj.get("kind") == "Pod":
        return spec.get("containers") or []
    return ((spec.get("template") or {}).get("spec") or {}).get("containers") or []


def ports_for(obj: dict) -> list[str]:
    if obj.get("kind") == "Service":
        return [str(p["port"]) for p in (obj.get("spec") or {}).get("ports") or []]
    return [str(p["containerPort"]) for c in _containers(obj) for p in c.get("ports") or []]


def protocols_for(obj: dict) -> dict:
    if obj.get("kind") == "Service":
        return {str(p["port"]): p.get("protocol", "TCP") for p in (obj.get("spec") or {}).get("ports") or []}
    return {str(p["containerPort"]): p.get("protocol", "TCP") for c in _containers(obj) for p in c.get("ports") or []}


def generate_service_v2(params: dict) -> dict:
    """ServiceGeneratorV2.Generate from string parameters."""
    sel_s = params.get("selector") or ""
    if not sel_s:
        raise GenerateError("'selector' is a required parameter.")
    selector = parse_labels_spec(sel_s)
    labels = parse_labels_spec(params["labels"]) if params.get("labels") else None
    name = params.get("name") or params.get("default-name")
    if not name:
        raise GenerateError("'name' is a required parameter.")
    headless = params.get("cluster-ip") == "None"
    proto_map = {}
    if params.get("protocols"):
        for item in params["protocols"].split(","):
            pp = item.split("/")
            if len(pp) != 2:
                raise GenerateError(f"unexpected port protocol mapping: {item}")
            if not pp[0]:
                raise GenerateError("unexpected empty port")
            if not pp[1]:
                raise GenerateError("unexpected empty protocol")
            proto_map[pp[0]] = pp[1]
    port_s = params.get("ports") if "ports" in params else params.get("port")
    if port_s is None and not headless:
        raise GenerateError("'ports' or 'port' is a required parameter.")
    ports = []
    if port_s:
        parts = port_s.split(",")
        for i, ps in enumerate(parts):
            try:
                port = int(ps)
            except ValueError:
                raise GenerateError(f'strconv.Atoi: parsing "{ps}": invalid syntax') from None
            proto = params.get("protocol") or ""
            if not proto:
                proto = proto_map.get(ps, "TCP") if proto_map else "TCP"
            p = {"port": port, "protocol": proto}
            name_p = f"port-{i + 1}" if len(parts) > 1 else (params.get("port-name") or "")
            if name_p:
                p = {"name": name_p, **p}
            ports.append(p)
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name}, "spec": {"selector": selector, "ports": ports}}
    if labels:
        svc["metadata"]["labels"] = labels
    target = params.get("target-port") or params.get("container-port") or ""
    for p in ports:
        p["targetPort"] = (int(target) if target.isdigit() else target) if target else p["port"]
    if params.get("external-ip"):
        svc["spec"]["externalIPs"] = [params["external-ip"]]
    if params.get("type"):
        svc["spec"]["type"] = params["type"]
    if svc["spec"].get("type") == "LoadBalancer" and params.get("load-balancer-ip"):
        svc["spec"]["loadBalancerIP"] = params["load-balancer-ip"]
    aff = params.get("session-affinity")
    if aff:
        if aff not in ("None", "ClientIP"):
            raise GenerateError(f"unknown session affinity: {aff}")
        svc["spec"]["sessionAffinity"] = aff
    if params.get("cluster-ip"):
        svc["spec"]["clusterIP"] = params["cluster-ip"]
    return svc


async def cmd_expose(c, a):
    from ..api.strategicpatch import apply as strategic_merge
    from .metacmds import resolve_targets
    try:
        targets = await resolve_targets(c, a, list(a.args), a.namespace or "default")
        if not targets:
            raise UsageError("You must provide one or more resources by argument or filename.")
        for ri, obj in targets:
            obj.setdefault("kind", ri.kind)
            if ri.kind not in EXPOSABLE:
                raise UsageError(f"cannot expose a {{{ri.group} {ri.kind}}}")
            name = m.name_of(obj)[:63]
            params = {"default-name": name, "name": a.name or "", "selector": getattr(a, "expose_selector", None) or "",
                      "labels": getattr(a, "expose_labels", None) or "", "port": a.port or "",
                      "protocol": a.protocol or "", "target-port": a.target_port or "",
                      "container-port": getattr(a, "container_port", None) or "",
                      "external-ip": getattr(a, "external_ip", None) or "", "load-balancer-ip": getattr(a, "load_balancer_ip", None) or "",
                      "type": "" if a.type in PATCH_TYPES else (a.type or ""),
                      "session-affinity": getattr(a, "session_affinity", None) or "",
                      "cluster-ip": getattr(a, "cluster_ip", None) or "", "port-name": ""}
            if not params["selector"]:
                try:
                    params["selector"] = selector_for(obj)
                except UsageError as e:
                    raise UsageError(f"couldn't retrieve selectors via --selector flag or introspection: {e}") from None
            headless = params["cluster-ip"] == "None"
            if not params["port"]:
                ports = ports_for(obj)
                if not ports and not headless:
                    raise UsageError("couldn't find port via --port flag or introspection")
                if len(ports) == 1:
                    params["port"] = ports[0]
                elif ports:
                    params["ports"] = ",".join(ports)
                elif headless:
                    params.pop("port")
            if not params["protocol"]:
                pm = protocols_for(obj)
                if pm:
                    params["protocols"] = ",".join(f"{k}/{v}" for k, v in pm.items())
            if not params["labels"]:
                params["labels"] = ",".join(f"{k}={v}" for k, v in m.labels_of(obj).items())
            svc = generate_service_v2(params)
            if getattr(a, "overrides", None):
                svc = strategic_merge(svc, json.loads(a.overrides))
            if a.dry_run:
                if a.output:
                    from .run import _print
                    _print(svc, a.output)
                else:
                    print_success("service", m.name_of(svc), "exposed", True)
                continue
            out = await c.create(svc, a.namespace or "default")
            if a.output:
                from .run import _print
                _print(out, a.output)
            else:
                print_success("service", m.name_of(out), "exposed")
    except (UsageError, GenerateError) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    return 0


def rewrite_flags(argv: list[str]) -> list[str]:
    """In `expose`, -l/--labels are the service's labels and --selector the pod selector."""
    if "expose" not in argv:
        return argv
    i = argv.index("expose")
    out = argv[:i + 1]
    for t in argv[i + 1:]:
        if t in ("-l", "--labels"):
            out.append("--expose-labels")
        elif t.startswith("--labels="):
            out.append("--expose-labels=" + t.split("=", 1)[1])
        elif t == "--selector":
            out.append("--expose-selector")
        elif t.startswith("--selector="):
            out.append("--expose-selector=" + t.split("=", 1)[1])
        else:
            out.append(t)
    return out


def add_arguments(sp):
    sp.add_argument("--expose-labels", default=None)
    sp.add_argument("--expose-selector", default=None)
    sp.add_argument("--container-port", default=None)
    sp.add_argument("--external-ip", default=None)
    sp.add_argument("--load-balancer-ip", default=None)
    sp.add_argument("--session-affinity", default=None)
    sp.add_argument("--cluster-ip", default=None)
