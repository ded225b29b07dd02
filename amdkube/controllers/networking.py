"""Networking controllers: Endpoints and node IPAM (pod CIDR per node).

Reference:
  * pkg/controller/endpoint/endpoints_controller.go — syncService: for a service with a
    selector, every pod with a podIP that matches it (not being deleted, unless the service
    tolerates unready endpoints) contributes one address per service port (targetPort by
    number or container-port name, podutil.FindPort; a headless service without ports gets
    port 0); ready pods go to `addresses`, unready ones to `notReadyAddresses` if
    shouldPodBeInEndpoints; subsets are repacked (pkg/api/v1/endpoints RepackSubsets: per
    port, not-ready trumping ready, ports with the same addresses merged); the Endpoints
    object is created, or updated only when subsets or labels changed, and deleted with its
    service; updatePod enqueues per podChanged / determineNeededServiceUpdates, and leftover
    Endpoints are re-synced at start.
  * pkg/controller/node/ipam/range_allocator.go — `--allocate-node-cidrs`: each node gets
    the next free `--node-cidr-mask-size` block of `--cluster-cidr` in spec.podCIDR; the
    in-use set is rebuilt from existing nodes, and a deleted node's CIDR is released.
"""
from __future__ import annotations

import ipaddress

from ..api import meta as m
from ..api.helpers import is_pod_ready
from ..api.labels import selector_from_set
from .base import Controller, split_key

TOLERATE_UNREADY = "service.alpha.kubernetes.io/tolerate-unready-endpoints"
LEADER_ANNOTATION = "control-plane.alpha.kubernetes.io/leader"


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


def should_pod_be_in_endpoints(pod: dict) -> bool:
    """shouldPodBeInEndpoints: a pod that will not run again (restartPolicy Never and done, or
    OnFailure and succeeded) is not even a not-ready address."""
    rp = (pod.get("spec") or {}).get("restartPolicy", "Always")
    phase = (pod.get("status") or {}).get("phase", "")
    if rp == "Never":
        return phase not in ("Failed", "Succeeded")
    if rp == "OnFailure":
        return phase != "Succeeded"
    return True


def pod_to_endpoint_address(pod: dict) -> dict:
    md = pod.get("metadata") or {}
    ref = {"kind": "Pod", "namespace": md.get("namespace", ""), "name": md.get("name", "")}
    if md.get("uid"):
        ref["uid"] = md["uid"]
    if md.get("resourceVersion"):
        ref["resourceVersion"] = md["resourceVersion"]
    return {"ip": (pod.get("status") or {}).get("podIP", ""), "nodeName": (pod.get("spec") or {}).get("nodeName", ""),
            "targetRef": ref}


def _canon(o) -> str:
    import json
    return json.dumps(o, sort_keys=True, separators=(",", ":"))


def _addr_order(a: dict):
    """LessEndpointAddress: by IP, an address without a targetRef first, then by UID."""
    ref = a.get("targetRef")
    return (a.get("ip", ""), ref is not None, (ref or {}).get("uid", ""))


def sort_subsets(subsets: list[dict]) -> list[dict]:
    """SortSubsets: addresses by IP and UID; ports and subsets in a canonical order (the reference
    orders them by the md5 of Go's struct dump, which has no meaning beyond being stable)."""
    for ss in subsets:
        for k in ("addresses", "notReadyAddresses"):
            if ss.get(k):
                ss[k].sort(key=_addr_order)
        if ss.get("ports"):
            ss["ports"].sort(key=_canon)
    subsets.sort(key=_canon)
    return subsets


def repack_subsets(subsets: list[dict]) -> list[dict]:
    """endpoints.RepackSubsets: every (address, port) pair — addresses keyed by IP and target UID,
    the first occurrence's address kept, not-ready trumping ready for the same port — regrouped
    so ports served by exactly the same addresses share a subset."""
    addrs: dict[tuple, dict] = {}
    port_to_addrs: dict[str, tuple[dict, dict]] = {}       # canonical port -> (port, {addr key: ready})
    for ss in subsets:
        for port in ss.get("ports") or []:
            for field, ready in (("addresses", True), ("notReadyAddresses", False)):
                for a in ss.get(field) or []:
                    key = (a.get("ip", ""), (a.get("targetRef") or {}).get("uid", ""))
                    addrs.setdefault(key, a)
                    _, amap = port_to_addrs.setdefault(_canon(port), (port, {}))
                    if amap.get(key, True):
                        amap[key] = ready
    groups: dict[str, tuple[dict, list]] = {}
    for port, amap in port_to_addrs.values():
        gk = _canon(sorted([list(k), r] for k, r in amap.items()))
        groups.setdefault(gk, (amap, []))[1].append(port)
    out = []
    for amap, ports in groups.values():
        ss = {}
        ready = [addrs[k] for k, r in amap.items() if r]
        not_ready = [addrs[k] for k, r in amap.items() if not r]
        if ready:
            ss["addresses"] = [dict(a) for a in ready]
        if not_ready:
            ss["notReadyAddresses"] = [dict(a) for a in not_ready]
        ss["ports"] = [dict(p) for p in ports]
        out.append(ss)
    return sort_subsets(out)


def _subsets_equal(a, b) -> bool:
    """apiequality.Semantic.DeepEqual of two subset lists (nil and empty alike)."""
    def norm(x):
        if isinstance(x, dict):
            return {k: norm(v) for k, v in x.items() if v not in (None, [], {}, "")}
        if isinstance(x, list):
            return [norm(v) for v in x]
        return x
    return norm(a or []) == norm(b or [])


def _parse_bool(v: str) -> bool | None:
    """strconv.ParseBool."""
    if v in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if v in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    return None


def pod_changed(old: dict, new: dict) -> bool:
    """podChanged: deletion started, readiness flipped, or the pod's endpoint address (IP, node,
    name, namespace, UID; not its resourceVersion) differs."""
    if ((old.get("metadata") or {}).get("deletionTimestamp")) != ((new.get("metadata") or {}).get("deletionTimestamp")):
        return True
    if is_pod_ready(old) != is_pod_ready(new):
        return True
    a, b = pod_to_endpoint_address(old), pod_to_endpoint_address(new)
    a["targetRef"].pop("resourceVersion", None)
    b["targetRef"].pop("resourceVersion", None)
    return a != b


def determine_needed_service_updates(old: set, new: set, changed: bool) -> set:
    """determineNeededServiceUpdates: all services of both sets when the pod itself changed,
    otherwise only those it joined or left."""
    return (new | old) if changed else (new - old) | (old - new)


def _host_and_domain_equal(a: dict, b: dict) -> bool:
    sa, sb = a.get("spec") or {}, b.get("spec") or {}
    return sa.get("hostname", "") == sb.get("hostname", "") and sa.get("subdomain", "") == sb.get("subdomain", "")


class EndpointsController(Controller):
    """pkg/controller/endpoint/endpoints_controller.go."""
    name = "endpoint"
    workers = 4

    def setup(self):
        f = self.mgr.factory
        self.svc_inf = f.informer("services")
        self.ep_inf = f.informer("endpoints")
        self.pod_inf = self.mgr.pods
        self.svc_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.pod_inf.add_handler(on_add=self._pod, on_update=self._pod_update, on_delete=self._pod)

    async def start(self):
        self.check_leftover_endpoints()
        await super().start()

    def check_leftover_endpoints(self):
        """checkLeftoverEndpoints: every Endpoints object (but leader-election records) is synced
        once at start, so one whose Service went away while the controller was down is deleted."""
        for ep in self.ep_inf.list():
            if LEADER_ANNOTATION in m.annotations_of(ep):
                continue
            self.enqueue(ep)

    def pod_services(self, pod) -> set[str]:
        """getPodServiceMemberships: services of the pod's namespace whose (non-nil) selector matches."""
        ns, labels = m.namespace_of(pod), m.labels_of(pod)
        out = set()
        for svc in self.svc_inf.list():
            if m.namespace_of(svc) != ns:
                continue
            sel = (svc.get("spec") or {}).get("selector")
            if sel and selector_from_set(sel).matches(labels):
                out.add(m.key_of(svc))
        return out

    def _pod(self, pod):
        for key in self.pod_services(pod):
            self.enqueue(key)

    def _pod_update(self, old, new):
        """updatePod: nothing for a resync of the same version; the pod's services when it changed
        in a way its endpoints show; the services it joined or left when its labels (or
        hostname/subdomain) changed."""
        if (old.get("metadata") or {}).get("resourceVersion") == (new.get("metadata") or {}).get("resourceVersion"):
            return
        changed = pod_changed(old, new)
        labels_changed = m.labels_of(old) != m.labels_of(new) or not _host_and_domain_equal(old, new)
        if not changed and not labels_changed:
            return
        services = self.pod_services(new)
        if labels_changed:
            services = determine_needed_service_updates(self.pod_services(old), services, changed)
        for key in services:
            self.enqueue(key)

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
            # services without a selector get their endpoints out of band (an empty selector is
            # dropped on the way through the API, so it is no selector either)
            return
        sel = selector_from_set(spec["selector"])
        tolerate = bool(_parse_bool(m.annotations_of(svc).get(TOLERATE_UNREADY, "")))
        subsets = []
        for pod in self.pod_inf.list():
            if m.namespace_of(pod) != ns or not sel.matches(m.labels_of(pod)):
                continue
            if not (pod.get("status") or {}).get("podIP"):
                continue
            if not tolerate and (pod.get("metadata") or {}).get("deletionTimestamp"):
                continue
            epa = pod_to_endpoint_address(pod)
            pspec = pod.get("spec") or {}
            if pspec.get("hostname") and pspec.get("subdomain") == m.name_of(svc):
                epa["hostname"] = pspec["hostname"]   # per-pod DNS names of a headless service
            ports = []
            if not spec.get("ports"):
                if spec.get("clusterIP") == "None":   # a headless service may have no ports
                    ports.append({"port": 0, "protocol": "TCP"})
            else:
                for sp in spec["ports"]:
                    num = find_port(pod, sp)
                    if num is None:
                        continue
                    epp = {"port": num, "protocol": sp.get("protocol", "TCP")}
                    if sp.get("name"):
                        epp["name"] = sp["name"]
                    ports.append(epp)
            for epp in ports:                          # addEndpointSubset
                if tolerate or is_pod_ready(pod):
                    subsets.append({"addresses": [dict(epa)], "ports": [epp]})
                elif should_pod_be_in_endpoints(pod):
                    subsets.append({"notReadyAddresses": [dict(epa)], "ports": [epp]})
        subsets = repack_subsets(subsets)
        cur = self.ep_inf.get(key)
        want_labels = m.labels_of(svc)
        if cur is not None and _subsets_equal(cur.get("subsets"), subsets) and m.labels_of(cur) == want_labels:
            return
        if cur is None:
            body = {"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": name, "namespace": ns}, "subsets": subsets}
            if want_labels:
                body["metadata"]["labels"] = want_labels
            try:
                await self.client.create(body, ns)
                return
            except m.StatusError as e:
                if not m.is_already_exists(e):
                    raise
                cur = await self.client.get("endpoints", name, ns)
        new = dict(cur, subsets=subsets)
        new["metadata"] = dict(cur.get("metadata") or {}, labels=want_labels)
        if not want_labels:
            new["metadata"].pop("labels", None)
        await self.client.update(new)


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
