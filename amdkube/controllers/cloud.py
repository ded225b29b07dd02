"""Cloud-backed controllers: service load balancers and pod-CIDR routes.

Reference:
  * pkg/controller/service/service_controller.go — a Service of type LoadBalancer gets
    EnsureLoadBalancer(cluster, service, ready non-master nodes) and the result in
    status.loadBalancer; a service that stops being a LoadBalancer, or is deleted, gets
    EnsureLoadBalancerDeleted; node-set changes call UpdateLoadBalancer for every balancer.
  * pkg/controller/route/route_controller.go — every node with a spec.podCIDR gets a cloud
    route <cluster>-<node uid> → podCIDR; routes whose node is gone are deleted; the node's
    NetworkUnavailable condition goes False once its route exists.
"""
from __future__ import annotations

import asyncio
import ipaddress
import logging

from ..api import meta as m
from ..api.helpers import is_node_ready
from ..cloudprovider import Route
from .base import Controller, split_key

log = logging.getLogger("amdkube.controllers.cloud")
MASTER_LABEL = "node-role.kubernetes.io/master"


class ServiceLBController(Controller):
    name = "service"
    workers = 1

    def __init__(self, mgr, cloud, cluster_name: str = "kubernetes"):
        super().__init__(mgr)
        self.cloud, self.cluster = cloud, cluster_name
        self.known: dict[str, dict] = {}   # services with a balancer

    def setup(self):
        self.svc_inf = self.mgr.factory.informer("services")
        self.node_inf = self.mgr.nodes
        self.svc_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n), on_delete=self.enqueue)
        self.node_inf.add_handler(on_add=lambda n: self._nodes(), on_delete=lambda n: self._nodes(),
                                  on_update=lambda o, n: self._nodes() if is_node_ready(o) != is_node_ready(n) else None)

    def _nodes(self):
        self.enqueue("@nodes")

    def lb_nodes(self):
        return [n for n in self.node_inf.list() if is_node_ready(n) and MASTER_LABEL not in m.labels_of(n)]

    async def sync(self, key):
        lb = self.cloud.load_balancer() if self.cloud else None
        if lb is None:
            return
        if key == "@nodes":
            nodes = self.lb_nodes()
            for k, svc in list(self.known.items()):
                await asyncio.to_thread(lb.update, self.cluster, svc, nodes)
            return
        svc = self.svc_inf.get(key)
        wants = svc is not None and (svc.get("spec") or {}).get("type") == "LoadBalancer" \
            and not (svc.get("metadata") or {}).get("deletionTimestamp")
        if not wants:
            old = self.known.pop(key, None)
            if old is not None:
                await asyncio.to_thread(lb.ensure_deleted, self.cluster, old)
                if svc is not None and ((svc.get("status") or {}).get("loadBalancer") or {}).get("ingress"):
                    ns, name = split_key(key)
                    await self.client.patch("services", name, {"status": {"loadBalancer": {}}}, ns, sub="status")
            return
        st = await asyncio.get_running_loop().run_in_executor(None, lb.ensure, self.cluster, svc, self.lb_nodes())
        self.known[key] = svc
        if ((svc.get("status") or {}).get("loadBalancer") or {}) != st:
            ns, name = split_key(key)
            await self.client.patch("services", name, {"status": {"loadBalancer": st}}, ns, sub="status")


class RouteController(Controller):
    name = "route"
    workers = 1
    period = 10.0

    def __init__(self, mgr, cloud, cluster_name: str = "kubernetes", cluster_cidr: str = "10.244.0.0/16"):
        super().__init__(mgr)
        self.cloud, self.cluster = cloud, cluster_name
        self.cluster_cidr = ipaddress.ip_network(cluster_cidr, strict=False)
        self._poll = None

    def responsible_for(self, r) -> bool:
        """route_controller.go:264-275 isResponsibleForRoute: only routes whose destination
        (first and last address) lies inside --cluster-cidr are ours to delete — a NAT default
        route or a tenant route in the same table is never touched."""
        try:
            net = ipaddress.ip_network(r.destination_cidr, strict=False)
        except ValueError:
            return False
        c = self.cluster_cidr
        return net.version == c.version and c[0] <= net[0] and net[-1] <= c[-1]

    def setup(self):
        self.node_inf = self.mgr.nodes
        self.node_inf.add_handler(on_add=lambda n: self.enqueue("@all"), on_update=lambda o, n: self.enqueue("@all")
                                  if (o.get("spec") or {}).get("podCIDR") != (n.get("spec") or {}).get("podCIDR") else None,
                                  on_delete=lambda n: self.enqueue("@all"))

    async def start(self):
        await super().start()
        self._poll = asyncio.create_task(self._loop())

    async def stop(self):
        if self._poll:
            self._poll.cancel()
        await super().stop()

    async def _loop(self):
        while True:
            await asyncio.sleep(self.period)
            self.enqueue("@all")

    async def sync(self, key):
        """route_controller.go reconcile: one route per node with a podCIDR (compared by target
        node and CIDR, the way cloud route tables are keyed), stale ones removed."""
        routes = self.cloud.routes() if self.cloud else None
        if routes is None:
            return
        have = await asyncio.to_thread(routes.list, self.cluster)
        want = {}
        for n in self.node_inf.list():
            cidr = (n.get("spec") or {}).get("podCIDR")
            if cidr:
                want[m.name_of(n)] = Route(f"{self.cluster}-{m.uid_of(n)}", m.name_of(n), cidr)
                ip = next((a["address"] for a in (n.get("status") or {}).get("addresses") or [] if a.get("type") == "InternalIP"), None)
                if ip and hasattr(routes, "node_ips"):
                    routes.node_ips[m.name_of(n)] = ip
        present = {(r.target_node, r.destination_cidr) for r in have}
        for node, r in want.items():
            if (node, r.destination_cidr) not in present:
                await asyncio.to_thread(routes.create, self.cluster, r.name, r)
        for r in have:
            w = want.get(r.target_node)
            if (w is None or w.destination_cidr != r.destination_cidr) and self.responsible_for(r):
                await asyncio.to_thread(routes.delete, self.cluster, r)
        for n in self.node_inf.list():
            if m.name_of(n) not in want:
                continue
            conds = (n.get("status") or {}).get("conditions") or []
            cur = next((c for c in conds if c.get("type") == "NetworkUnavailable"), None)
            if cur is None or cur.get("status") != "False":
                cond = {"type": "NetworkUnavailable", "status": "False", "reason": "RouteCreated",
                        "message": "RouteController created a route", "lastTransitionTime": m.now_rfc3339()}
                await self.client.patch("nodes", m.name_of(n), {"status": {"conditions": [cond]}}, sub="status",
                                        patch_type="application/strategic-merge-patch+json")


CLOUD_TAINT = "node.cloudprovider.kubernetes.io/uninitialized"
PROVIDED_IP_ANN = "alpha.kubernetes.io/provided-node-ip"
INSTANCE_TYPE_LABEL = "beta.kubernetes.io/instance-type"
ZONE_LABEL = "failure-domain.beta.kubernetes.io/zone"
REGION_LABEL = "failure-domain.beta.kubernetes.io/region"
PVL_INITIALIZER = "pvl.kubernetes.io"


class CloudNodeController(Controller):
    """pkg/controller/cloud/node_controller.go (cloud-controller-manager): a kubelet started
    with --cloud-provider=external registers tainted `node.cloudprovider.kubernetes.io/
    uninitialized`; this controller then fills in what only the cloud knows — spec.providerID,
    status.addresses (keeping the kubelet's --node-ip, annotated alpha.kubernetes.io/
    provided-node-ip, and the hostname), the instance-type label and zone/region labels — and
    removes the taint. Every `status_period` it refreshes addresses; every `monitor_period` it
    deletes nodes that are not Ready and that the cloud says no longer exist."""
    name = "cloud-node"
    workers = 1

    def __init__(self, mgr, cloud, status_period: float = 300.0, monitor_period: float = 5.0):
        super().__init__(mgr)
        self.cloud = cloud
        self.status_period, self.monitor_period = status_period, monitor_period
        self._loops: list[asyncio.Task] = []

    def setup(self):
        self.node_inf = self.mgr.nodes
        self.node_inf.add_handler(on_add=self.enqueue, on_update=lambda o, n: self.enqueue(n)
                                  if _cloud_taint(n) is not None else None)

    async def start(self):
        await super().start()
        self._loops = [asyncio.create_task(self._every(self.status_period, self.update_node_status)),
                       asyncio.create_task(self._every(self.monitor_period, self.monitor_nodes))]

    async def stop(self):
        for t in self._loops:
            t.cancel()
        await super().stop()

    async def _every(self, period, fn):
        while True:
            await asyncio.sleep(period)
            try:
                await fn()
            except Exception as e:
                import logging
                logging.getLogger("amdkube.controllers.cloud").warning("%s: %r", fn.__name__, e)

    @staticmethod
    def _addresses(node, addrs: list[dict]) -> list[dict] | None:
        """ensureNodeProvidedIPExists + hostname preservation; None: the provided IP is not
        among the cloud's addresses (leave the node alone)."""
        addrs = [dict(a) for a in addrs]
        if not any(a.get("type") == "Hostname" for a in addrs):
            addrs += [a for a in (node.get("status") or {}).get("addresses") or [] if a.get("type") == "Hostname"]
        provided = m.annotations_of(node).get(PROVIDED_IP_ANN)
        if provided:
            hit = next((a for a in addrs if a.get("address") == provided), None)
            if hit is None:
                return None
            addrs = [hit] + [a for a in addrs if a.get("type") == "Hostname"]
        return addrs

    async def sync(self, key):
        _, name = split_key(key)
        node = self.node_inf.get(name)
        if node is None or _cloud_taint(node) is None:
            return
        inst = self.cloud.instances() if self.cloud else None
        if inst is None:
            return
        node = await self.client.get("nodes", name)
        spec = dict(node.get("spec") or {})
        if not spec.get("providerID"):
            spec["providerID"] = await inst.instance_id(name)
        addrs = self._addresses(node, await inst.node_addresses(name))
        if addrs is None:
            return           # the kubelet's --node-ip is not one of the instance's addresses
        labels = dict(m.labels_of(node))
        itype = await inst.instance_type(name)
        if itype:
            labels[INSTANCE_TYPE_LABEL] = itype
        zone = await asyncio.to_thread(self.cloud.zone_for_node, name) if hasattr(self.cloud, "zone_for_node") \
            else self.cloud.zones()
        if zone is not None and zone.failure_domain:
            labels[ZONE_LABEL] = zone.failure_domain
        if zone is not None and zone.region:
            labels[REGION_LABEL] = zone.region
        spec["taints"] = [t for t in spec.get("taints") or [] if t.get("key") != CLOUD_TAINT] or None
        await self.client.patch("nodes", name, {"metadata": {"labels": labels}, "spec": {"providerID": spec["providerID"],
                                                                                        "taints": spec["taints"]}})
        if addrs and addrs != ((node.get("status") or {}).get("addresses") or []):
            await self.client.patch("nodes", name, {"status": {"addresses": addrs}}, sub="status")
        self.mgr.recorder.event({"kind": "Node", "metadata": {"name": name, "uid": m.uid_of(node)}}, "Normal",
                                "Initialized", f"Node {name} initialized by the {getattr(self.cloud, 'name', 'cloud')} provider")

    async def update_node_status(self):
        inst = self.cloud.instances() if self.cloud else None
        if inst is None:
            return
        for node in self.node_inf.list():
            if _cloud_taint(node) is not None:
                continue
            name = m.name_of(node)
            try:
                if not await inst.instance_exists(name):
                    continue
                addrs = self._addresses(node, await inst.node_addresses(name))
            except LookupError:
                continue
            if addrs and addrs != ((node.get("status") or {}).get("addresses") or []):
                await self.client.patch("nodes", name, {"status": {"addresses": addrs}}, sub="status")

    async def monitor_nodes(self):
        inst = self.cloud.instances() if self.cloud else None
        if inst is None:
            return
        for node in self.node_inf.list():
            ready = next((c for c in (node.get("status") or {}).get("conditions") or [] if c.get("type") == "Ready"), None)
            if ready is None or ready.get("status") == "True":
                continue
            pid = (node.get("spec") or {}).get("providerID")
            try:
                exists = await inst.instance_exists_by_provider_id(pid) if pid and hasattr(inst, "instance_exists_by_provider_id") \
                    else await inst.instance_exists(m.name_of(node))
            except Exception as e:      # noqa: BLE001 — a cloud that cannot tell (or is unreachable) keeps the node
                log.warning("cloud existence check for node %s: %r", m.name_of(node), e)
                continue
            if exists:
                continue
            self.mgr.recorder.event({"kind": "Node", "metadata": {"name": m.name_of(node), "uid": m.uid_of(node)}}, "Normal",
                                    "DeletingNode", f"Deleting Node {m.name_of(node)} because it's not present according to "
                                                    "cloud provider")
            try:
                await self.client.delete("nodes", m.name_of(node))
            except m.StatusError as e:
                if not m.is_not_found(e):
                    raise


def _cloud_taint(node):
    return next((t for t in (node.get("spec") or {}).get("taints") or [] if t.get("key") == CLOUD_TAINT), None)


class PersistentVolumeLabelController(Controller):
    """pkg/controller/cloud/pvlcontroller.go: PersistentVolumes created with the pending
    initializer `pvl.kubernetes.io` get the cloud's labels for them (zone / region) and the
    initializer removed, which publishes them."""
    name = "persistentvolume-labeler"
    workers = 1

    def __init__(self, mgr, cloud, period: float = 0.5):
        super().__init__(mgr)
        self.cloud, self.period = cloud, period
        self._poll = None
        self.pending: dict[str, dict] = {}

    async def start(self):
        await super().start()
        self._poll = asyncio.create_task(self._loop())

    async def stop(self):
        if self._poll:
            self._poll.cancel()
        await super().stop()

    async def _loop(self):
        """Uninitialized objects are invisible to ordinary lists and watches: poll with
        includeUninitialized for the volumes still waiting on this initializer."""
        while True:
            try:
                lst = await self.client.request("GET", "/api/v1/persistentvolumes", params={"includeUninitialized": "true"})
                for pv in lst.get("items") or []:
                    pend = (((pv.get("metadata") or {}).get("initializers")) or {}).get("pending") or []
                    if pend and pend[0].get("name") == PVL_INITIALIZER:
                        self.pending[m.name_of(pv)] = pv
                        self.enqueue(m.name_of(pv))
            except Exception as e:
                import logging
                logging.getLogger("amdkube.controllers.cloud").debug("pvl list: %r", e)
            await asyncio.sleep(self.period)

    async def sync(self, key):
        _, name = split_key(key)
        pv = self.pending.pop(name, None)
        pending = (((pv or {}).get("metadata") or {}).get("initializers") or {}).get("pending") or []
        if not pending or pending[0].get("name") != PVL_INITIALIZER:
            return
        labels = await asyncio.to_thread(self.cloud.labels_for_volume, pv) if hasattr(self.cloud, "labels_for_volume") else {}
        rest = [p for p in pending if p.get("name") != PVL_INITIALIZER]
        patch = {"metadata": {"initializers": {"pending": rest} if rest else None}}
        if labels:
            patch["metadata"]["labels"] = {**m.labels_of(pv), **labels}
        await self.client.request("PATCH", f"/api/v1/persistentvolumes/{name}", params={"includeUninitialized": "true"},
                                  body=patch, content_type="application/merge-patch+json")
