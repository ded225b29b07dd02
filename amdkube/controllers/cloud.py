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

from ..api import meta as m
from ..api.helpers import is_node_ready
from ..cloudprovider import Route
from .base import Controller, split_key

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
                lb.update(self.cluster, svc, nodes)
            return
        svc = self.svc_inf.get(key)
        wants = svc is not None and (svc.get("spec") or {}).get("type") == "LoadBalancer" \
            and not (svc.get("metadata") or {}).get("deletionTimestamp")
        if not wants:
            old = self.known.pop(key, None)
            if old is not None:
                lb.ensure_deleted(self.cluster, old)
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

    def __init__(self, mgr, cloud, cluster_name: str = "kubernetes"):
        super().__init__(mgr)
        self.cloud, self.cluster = cloud, cluster_name
        self._poll = None

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
        routes = self.cloud.routes() if self.cloud else None
        if routes is None:
            return
        have = {r.name: r for r in routes.list(self.cluster)}
        want = {}
        for n in self.node_inf.list():
            cidr = (n.get("spec") or {}).get("podCIDR")
            if cidr:
                want[f"{self.cluster}-{m.uid_of(n)}"] = Route(f"{self.cluster}-{m.uid_of(n)}", m.name_of(n), cidr)
                ip = next((a["address"] for a in (n.get("status") or {}).get("addresses") or [] if a.get("type") == "InternalIP"), None)
                if ip and hasattr(routes, "node_ips"):
                    routes.node_ips[m.name_of(n)] = ip
        for name, r in want.items():
            if have.get(name) != r:
                routes.create(self.cluster, name, r)
        for name, r in have.items():
            if name.startswith(self.cluster + "-") and name not in want:
                routes.delete(self.cluster, r)
        for n in self.node_inf.list():
            if f"{self.cluster}-{m.uid_of(n)}" not in want:
                continue
            conds = (n.get("status") or {}).get("conditions") or []
            cur = next((c for c in conds if c.get("type") == "NetworkUnavailable"), None)
            if cur is None or cur.get("status") != "False":
                cond = {"type": "NetworkUnavailable", "status": "False", "reason": "RouteCreated",
                        "message": "RouteController created a route", "lastTransitionTime": m.now_rfc3339()}
                await self.client.patch("nodes", m.name_of(n), {"status": {"conditions": [cond]}}, sub="status",
                                        patch_type="application/strategic-merge-patch+json")
