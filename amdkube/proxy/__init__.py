"""kube-proxy equivalent (reference cmd/kube-proxy, pkg/proxy).

ProxyServer watches services and endpoints and drives one proxier:
  * `userspace`: real listeners per service port with round-robin / ClientIP affinity;
  * `iptables`: the reference's nat/filter ruleset, applied with iptables-restore when
    privileged, otherwise rendered (dry run);
  * `ipvs`: IPVS virtual servers plus the iptables masquerade linkage.
For externalTrafficPolicy=Local services it serves each healthCheckNodePort
(proxy/healthcheck.py).
It serves /healthz on --healthz-port (reference healthcheck.go: 503 once the last
successful sync is older than 2 × the sync period) and /metrics with
kubeproxy_sync_proxy_rules_latency_microseconds.
"""
from __future__ import annotations

import asyncio
import logging
import time

from aiohttp import web

from ..client import Client, Informer
from ..utils.metrics import CONTENT_TYPE, MICRO_BUCKETS, Histogram, new_registry, render
from .config import ChangeTracker, ServiceInfo, ServicePortName  # noqa: F401
from .iptables import IptablesProxier
from .userspace import LoadBalancerRR, UserspaceProxier  # noqa: F401
from ..utils import wait_event

log = logging.getLogger("amdkube.proxy")


class ProxyServer:
    def __init__(self, client: Client, mode: str = "userspace", node_ip: str = "0.0.0.0", cluster_cidr: str = "",
                 sync_period: float = 30.0, min_sync_period: float = 0.0, healthz_port: int | None = None,
                 iptables_dump: str | None = None, bind_cluster_ips: bool = True, ipvs_scheduler: str = "rr",
                 masquerade_all: bool = False, masquerade_bit: int = 14, healthz_address: str = "127.0.0.1",
                 udp_idle_timeout: float = 0.25, metrics_address: tuple | None = None, hostname: str = ""):
        self.client = client
        self.hostname = hostname
        nip = node_ip if node_ip not in ("", "0.0.0.0") else ""
        if mode == "iptables":
            self.proxier = IptablesProxier(cluster_cidr, dump_path=iptables_dump, masquerade_all=masquerade_all,
                                           masquerade_bit=masquerade_bit, hostname=hostname, node_ip=nip)
        elif mode == "ipvs":
            from .ipvs import IPVSProxier
            self.proxier = IPVSProxier(cluster_cidr, ipvs_scheduler, node_ips=[nip] if nip else [],
                                       masquerade_all=masquerade_all, dump_path=iptables_dump, hostname=hostname,
                                       masquerade_bit=masquerade_bit)
        elif mode == "userspace":
            self.proxier = UserspaceProxier(node_ip, bind_cluster_ips=bind_cluster_ips, udp_idle_timeout=udp_idle_timeout)
        else:
            raise ValueError(f"unknown proxy mode {mode!r} (userspace|iptables|ipvs)")
        self.tracker = ChangeTracker()
        # healthCheckNodePort listeners for externalTrafficPolicy=Local (iptables and ipvs modes)
        from .healthcheck import HealthCheckServer
        self.health = HealthCheckServer(hostname) if mode in ("iptables", "ipvs") else None
        self.sync_period, self.min_sync_period = sync_period, min_sync_period
        self.healthz_port = healthz_port
        self.healthz_address = healthz_address
        self.metrics_address = metrics_address          # --metrics-bind-address (host, port) or None
        self.metrics = new_registry()
        self.m_sync = Histogram("kubeproxy_sync_proxy_rules_latency_microseconds", "SyncProxyRules latency",
                                buckets=MICRO_BUCKETS, registry=self.metrics)
        self._wake = asyncio.Event()
        self.last_sync = 0.0
        self._tasks: list[asyncio.Task] = []
        self._runner = None
        self.svc_inf = Informer(client, "services")
        self.ep_inf = Informer(client, "endpoints")

    def _changed(self):
        self._wake.set()

    async def start(self):
        t = self.tracker
        self.svc_inf.add_handler(on_add=lambda o: (t.on_service(o), self._changed()),
                                 on_update=lambda o, n: (t.on_service(n), self._changed()),
                                 on_delete=lambda o: (t.on_service(o, deleted=True), self._changed()))
        self.ep_inf.add_handler(on_add=lambda o: (t.on_endpoints(o), self._changed()),
                                on_update=lambda o, n: (t.on_endpoints(n), self._changed()),
                                on_delete=lambda o: (t.on_endpoints(o, deleted=True), self._changed()))
        self.svc_inf.start()
        self.ep_inf.start()
        await self.svc_inf.wait_synced(30)
        await self.ep_inf.wait_synced(30)
        await self.sync()
        self._tasks.append(asyncio.create_task(self._loop(), name="proxy-sync"))
        if self.healthz_port is not None:
            app = web.Application()
            app.router.add_get("/healthz", self._healthz)
            app.router.add_get("/metrics", self._metrics)
            self._runner = web.AppRunner(app, access_log=None)
            await self._runner.setup()
            site = web.TCPSite(self._runner, self.healthz_address, self.healthz_port)
            await site.start()
            self.healthz_port = site._server.sockets[0].getsockname()[1]
            if self.metrics_address and self.metrics_address[1]:
                try:
                    await web.TCPSite(self._runner, *self.metrics_address).start()
                except OSError as e:
                    log.warning("metrics listener %s: %s", self.metrics_address, e)
        return self

    async def sync(self):
        t0 = time.perf_counter()
        self.tracker.dirty = False
        svcs, eps = self.tracker.service_map(), self.tracker.endpoint_map()
        await self.proxier.sync(svcs, eps)
        if self.health is not None:
            from .iptables import health_check_state
            hc_svcs, hc_eps = health_check_state(svcs, eps, self.hostname)
            await self.health.sync_services(hc_svcs)
            self.health.sync_endpoints(hc_eps)
        self.last_sync = time.time()
        self.m_sync.observe((time.perf_counter() - t0) * 1e6)

    async def _loop(self):
        while True:
            await wait_event(self._wake, self.sync_period)
            self._wake.clear()
            if self.min_sync_period:
                wait = self.last_sync + self.min_sync_period - time.time()
                if wait > 0:
                    await asyncio.sleep(wait)   # BoundedFrequencyRunner minInterval
            try:
                await self.sync()
            except Exception as e:
                log.warning("proxy sync failed: %r", e)
                await asyncio.sleep(1.0)
                self._wake.set()

    async def _healthz(self, request):
        age = time.time() - self.last_sync
        ok = age < max(2 * self.sync_period, 1.0) or not self.tracker.dirty
        body = {"lastUpdated": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(self.last_sync)),
                "currentTime": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
        return web.json_response(body, status=200 if ok else 503)

    async def _metrics(self, request):
        return web.Response(body=render(self.metrics), headers={"Content-Type": CONTENT_TYPE})

    async def stop(self):
        for t in self._tasks:
            t.cancel()
        await self.svc_inf.stop()
        await self.ep_inf.stop()
        await self.proxier.stop()
        if self.health is not None:
            await self.health.stop()
        if self._runner:
            await self._runner.cleanup()
