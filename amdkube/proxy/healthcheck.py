"""Service health checks for externalTrafficPolicy=Local (pkg/proxy/healthcheck/healthcheck.go).

A LoadBalancer service with externalTrafficPolicy=Local gets a `spec.healthCheckNodePort`
from the apiserver. Every kube-proxy serves HTTP on that port; the cloud load balancer probes
it on each node and only sends traffic to nodes that answer 200, i.e. nodes running at least
one of the service's endpoints (KUBE-XLB drops it elsewhere). The answer (:173-185):

    {"service": {"namespace": "<ns>", "name": "<name>"}, "localEndpoints": <n>}

with status 200 when n > 0, else 503.

`sync_services({(ns, name): port})` opens / closes one listener per service (SyncServices
:97-150; a port that cannot be bound is reported and skipped), and `sync_endpoints({(ns,
name): n})` sets the counts (SyncEndpoints :188-207: a service missing from the map has 0).
"""
from __future__ import annotations

import json
import logging

from aiohttp import web

log = logging.getLogger("amdkube.proxy.healthcheck")


class HealthCheckServer:
    def __init__(self, hostname: str = "", address: str = "0.0.0.0", recorder=None):
        self.hostname, self.address, self.recorder = hostname, address, recorder
        self.services: dict[tuple[str, str], dict] = {}     # nsn -> {port, runner, endpoints}

    def body(self, nsn) -> tuple[int, str]:
        svc = self.services.get(nsn)
        count = svc["endpoints"] if svc else 0
        text = json.dumps({"service": {"namespace": nsn[0], "name": nsn[1]}, "localEndpoints": count}, indent="\t")
        return (200 if count else 503), text

    async def sync_services(self, new: dict[tuple[str, str], int]):
        for nsn in list(self.services):
            svc = self.services[nsn]
            if new.get(nsn) != svc["port"]:
                log.info("closing healthcheck %s/%s on port %d", *nsn, svc["port"])
                await svc["runner"].cleanup()
                del self.services[nsn]
        for nsn, port in new.items():
            if nsn in self.services:
                continue
            app = web.Application()

            async def handle(request, nsn=nsn):
                status, text = self.body(nsn)
                return web.Response(status=status, text=text, content_type="application/json")
            app.router.add_route("GET", "/{tail:.*}", handle)
            runner = web.AppRunner(app, access_log=None)
            await runner.setup()
            try:
                site = web.TCPSite(runner, self.address, port, reuse_address=True)
                await site.start()
            except OSError as e:
                await runner.cleanup()
                msg = f"node {self.hostname} failed to start healthcheck \"{nsn[0]}/{nsn[1]}\" on port {port}: {e}"
                log.error(msg)
                if self.recorder is not None:
                    self.recorder.event({"kind": "Service", "namespace": nsn[0], "name": nsn[1]}, "Warning",
                                        "FailedToStartServiceHealthcheck", msg)
                continue
            log.info("opened healthcheck %s/%s on port %d", *nsn, port)
            self.services[nsn] = {"port": port, "runner": runner, "endpoints": 0}

    def sync_endpoints(self, counts: dict[tuple[str, str], int]):
        for nsn, svc in self.services.items():
            svc["endpoints"] = int(counts.get(nsn, 0))

    async def stop(self):
        await self.sync_services({})
