"""userspace proxy mode: one proxy socket per service port, round-robin with ClientIP affinity.

Reference: pkg/proxy/userspace/proxier.go (a proxy socket per ServicePortName; iptables
"portals" redirect clusterIP:port and nodePort to it), proxysocket.go (tcpProxySocket:
tryConnect over up to len(endpoints) endpoints with back-off timeouts 250 ms, 500 ms,
1 s, 2 s, then copyBytes both ways; udpProxySocket: per-client "connection" kept for
--udp-timeout), roundrobin.go (LoadBalancerRR: NextEndpoint with ClientIP session
affinity and TTL, endpoints shuffled on update, affinity entries dropped when their
endpoint goes away).

MI355X-node specifics: amdkube cannot assume it may program iptables (the GPU box and CI
run unprivileged), so portals are real listeners. The NodePort binds on the node address,
and the ClusterIP binds directly when the address is local. A service CIDR inside
127.0.0.0/8, as `local-up` uses, makes every ClusterIP reachable on the node with no NAT
at all. Otherwise the proxier records an ephemeral proxy port per portal (`portals`), which
is exactly what the reference's iptables REDIRECT would target.
"""
from __future__ import annotations

import asyncio
import errno
import logging
import random
import socket
import time

from .config import ServiceInfo, ServicePortName

log = logging.getLogger("amdkube.proxy")

CONNECT_TIMEOUTS = (0.25, 0.5, 1.0, 2.0)   # proxysocket.go EndpointDialTimeouts


class _SvcState:
    __slots__ = ("endpoints", "index", "affinity", "affinity_type", "ttl")

    def __init__(self, affinity_type="None", ttl=10800):
        self.endpoints: list[str] = []
        self.index = 0
        self.affinity: dict[str, tuple[str, float]] = {}
        self.affinity_type = affinity_type
        self.ttl = ttl


class LoadBalancerRR:
    def __init__(self, rng: random.Random | None = None):
        self.services: dict[ServicePortName, _SvcState] = {}
        self.rng = rng or random.Random()

    def new_service(self, spn: ServicePortName, affinity_type: str = "None", ttl: int = 10800):
        st = self.services.get(spn)
        if st is None:
            self.services[spn] = _SvcState(affinity_type, ttl)
        else:
            st.affinity_type, st.ttl = affinity_type, ttl

    def delete_service(self, spn: ServicePortName):
        self.services.pop(spn, None)

    def on_endpoints_update(self, eps: dict[ServicePortName, list]):
        for spn, lst in eps.items():
            st = self.services.setdefault(spn, _SvcState())
            new = sorted(f"{ip}:{port}" for ip, port, _ in lst)
            if sorted(st.endpoints) != new:
                self.rng.shuffle(new)
                st.endpoints, st.index = new, 0
                live = set(new)
                st.affinity = {c: v for c, v in st.affinity.items() if v[0] in live}
        for spn, st in self.services.items():
            if spn not in eps and st.endpoints:
                st.endpoints, st.index, st.affinity = [], 0, {}

    def next_endpoint(self, spn: ServicePortName, client_ip: str | None, reset_affinity: bool = False) -> str:
        st = self.services.get(spn)
        if st is None or not st.endpoints:
            raise LookupError(f"missing service entry for {spn}")
        now = time.monotonic()
        sticky = st.affinity_type == "ClientIP" and client_ip
        if sticky and not reset_affinity:
            hit = st.affinity.get(client_ip)
            if hit and now - hit[1] < st.ttl:
                st.affinity[client_ip] = (hit[0], now)
                return hit[0]
        ep = st.endpoints[st.index % len(st.endpoints)]
        st.index = (st.index + 1) % len(st.endpoints)
        if sticky:
            st.affinity[client_ip] = (ep, now)
        return ep


async def _pipe(r: asyncio.StreamReader, w: asyncio.StreamWriter):
    try:
        while True:
            b = await r.read(65536)
            if not b:
                break
            w.write(b)
            await w.drain()
    except (ConnectionError, asyncio.CancelledError):
        pass
    finally:
        try:
            if w.can_write_eof():
                w.write_eof()
        except (OSError, RuntimeError):
            pass


class _TCPSocket:
    def __init__(self, proxier, spn: ServicePortName):
        self.proxier, self.spn = proxier, spn
        self.servers: list[asyncio.AbstractServer] = []
        self.conns: set[asyncio.Task] = set()

    async def listen(self, host, port) -> int:
        srv = await asyncio.start_server(self._handle, host, port, reuse_address=True)
        self.servers.append(srv)
        return srv.sockets[0].getsockname()[1]

    async def _connect(self, client_ip):
        for i, timeout in enumerate(CONNECT_TIMEOUTS):
            try:
                ep = self.proxier.lb.next_endpoint(self.spn, client_ip, reset_affinity=i > 0)
            except LookupError:
                return None
            host, _, port = ep.rpartition(":")
            try:
                return await asyncio.wait_for(asyncio.open_connection(host, int(port)), timeout)
            except (OSError, asyncio.TimeoutError) as e:
                log.debug("dial %s for %s failed: %r", ep, self.spn, e)
        return None

    async def _handle(self, reader, writer):
        task = asyncio.current_task()
        self.conns.add(task)
        peer = writer.get_extra_info("peername") or ("", 0)
        try:
            up = await self._connect(peer[0])
            if up is None:
                self.proxier.failed_connects += 1
                return
            ur, uw = up
            self.proxier.connections += 1
            await asyncio.gather(_pipe(reader, uw), _pipe(ur, writer))
            uw.close()
        finally:
            writer.close()
            self.conns.discard(task)

    async def close(self):
        for s in self.servers:
            s.close()
        for t in list(self.conns):
            t.cancel()
        for s in self.servers:
            try:
                await s.wait_closed()
            except Exception:
                pass


class _UDPRelay(asyncio.DatagramProtocol):
    def __init__(self, owner, client_addr):
        self.owner, self.client_addr, self.transport, self.last = owner, client_addr, None, time.monotonic()

    def connection_made(self, transport):
        self.transport = transport

    def datagram_received(self, data, addr):
        self.last = time.monotonic()
        if self.owner.transport is not None:
            self.owner.transport.sendto(data, self.client_addr)


class _UDPSocket(asyncio.DatagramProtocol):
    def __init__(self, proxier, spn, idle_timeout=0.25):
        self.proxier, self.spn, self.idle = proxier, spn, idle_timeout
        self.transport = None
        self.transports: list = []
        self.clients: dict[tuple, _UDPRelay] = {}
        self._reaper = None

    async def listen(self, host, port) -> int:
        loop = asyncio.get_running_loop()
        t, _ = await loop.create_datagram_endpoint(lambda: self, local_addr=(host, port), reuse_port=False)
        self.transports.append(t)
        if self._reaper is None:
            self._reaper = asyncio.create_task(self._reap())
        return t.get_extra_info("sockname")[1]

    def connection_made(self, transport):
        self.transport = transport

    def datagram_received(self, data, addr):
        asyncio.ensure_future(self._forward(data, addr))

    async def _forward(self, data, addr):
        relay = self.clients.get(addr)
        if relay is None or relay.transport is None or relay.transport.is_closing():
            try:
                ep = self.proxier.lb.next_endpoint(self.spn, addr[0])
            except LookupError:
                return
            host, _, port = ep.rpartition(":")
            loop = asyncio.get_running_loop()
            _, relay = await loop.create_datagram_endpoint(lambda: _UDPRelay(self, addr), remote_addr=(host, int(port)))
            self.clients[addr] = relay
        relay.last = time.monotonic()
        relay.transport.sendto(data)

    async def _reap(self):
        while True:
            await asyncio.sleep(max(self.idle, 1.0))
            now = time.monotonic()
            for a, r in list(self.clients.items()):
                if now - r.last > max(self.idle, 1.0) * 4:
                    r.transport.close()
                    del self.clients[a]

    async def close(self):
        if self._reaper:
            self._reaper.cancel()
        for r in self.clients.values():
            r.transport.close()
        for t in self.transports:
            t.close()


class UserspaceProxier:
    mode = "userspace"

    def __init__(self, node_ip: str = "0.0.0.0", bind_cluster_ips: bool = True, udp_idle_timeout: float = 0.25):
        self.node_ip = node_ip
        self.bind_cluster_ips = bind_cluster_ips
        self.udp_idle = udp_idle_timeout
        self.lb = LoadBalancerRR()
        self.sockets: dict[ServicePortName, tuple[ServiceInfo, object]] = {}
        self.portals: dict[tuple[str, int, str], int] = {}   # (ip, port, proto) -> local listening port
        self.connections = 0
        self.failed_connects = 0
        self.syncs = 0

    async def _open(self, spn: ServicePortName, info: ServiceInfo):
        sock = _TCPSocket(self, spn) if info.protocol == "TCP" else _UDPSocket(self, spn, self.udp_idle)
        portals = [(ip, info.port) for ip in [info.cluster_ip, *info.external_ips, *info.lb_ingress]]
        for ip, port in portals:
            bound = None
            if self.bind_cluster_ips:
                try:
                    bound = await sock.listen(ip, port)
                except OSError as e:
                    if e.errno not in (errno.EADDRNOTAVAIL, errno.EACCES, errno.EADDRINUSE, errno.EPERM):
                        raise
            if bound is None:  # the reference's REDIRECT target: an ephemeral proxy port
                bound = await sock.listen("127.0.0.1", 0)
            self.portals[(ip, port, info.protocol)] = bound
        if info.node_port:
            try:
                await sock.listen(self.node_ip, info.node_port)
                self.portals[(self.node_ip, info.node_port, info.protocol)] = info.node_port
            except OSError as e:
                log.warning("cannot open nodePort %d for %s: %r", info.node_port, spn, e)
        return sock

    async def sync(self, services: dict[ServicePortName, ServiceInfo], endpoints: dict[ServicePortName, list]):
        self.syncs += 1
        for spn in list(self.sockets):
            info, sock = self.sockets[spn]
            if services.get(spn) != info:
                await sock.close()
                del self.sockets[spn]
                self.lb.delete_service(spn)
                self.portals = {k: v for k, v in self.portals.items()
                                if k[:2] not in [(ip, info.port) for ip in [info.cluster_ip, *info.external_ips, *info.lb_ingress]]
                                and k[:2] != (self.node_ip, info.node_port)}
        for spn, info in services.items():
            if spn not in self.sockets:
                self.lb.new_service(spn, info.session_affinity, info.affinity_timeout)
                self.sockets[spn] = (info, await self._open(spn, info))
        self.lb.on_endpoints_update({k: v for k, v in endpoints.items() if k in services})

    def portal(self, ip: str, port: int, proto: str = "TCP") -> tuple[str, int] | None:
        """Where a client on this node reaches ip:port (the REDIRECT target)."""
        p = self.portals.get((ip, port, proto))
        if p is None:
            return None
        try:
            socket.inet_aton(ip)
            with socket.socket() as s:
                s.settimeout(0.2)
                if s.connect_ex((ip, port)) == 0:
                    return ip, port
        except OSError:
            pass
        return "127.0.0.1", p

    async def stop(self):
        for _, sock in self.sockets.values():
            await sock.close()
        self.sockets.clear()
