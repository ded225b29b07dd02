"""Host ports of pods that live in their own network namespace (pkg/kubelet/network/hostport:
hostport_manager.go opens and holds every host port a pod maps, so nothing else can take it,
and DNATs it to the pod IP).

This node has no iptables to DNAT with, so the held socket itself forwards: a TCP listener per
(hostIP, hostPort) splices each accepted connection to podIP:containerPort, and a UDP socket
relays datagrams through one upstream socket per client (the userland proxy the container
runtimes use when NAT is unavailable). A port already held — by another pod or any other
process — makes the sandbox fail ("hostport already in use"), as in the reference.
"""
from __future__ import annotations

import asyncio
import logging
import socket

log = logging.getLogger("amdkube.rocshim.hostport")


class HostPortError(RuntimeError):
    pass


async def _pipe(reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
    try:
        while True:
            b = await reader.read(65536)
            if not b:
                break
            writer.write(b)
            await writer.drain()
    except (ConnectionError, asyncio.CancelledError):
        pass
    finally:
        try:
            writer.close()
        except Exception:
            pass


class _UDPRelay(asyncio.DatagramProtocol):
    def __init__(self, target):
        self.target = target
        self.transport = None
        self.upstream: dict[tuple, asyncio.DatagramTransport] = {}

    def connection_made(self, transport):
        self.transport = transport

    def datagram_received(self, data, addr):
        up = self.upstream.get(addr)
        if up is not None:
            up.sendto(data)
            return

        relay = self

        class Back(asyncio.DatagramProtocol):
            def datagram_received(self, d, _a):
                if relay.transport is not None:
                    relay.transport.sendto(d, addr)

        async def open_up():
            t, _ = await asyncio.get_running_loop().create_datagram_endpoint(Back, remote_addr=self.target)
            self.upstream[addr] = t
            t.sendto(data)
        asyncio.ensure_future(open_up())

    def close(self):
        for t in self.upstream.values():
            t.close()
        if self.transport is not None:
            self.transport.close()


class HostPortManager:
    def __init__(self):
        self.held: dict[tuple[str, int, str], object] = {}     # (hostIP, port, proto) -> server / relay
        self.by_sandbox: dict[str, list[tuple[str, int, str]]] = {}

    async def add(self, sid: str, pod_ip: str, mappings: list[dict]):
        """mappings: [{"host_ip", "host_port", "container_port", "protocol"}] (host_port 0 = none)."""
        opened = []
        try:
            for pm in mappings:
                hp = int(pm.get("host_port") or 0)
                if not hp:
                    continue
                proto = (pm.get("protocol") or "TCP").upper()
                hip = pm.get("host_ip") or "0.0.0.0"
                key = (hip, hp, proto)
                if key in self.held:
                    raise HostPortError(f"hostport {hp}/{proto} on {hip} is already in use")
                target = (pod_ip, int(pm["container_port"]))
                try:
                    if proto == "UDP":
                        relay = _UDPRelay(target)
                        await asyncio.get_running_loop().create_datagram_endpoint(lambda r=relay: r, local_addr=(hip, hp),
                                                                                  reuse_port=False)
                        self.held[key] = relay
                    else:
                        async def handle(r, w, target=target):
                            try:
                                ur, uw = await asyncio.open_connection(*target)
                            except OSError:
                                w.close()
                                return
                            await asyncio.gather(_pipe(r, uw), _pipe(ur, w))
                        srv = await asyncio.start_server(handle, hip, hp, family=socket.AF_INET, reuse_address=True)
                        self.held[key] = srv
                except OSError as e:
                    raise HostPortError(f"cannot open hostport {hp}/{proto} on {hip}: {e.strerror or e}")
                opened.append(key)
        except HostPortError:
            await self._close(opened)
            raise
        if opened:
            self.by_sandbox[sid] = opened
            log.info("sandbox %s holds host ports %s", sid[:12], [f"{k[1]}/{k[2]}" for k in opened])

    async def _close(self, keys):
        for k in keys:
            h = self.held.pop(k, None)
            if h is None:
                continue
            h.close()
            if isinstance(h, asyncio.AbstractServer):
                await h.wait_closed()

    async def remove(self, sid: str):
        await self._close(self.by_sandbox.pop(sid, []))

    async def close(self):
        for sid in list(self.by_sandbox):
            await self.remove(sid)
