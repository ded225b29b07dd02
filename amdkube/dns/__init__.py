"""Cluster DNS (the kube-dns / CoreDNS addon that local-up-cluster starts).

Reference behaviour: cluster/addons/dns (kube-dns manifests) and the Kubernetes DNS
specification the kubelet's resolv.conf targets (pkg/kubelet/network/dns/dns.go):
  * `<svc>.<ns>.svc.<domain>` A → the ClusterIP; headless services (clusterIP None) → the
    ready endpoint IPs; ExternalName → CNAME;
  * `<hostname>.<svc>.<ns>.svc.<domain>` A for endpoints that carry a hostname (StatefulSet
    pods with spec.subdomain);
  * `_<port>._<proto>.<svc>.<ns>.svc.<domain>` SRV for named service ports;
  * `<a-b-c-d>.<ns>.pod.<domain>` A → a.b.c.d ("pods insecure");
  * PTR for ClusterIPs and endpoint IPs;
  * names outside the cluster domain go to the upstream servers of the host's resolv.conf.
UDP and TCP, RFC 1035 wire format with name compression in answers; negative answers carry
an SOA for the cluster domain so resolvers cache NXDOMAIN for 30 s.
"""
from __future__ import annotations

import asyncio
import ipaddress
import logging
import struct

from ..client import Client, Informer

log = logging.getLogger("amdkube.dns")

A, NS, CNAME, SOA, PTR, TXT, AAAA, SRV, ANY = 1, 2, 5, 6, 12, 16, 28, 33, 255
NOERROR, FORMERR, SERVFAIL, NXDOMAIN, NOTIMP, REFUSED = 0, 1, 2, 3, 4, 5
TTL = 30


# ------------------------------------------------------------------ wire format
def encode_name(name: str) -> bytes:
    out = b""
    for label in name.rstrip(".").split("."):
        if label:
            b = label.encode()
            if len(b) > 63:
                raise ValueError("label too long")
            out += bytes([len(b)]) + b
    return out + b"\x00"


def decode_name(msg: bytes, off: int) -> tuple[str, int]:
    labels, jumped, end, hops = [], False, off, 0
    while True:
        n = msg[off]
        if n & 0xC0 == 0xC0:
            ptr = ((n & 0x3F) << 8) | msg[off + 1]
            if not jumped:
                end = off + 2
            off, jumped = ptr, True
            hops += 1
            if hops > 32:
                raise ValueError("compression loop")
            continue
        if n == 0:
            if not jumped:
                end = off + 1
            break
        labels.append(msg[off + 1:off + 1 + n].decode(errors="replace"))
        off += 1 + n
    return ".".join(labels).lower(), end


def parse_query(msg: bytes):
    qid, flags, qd, _an, _ns, _ar = struct.unpack("!6H", msg[:12])
    name, off = decode_name(msg, 12)
    qtype, qclass = struct.unpack("!2H", msg[off:off + 4])
    return qid, flags, name, qtype, qclass, off + 4


def rr(name: str, rtype: int, rdata: bytes, ttl: int = TTL, qname: str | None = None) -> bytes:
    owner = b"\xc0\x0c" if qname is not None and name == qname else encode_name(name)
    return owner + struct.pack("!HHIH", rtype, 1, ttl, len(rdata)) + rdata


def build_response(query: bytes, qend: int, rcode: int, answers=(), authority=(), aa=True) -> bytes:
    qid, flags = struct.unpack("!2H", query[:4])
    rd = flags & 0x0100
    out_flags = 0x8000 | (0x0400 if aa else 0) | rd | 0x0080 | rcode
    head = struct.pack("!6H", qid, out_flags, 1, len(answers), len(authority), 0)
    return head + query[12:qend] + b"".join(answers) + b"".join(authority)


def build_query(name: str, qtype: int, qid: int = 0x1234) -> bytes:
    return struct.pack("!6H", qid, 0x0100, 1, 0, 0, 0) + encode_name(name) + struct.pack("!2H", qtype, 1)


def parse_response(msg: bytes):
    """(rcode, [(name, type, value)]) — for tests and the kubectl-side resolver helper."""
    _qid, flags, qd, an, _ns, _ar = struct.unpack("!6H", msg[:12])
    off = 12
    for _ in range(qd):
        _, off = decode_name(msg, off)
        off += 4
    out = []
    for _ in range(an):
        name, off = decode_name(msg, off)
        rtype, _cls, _ttl, rdlen = struct.unpack("!HHIH", msg[off:off + 10])
        off += 10
        rdata = msg[off:off + rdlen]
        if rtype == A:
            val = str(ipaddress.IPv4Address(rdata))
        elif rtype in (CNAME, PTR, NS):
            val = decode_name(msg, off)[0]
        elif rtype == SRV:
            prio, weight, port = struct.unpack("!3H", rdata[:6])
            val = (prio, weight, port, decode_name(msg, off + 6)[0])
        else:
            val = rdata
        out.append((name, rtype, val))
        off += rdlen
    return flags & 0xF, out


# ------------------------------------------------------------------ records
class Records:
    """Name → records view over services and endpoints, rebuilt on every change."""

    def __init__(self, domain: str):
        self.domain = domain.strip(".").lower()
        self.a: dict[str, list[str]] = {}
        self.cname: dict[str, str] = {}
        self.srv: dict[str, list[tuple[int, str]]] = {}
        self.ptr: dict[str, str] = {}
        self.names: set[str] = set()   # every existing name (NODATA vs NXDOMAIN)

    def rebuild(self, services: list[dict], endpoints: list[dict]):
        a, cname, srv, ptr = {}, {}, {}, {}
        eps = {((e.get("metadata") or {}).get("namespace"), (e.get("metadata") or {}).get("name")): e for e in endpoints}
        for s in services:
            md, spec = s.get("metadata") or {}, s.get("spec") or {}
            ns, name = md.get("namespace") or "default", md.get("name")
            fq = f"{name}.{ns}.svc.{self.domain}"
            if spec.get("type") == "ExternalName":
                cname[fq] = spec.get("externalName", "").rstrip(".").lower()
                continue
            cip = spec.get("clusterIP")
            headless = cip in (None, "", "None")
            addrs = []
            for sub in (eps.get((ns, name)) or {}).get("subsets") or []:
                for ad in sub.get("addresses") or []:
                    addrs.append((ad, sub.get("ports") or []))
            if not headless:
                a[fq] = [cip]
                ptr[_rev(cip)] = fq
            else:
                a[fq] = sorted({ad["ip"] for ad, _ in addrs})
            for ad, _ in addrs:
                host = ad.get("hostname")
                if host:
                    a.setdefault(f"{host}.{fq}", []).append(ad["ip"])
                    ptr.setdefault(_rev(ad["ip"]), f"{host}.{fq}")
            for p in spec.get("ports") or []:
                if not p.get("name"):
                    continue
                key = f"_{p['name']}._{(p.get('protocol') or 'TCP').lower()}.{fq}"
                if not headless:
                    srv[key] = [(int(p["port"]), fq)]
                else:
                    lst = []
                    for ad, ports in addrs:
                        ep_port = next((x["port"] for x in ports if x.get("name") == p["name"]), None)
                        if ep_port is None:
                            continue
                        target = f"{ad['hostname']}.{fq}" if ad.get("hostname") else f"{ad['ip'].replace('.', '-')}.{fq}"
                        a.setdefault(target, [ad["ip"]])
                        lst.append((int(ep_port), target))
                    srv[key] = lst
        self.a, self.cname, self.srv, self.ptr = a, cname, srv, ptr
        names = set(a) | set(cname) | set(srv)
        for n in list(names):   # parents (svc.<domain>, <ns>.svc.<domain>, …) exist as empty non-terminals
            parts = n.split(".")
            for i in range(1, len(parts)):
                names.add(".".join(parts[i:]))
        self.names = names

    def in_domain(self, q: str) -> bool:
        return q == self.domain or q.endswith("." + self.domain) or q.endswith(".in-addr.arpa")

    def lookup(self, q: str, qtype: int):
        """(rcode, [(name, type, rdata bytes)])"""
        ans = []
        if q.endswith(".in-addr.arpa"):
            if q in self.ptr and qtype in (PTR, ANY):
                return NOERROR, [(q, PTR, encode_name(self.ptr[q]))]
            return (NOERROR if q in self.ptr else NXDOMAIN), []
        pod = self._pod_ip(q)
        if pod is not None:
            return NOERROR, ([(q, A, ipaddress.IPv4Address(pod).packed)] if qtype in (A, ANY) else [])
        if q in self.cname:
            tgt = self.cname[q]
            ans.append((q, CNAME, encode_name(tgt)))
            return NOERROR, ans
        if qtype in (A, ANY) and q in self.a:
            ans += [(q, A, ipaddress.IPv4Address(ip).packed) for ip in self.a[q] if _v4(ip)]
        if qtype in (SRV, ANY) and q in self.srv:
            ans += [(q, SRV, struct.pack("!3H", 10, 100 // max(1, len(self.srv[q])), port) + encode_name(t))
                    for port, t in self.srv[q]]
        if ans or q in self.names:
            return NOERROR, ans
        return NXDOMAIN, []

    def _pod_ip(self, q: str):
        suffix = f".pod.{self.domain}"
        if not q.endswith(suffix):
            return None
        head = q[:-len(suffix)].split(".")
        if len(head) != 2:
            return None
        ip = head[0].replace("-", ".")
        return ip if _v4(ip) else None

    def soa(self) -> bytes:
        d = self.domain
        rdata = encode_name(f"ns.dns.{d}") + encode_name(f"hostmaster.{d}") + struct.pack("!5I", 1, 7200, 1800, 86400, TTL)
        return rr(d, SOA, rdata)


def _v4(ip: str) -> bool:
    try:
        return isinstance(ipaddress.ip_address(ip), ipaddress.IPv4Address)
    except ValueError:
        return False


def _rev(ip: str) -> str:
    return ".".join(reversed(ip.split("."))) + ".in-addr.arpa"


# ------------------------------------------------------------------ server
class DNSServer:
    def __init__(self, client: Client, domain: str = "cluster.local", address: str = "127.0.0.1", port: int = 53,
                 upstream: list[str] | None = None, resolv_conf: str = "/etc/resolv.conf"):
        self.client = client
        self.records = Records(domain)
        self.address, self.port = address, port
        if upstream is None:
            from ..kubelet.dns import parse_resolv_conf
            try:
                upstream = parse_resolv_conf(open(resolv_conf).read())[0]
            except OSError:
                upstream = []
        self.upstream = [u for u in upstream if u not in ("127.0.0.1", address)]
        self.svc_inf = Informer(client, "services")
        self.ep_inf = Informer(client, "endpoints")
        self._udp = self._tcp = None
        self.queries = 0

    def _rebuild(self, *_):
        self.records.rebuild(self.svc_inf.list(), self.ep_inf.list())

    async def start(self):
        for inf in (self.svc_inf, self.ep_inf):
            inf.add_handler(on_add=self._rebuild, on_update=self._rebuild, on_delete=self._rebuild)
            inf.start()
        await self.svc_inf.wait_synced(30)
        await self.ep_inf.wait_synced(30)
        self._rebuild()
        loop = asyncio.get_running_loop()
        want = self.port
        for attempt in range(20):   # port 0: UDP picks a port, TCP must get the same number
            self._udp, _ = await loop.create_datagram_endpoint(lambda: _UDP(self), local_addr=(self.address, want))
            self.port = self._udp.get_extra_info("sockname")[1]
            try:
                self._tcp = await asyncio.start_server(self._tcp_conn, self.address, self.port)
                break
            except OSError:
                self._udp.close()
                if want != 0 or attempt == 19:
                    raise
        log.info("cluster DNS for %s on %s:%d", self.records.domain, self.address, self.port)
        return self

    async def stop(self):
        if self._udp is not None:
            self._udp.close()
        if self._tcp is not None:
            self._tcp.close()
        await self.svc_inf.stop()
        await self.ep_inf.stop()

    async def answer(self, msg: bytes) -> bytes | None:
        self.queries += 1
        try:
            _qid, flags, q, qtype, _qclass, qend = parse_query(msg)
        except (struct.error, IndexError, ValueError):
            return None
        if flags & 0x8000:
            return None
        if not self.records.in_domain(q):
            return await self._forward(msg, qend)
        rcode, ans = self.records.lookup(q, qtype)
        answers = [rr(n, t, d, qname=q) for n, t, d in ans]
        auth = [self.records.soa()] if not answers else []
        return build_response(msg, qend, rcode, answers, auth)

    async def _forward(self, msg: bytes, qend: int) -> bytes:
        loop = asyncio.get_running_loop()
        for up in self.upstream:
            fut = loop.create_future()

            class _P(asyncio.DatagramProtocol):
                def datagram_received(self, data, addr):
                    if not fut.done():
                        fut.set_result(data)
            try:
                tr, _ = await loop.create_datagram_endpoint(_P, remote_addr=(up, 53))
            except OSError:
                continue
            try:
                tr.sendto(msg)
                return await asyncio.wait_for(fut, 2.0)
            except asyncio.TimeoutError:
                continue
            finally:
                tr.close()
        return build_response(msg, qend, SERVFAIL, aa=False)

    async def _tcp_conn(self, r, w):
        try:
            while True:
                n = struct.unpack("!H", await r.readexactly(2))[0]
                out = await self.answer(await r.readexactly(n))
                if out is None:
                    break
                w.write(struct.pack("!H", len(out)) + out)
                await w.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            w.close()


class _UDP(asyncio.DatagramProtocol):
    def __init__(self, srv: DNSServer):
        self.srv = srv
        self.tr = None

    def connection_made(self, tr):
        self.tr = tr

    def datagram_received(self, data, addr):
        async def go():
            out = await self.srv.answer(data)
            if out is not None:
                if len(out) > 512:   # truncated (TC): header + question only, the client retries over TCP
                    qend = parse_query(data)[5]
                    flags = struct.unpack("!H", out[2:4])[0] | 0x0200
                    out = out[:2] + struct.pack("!5H", flags, 1, 0, 0, 0) + data[12:qend]
                self.tr.sendto(out, addr)
        asyncio.ensure_future(go())


async def resolve(name: str, qtype: int = A, server: tuple[str, int] = ("127.0.0.1", 53), timeout: float = 2.0):
    """A one-shot UDP DNS query (tests, health checks)."""
    loop = asyncio.get_running_loop()
    fut = loop.create_future()

    class _P(asyncio.DatagramProtocol):
        def datagram_received(self, data, addr):
            if not fut.done():
                fut.set_result(data)
    tr, _ = await loop.create_datagram_endpoint(_P, remote_addr=server)
    try:
        tr.sendto(build_query(name, qtype))
        return parse_response(await asyncio.wait_for(fut, timeout))
    finally:
        tr.close()
