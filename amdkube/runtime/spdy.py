"""SPDY/3.1 streams for exec / attach / port-forward, next to the WebSocket channel protocol.

A v1.9 kubectl negotiates `Upgrade: SPDY/3.1` for `exec`, `attach` and `port-forward`
(reference staging/src/k8s.io/apimachinery/pkg/util/httpstream/spdy/{roundtripper,upgrade,
connection}.go over vendor/github.com/docker/spdystream), then multiplexes one stream per
channel: remotecommand (pkg/kubelet/server/remotecommand/httpstream.go) opens `streamtype`
error/stdin/stdout/stderr/resize streams, port-forward (pkg/kubelet/server/portforward/
httpstream.go) a data+error pair per forwarded connection keyed by `requestid`.

This module is amdkube's own asyncio implementation of that wire:

* frames — control frames `1|version(15)|type(16)|flags(8)|length(24)`, data frames
  `0|stream-id(31)|flags(8)|length(24)`; SYN_STREAM / SYN_REPLY / RST_STREAM / SETTINGS / PING /
  GOAWAY / HEADERS / WINDOW_UPDATE;
* header blocks — SPDY/3 name/value blocks (32-bit counts and lengths, lower-case names, multiple
  values joined by NUL) in ONE zlib stream per direction per session, primed with the SPDY/3
  dictionary and sync-flushed per frame;
* flow control is left to TCP, as spdystream does (WINDOW_UPDATE is accepted and ignored, no
  send window is enforced, so a Go peer that never sends WINDOW_UPDATE cannot stall us);
* `Session` runs over either a hijacked aiohttp server connection (`accept`) or a client socket
  (`connect`); `upgrade_proxy` is the apiserver/kubelet hop: it forwards the upgrade request and
  then splices raw bytes, like the reference's UpgradeAwareHandler, so SPDY is parsed only at
  the ends.
"""
from __future__ import annotations

import asyncio
import json
import ssl as _ssl
import struct
import zlib
from urllib.parse import quote, urlsplit

from aiohttp import web

UPGRADE = "SPDY/3.1"
PROTOCOL_HEADER = "X-Stream-Protocol-Version"
ACCEPTED_HEADER = "X-Accepted-Stream-Protocol-Versions"
EXEC_PROTOCOLS = ("v4.channel.k8s.io", "v3.channel.k8s.io", "v2.channel.k8s.io", "channel.k8s.io")
PORTFORWARD_PROTOCOLS = ("portforward.k8s.io",)
STREAM_CREATION_TIMEOUT = 30.0
MAX_DATA = 64 * 1024
MAX_HEADER_BLOCK = 1 << 20     # inflated name/value block bound (a small compressed block can expand ~1000x)

SYN_STREAM, SYN_REPLY, RST_STREAM, SETTINGS, PING, GOAWAY, HEADERS, WINDOW_UPDATE = 1, 2, 3, 4, 6, 7, 8, 9
FLAG_FIN, FLAG_UNIDIRECTIONAL = 0x01, 0x02
RST_PROTOCOL_ERROR, RST_REFUSED_STREAM, RST_CANCEL = 1, 3, 5


def _dictionary() -> bytes:
    """The SPDY/3 header-compression dictionary (draft-mbelshe-httpbis-spdy-00 §2.6.10.1):
    length-prefixed common header names/values, then a run of status lines, dates and media types."""
    words = ("options head post put delete trace accept accept-charset accept-encoding accept-language "
             "accept-ranges age allow authorization cache-control connection content-base content-encoding "
             "content-language content-length content-location content-md5 content-range content-type date "
             "etag expect expires from host if-match if-modified-since if-none-match if-range "
             "if-unmodified-since last-modified location max-forwards pragma proxy-authenticate "
             "proxy-authorization range referer retry-after server te trailer transfer-encoding upgrade "
             "user-agent vary via warning www-authenticate method get status").split()
    words += ["200 OK", "version", "HTTP/1.1", "url", "public", "set-cookie", "keep-alive", "origin"]
    head = b"".join(struct.pack(">I", len(w)) + w.encode() for w in words)
    codes = "100101201202205206300302303304305306307402405406407408409410411412413414415416417502504505"
    reasons = ("203 Non-Authoritative Information", "204 No Content", "301 Moved Permanently", "400 Bad Request",
               "401 Unauthorized", "403 Forbidden", "404 Not Found", "500 Internal Server Error",
               "501 Not Implemented", "503 Service Unavailable")
    tail = (codes + "".join(reasons) + "Jan Feb Mar Apr May Jun Jul Aug Sept Oct Nov Dec 00:00:00 "
            "Mon, Tue, Wed, Thu, Fri, Sat, Sun, GMT"
            "chunked,text/html,image/png,image/jpg,image/gif,application/xml,application/xhtml+xml,"
            "text/plain,text/javascript,publicprivatemax-age=gzip,deflate,sdch"
            "charset=utf-8charset=iso-8859-1,utf-,*,enq=0.")
    return head + tail.encode()


DICTIONARY = _dictionary()


def encode_headers(headers: dict) -> bytes:
    """{name: str | list[str]} -> uncompressed SPDY/3 name/value block."""
    out = [struct.pack(">I", len(headers))]
    for k, v in headers.items():
        name = k.lower().encode()
        val = "\x00".join(v if isinstance(v, (list, tuple)) else [str(v)]).encode()
        out += [struct.pack(">I", len(name)), name, struct.pack(">I", len(val)), val]
    return b"".join(out)


def decode_headers(block: bytes) -> dict[str, list[str]]:
    (n,), i, out = struct.unpack_from(">I", block), 4, {}
    for _ in range(n):
        (ln,) = struct.unpack_from(">I", block, i)
        name = block[i + 4:i + 4 + ln].decode().lower()
        i += 4 + ln
        (lv,) = struct.unpack_from(">I", block, i)
        out.setdefault(name, []).extend(block[i + 4:i + 4 + lv].decode().split("\x00"))
        i += 4 + lv
    return out


def control_frame(ftype: int, payload: bytes, flags: int = 0) -> bytes:
    return struct.pack(">HHI", 0x8000 | 3, ftype, flags << 24 | len(payload)) + payload


def data_frame(sid: int, data: bytes, flags: int = 0) -> bytes:
    return struct.pack(">II", sid & 0x7FFFFFFF, flags << 24 | len(data)) + data


class SpdyError(Exception):
    pass


class UpgradeRefused(SpdyError):
    """The server answered the upgrade with an error (its body: a metav1.Status, usually)."""

    def __init__(self, status: int, body: str):
        super().__init__(f"upgrade refused: {status}: {body}")
        self.status_code, self.body = status, body

    def status_error(self):
        """The API error the body carries (meta.StatusError), or None."""
        import json
        from ..api import meta as m
        try:
            st = json.loads(self.body)
        except ValueError:
            return None
        return m.StatusError.from_status(st) if isinstance(st, dict) and st.get("kind") == "Status" else None


class Stream:
    """One SPDY stream: a byte pipe with half-close (FIN) in each direction."""

    def __init__(self, session: "Session", sid: int, headers: dict[str, list[str]]):
        self.session, self.id, self.headers = session, sid, headers
        self._q: asyncio.Queue[bytes] = asyncio.Queue()
        self.remote_closed = self.local_closed = self.reset = False
        self.replied = asyncio.get_running_loop().create_future()

    def header(self, name: str, default: str = "") -> str:
        v = self.headers.get(name.lower())
        return v[0] if v else default

    def _feed(self, data: bytes, fin: bool):
        if data and not self.remote_closed:
            self._q.put_nowait(data)
        if fin and not self.remote_closed:
            self.remote_closed = True
            self._q.put_nowait(b"")

    async def read(self) -> bytes:
        """The next chunk, b"" once the peer half-closed (or the session ended)."""
        data = await self._q.get()
        if not data:
            self._q.put_nowait(b"")      # EOF is sticky
        return data

    async def read_all(self) -> bytes:
        out = bytearray()
        while True:
            chunk = await self.read()
            if not chunk:
                return bytes(out)
            out += chunk

    async def write(self, data: bytes):
        if self.local_closed or self.reset:
            raise SpdyError(f"write on closed stream {self.id}")
        for i in range(0, len(data), MAX_DATA):
            await self.session._send(data_frame(self.id, data[i:i + MAX_DATA]))

    async def close(self):
        """Half-close our direction (empty DATA frame with FIN)."""
        if not self.local_closed and not self.reset and not self.session.closed.is_set():
            self.local_closed = True
            await self.session._send(data_frame(self.id, b"", FLAG_FIN))
        self.local_closed = True
        self.session._maybe_forget(self)

    async def reply(self, headers: dict | None = None, fin: bool = False):
        await self.session._send_control(SYN_REPLY, struct.pack(">I", self.id), headers or {}, FLAG_FIN if fin else 0)
        if fin:
            self.local_closed = True

    async def rst(self, status: int = RST_CANCEL):
        self.reset = True
        await self.session._send(control_frame(RST_STREAM, struct.pack(">II", self.id, status)))
        self._feed(b"", True)
        self.session.streams.pop(self.id, None)


class Session:
    """Both ends of a SPDY/3.1 connection. `feed()` takes received bytes (the transport is
    push-based on the server side); `write`/`drain`/`close_transport` are the way out."""

    def __init__(self, server: bool, on_stream=None):
        self.server, self.on_stream = server, on_stream
        self.next_id = 2 if server else 1
        self.next_ping = 2 if server else 1
        self.streams: dict[int, Stream] = {}
        self.closed = asyncio.Event()
        self._buf = bytearray()
        self._inflate = zlib.decompressobj(zdict=DICTIONARY)
        self._deflate = zlib.compressobj(zlib.Z_DEFAULT_COMPRESSION, zlib.DEFLATED, 15, zdict=DICTIONARY)
        self._wlock = asyncio.Lock()
        self._pings: dict[int, asyncio.Future] = {}
        self._tasks: set[asyncio.Task] = set()
        self.write = self.drain = self.close_transport = None
        self.goaway = False
        self._reader: asyncio.Task | None = None     # client side: the socket-reading task

    def attach(self, write, drain, close_transport):
        self.write, self.drain, self.close_transport = write, drain, close_transport

    # -------------------------------------------------------------------- outbound
    def _header_block(self, headers: dict) -> bytes:
        return self._deflate.compress(encode_headers(headers)) + self._deflate.flush(zlib.Z_SYNC_FLUSH)

    async def _send(self, frame: bytes):
        if self.closed.is_set():
            raise SpdyError("session closed")
        self.write(frame)
        await self.drain()

    async def _send_control(self, ftype: int, prefix: bytes, headers: dict, flags: int = 0):
        async with self._wlock:        # header blocks share one zlib stream: compress+write in order
            await self._send(control_frame(ftype, prefix + self._header_block(headers), flags))

    async def open_stream(self, headers: dict, fin: bool = False, timeout: float = STREAM_CREATION_TIMEOUT) -> Stream:
        async with self._wlock:        # ids must reach the wire in increasing order
            sid, self.next_id = self.next_id, self.next_id + 2
            st = self.streams[sid] = Stream(self, sid, {k.lower(): (v if isinstance(v, list) else [str(v)]) for k, v in headers.items()})
            await self._send(control_frame(SYN_STREAM, struct.pack(">IIBB", sid, 0, 0, 0) + self._header_block(headers),
                                           FLAG_FIN if fin else 0))
        st.local_closed = fin
        try:
            await asyncio.wait_for(asyncio.shield(st.replied), timeout)
        except asyncio.TimeoutError:
            raise SpdyError(f"timed out waiting for a reply to stream {sid}") from None
        if st.reset:
            raise SpdyError(f"stream {sid} was reset by the peer")
        return st

    async def ping(self, timeout: float = 10.0) -> float:
        pid, self.next_ping = self.next_ping, self.next_ping + 2
        fut = self._pings[pid] = asyncio.get_running_loop().create_future()
        t0 = asyncio.get_running_loop().time()
        await self._send(control_frame(PING, struct.pack(">I", pid)))
        try:
            await asyncio.wait_for(fut, timeout)
        finally:
            self._pings.pop(pid, None)
        return asyncio.get_running_loop().time() - t0

    async def close(self):
        """GOAWAY, then drop the transport; every stream reads EOF."""
        if not self.closed.is_set():
            last = max((s for s in self.streams if (s % 2 == 0) != self.server), default=0)
            try:
                await self._send(control_frame(GOAWAY, struct.pack(">II", last, 0)))
            except (SpdyError, ConnectionError, RuntimeError):
                pass
        self.connection_lost()
        if self.close_transport is not None:
            self.close_transport()

    async def aclose(self):
        """close() and wait for the reading side to wind down."""
        await self.close()
        if self._reader is not None:
            await asyncio.gather(self._reader, return_exceptions=True)

    def connection_lost(self):
        if self.closed.is_set():
            return
        self.closed.set()
        for st in list(self.streams.values()):
            st._feed(b"", True)
            if not st.replied.done():
                st.reset = True
                st.replied.set_result(None)
        for f in self._pings.values():
            if not f.done():
                f.set_exception(SpdyError("session closed"))
        for t in self._tasks:
            t.cancel()

    def _maybe_forget(self, st: Stream):
        if st.local_closed and st.remote_closed:
            self.streams.pop(st.id, None)

    # -------------------------------------------------------------------- inbound
    def feed(self, data: bytes):
        self._buf += data
        buf = self._buf
        while len(buf) >= 8:
            w0, w1 = struct.unpack_from(">II", buf)
            length = w1 & 0xFFFFFF
            if len(buf) < 8 + length:
                break
            payload, flags = bytes(buf[8:8 + length]), w1 >> 24
            del buf[:8 + length]
            if w0 & 0x80000000:
                version, ftype = (w0 >> 16) & 0x7FFF, w0 & 0xFFFF
                if version != 3:
                    self._spawn(self.close())
                    return
                try:
                    self._control(ftype, flags, payload)
                except (struct.error, zlib.error, UnicodeDecodeError) as e:   # malformed header block
                    raise SpdyError(f"malformed SPDY control frame: {e}") from e
            else:
                st = self.streams.get(w0 & 0x7FFFFFFF)
                if st is not None:
                    st._feed(payload, bool(flags & FLAG_FIN))
                    self._maybe_forget(st)

    def _spawn(self, coro):
        t = asyncio.get_running_loop().create_task(coro)
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)

    def _headers(self, block: bytes) -> dict:
        if not block:
            return {}
        raw = self._inflate.decompress(block, MAX_HEADER_BLOCK)
        if self._inflate.unconsumed_tail:       # a header block that inflates past the bound
            raise SpdyError(f"SPDY header block inflates beyond {MAX_HEADER_BLOCK} bytes")
        return decode_headers(raw)

    def _control(self, ftype: int, flags: int, p: bytes):
        if ftype == SYN_STREAM:
            sid = struct.unpack_from(">I", p)[0] & 0x7FFFFFFF
            st = Stream(self, sid, self._headers(p[10:]))
            if self.goaway or sid in self.streams or (sid % 2 == 0) == self.server:
                self._spawn(st.rst(RST_PROTOCOL_ERROR))
                return
            st.replied.set_result(None)
            if flags & FLAG_UNIDIRECTIONAL:
                st.local_closed = True
            self.streams[sid] = st
            if flags & FLAG_FIN:
                st._feed(b"", True)
            if self.on_stream is None:
                self._spawn(st.rst(RST_REFUSED_STREAM))
            else:
                self._spawn(self.on_stream(st))
        elif ftype in (SYN_REPLY, HEADERS):
            sid = struct.unpack_from(">I", p)[0] & 0x7FFFFFFF
            hdrs = self._headers(p[4:])
            st = self.streams.get(sid)
            if st is None:
                return
            if ftype == SYN_REPLY and not st.replied.done():
                st.headers.update({f"reply:{k}": v for k, v in hdrs.items()})
                st.replied.set_result(None)
            if flags & FLAG_FIN:
                st._feed(b"", True)
                self._maybe_forget(st)
        elif ftype == RST_STREAM:
            sid = struct.unpack_from(">I", p)[0] & 0x7FFFFFFF
            st = self.streams.pop(sid, None)
            if st is not None:
                st.reset = True
                st._feed(b"", True)
                if not st.replied.done():
                    st.replied.set_result(None)
        elif ftype == PING:
            (pid,) = struct.unpack_from(">I", p)
            if (pid % 2 == 0) == self.server:      # our own ping coming back
                fut = self._pings.get(pid)
                if fut is not None and not fut.done():
                    fut.set_result(None)
            else:
                self._spawn(self._send(control_frame(PING, p[:4])))
        elif ftype == GOAWAY:
            self.goaway = True
        # SETTINGS and WINDOW_UPDATE: accepted, nothing to do (flow control is TCP's)


# ------------------------------------------------------------------------ HTTP upgrade
def is_upgrade(request) -> bool:
    return request.headers.get("Upgrade", "").lower() == UPGRADE.lower()


def negotiate(client: list[str], server) -> str | None:
    """httpstream.Handshake: the first client-offered protocol the server speaks; "" for a
    client that offers none (pre-1.1 kubectl), None when nothing matches."""
    if not client:
        return ""
    for c in client:
        for s in server:
            if c.strip() == s:
                return c.strip()
    return None


class _Feed:
    """aiohttp payload-parser hook: bytes arriving on the hijacked connection go to the session."""

    def __init__(self, sink, on_eof):
        self.sink, self.on_eof = sink, on_eof

    def feed_data(self, data: bytes):
        try:
            self.sink(data)
        except SpdyError:              # protocol violation by the peer: end the session, not the server
            self.on_eof()
        return False, b""

    def feed_eof(self):
        self.on_eof()


async def accept(request: web.Request, protocols, on_stream=None) -> tuple[Session | None, str, web.StreamResponse]:
    """Server side of the upgrade (spdy/upgrade.go). Returns (session, protocol, response); the
    session is None and the response a 400/403 when the request cannot be upgraded."""
    offered = [p.strip() for v in request.headers.getall(PROTOCOL_HEADER, []) for p in v.split(",") if p.strip()]
    proto = negotiate(offered, protocols)
    if proto is None:
        r = web.Response(status=403, text=f"unable to upgrade: unable to negotiate protocol: client supports {offered}, "
                                          f"server accepts {list(protocols)}")
        for p in protocols:
            r.headers.add(ACCEPTED_HEADER, p)
        return None, "", r
    if "upgrade" not in request.headers.get("Connection", "").lower():
        return None, "", web.Response(status=400, text="unable to upgrade: missing upgrade headers in request")
    hdrs = {"Connection": "Upgrade", "Upgrade": UPGRADE}
    if proto:
        hdrs[PROTOCOL_HEADER] = proto
    resp = web.StreamResponse(status=101, reason="Switching Protocols", headers=hdrs)
    resp.force_close()
    sess = Session(server=True, on_stream=on_stream)
    request.protocol.set_parser(_Feed(sess.feed, sess.connection_lost))
    writer = await resp.prepare(request)
    tr = request.transport
    sess.attach(tr.write, writer.drain, tr.close)
    return sess, proto, resp


async def _open(url: str, ssl=None):
    u = urlsplit(url)
    tls = u.scheme in ("https", "wss")
    port = u.port or (443 if tls else 80)
    ctx = None
    if tls:
        ctx = ssl if isinstance(ssl, _ssl.SSLContext) else _ssl.create_default_context()
        if ssl is False:
            ctx.check_hostname, ctx.verify_mode = False, _ssl.CERT_NONE
    reader, writer = await asyncio.open_connection(u.hostname, port, ssl=ctx)
    return u, reader, writer


def _request_head(method: str, u, headers: list[tuple[str, str]]) -> bytes:
    target = quote((u.path or "/") + (f"?{u.query}" if u.query else ""), safe="/?&=%+:@,;!$'()*~-._")
    lines = [f"{method} {target} HTTP/1.1", f"Host: {u.netloc}"] + [f"{k}: {v}" for k, v in headers]
    return ("\r\n".join(lines) + "\r\n\r\n").encode()


async def _response_head(reader) -> tuple[int, list[tuple[str, str]], bytes]:
    head = await reader.readuntil(b"\r\n\r\n")
    lines = head.decode("latin-1").split("\r\n")
    status = int(lines[0].split()[1])
    hdrs = [(k.strip(), v.strip()) for k, _, v in (ln.partition(":") for ln in lines[1:] if ln)]
    body = b""
    if status != 101:
        n = next((int(v) for k, v in hdrs if k.lower() == "content-length"), None)
        try:
            body = await (reader.readexactly(n) if n is not None else asyncio.wait_for(reader.read(65536), 5))
        except (asyncio.IncompleteReadError, asyncio.TimeoutError):
            pass
    return status, hdrs, body


async def connect(url: str, protocols, headers: dict | None = None, ssl=None, method: str = "POST",
                  on_stream=None) -> tuple[Session, str]:
    """Client side (spdy/roundtripper.go): upgrade `url` and return the session and the
    negotiated protocol. Raises SpdyError with the server's body when it refuses."""
    u, reader, writer = await _open(url, ssl)
    hl = [("Connection", "Upgrade"), ("Upgrade", UPGRADE), ("Content-Length", "0")]
    hl += [(PROTOCOL_HEADER, p) for p in protocols] + list((headers or {}).items())
    writer.write(_request_head(method, u, hl))
    await writer.drain()
    status, rh, body = await _response_head(reader)
    if status != 101:
        writer.close()
        raise UpgradeRefused(status, body.decode(errors="replace").strip())
    proto = next((v for k, v in rh if k.lower() == PROTOCOL_HEADER.lower()), "")
    sess = Session(server=False, on_stream=on_stream)
    sess.attach(writer.write, writer.drain, writer.close)

    async def pump():
        try:
            while True:
                data = await reader.read(65536)
                if not data:
                    break
                sess.feed(data)
        except (ConnectionError, OSError, SpdyError):
            pass
        finally:
            sess.connection_lost()
    sess._reader = asyncio.get_running_loop().create_task(pump())
    return sess, proto


_HOP = {"host", "content-length", "transfer-encoding", "authorization", "connection", "upgrade", "keep-alive",
        "proxy-connection", "te", "trailer"}


async def upgrade_proxy(request: web.Request, url: str, ssl=None, headers: dict | None = None) -> web.StreamResponse:
    """The relay hop (apiserver → kubelet, kubelet → runtime): forward the upgrade request, pass a
    refusal back as an ordinary response, otherwise complete the client's upgrade with the
    upstream's 101 headers and splice raw bytes both ways until either side closes."""
    u, reader, writer = await _open(url, ssl)
    hl = [("Connection", "Upgrade"), ("Upgrade", request.headers.get("Upgrade", UPGRADE)), ("Content-Length", "0")]
    hl += [(k, v) for k, v in request.headers.items() if k.lower() not in _HOP]
    hl += list((headers or {}).items())
    writer.write(_request_head(request.method, u, hl))
    await writer.drain()
    try:
        status, rh, body = await _response_head(reader)
    except (asyncio.IncompleteReadError, ConnectionError) as e:
        writer.close()
        return web.Response(status=502, text=f"upgrade upstream failed: {e}")
    if status != 101:
        writer.close()
        ctype = next((v for k, v in rh if k.lower() == "content-type"), "text/plain")
        r = web.Response(status=status, body=body, headers={"Content-Type": ctype})
        for k, v in rh:
            if k.lower() == ACCEPTED_HEADER.lower():
                r.headers.add(k, v)
        return r
    resp = web.StreamResponse(status=101, reason="Switching Protocols",
                              headers={k: v for k, v in rh if k.lower() not in ("content-length", "date", "server")})
    resp.force_close()
    done = asyncio.Event()
    client_tr = request.transport
    up_tr = writer.transport

    def upward(data: bytes):
        up_tr.write(data)
        if up_tr.get_write_buffer_size() > 4 << 20 and client_tr is not None:
            client_tr.pause_reading()            # slow upstream: stop reading the client until it drains

            async def resume():
                try:
                    await writer.drain()
                finally:
                    if not client_tr.is_closing():
                        client_tr.resume_reading()
            asyncio.get_running_loop().create_task(resume())

    def client_eof():
        if not up_tr.is_closing() and up_tr.can_write_eof():
            up_tr.write_eof()
        done.set()
    request.protocol.set_parser(_Feed(upward, client_eof))
    out = await resp.prepare(request)
    try:
        while True:
            data = await reader.read(65536)
            if not data:
                break
            client_tr.write(data)
            await out.drain()
    except (ConnectionError, OSError):
        pass
    finally:
        writer.close()
        if client_tr is not None and not client_tr.is_closing():
            client_tr.close()
    return resp


# ------------------------------------------------------------------------ remotecommand helpers
def exec_streams_expected(proto: str, stdin: bool, stdout: bool, stderr: bool, tty: bool) -> set[str]:
    """Which streams the client opens (remotecommand/httpstream.go createStreams): the error
    stream always, stdio as requested (no stderr under a tty), resize from v3 on when tty."""
    want = {"error"}
    if stdin:
        want.add("stdin")
    if stdout:
        want.add("stdout")
    if stderr and not tty:
        want.add("stderr")
    if tty and proto in ("v3.channel.k8s.io", "v4.channel.k8s.io"):
        want.add("resize")
    return want


def split_json(text: str) -> tuple[list, str]:
    """Complete JSON objects at the head of `text` and the unparsed rest (a resize stream is a
    json.Encoder stream of TerminalSize objects)."""
    dec, out, i = json.JSONDecoder(), [], 0
    while True:
        while i < len(text) and text[i].isspace():
            i += 1
        if i >= len(text):
            return out, ""
        try:
            obj, i = dec.raw_decode(text, i)
        except ValueError:
            return out, text[i:]
        out.append(obj)
