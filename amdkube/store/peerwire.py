"""Member-to-member transport of the raft group: length-prefixed protobuf frames over one TCP
(optionally mutual-TLS) connection per peer, calls multiplexed by id.

etcd does not run raft over gRPC either: its peers talk rafthttp, long-lived HTTP streams of
raft messages (vendor/github.com/coreos/etcd/rafthttp/stream.go). The reason holds here too:
Python gRPC aio costs about a millisecond per unary round trip on loopback, which put one
full millisecond into every commit (leader → follower AppendEntries → ack). This transport
costs a tenth of that, so a commit is bounded by the follower's fdatasync, not the RPC stack.

The same framing also carries the etcd client API between `amdkube etcd` and the apiserver's
Etcd3Store (the "wire lane", EtcdServer.start(wire_address=...)): the apiserver makes one
blocking KV call per write, and gRPC's per-call cost on both ends was most of an etcd-1 Txn.
gRPC stays the public client API; the lane is advertised to clients in the `amdkube-wire`
initial metadata of Maintenance.Status and used only by clients that see it.

Frames: u32 big-endian length, then
  request   u8 0 | u32 id | u8 len(path) | path "/pkg.Service/Method" | request message
  response  u8 1 | u32 id | response message
  error     u8 2 | u32 id | u8 grpc status code | utf-8 message
  message   u8 3 | u32 id | one server-stream message          (streaming methods)
  end       u8 4 | u32 id                                      (stream finished)
  cancel    u8 5 | u32 id                                      (client ends its stream)
  cmessage  u8 6 | u32 id | one more client-stream message     (bidi methods)
The server dispatches each request to its own task (handlers may wait on raft), so replies can
come back out of order; the client matches them by id. Failures surface as `PeerRpcError`, a
grpc.RpcError with code()/details(), so raft and the etcd server handle them as before.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import socket
import ssl
import struct
import threading

import grpc

log = logging.getLogger("amdkube.peerwire")

REQ, RESP, ERR, MSG, END, CANCEL, CMSG = 0, 1, 2, 3, 4, 5, 6
MAX_FRAME = 256 << 20


class PeerRpcError(grpc.RpcError):
    def __init__(self, code: grpc.StatusCode, details: str):
        super().__init__(f"{code.name}: {details}")
        self._code, self._details = code, details

    def code(self):
        return self._code

    def details(self):
        return self._details


_CODES = {c.value[0]: c for c in grpc.StatusCode}


def server_ssl(cert: str, key: str, ca: str | None) -> ssl.SSLContext:
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(cert, key)
    if ca:
        ctx.load_verify_locations(ca)
        ctx.verify_mode = ssl.CERT_REQUIRED          # members only
    return ctx


def client_ssl(cert: str | None, key: str | None, ca: str | None) -> ssl.SSLContext:
    ctx = ssl.create_default_context(ssl.Purpose.SERVER_AUTH, cafile=ca)
    if cert and key:
        ctx.load_cert_chain(cert, key)
    return ctx


class _Ctx:
    """The handler context a PeerServer passes where gRPC passes its ServicerContext."""

    async def abort(self, code, details):
        raise PeerRpcError(code, details)

    def invocation_metadata(self):
        return ()


_CTX = _Ctx()


def _frame(kind: int, cid: int, body: bytes = b"") -> bytes:
    return struct.pack(">IBI", 5 + len(body), kind, cid) + body


def _err_frame(cid: int, code: grpc.StatusCode, msg: str) -> bytes:
    return _frame(ERR, cid, bytes([code.value[0]]) + msg[:4000].encode())


async def _read_frame(reader: asyncio.StreamReader) -> bytes:
    (n,) = struct.unpack(">I", await reader.readexactly(4))
    if n < 5 or n > MAX_FRAME:
        raise ConnectionError(f"bad peer frame length {n}")
    return await reader.readexactly(n)


class PeerServer:
    """Serves the methods of `bindings` [(compiler.Service, impl)] to member connections."""

    def __init__(self, bindings, ssl_ctx: ssl.SSLContext | None = None):
        self.methods = {}
        self.streams = {}               # streaming methods: path -> (req_cls, fn, client_streaming)
        for svc, impl in bindings:
            for name, req, _resp, stream, cstream in svc.methods:
                fn = getattr(impl, name, None)
                if fn is None:
                    continue
                if stream or cstream:
                    self.streams[f"/{svc.full_name}/{name}"] = (req, fn, cstream)
                else:
                    self.methods[f"/{svc.full_name}/{name}"] = (req, fn)
        self.ssl = ssl_ctx
        self.server: asyncio.AbstractServer | None = None
        self._conns: set[asyncio.Task] = set()
        self.port = 0

    async def start(self, address: str) -> int:
        host, _, port = address.rpartition(":")
        self.server = await asyncio.start_server(self._serve, host or "127.0.0.1", int(port), ssl=self.ssl,
                                                 limit=1 << 20, reuse_address=True)
        self.port = self.server.sockets[0].getsockname()[1]
        return self.port

    async def stop(self):
        if self.server is not None:
            self.server.close()
        for t in list(self._conns):
            t.cancel()
        for t in list(self._conns):
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        if self.server is not None:
            await self.server.wait_closed()

    async def _serve(self, reader, writer):
        task = asyncio.current_task()
        self._conns.add(task)
        inflight: set[asyncio.Task] = set()
        streams: dict[int, tuple] = {}           # id -> (task, request queue, request class)
        try:
            while True:
                frame = await _read_frame(reader)
                kind, cid = frame[0], struct.unpack_from(">I", frame, 1)[0]
                if kind == REQ and (len(frame) < 6 or len(frame) < 6 + frame[5]):
                    raise ConnectionError("truncated request frame")
                if kind == CMSG or kind == CANCEL:
                    ent = streams.get(cid)
                    if ent is not None:
                        if kind == CANCEL:
                            ent[0].cancel()
                        else:
                            ent[1].put_nowait(ent[2].FromString(frame[5:]))
                    continue
                if kind != REQ:
                    raise ConnectionError("peer sent a non-request frame")
                plen = frame[5]
                path = frame[6:6 + plen].decode(errors="replace")
                sm = self.streams.get(path)
                if sm is not None:
                    q: asyncio.Queue = asyncio.Queue()
                    q.put_nowait(sm[0].FromString(frame[6 + plen:]))
                    t = asyncio.create_task(self._stream(writer, cid, sm, q))
                    streams[cid] = (t, q, sm[0])
                    t.add_done_callback(lambda _t, c=cid: streams.pop(c, None))
                else:
                    t = asyncio.create_task(self._one(writer, cid, path, frame[6 + plen:]))
                inflight.add(t)
                t.add_done_callback(inflight.discard)
        except (asyncio.IncompleteReadError, ConnectionError, ssl.SSLError, OSError):
            pass
        except asyncio.CancelledError:
            pass
        except Exception as e:       # noqa: BLE001 — a malformed message ends this connection only
            log.debug("peer connection dropped: %r", e)
        finally:
            for t in list(inflight):
                t.cancel()
            writer.close()
            self._conns.discard(task)

    async def _one(self, writer, cid: int, path: str, payload: bytes):
        ent = self.methods.get(path)
        if ent is None:
            body = bytes([ERR]) + struct.pack(">IB", cid, grpc.StatusCode.UNIMPLEMENTED.value[0]) + f"no method {path}".encode()
        else:
            req_cls, fn = ent
            try:
                resp = await fn(req_cls.FromString(payload), _CTX)
                body = bytes([RESP]) + struct.pack(">I", cid) + resp.SerializeToString()
            except asyncio.CancelledError:
                raise
            except PeerRpcError as e:
                body = bytes([ERR]) + struct.pack(">IB", cid, e.code().value[0]) + e.details()[:4000].encode()
            except Exception as e:   # noqa: BLE001 — the caller gets the error, the connection lives on
                log.debug("peer method %s failed: %r", path, e)
                body = bytes([ERR]) + struct.pack(">IB", cid, grpc.StatusCode.UNKNOWN.value[0]) + str(e)[:4000].encode()
        try:
            writer.write(struct.pack(">I", len(body)) + body)
            if len(body) > 1 << 16:
                await writer.drain()
        except (ConnectionError, RuntimeError):
            pass

    async def _stream(self, writer, cid: int, ent, q: asyncio.Queue):
        """A streaming method: its responses go out as MSG frames, then END (or ERR)."""
        req_cls, fn, client_streaming = ent

        async def requests():
            while True:
                yield await q.get()

        try:
            gen = fn(requests() if client_streaming else q.get_nowait(), _CTX)
            async for resp in gen:
                writer.write(_frame(MSG, cid, resp.SerializeToString()))
                if writer.transport.get_write_buffer_size() > 1 << 20:
                    await writer.drain()                 # a slow reader holds the stream, not memory
            writer.write(_frame(END, cid))
        except asyncio.CancelledError:
            pass
        except PeerRpcError as e:
            writer.write(_err_frame(cid, e.code(), e.details()))
        except (ConnectionError, RuntimeError):
            pass
        except Exception as e:   # noqa: BLE001
            log.debug("peer stream %d failed: %r", cid, e)
            try:
                writer.write(_err_frame(cid, grpc.StatusCode.UNKNOWN, str(e)))
            except (ConnectionError, RuntimeError):
                pass


class SyncChannel:
    """A blocking client of a PeerServer for callers that block anyway (Etcd3Store's writes,
    its watch thread): one call in flight per channel, no event loop involved. A stream gets
    a channel of its own. Connection and protocol failures are PeerRpcError(UNAVAILABLE) and
    drop the socket; the next call reconnects."""

    def __init__(self, target: str, ssl_ctx: ssl.SSLContext | None = None, connect_timeout: float = 3.0):
        self.target = target.split("://", 1)[-1].rstrip("/")
        self.ssl = ssl_ctx
        self.connect_timeout = connect_timeout
        self._sock: socket.socket | None = None
        self._ids = itertools.count(1)
        self._lock = threading.Lock()

    def _connect(self) -> socket.socket:
        if self._sock is None:
            host, _, port = self.target.rpartition(":")
            try:
                s = socket.create_connection((host, int(port)), timeout=self.connect_timeout)
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                if self.ssl is not None:
                    s = self.ssl.wrap_socket(s, server_hostname=host)
            except (OSError, ssl.SSLError) as e:
                raise PeerRpcError(grpc.StatusCode.UNAVAILABLE, f"connect {self.target}: {e}") from None
            self._sock = s
        return self._sock

    def _drop(self):
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
            self._sock = None

    def _recv(self, s: socket.socket, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = s.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("connection closed")
            buf += chunk
        return bytes(buf)

    def _read(self, s: socket.socket) -> bytes:
        (n,) = struct.unpack(">I", self._recv(s, 4))
        if n < 5 or n > MAX_FRAME:
            raise ConnectionError(f"bad peer frame length {n}")
        return self._recv(s, n)

    def _send_req(self, s: socket.socket, cid: int, path: str, payload: bytes):
        p = path.encode()
        s.sendall(_frame(REQ, cid, bytes([len(p)]) + p + payload))

    def call(self, path: str, payload: bytes, timeout: float | None = None) -> bytes:
        with self._lock:
            s = self._connect()
            cid = next(self._ids) & 0xFFFFFFFF
            try:
                s.settimeout(timeout)
                self._send_req(s, cid, path, payload)
                while True:
                    frame = self._read(s)
                    if struct.unpack_from(">I", frame, 1)[0] == cid:
                        break
            except socket.timeout:
                self._drop()              # a late reply must not be read as the next call's
                raise PeerRpcError(grpc.StatusCode.DEADLINE_EXCEEDED, f"{path} to {self.target} timed out") from None
            except (OSError, ConnectionError, ssl.SSLError) as e:
                self._drop()
                raise PeerRpcError(grpc.StatusCode.UNAVAILABLE, f"{path} to {self.target}: {e}") from None
        if frame[0] == RESP:
            return frame[5:]
        if frame[0] == ERR:
            raise PeerRpcError(_CODES.get(frame[5], grpc.StatusCode.UNKNOWN), frame[6:].decode(errors="replace"))
        self._drop()
        raise PeerRpcError(grpc.StatusCode.UNAVAILABLE, f"{path}: unexpected frame kind {frame[0]}")

    def stream(self, path: str, payload: bytes):
        """Open a streaming call; yields each response message's bytes until the server ends
        it. close() from another thread unblocks the reader (as a cancelled call)."""
        s = self._connect()
        cid = next(self._ids) & 0xFFFFFFFF
        try:
            s.settimeout(None)
            self._send_req(s, cid, path, payload)
            while True:
                frame = self._read(s)
                if struct.unpack_from(">I", frame, 1)[0] != cid:
                    continue
                if frame[0] == MSG:
                    yield frame[5:]
                elif frame[0] == END:
                    return
                elif frame[0] == ERR:
                    raise PeerRpcError(_CODES.get(frame[5], grpc.StatusCode.UNKNOWN), frame[6:].decode(errors="replace"))
                else:
                    raise ConnectionError(f"unexpected frame kind {frame[0]}")
        except (OSError, ConnectionError, ssl.SSLError) as e:
            closed = self._sock is None
            self._drop()
            raise PeerRpcError(grpc.StatusCode.CANCELLED if closed else grpc.StatusCode.UNAVAILABLE,
                               f"{path} stream to {self.target}: {e}") from None

    def close(self):
        s, self._sock = self._sock, None
        if s is not None:
            try:
                s.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            s.close()


class PeerChannel:
    """One lazily (re)connected connection to a member's peer listener."""

    def __init__(self, target: str, ssl_ctx: ssl.SSLContext | None = None):
        self.target = target.split("://", 1)[-1].rstrip("/")
        self.ssl = ssl_ctx
        self._reader = self._writer = None
        self._rtask: asyncio.Task | None = None
        self._pending: dict[int, asyncio.Future] = {}
        self._ids = itertools.count(1)
        self._lock = asyncio.Lock()
        self.closed = False

    async def _connect(self):
        async with self._lock:
            if self._writer is not None:
                return
            if self.closed:
                raise PeerRpcError(grpc.StatusCode.CANCELLED, "channel closed")
            host, _, port = self.target.rpartition(":")
            try:
                self._reader, self._writer = await asyncio.open_connection(
                    host, int(port), ssl=self.ssl, server_hostname=host if self.ssl else None, limit=1 << 20)
            except (OSError, ssl.SSLError) as e:
                raise PeerRpcError(grpc.StatusCode.UNAVAILABLE, f"connect {self.target}: {e}") from None
            self._rtask = asyncio.create_task(self._read_loop(self._reader, self._writer), name=f"peer-{self.target}")

    async def _read_loop(self, reader, writer):
        err = PeerRpcError(grpc.StatusCode.UNAVAILABLE, f"connection to {self.target} lost")
        try:
            while True:
                frame = await _read_frame(reader)
                kind, cid = frame[0], struct.unpack_from(">I", frame, 1)[0]
                fut = self._pending.pop(cid, None)
                if fut is None or fut.done():
                    continue
                if kind == RESP:
                    fut.set_result(frame[5:])
                else:
                    code = _CODES.get(frame[5], grpc.StatusCode.UNKNOWN)
                    fut.set_exception(PeerRpcError(code, frame[6:].decode(errors="replace")))
        except (asyncio.IncompleteReadError, ConnectionError, ssl.SSLError, OSError):
            pass
        except asyncio.CancelledError:
            err = PeerRpcError(grpc.StatusCode.CANCELLED, "channel closed")
        finally:
            if self._writer is writer:
                self._reader = self._writer = None
            writer.close()
            for fut in self._pending.values():
                if not fut.done():
                    fut.set_exception(err)
            self._pending.clear()

    async def call(self, path: str, payload: bytes, timeout: float | None = None) -> bytes:
        if self._writer is None:
            await self._connect()
        cid = next(self._ids) & 0xFFFFFFFF
        fut = asyncio.get_running_loop().create_future()
        self._pending[cid] = fut
        p = path.encode()
        body = struct.pack(">BIB", REQ, cid, len(p)) + p + payload
        try:
            self._writer.write(struct.pack(">I", len(body)) + body)
            if len(body) > 1 << 16:
                await self._writer.drain()
        except (ConnectionError, AttributeError, RuntimeError) as e:
            self._pending.pop(cid, None)
            raise PeerRpcError(grpc.StatusCode.UNAVAILABLE, f"send to {self.target}: {e}") from None
        try:
            return await asyncio.wait_for(fut, timeout)
        except asyncio.TimeoutError:
            self._pending.pop(cid, None)
            raise PeerRpcError(grpc.StatusCode.DEADLINE_EXCEEDED, f"{path} to {self.target} timed out") from None

    async def close(self):
        self.closed = True
        if self._rtask is not None:
            self._rtask.cancel()
            try:
                await self._rtask
            except (asyncio.CancelledError, Exception):
                pass
        if self._writer is not None:
            self._writer.close()
            self._writer = None

    async def __aenter__(self):
        return self

    async def __aexit__(self, *exc):
        await self.close()


class _Stub:
    def __init__(self, svc, channel: PeerChannel):
        for name, req, resp, stream, cstream in svc.methods:
            if stream or cstream:
                continue
            setattr(self, name, self._method(channel, f"/{svc.full_name}/{name}", resp))

    @staticmethod
    def _method(channel, path, resp_cls):
        async def call(request, timeout: float | None = None):
            return resp_cls.FromString(await channel.call(path, request.SerializeToString(), timeout))
        return call


def stub(svc, channel: PeerChannel) -> _Stub:
    """`svc` (a grpcdesc.compiler.Service)'s unary methods as coroutines over `channel`."""
    return _Stub(svc, channel)
