"""CRI streaming: exec / attach / port-forward over WebSocket or SPDY/3.1 (runtime/spdy.py).

Reference: pkg/kubelet/server/streaming/server.go (the runtime's streaming server hands out
one-shot tokens from GetExec/GetAttach/GetPortForward, request_cache.go: 1 min TTL),
pkg/kubelet/server/remotecommand/websocket.go + apimachinery wsstream (channel protocol: one
byte of channel id per binary frame — 0 stdin, 1 stdout, 2 stderr, 3 error (v4: a JSON
metav1.Status), 4 resize), pkg/kubelet/server/portforward/websocket.go (per requested port:
data channel 2i and error channel 2i+1, each opened with the port as 2-byte little-endian).

The kubelet and the apiserver relay these WebSockets hop by hop (`bridge`), and SPDY upgrades
as raw byte splices (`spdy.upgrade_proxy`), so a client only ever talks to the apiserver, as in
the reference. exec and attach run the same code over either transport through a channel
adapter (`_WsChannels` / `_SpdyChannels`).
"""
from __future__ import annotations

import asyncio
import fcntl
import json
import os
import secrets
import struct
import termios
import time

from aiohttp import ClientSession, WSMsgType, web

from . import spdy

CHANNEL_PROTOCOLS = ("v4.channel.k8s.io", "channel.k8s.io")
PORTFORWARD_PROTOCOLS = ("portforward.k8s.io", "v4.channel.k8s.io")
STDIN, STDOUT, STDERR, ERROR, RESIZE = 0, 1, 2, 3, 4
TOKEN_TTL = 60.0


def exit_status(rc: int | None, message: str = "") -> bytes:
    """v4 error-channel payload (remotecommand/websocket.go writeStatus)."""
    if rc == 0:
        return json.dumps({"metadata": {}, "status": "Success"}).encode()
    if rc is None:
        return json.dumps({"metadata": {}, "status": "Failure", "message": message, "reason": "InternalError"}).encode()
    return json.dumps({"metadata": {}, "status": "Failure", "message": message or f"command terminated with non-zero exit code: {rc}",
                       "reason": "NonZeroExitCode",
                       "details": {"causes": [{"reason": "ExitCode", "message": str(rc)}]}}).encode()


def status_exit_code(payload: bytes) -> int:
    st = json.loads(payload or b"{}")
    if st.get("status") == "Success":
        return 0
    for c in (st.get("details") or {}).get("causes") or []:
        if c.get("reason") == "ExitCode":
            return int(c.get("message", "1"))
    return 1


async def bridge(ws_in: web.WebSocketResponse, url: str, protocols, headers=None, ssl=None):
    """Relay a server-side WebSocket to an upstream one (kubelet → runtime, apiserver → kubelet)."""
    async with ClientSession() as s:
        async with s.ws_connect(url, protocols=protocols, headers=headers or {}, ssl=ssl, max_msg_size=0) as up:
            async def down():
                async for msg in up:
                    if msg.type == WSMsgType.BINARY:
                        await ws_in.send_bytes(msg.data)
                    elif msg.type == WSMsgType.TEXT:
                        await ws_in.send_str(msg.data)
                    else:
                        break
                await ws_in.close()

            async def upward():
                async for msg in ws_in:
                    if msg.type == WSMsgType.BINARY:
                        await up.send_bytes(msg.data)
                    elif msg.type == WSMsgType.TEXT:
                        await up.send_str(msg.data)
                    else:
                        break
                await up.close()
            t1, t2 = asyncio.create_task(down()), asyncio.create_task(upward())
            done, pending = await asyncio.wait({t1, t2}, return_when=asyncio.FIRST_COMPLETED)
            if t1 in done:   # upstream finished: let the last frames drain, then stop reading the client
                t2.cancel()
            else:
                try:
                    await asyncio.wait_for(t1, 5)
                except asyncio.TimeoutError:
                    t1.cancel()
    return ws_in


class StreamingServer:
    """The runtime side: token → request, served on its own loopback HTTP port."""

    def __init__(self, shim, address: str = "127.0.0.1", port: int = 0):
        self.shim, self.address, self.port = shim, address, port
        self.requests: dict[str, tuple[str, dict, float]] = {}
        self.runner = None
        self.base = ""

    async def start(self):
        app = web.Application()
        for meth in ("GET", "POST"):       # WebSocket upgrades are GETs, SPDY ones POSTs
            app.router.add_route(meth, "/exec/{token}", self._exec)
            app.router.add_route(meth, "/attach/{token}", self._attach)
            app.router.add_route(meth, "/portforward/{token}", self._portforward)
        self.runner = web.AppRunner(app, access_log=None)
        await self.runner.setup()
        site = web.TCPSite(self.runner, self.address, self.port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        self.base = f"http://{self.address}:{self.port}"
        return self

    async def stop(self):
        if self.runner is not None:
            await self.runner.cleanup()

    def _token(self, kind: str, req: dict) -> str:
        now = time.monotonic()
        for k in [k for k, v in self.requests.items() if v[2] < now]:
            del self.requests[k]
        tok = secrets.token_urlsafe(12)
        self.requests[tok] = (kind, req, now + TOKEN_TTL)
        return f"{self.base}/{kind}/{tok}"

    def get_exec(self, cid, cmd, tty, stdin, stdout, stderr) -> str:
        return self._token("exec", {"cid": cid, "cmd": list(cmd), "tty": tty, "stdin": stdin, "stdout": stdout, "stderr": stderr})

    def get_attach(self, cid, tty, stdin, stdout, stderr) -> str:
        return self._token("attach", {"cid": cid, "tty": tty, "stdin": stdin, "stdout": stdout, "stderr": stderr})

    def get_portforward(self, sid, ports) -> str:
        return self._token("portforward", {"sid": sid, "ports": list(ports)})

    def _take(self, request, kind):
        ent = self.requests.pop(request.match_info["token"], None)
        if ent is None or ent[0] != kind or ent[2] < time.monotonic():
            raise web.HTTPNotFound(text="unknown or expired streaming token")
        return ent[1]

    # ---------------------------------------------------------------- transports
    async def _channels(self, request, req: dict, proto_ws):
        """Upgrade to whichever transport the client asked for and return the channel adapter
        (None after answering a refused upgrade)."""
        if spdy.is_upgrade(request):
            box: dict[str, spdy.Stream] = {}
            want = None
            arrived = asyncio.Event()

            async def on_stream(st):
                kind = st.header("streamtype")
                if kind not in _SPDY_CHANNELS or kind in box:
                    await st.rst(spdy.RST_PROTOCOL_ERROR)
                    return
                box[kind] = st
                await st.reply()
                if want is not None and want <= set(box):
                    arrived.set()
            sess, proto, resp = await spdy.accept(request, spdy.EXEC_PROTOCOLS, on_stream)
            if sess is None:
                return resp, None
            want = spdy.exec_streams_expected(proto, req.get("stdin", False), req.get("stdout", True),
                                              req.get("stderr", True), req.get("tty", False))
            if want <= set(box):
                arrived.set()
            try:
                await asyncio.wait_for(arrived.wait(), spdy.STREAM_CREATION_TIMEOUT)
            except asyncio.TimeoutError:
                await sess.close()
                return resp, None
            return resp, _SpdyChannels(sess, proto, box)
        ws = web.WebSocketResponse(protocols=proto_ws, max_msg_size=0)
        await ws.prepare(request)
        return ws, _WsChannels(ws)

    # ---------------------------------------------------------------- exec
    async def _exec(self, request):
        req = self._take(request, "exec")
        c = self.shim.containers.get(req["cid"])
        resp, ch = await self._channels(request, req, CHANNEL_PROTOCOLS)
        if ch is None:
            return resp
        if c is None or c.pid is None:
            await ch.finish(None, f"container {req['cid']} is not running")
            return resp
        env = dict(c.env)
        master = None
        # inside the container: its namespaces, cgroup and device guard (rocshim.exec_argv)
        argv = self.shim.exec_argv(c, req["cmd"]) if hasattr(self.shim, "exec_argv") else list(req["cmd"])
        cwd = self.shim.exec_cwd(c) if hasattr(self.shim, "exec_cwd") else c.cwd
        if req["tty"]:
            master, slave = os.openpty()
            proc = await asyncio.create_subprocess_exec(*argv, stdin=slave, stdout=slave, stderr=slave, env=env,
                                                        cwd=cwd, start_new_session=True)
            os.close(slave)
        else:
            try:
                proc = await asyncio.create_subprocess_exec(
                    *argv, env=env, cwd=cwd, start_new_session=True,
                    stdin=asyncio.subprocess.PIPE if req["stdin"] else asyncio.subprocess.DEVNULL,
                    stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE)
            except OSError as e:
                await ch.finish(None, f"exec failed: {e}")
                return resp
        loop = asyncio.get_running_loop()

        async def pump(reader, chan):
            while True:
                data = await reader.read(32768)
                if not data:
                    return
                await ch.send(chan, data)

        async def pump_pty():
            q: asyncio.Queue = asyncio.Queue()
            loop.add_reader(master, lambda: q.put_nowait(_read_nb(master)))
            try:
                while True:
                    data = await q.get()
                    if not data:
                        return
                    await ch.send(STDOUT, data)
            finally:
                loop.remove_reader(master)

        async def inbound():
            async for chan, data in ch.inbound():
                if chan == STDIN:
                    if master is not None:
                        if data:
                            os.write(master, data)
                    elif proc.stdin is not None:
                        if not data:     # EOF: zero-length stdin frame / v5 close / SPDY FIN
                            proc.stdin.close()
                        else:
                            proc.stdin.write(data)
                            await proc.stdin.drain()
                elif chan == RESIZE and master is not None:
                    sz = json.loads(data or b"{}")
                    fcntl.ioctl(master, termios.TIOCSWINSZ, struct.pack("HHHH", sz.get("Height", 24), sz.get("Width", 80), 0, 0))

        tasks = [asyncio.create_task(pump_pty())] if master is not None else \
            [asyncio.create_task(pump(proc.stdout, STDOUT)), asyncio.create_task(pump(proc.stderr, STDERR))]
        rx = asyncio.create_task(inbound())
        rc = await proc.wait()
        await asyncio.gather(*tasks, return_exceptions=True)
        rx.cancel()
        if master is not None:
            os.close(master)
        await ch.finish(rc)
        return resp

    # ---------------------------------------------------------------- attach
    async def _attach(self, request):
        req = self._take(request, "attach")
        c = self.shim.containers.get(req["cid"])
        resp, ch = await self._channels(request, req, CHANNEL_PROTOCOLS)
        if ch is None:
            return resp
        if c is None:
            await ch.finish(None, f"container {req['cid']} not found")
            return resp
        if req["stdin"]:
            await ch.finish(None, "containers run with stdin closed; attach is output-only")
            return resp
        # stream what the container writes from now on: its log file's records (the CRI log
        # format the log pump writes), each to its own stream
        from ..kubelet import logs as L
        try:
            off = os.path.getsize(c.log_path)
        except OSError:
            off = 0
        from ..grpcdesc.cri import CRI as C
        pending, parse = b"", None
        while not ch.closed():
            try:
                with open(c.log_path, "rb") as f:
                    f.seek(off)
                    data = f.read()
            except OSError:
                data = b""
            if data:
                off += len(data)
                pending += data
                cut = pending.rfind(b"\n") + 1
                lines, pending = pending[:cut].splitlines(keepends=True), pending[cut:]
                for ln in lines:
                    parse = parse or L.get_parse_func(ln, allow_raw=True)
                    try:
                        msg = parse(ln)
                    except ValueError:
                        continue
                    await ch.send(STDERR if msg.stream == L.STDERR else STDOUT, msg.log)
            if c.state == C.CONTAINER_EXITED and not data:
                if pending:
                    await ch.send(STDOUT, pending)
                await ch.finish(c.exit_code)
                break
            await asyncio.sleep(0.05)
        return resp

    # ---------------------------------------------------------------- port-forward
    async def _portforward(self, request):
        req = self._take(request, "portforward")
        s = self.shim.sandboxes.get(req["sid"])
        if spdy.is_upgrade(request):
            return await self._portforward_spdy(request, req, s)
        ws = web.WebSocketResponse(protocols=PORTFORWARD_PROTOCOLS, max_msg_size=0)
        await ws.prepare(request)
        ports = [int(p) for p in request.query.getall("port", [])] or req["ports"]
        if s is None or not ports:
            return await _close(ws)
        host = s.ip or self.shim.network.node_ip
        writers = {}
        for i, p in enumerate(ports):   # each channel opens with its port (websocket.go:handlePortForward)
            await ws.send_bytes(bytes([2 * i]) + struct.pack("<H", p))
            await ws.send_bytes(bytes([2 * i + 1]) + struct.pack("<H", p))
        readers = []
        for i, p in enumerate(ports):
            try:
                r, w = await asyncio.open_connection(host, p)
            except OSError as e:
                await ws.send_bytes(bytes([2 * i + 1]) + f"failed to connect to {host}:{p}: {e}".encode())
                continue
            writers[2 * i] = w

            async def pump(r=r, ch=2 * i):
                while True:
                    data = await r.read(65536)
                    if not data:
                        return
                    await ws.send_bytes(bytes([ch]) + data)
            readers.append(asyncio.create_task(pump()))

        async def inbound():
            async for msg in ws:
                if msg.type != WSMsgType.BINARY or not msg.data:
                    continue
                w = writers.get(msg.data[0])
                if w is not None and len(msg.data) > 1:
                    w.write(msg.data[1:])
                    await w.drain()
        rx = asyncio.create_task(inbound())
        if readers:
            both = asyncio.gather(*readers, return_exceptions=True)
            await asyncio.wait({rx, both}, return_when=asyncio.FIRST_COMPLETED)
            for w in writers.values():   # the client hung up or every target closed
                w.close()
            both.cancel()
        rx.cancel()
        return await _close(ws)


    async def _portforward_spdy(self, request, req, s):
        """portforward/httpstream.go: one upgraded connection carries any number of forwarded
        connections, each a (data, error) stream pair keyed by the `requestid` header."""
        host = (s.ip if s is not None else None) or self.shim.network.node_ip
        pairs: dict[str, dict] = {}
        jobs: set[asyncio.Task] = set()

        async def forward(data, err):
            port = int(data.header("port"))
            try:
                if s is None:
                    raise OSError("pod sandbox is gone")
                r, w = await asyncio.open_connection(host, port)
            except OSError as e:
                await err.write(f"error forwarding port {port} to pod sandbox {req['sid']}: {e}".encode())
                await err.close()
                await data.close()
                return

            async def upward():
                while True:
                    chunk = await data.read()
                    if not chunk:
                        break
                    w.write(chunk)
                    await w.drain()
                if w.can_write_eof():
                    w.write_eof()
            up = asyncio.create_task(upward())
            try:
                while True:
                    chunk = await r.read(65536)
                    if not chunk:
                        break
                    await data.write(chunk)
            except (spdy.SpdyError, ConnectionError):
                pass
            finally:
                up.cancel()
                w.close()
                for st in (data, err):
                    try:
                        await st.close()
                    except (spdy.SpdyError, ConnectionError):
                        pass

        async def on_stream(st):
            kind, port = st.header("streamtype"), st.header("port")
            if kind not in ("data", "error") or not port.isdigit():
                await st.rst(spdy.RST_PROTOCOL_ERROR)
                return
            rid = st.header("requestid") or str(st.id if kind == "error" else st.id - 2)   # pre-requestID clients
            pair = pairs.setdefault(rid, {})
            if kind in pair:
                await st.rst(spdy.RST_PROTOCOL_ERROR)
                return
            await st.reply()
            pair[kind] = st
            if len(pair) == 2:
                del pairs[rid]
                t = asyncio.create_task(forward(pair["data"], pair["error"]))
                jobs.add(t)
                t.add_done_callback(jobs.discard)
        sess, _, resp = await spdy.accept(request, spdy.PORTFORWARD_PROTOCOLS, on_stream)
        if sess is None:
            return resp
        try:
            await sess.closed.wait()
        finally:
            for t in list(jobs):
                t.cancel()
        return resp


_SPDY_CHANNELS = {"stdin": STDIN, "stdout": STDOUT, "stderr": STDERR, "error": ERROR, "resize": RESIZE}


class _WsChannels:
    """Channel-prefixed binary WebSocket frames (one byte of channel id per frame)."""

    def __init__(self, ws):
        self.ws = ws

    def closed(self) -> bool:
        return self.ws.closed

    async def send(self, ch: int, data: bytes):
        await self.ws.send_bytes(bytes([ch]) + data)

    async def inbound(self):
        async for msg in self.ws:
            if msg.type != WSMsgType.BINARY or not msg.data:
                continue
            ch, data = msg.data[0], msg.data[1:]
            if ch == 255 and data[:1]:           # v5 close(channel)
                yield data[0], b""
            else:
                yield ch, data

    async def finish(self, rc, message: str = ""):
        if not self.ws.closed:
            await self.ws.send_bytes(bytes([ERROR]) + exit_status(rc, message))
        await _close(self.ws)


class _SpdyChannels:
    """One SPDY stream per channel; EOF is the stream's FIN; the error stream carries a
    metav1.Status (v4) or the error text (v1-v3)."""

    def __init__(self, sess, proto: str, streams: dict):
        self.sess, self.proto = sess, proto
        self.by_ch = {_SPDY_CHANNELS[k]: st for k, st in streams.items()}

    def closed(self) -> bool:
        return self.sess.closed.is_set()

    async def send(self, ch: int, data: bytes):
        st = self.by_ch.get(ch)
        if st is not None and not st.local_closed and not self.closed():
            await st.write(data)

    async def inbound(self):
        q: asyncio.Queue = asyncio.Queue()

        async def rd(ch, st):
            buf = ""
            try:
                while True:
                    data = await st.read()
                    if ch == STDIN:
                        q.put_nowait((STDIN, data))
                    elif data:
                        objs, buf = spdy.split_json(buf + data.decode(errors="replace"))
                        for o in objs:
                            q.put_nowait((RESIZE, json.dumps(o).encode()))
                    if not data:
                        return
            finally:
                q.put_nowait(None)
        tasks = [asyncio.create_task(rd(ch, st)) for ch, st in self.by_ch.items() if ch in (STDIN, RESIZE)]
        try:
            if not tasks:
                await self.sess.closed.wait()
                return
            left = len(tasks)
            while left:
                item = await q.get()
                if item is None:
                    left -= 1
                else:
                    yield item
        finally:
            for t in tasks:
                t.cancel()

    async def finish(self, rc, message: str = ""):
        err = self.by_ch.get(ERROR)
        try:
            if err is not None and not self.closed():
                if self.proto == "v4.channel.k8s.io":
                    await err.write(exit_status(rc, message))
                elif rc != 0:
                    await err.write((message or f"command terminated with non-zero exit code: {rc}").encode())
            for st in self.by_ch.values():
                await st.close()
        except (spdy.SpdyError, ConnectionError):
            pass
        await self.sess.close()


def _read_nb(fd):
    try:
        return os.read(fd, 32768)
    except OSError:
        return b""


async def _close(ws):
    if not ws.closed:
        await ws.close()
    return ws
