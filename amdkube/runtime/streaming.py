"""CRI streaming: exec / attach / port-forward over WebSocket.

Reference: pkg/kubelet/server/streaming/server.go (the runtime's streaming server hands out
one-shot tokens from GetExec/GetAttach/GetPortForward, request_cache.go: 1 min TTL),
pkg/kubelet/server/remotecommand/websocket.go + apimachinery wsstream (channel protocol: one
byte of channel id per binary frame — 0 stdin, 1 stdout, 2 stderr, 3 error (v4: a JSON
metav1.Status), 4 resize), pkg/kubelet/server/portforward/websocket.go (per requested port:
data channel 2i and error channel 2i+1, each opened with the port as 2-byte little-endian).

The kubelet and the apiserver relay these WebSockets hop by hop (`bridge`), so a client only
ever talks to the apiserver, as in the reference.
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
        app.router.add_get("/exec/{token}", self._exec)
        app.router.add_get("/attach/{token}", self._attach)
        app.router.add_get("/portforward/{token}", self._portforward)
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

    # ---------------------------------------------------------------- exec
    async def _exec(self, request):
        req = self._take(request, "exec")
        c = self.shim.containers.get(req["cid"])
        ws = web.WebSocketResponse(protocols=CHANNEL_PROTOCOLS, max_msg_size=0)
        await ws.prepare(request)
        if c is None or c.pid is None:
            await ws.send_bytes(bytes([ERROR]) + exit_status(None, f"container {req['cid']} is not running"))
            await ws.close()
            return ws
        env = dict(c.env)
        master = None
        if req["tty"]:
            master, slave = os.openpty()
            proc = await asyncio.create_subprocess_exec(*req["cmd"], stdin=slave, stdout=slave, stderr=slave, env=env,
                                                        cwd=c.cwd, start_new_session=True)
            os.close(slave)
        else:
            try:
                proc = await asyncio.create_subprocess_exec(
                    *req["cmd"], env=env, cwd=c.cwd, start_new_session=True,
                    stdin=asyncio.subprocess.PIPE if req["stdin"] else asyncio.subprocess.DEVNULL,
                    stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE)
            except OSError as e:
                await ws.send_bytes(bytes([ERROR]) + exit_status(None, f"exec failed: {e}"))
                await ws.close()
                return ws
        loop = asyncio.get_running_loop()

        async def pump(reader, ch):
            while True:
                data = await reader.read(32768)
                if not data:
                    return
                await ws.send_bytes(bytes([ch]) + data)

        async def pump_pty():
            q: asyncio.Queue = asyncio.Queue()
            loop.add_reader(master, lambda: q.put_nowait(_read_nb(master)))
            try:
                while True:
                    data = await q.get()
                    if not data:
                        return
                    await ws.send_bytes(bytes([STDOUT]) + data)
            finally:
                loop.remove_reader(master)

        async def inbound():
            async for msg in ws:
                if msg.type != WSMsgType.BINARY or not msg.data:
                    continue
                ch, data = msg.data[0], msg.data[1:]
                if ch == STDIN:
                    if master is not None:
                        os.write(master, data)
                    elif proc.stdin is not None:
                        if not data:     # zero-length stdin frame: EOF
                            proc.stdin.close()
                        else:
                            proc.stdin.write(data)
                            await proc.stdin.drain()
                elif ch == 255 and data[:1] == bytes([STDIN]) and proc.stdin is not None:   # v5 close(stdin)
                    proc.stdin.close()
                elif ch == RESIZE and master is not None:
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
        await ws.send_bytes(bytes([ERROR]) + exit_status(rc))
        await ws.close()
        return ws

    # ---------------------------------------------------------------- attach
    async def _attach(self, request):
        req = self._take(request, "attach")
        c = self.shim.containers.get(req["cid"])
        ws = web.WebSocketResponse(protocols=CHANNEL_PROTOCOLS, max_msg_size=0)
        await ws.prepare(request)
        if c is None:
            await ws.send_bytes(bytes([ERROR]) + exit_status(None, f"container {req['cid']} not found"))
            return await _close(ws)
        if req["stdin"]:
            await ws.send_bytes(bytes([ERROR]) + exit_status(None, "containers run with stdin closed; attach is output-only"))
            return await _close(ws)
        # stream what the container writes from now on (its stdout/stderr share the log file)
        try:
            off = os.path.getsize(c.log_path)
        except OSError:
            off = 0
        from ..grpcdesc.cri import CRI as C
        while not ws.closed:
            try:
                with open(c.log_path, "rb") as f:
                    f.seek(off)
                    data = f.read()
            except OSError:
                data = b""
            if data:
                off += len(data)
                await ws.send_bytes(bytes([STDOUT]) + data)
            if c.state == C.CONTAINER_EXITED and not data:
                await ws.send_bytes(bytes([ERROR]) + exit_status(c.exit_code))
                break
            await asyncio.sleep(0.05)
        return await _close(ws)

    # ---------------------------------------------------------------- port-forward
    async def _portforward(self, request):
        req = self._take(request, "portforward")
        s = self.shim.sandboxes.get(req["sid"])
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


def _read_nb(fd):
    try:
        return os.read(fd, 32768)
    except OSError:
        return b""


async def _close(ws):
    if not ws.closed:
        await ws.close()
    return ws
