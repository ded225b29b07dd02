"""Client side of exec / attach / port-forward through the apiserver, over the WebSocket
channel protocols or SPDY/3.1 (reference staging/src/k8s.io/client-go/tools/remotecommand
{v4,v3,v2}.go and tools/portforward/portforward.go). See runtime/streaming.py and
runtime/spdy.py for the framing; `transport="spdy"` is what a v1.9 kubectl speaks."""
from __future__ import annotations

import asyncio
import json
from urllib.parse import urlencode

from aiohttp import WSMsgType

from ..runtime import spdy
from ..runtime.streaming import CHANNEL_PROTOCOLS, ERROR, PORTFORWARD_PROTOCOLS, STDERR, STDIN, STDOUT, status_exit_code


def _path(ns, pod, sub):
    return f"/api/v1/namespaces/{ns}/pods/{pod}/{sub}"


def _auth(client) -> dict:
    return {k: v for k, v in client.headers.items() if k in ("Authorization", "User-Agent")}


async def _stdin_chunks(stdin):
    if isinstance(stdin, (bytes, bytearray)):
        if stdin:
            yield bytes(stdin)
    else:
        async for chunk in stdin:
            yield chunk


async def _exec_spdy(client, url, stdin, tty, on_stdout, on_stderr, resize) -> int:
    """remotecommand over SPDY: one stream per channel, the error stream first (v2+)."""
    sess, proto = await spdy.connect(url, spdy.EXEC_PROTOCOLS, headers=_auth(client), ssl=client.ssl)
    try:
        err = await sess.open_stream({"streamtype": "error"})
        await err.close()                       # the client never writes to it
        sin = await sess.open_stream({"streamtype": "stdin"}) if stdin is not None else None
        sout = await sess.open_stream({"streamtype": "stdout"})
        serr = None if tty else await sess.open_stream({"streamtype": "stderr"})
        rsz = await sess.open_stream({"streamtype": "resize"}) if tty and proto in ("v3.channel.k8s.io", "v4.channel.k8s.io") else None

        async def copy(st, sink):
            while True:
                data = await st.read()
                if not data:
                    return
                sink(data)

        async def feed():
            async for chunk in _stdin_chunks(stdin):
                await sin.write(chunk)
            await sin.close()
        tasks = [asyncio.create_task(copy(sout, on_stdout))] + ([asyncio.create_task(copy(serr, on_stderr))] if serr else [])
        feeder = asyncio.create_task(feed()) if sin is not None else None
        if rsz is not None and resize:
            await rsz.write(json.dumps({"Width": resize[0], "Height": resize[1]}).encode())
        status = await err.read_all()
        await asyncio.gather(*tasks)
        if feeder is not None:
            feeder.cancel()
        if proto == "v4.channel.k8s.io":
            st = json.loads(status or b"{}")
            if st.get("status") == "Failure" and st.get("reason") != "NonZeroExitCode" and st.get("message"):
                on_stderr((st["message"] + "\n").encode())
            return status_exit_code(status) if status else 0
        if status:
            on_stderr(status + b"\n")
            text = status.decode(errors="replace")
            return int(text.rsplit(":", 1)[1]) if "non-zero exit code" in text and text.rsplit(":", 1)[1].strip().isdigit() else 1
        return 0
    finally:
        await sess.aclose()


async def exec_stream(client, ns: str, pod: str, command: list[str], container: str | None = None, stdin=None,
                      tty: bool = False, on_stdout=None, on_stderr=None, attach: bool = False,
                      transport: str = "websocket", resize: tuple[int, int] | None = None) -> int:
    """Run `command` in the container (or attach to it) and return its exit code. `stdin` is
    bytes (sent, then EOF), an async iterator of bytes (interactive), or None. `transport` is
    "websocket" or "spdy"; `resize` = (width, height) of the tty (SPDY v3+ resize stream)."""
    params = [("stdout", "true"), ("stderr", "true"), ("tty", "true" if tty else "false"),
              ("stdin", "true" if stdin is not None else "false")]
    if container:
        params.append(("container", container))
    if not attach:
        params += [("command", c) for c in command]
    url = client.server + _path(ns, pod, "attach" if attach else "exec") + "?" + urlencode(params)
    out, err = bytearray(), bytearray()
    on_stdout = on_stdout or out.extend
    on_stderr = on_stderr or err.extend
    rc = 1
    if transport == "spdy":
        rc = await _exec_spdy(client, url, stdin, tty, on_stdout, on_stderr, resize)
        exec_stream.last_output = (bytes(out), bytes(err))
        return rc
    async with client.session.ws_connect(url, protocols=CHANNEL_PROTOCOLS, ssl=client.ssl, max_msg_size=0) as ws:
        async def feed():
            if isinstance(stdin, (bytes, bytearray)):
                if stdin:
                    await ws.send_bytes(bytes([STDIN]) + bytes(stdin))
                await ws.send_bytes(bytes([STDIN]))   # zero-length frame: EOF
            elif stdin is not None:
                async for chunk in stdin:
                    await ws.send_bytes(bytes([STDIN]) + chunk)
                await ws.send_bytes(bytes([STDIN]))
        feeder = asyncio.create_task(feed()) if stdin is not None else None
        async for msg in ws:
            if msg.type != WSMsgType.BINARY or not msg.data:
                if msg.type in (WSMsgType.CLOSE, WSMsgType.CLOSED, WSMsgType.ERROR):
                    break
                continue
            ch, data = msg.data[0], msg.data[1:]
            if ch == STDOUT:
                on_stdout(data)
            elif ch == STDERR:
                on_stderr(data)
            elif ch == ERROR:
                st = json.loads(data or b"{}")
                rc = status_exit_code(data)
                if st.get("status") == "Failure" and st.get("reason") != "NonZeroExitCode" and st.get("message"):
                    on_stderr((st["message"] + "\n").encode())
        if feeder is not None:
            feeder.cancel()
    exec_stream.last_output = (bytes(out), bytes(err))
    return rc


async def port_forward(client, ns: str, pod: str, mappings: list[str], ready=None, stop: asyncio.Event | None = None,
                       address: str = "127.0.0.1", transport: str = "websocket"):
    """`LOCAL:REMOTE` listeners. Over WebSocket every accepted connection opens its own
    portforward WebSocket; over SPDY one upgraded connection carries them all, a (data, error)
    stream pair per accepted connection keyed by `requestID` (portforward.go handleConnection)."""
    servers = []
    if transport == "spdy":
        return await _port_forward_spdy(client, ns, pod, mappings, ready, stop, address)

    async def handle(r, w, remote):
        url = client.server + _path(ns, pod, "portforward") + "?" + urlencode([("ports", str(remote))])
        try:
            async with client.session.ws_connect(url, protocols=PORTFORWARD_PROTOCOLS, ssl=client.ssl, max_msg_size=0) as ws:
                async def up():
                    while True:
                        data = await r.read(65536)
                        if not data:
                            return
                        await ws.send_bytes(bytes([0]) + data)

                async def down():
                    seen = set()
                    async for msg in ws:
                        if msg.type != WSMsgType.BINARY or not msg.data:
                            if msg.type in (WSMsgType.CLOSE, WSMsgType.CLOSED, WSMsgType.ERROR):
                                return
                            continue
                        ch, data = msg.data[0], msg.data[1:]
                        if ch not in seen:     # each channel opens with the port number
                            seen.add(ch)
                            continue
                        if ch == 0:
                            w.write(data)
                            await w.drain()
                        elif ch == 1 and data:
                            return
                t1, t2 = asyncio.create_task(up()), asyncio.create_task(down())
                await asyncio.wait({t1, t2}, return_when=asyncio.FIRST_COMPLETED)
                t1.cancel()
                t2.cancel()
        finally:
            w.close()

    for mp in mappings:
        local, _, remote = mp.partition(":")
        remote = int(remote or local)
        srv = await asyncio.start_server(lambda r, w, remote=remote: handle(r, w, remote), address, int(local or 0))
        servers.append(srv)
        print(f"Forwarding from {address}:{srv.sockets[0].getsockname()[1]} -> {remote}", flush=True)
    if ready is not None:
        ready.set_result([s.sockets[0].getsockname()[1] for s in servers])
    try:
        await (stop.wait() if stop is not None else asyncio.Event().wait())
    finally:
        for s in servers:
            s.close()


async def _port_forward_spdy(client, ns, pod, mappings, ready, stop, address):
    url = client.server + _path(ns, pod, "portforward")
    sess, _ = await spdy.connect(url, spdy.PORTFORWARD_PROTOCOLS, headers=_auth(client), ssl=client.ssl)
    next_id = iter(range(1 << 31))
    conns: set[asyncio.Task] = set()

    async def handle(r, w, remote):
        rid = str(next(next_id))
        try:
            err = await sess.open_stream({"streamtype": "error", "port": str(remote), "requestid": rid})
            await err.close()
            data = await sess.open_stream({"streamtype": "data", "port": str(remote), "requestid": rid})
        except spdy.SpdyError:
            w.close()
            return

        async def up():
            while True:
                chunk = await r.read(65536)
                if not chunk:
                    break
                await data.write(chunk)
            await data.close()

        async def down():
            while True:
                chunk = await data.read()
                if not chunk:
                    return
                w.write(chunk)
                await w.drain()

        async def errors():
            msg = await err.read_all()
            if msg:
                print(f"E portforward {remote}: {msg.decode(errors='replace')}", flush=True)
        t_up, t_down, t_err = asyncio.create_task(up()), asyncio.create_task(down()), asyncio.create_task(errors())
        try:
            await t_down
        except (spdy.SpdyError, ConnectionError):
            pass
        finally:
            t_up.cancel()
            await asyncio.gather(t_err, return_exceptions=True)
            w.close()

    def accepted(r, w, remote):
        t = asyncio.create_task(handle(r, w, remote))
        conns.add(t)
        t.add_done_callback(conns.discard)
    servers = []
    for mp in mappings:
        local, _, remote = mp.partition(":")
        remote = int(remote or local)
        srv = await asyncio.start_server(lambda r, w, remote=remote: accepted(r, w, remote), address, int(local or 0))
        servers.append(srv)
        print(f"Forwarding from {address}:{srv.sockets[0].getsockname()[1]} -> {remote}", flush=True)
    if ready is not None:
        ready.set_result([s.sockets[0].getsockname()[1] for s in servers])
    try:
        waits = [asyncio.create_task(sess.closed.wait())]
        if stop is not None:
            waits.append(asyncio.create_task(stop.wait()))
        await asyncio.wait(waits, return_when=asyncio.FIRST_COMPLETED)
        for t in waits:
            t.cancel()
    finally:
        for s in servers:
            s.close()
        for t in list(conns):
            t.cancel()
        await asyncio.gather(*conns, return_exceptions=True)
        await sess.aclose()


__all__ = ["exec_stream", "port_forward"]
