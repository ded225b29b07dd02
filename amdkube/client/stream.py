"""Client side of exec / attach / port-forward through the apiserver (WebSocket channel
protocols; reference staging/src/k8s.io/client-go/tools/remotecommand and
tools/portforward, websocket variants). See runtime/streaming.py for the framing."""
from __future__ import annotations

import asyncio
import json
from urllib.parse import urlencode

from aiohttp import WSMsgType

from ..runtime.streaming import CHANNEL_PROTOCOLS, ERROR, PORTFORWARD_PROTOCOLS, STDERR, STDIN, STDOUT, status_exit_code


def _path(ns, pod, sub):
    return f"/api/v1/namespaces/{ns}/pods/{pod}/{sub}"


async def exec_stream(client, ns: str, pod: str, command: list[str], container: str | None = None, stdin=None,
                      tty: bool = False, on_stdout=None, on_stderr=None, attach: bool = False) -> int:
    """Run `command` in the container (or attach to it) and return its exit code. `stdin` is
    bytes (sent, then EOF), an async iterator of bytes (interactive), or None."""
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
                       address: str = "127.0.0.1"):
    """`LOCAL:REMOTE` listeners; every accepted connection opens its own portforward WebSocket."""
    servers = []

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


__all__ = ["exec_stream", "port_forward"]
