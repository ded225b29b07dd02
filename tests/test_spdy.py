"""SPDY/3.1 exec / attach / port-forward (reference: vendor/github.com/docker/spdystream framing,
staging/src/k8s.io/apimachinery/pkg/util/httpstream/spdy/{connection,upgrade}_test.go,
pkg/kubelet/server/remotecommand/httpstream.go stream set-up, pkg/kubelet/server/portforward/
httpstream_test.go request-ID pairing). The in-repo client (client/stream.py, transport="spdy")
drives the same path a v1.9 kubectl does: apiserver → kubelet → runtime streaming server, the two
relays splicing raw bytes."""
import asyncio
import json
import os
import socket
import struct
import zlib

import pytest

from amdkube.client.stream import exec_stream, port_forward
from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.runtime import spdy


def test_dictionary_and_header_blocks():
    # the zlib DICTID every SPDY/3 header stream announces (RFC 1950 FDICT = Adler-32 of the dictionary)
    assert len(spdy.DICTIONARY) == 1423 and zlib.adler32(spdy.DICTIONARY) == 0xE3C6A7C2
    hdrs = {"streamtype": "stdin", "port": ["8080"], "multi": ["a", "b"]}
    blk = spdy.encode_headers(hdrs)
    assert blk[:4] == struct.pack(">I", 3) and spdy.decode_headers(blk) == {"streamtype": ["stdin"], "port": ["8080"],
                                                                             "multi": ["a", "b"]}
    c = zlib.compressobj(zlib.Z_DEFAULT_COMPRESSION, zlib.DEFLATED, 15, zdict=spdy.DICTIONARY)
    z = c.compress(blk) + c.flush(zlib.Z_SYNC_FLUSH)
    assert z[1] & 0x20 and struct.unpack(">I", z[2:6])[0] == 0xE3C6A7C2     # FDICT set, DICTID present
    # control frame layout: 1 | version 3 | type ; flags | 24-bit length
    f = spdy.control_frame(spdy.PING, struct.pack(">I", 7))
    assert f == bytes([0x80, 0x03, 0x00, 0x06, 0x00, 0x00, 0x00, 0x04, 0, 0, 0, 7])
    assert spdy.data_frame(5, b"hi", spdy.FLAG_FIN) == bytes([0, 0, 0, 5, 1, 0, 0, 2]) + b"hi"
    assert spdy.split_json('{"Width":80,"Height":24}\n{"Width":1') == ([{"Width": 80, "Height": 24}], '{"Width":1')


def _pipe():
    """Two sessions wired back to back in memory (writes of one are the other's input)."""
    srv_streams = []

    async def on_stream(st):
        srv_streams.append(st)
        await st.reply()
    server, client = spdy.Session(True, on_stream), spdy.Session(False)

    async def nodrain():
        await asyncio.sleep(0)
    server.attach(lambda b: client.feed(b), nodrain, lambda: client.connection_lost())
    client.attach(lambda b: server.feed(b), nodrain, lambda: server.connection_lost())
    return server, client, srv_streams


async def test_session_streams_half_close_ping_reset():
    server, client, got = _pipe()
    a = await client.open_stream({"streamtype": "stdin"})
    b = await client.open_stream({"streamtype": "stdout"})
    assert (a.id, b.id) == (1, 3) and [s.header("streamtype") for s in got] == ["stdin", "stdout"]
    await a.write(b"x" * 200_000)                 # > one data frame
    await a.close()
    assert await got[0].read_all() == b"x" * 200_000
    await got[1].write(b"out")
    await got[1].close()
    assert await b.read_all() == b"out"
    assert await client.ping() >= 0 and await server.ping() >= 0
    c = await client.open_stream({"streamtype": "stderr"})
    await got[2].rst()
    await asyncio.sleep(0)
    assert c.reset and await c.read() == b""
    # many header blocks share one zlib context per direction
    for i in range(20):
        await client.open_stream({"streamtype": "data", "requestid": str(i), "port": "80"})
    assert [s.header("requestid") for s in got[3:]] == [str(i) for i in range(20)]
    await client.close()
    assert server.closed.is_set() and client.closed.is_set()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _raw_upgrade(url, token, protocols):
    """A bare upgrade request, to see what a refused negotiation answers."""
    try:
        await spdy.connect(url, protocols, headers={"Authorization": f"Bearer {token}"})
    except spdy.SpdyError as e:
        return str(e)
    return "upgraded"


@pytest.mark.timeout(120)
async def test_spdy_exec_attach_port_forward_through_apiserver():
    port = _free_port()
    async with LocalCluster(gpus="none", relist_period=0.2) as lc:
        c = lc.client
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "sh"},
                        "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}, "default")
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "web"},
                        "spec": {"containers": [{"name": "w", "image": "python:3",
                                                 "command": ["python3", "-m", "http.server", str(port), "--bind", "127.0.0.1"],
                                                 "ports": [{"containerPort": port}]}]}}, "default")
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "ticker"},
                        "spec": {"restartPolicy": "Never", "containers": [{"name": "t", "image": "busybox", "command": [
                            "sh", "-c", "sleep 1; for i in 1 2 3; do echo tick$i; sleep 0.2; done; exit 4"]}]}}, "default")
        for n in ("sh", "web", "ticker"):
            await wait_pod(c, "default", n, ("Running",), 20)

        # stdin + stdout + stderr + error streams, non-zero exit through the v4 Status
        out, err = bytearray(), bytearray()
        rc = await exec_stream(c, "default", "sh", ["sh", "-c", "cat; echo oops >&2; exit 3"], stdin=b"ping" * 50000,
                               on_stdout=out.extend, on_stderr=err.extend, transport="spdy")
        assert (rc, bytes(out), bytes(err)) == (3, b"ping" * 50000, b"oops\n")
        # tty + resize stream (v3+): the window size reaches the pty before the command reads it
        out = bytearray()
        rc = await exec_stream(c, "default", "sh", ["sh", "-c", "sleep 0.5; stty size"], tty=True, resize=(132, 43),
                               on_stdout=out.extend, transport="spdy")
        assert rc == 0 and bytes(out).strip() == b"43 132"
        # attach over SPDY follows output until exit
        out = bytearray()
        rc = await exec_stream(c, "default", "ticker", [], attach=True, on_stdout=out.extend, transport="spdy")
        assert rc == 4 and b"tick1\ntick2\ntick3\n" in bytes(out)

        # kubectl cp (upload through stdin, download through stdout) rides SPDY by default
        import tempfile
        from amdkube.kubectl.main import main as kubectl
        d = tempfile.mkdtemp(prefix="spdycp", dir="/tmp")
        src, back = os.path.join(d, "src.bin"), os.path.join(d, "back.bin")
        with open(src, "wb") as f:
            f.write(os.urandom(300_000))
        args = ["--server", c.server, "--token", c.headers["Authorization"].split(" ", 1)[1]]
        assert await asyncio.to_thread(kubectl, args + ["cp", src, f"default/sh:{d}/in-pod.bin"]) in (0, None)
        assert await asyncio.to_thread(kubectl, args + ["cp", f"default/sh:{d}/in-pod.bin", back]) in (0, None)
        assert open(back, "rb").read() == open(src, "rb").read()

        # older protocol versions: v2 reports the exit as error-stream text
        url = (f"{c.server}/api/v1/namespaces/default/pods/sh/exec?command=sh&command=-c&command=exit+5"
               f"&stdout=true&stderr=true")
        sess, proto = await spdy.connect(url, ["v2.channel.k8s.io"], headers={"Authorization": c.headers["Authorization"]})
        try:
            assert proto == "v2.channel.k8s.io"
            e = await sess.open_stream({"streamtype": "error"})
            o = await sess.open_stream({"streamtype": "stdout"})
            await sess.open_stream({"streamtype": "stderr"})
            assert b"non-zero exit code: 5" in await e.read_all()
            assert await o.read_all() == b""
        finally:
            await sess.aclose()
        # an unknown protocol is refused with 403 and the accepted list, relayed back through both hops
        msg = await _raw_upgrade(url, lc.api.loopback_token, ["v9.channel.k8s.io"])
        assert "403" in msg and "unable to negotiate protocol" in msg

        # port-forward: one SPDY connection, a stream pair per forwarded TCP connection
        for _ in range(50):
            try:
                _r, _w = await asyncio.open_connection("127.0.0.1", port)
                _w.close()
                break
            except OSError:
                await asyncio.sleep(0.1)
        ready, stop = asyncio.get_running_loop().create_future(), asyncio.Event()
        t = asyncio.create_task(port_forward(c, "default", "web", [f"0:{port}"], ready=ready, stop=stop, transport="spdy"))
        [local] = await ready

        async def get():
            r, w = await asyncio.open_connection("127.0.0.1", local)
            w.write(b"GET / HTTP/1.0\r\n\r\n")
            await w.drain()
            data = await asyncio.wait_for(r.read(), 10)
            w.close()
            return data
        bodies = await asyncio.gather(get(), get(), get())
        assert all(b.startswith(b"HTTP/1.0 200") and b"Directory listing" in b for b in bodies)
        stop.set()
        await asyncio.wait_for(t, 10)
        # a port nothing listens on: the error stream says so and the data stream ends
        ready, stop = asyncio.get_running_loop().create_future(), asyncio.Event()
        t = asyncio.create_task(port_forward(c, "default", "web", [f"0:{_free_port()}"], ready=ready, stop=stop,
                                             transport="spdy"))
        [local] = await ready
        r, w = await asyncio.open_connection("127.0.0.1", local)
        assert await asyncio.wait_for(r.read(), 10) == b""
        w.close()
        stop.set()
        await asyncio.wait_for(t, 10)


async def test_spdy_refuses_bad_streams():
    """portforward/httpstream.go: streams without a port header or with an unknown type are reset."""
    server, client, got = _pipe()
    server.on_stream = None                       # no handler: every stream is refused
    with pytest.raises(spdy.SpdyError, match="reset"):
        await client.open_stream({"streamtype": "data"}, timeout=5)
    await client.close()
    assert json.dumps(spdy.exec_streams_expected("v4.channel.k8s.io", True, True, True, True), default=sorted) == \
        json.dumps(["error", "resize", "stdin", "stdout"])


def test_header_block_bombs_and_garbage_end_the_session():
    """A SYN_STREAM whose header block inflates past MAX_HEADER_BLOCK, or a truncated block,
    is a SpdyError (the session ends) rather than unbounded memory or an unhandled error."""

    def syn(block):
        return spdy.control_frame(spdy.SYN_STREAM, struct.pack(">IIH", 1, 0, 0) + block)

    bomb = struct.pack(">I", 1) + struct.pack(">I", 1) + b"x" + struct.pack(">I", 4 << 20) + b"a" * (4 << 20)
    z = zlib.compressobj(zlib.Z_DEFAULT_COMPRESSION, zlib.DEFLATED, 15, zdict=spdy.DICTIONARY)
    packed = z.compress(bomb) + z.flush(zlib.Z_SYNC_FLUSH)
    assert len(packed) < (1 << 24)

    async def run():
        for frame in (syn(packed), syn(b"\x00garbage")):
            sess = spdy.Session(server=True)
            with pytest.raises(spdy.SpdyError):
                sess.feed(frame)
    asyncio.run(run())
