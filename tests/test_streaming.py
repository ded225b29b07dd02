"""exec / attach / port-forward / proxy through the apiserver (reference
pkg/kubelet/server/streaming/server_test.go, remotecommand websocket tests,
test/e2e/kubectl port-forward and exec cases, registry pod subresource proxy tests)."""
import asyncio
import socket

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.client.stream import exec_stream, port_forward
from amdkube.localcluster import LocalCluster, wait_pod


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def test_exec_attach_port_forward_proxy(tmp_path):
    port = _free_port()
    async with LocalCluster(gpus="none", relist_period=0.2, api_kw={"authorization_mode": "RBAC",
                                                                     "token_auth": {"viewer-token": {"name": "viewer"}}}) as lc:
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
        out, err = bytearray(), bytearray()
        rc = await exec_stream(c, "default", "sh", ["sh", "-c", "echo hi; echo oops >&2; exit 3"],
                               on_stdout=out.extend, on_stderr=err.extend)
        assert (rc, bytes(out), bytes(err)) == (3, b"hi\n", b"oops\n")
        out = bytearray()
        assert await exec_stream(c, "default", "sh", ["cat"], stdin=b"x" * 100000, on_stdout=out.extend) == 0
        assert bytes(out) == b"x" * 100000
        out = bytearray()
        assert await exec_stream(c, "default", "sh", ["tty"], tty=True, on_stdout=out.extend) == 0
        assert bytes(out).startswith(b"/dev/pts/")
        # attach follows the container's output until it exits
        out = bytearray()
        rc = await exec_stream(c, "default", "ticker", [], attach=True, on_stdout=out.extend)
        assert rc == 4 and b"tick1\ntick2\ntick3\n" in bytes(out)
        # port-forward through apiserver → kubelet → runtime
        for _ in range(50):
            try:
                _r, _w = await asyncio.open_connection("127.0.0.1", port)
                _w.close()
                break
            except OSError:
                await asyncio.sleep(0.1)
        ready, stop = asyncio.get_running_loop().create_future(), asyncio.Event()
        t = asyncio.create_task(port_forward(c, "default", "web", [f"0:{port}"], ready=ready, stop=stop))
        [local] = await ready
        r, w = await asyncio.open_connection("127.0.0.1", local)
        w.write(b"GET / HTTP/1.0\r\n\r\n")
        await w.drain()
        data = await asyncio.wait_for(r.read(), 10)
        assert data.startswith(b"HTTP/1.0 200") and b"Directory listing" in data
        w.close()
        stop.set()
        await t
        # pods/{name}:{port}/proxy/ → the pod's HTTP server
        body = await c.request("GET", f"/api/v1/namespaces/default/pods/web:{port}/proxy/", raw=True)
        assert b"Directory listing" in body
        # exec needs create on pods/exec: a token without RBAC grants is refused
        viewer = Client(c.server, token="viewer-token")
        try:
            await exec_stream(viewer, "default", "sh", ["true"])
            raise AssertionError("exec must be forbidden")
        except Exception as e:
            assert "403" in str(e) or isinstance(e, m.StatusError)
        finally:
            await viewer.close()
