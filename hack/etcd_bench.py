"""Write latency/throughput of the store topologies (CPU only).

  embedded   MVCCStore.put in process (the default apiserver store)
  etcd-1     Etcd3Store fenced CAS Txn against one `amdkube etcd` process
  raft-3     the same against a 3-member raft group (client talks to a follower: forward + commit)
  apiserver  pod creates/s through APIServer over each backend: one serial client, and 32
             concurrent clients (writes from concurrent requests group-commit into shared Txns)

  python hack/etcd_bench.py            prints one JSON object
"""
import asyncio
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import grpc  # noqa: E402

from amdkube.apiserver import APIServer  # noqa: E402
from amdkube.client import Client  # noqa: E402
from amdkube.grpcdesc.etcd import ETCD as E  # noqa: E402
from amdkube.store import MVCCStore  # noqa: E402
from amdkube.store.etcd3 import Etcd3Store  # noqa: E402

N = 2000
VALUE = b'{"kind":"Pod","metadata":{"name":"x","resourceVersion":"1"},"spec":{"containers":[{"name":"c","image":"busybox"}]}}'


def ports(n):
    ss = [socket.socket() for _ in range(n)]
    for s in ss:
        s.bind(("127.0.0.1", 0))
    out = [s.getsockname()[1] for s in ss]
    for s in ss:
        s.close()
    return out


def spawn(tmp, n):
    ps = ports(2 * n)
    names = [f"m{i}" for i in range(n)]
    client = {nm: f"127.0.0.1:{ps[i]}" for i, nm in enumerate(names)}
    peer = {nm: f"127.0.0.1:{ps[n + i]}" for i, nm in enumerate(names)}
    procs = []
    for nm in names:
        args = [sys.executable, "-m", "amdkube", "etcd", "--listen-client-urls", f"http://{client[nm]}",
                "--data-dir", os.path.join(tmp, nm)]
        if n > 1:
            args += ["--name", nm, "--initial-cluster", ",".join(f"{k}=http://{v}" for k, v in peer.items()),
                     "--listen-peer-urls", f"http://{peer[nm]}"]
        procs.append(subprocess.Popen(args, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
    for nm in names:                      # wait for every member, then for a leader
        end = time.time() + 30
        while True:
            try:
                with grpc.insecure_channel(client[nm]) as ch:
                    st = E.Maintenance.stub(ch).Status(E.StatusRequest(), timeout=1)
                if st.leader:
                    break
            except grpc.RpcError:
                pass
            if time.time() > end:
                raise RuntimeError(f"{nm} not ready")
            time.sleep(0.1)
    return procs, client


def timed_puts(store, n=N):
    lat = []
    t0 = time.perf_counter()
    for i in range(n):
        a = time.perf_counter()
        store.put(f"/registry/bench/default/k{i}", VALUE)
        lat.append(time.perf_counter() - a)
    el = time.perf_counter() - t0
    lat.sort()
    return {"puts": n, "puts_per_s": round(n / el, 1), "p50_ms": round(lat[n // 2] * 1e3, 3),
            "p99_ms": round(lat[int(n * 0.99)] * 1e3, 3)}


async def concurrent_puts(endpoint, writers=64, n=4000):
    """Raw etcd Puts from `writers` concurrent clients (one aio channel each) through `endpoint`."""
    chans = [grpc.aio.insecure_channel(endpoint) for _ in range(writers)]
    lat = []

    async def writer(w):
        kv = E.KV.stub(chans[w])
        for i in range(w, n, writers):
            a = time.perf_counter()
            await kv.Put(E.PutRequest(key=f"/registry/conc/k{i}".encode(), value=VALUE), timeout=30)
            lat.append(time.perf_counter() - a)
    t0 = time.perf_counter()
    await asyncio.gather(*(writer(w) for w in range(writers)))
    el = time.perf_counter() - t0
    for c in chans:
        await c.close()
    lat.sort()
    return {"writers": writers, "puts": n, "puts_per_s": round(n / el, 1), "p50_ms": round(lat[n // 2] * 1e3, 3),
            "p99_ms": round(lat[int(n * 0.99)] * 1e3, 3)}


async def pod_creates(store, n=500, clients=1):
    srv = await APIServer(store).start()
    cs = [Client(srv.url, token=srv.loopback_token) for _ in range(clients)]

    async def one(k):
        for i in range(k, n, clients):
            await cs[k].create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{clients}-{i}", "namespace": "default"},
                                "spec": {"containers": [{"name": "c", "image": "busybox"}]}}, "default")
    try:
        t0 = time.perf_counter()
        await asyncio.gather(*(one(k) for k in range(clients)))
        return round(n / (time.perf_counter() - t0), 1)
    finally:
        for c in cs:
            await c.close()
        await srv.stop()


async def main():
    out = {}
    out["embedded"] = timed_puts(MVCCStore())
    out["embedded"]["apiserver_pod_creates_per_s"] = await pod_creates(MVCCStore())
    out["embedded"]["apiserver_pod_creates_per_s_32_clients"] = await pod_creates(MVCCStore(), 1000, 32)
    for label, n in (("etcd-1", 1), ("raft-3", 3)):
        with tempfile.TemporaryDirectory() as tmp:
            procs, client = spawn(tmp, n)
            try:
                eps = list(client.values())
                s = await asyncio.to_thread(Etcd3Store, eps[-1:] + eps[:-1])   # a follower first in raft-3
                s.start(asyncio.get_running_loop())
                out[label] = timed_puts(s)
                s.close()
                out[label]["concurrent"] = await concurrent_puts(eps[-1])
                s = await asyncio.to_thread(Etcd3Store, eps[-1:] + eps[:-1])
                out[label]["transport"] = s.transport
                out[label]["apiserver_pod_creates_per_s"] = await pod_creates(s)
                out[label]["apiserver_pod_creates_per_s_32_clients"] = await pod_creates(s, 1000, 32)
                s.close()
            finally:
                for p in procs:
                    p.terminate()
                for p in procs:
                    p.wait(10)
    print(json.dumps(out))


if __name__ == "__main__":
    asyncio.run(main())
