"""apiserver CPU per request, JSON vs protobuf responses, JSON vs protobuf storage.

In-process APIServer, 200 GPU pods; raw aiohttp reads (bodies are not decoded), so the
process CPU time is the server's. Prints one JSON object.   python hack/proto_vs_json.py
"""
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import aiohttp  # noqa: E402

from amdkube.api import protobuf as pb  # noqa: E402
from amdkube.apiserver import APIServer  # noqa: E402
from amdkube.client import Client  # noqa: E402

N_PODS, N_GET, N_LIST = 200, 400, 20


def pod(i):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i:04d}", "namespace": "default", "labels": {"app": "x"}},
            "spec": {"containers": [{"name": "c", "image": "rocm/vector-add", "resources": {"limits": {"amd.com/gpu": "1", "cpu": "1"}}}]}}


async def measure(storage):
    srv = await APIServer(options={"storage_media_type": storage}).start()
    c = Client(srv.url, token=srv.loopback_token)
    out = {}
    try:
        for i in range(N_PODS):
            await c.create(pod(i))
        async with aiohttp.ClientSession() as s:
            for accept in ("application/json", pb.MEDIA_TYPE):
                h = {"Accept": accept, "Authorization": f"Bearer {srv.loopback_token}"}

                async def get(path):
                    async with s.get(srv.url + path, headers=h) as r:
                        return len(await r.read())
                await get("/api/v1/namespaces/default/pods/p0000")
                c0 = time.process_time()
                for i in range(N_GET):
                    size = await get(f"/api/v1/namespaces/default/pods/p{i % N_PODS:04d}")
                g = (time.process_time() - c0) / N_GET * 1e6
                c0 = time.process_time()
                for _ in range(N_LIST):
                    lsize = await get("/api/v1/namespaces/default/pods")
                lst = (time.process_time() - c0) / N_LIST * 1e3
                out[accept] = {"get_cpu_us": round(g, 1), "get_bytes": size, "list200_cpu_ms": round(lst, 2),
                               "list200_bytes": lsize}
    finally:
        await c.close()
        await srv.stop()
    return out


async def main():
    res = {"pods": N_PODS, "storage_json": await measure("application/json"),
           "storage_protobuf": await measure(pb.MEDIA_TYPE)}
    print(json.dumps(res))


if __name__ == "__main__":
    asyncio.run(main())
