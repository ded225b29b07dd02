"""Debug (round 4): a gpu-burn pod on the MI355X node, its status and log after a few seconds."""
import asyncio, json, sys, time
sys.path.insert(0, ".")
from amdkube.localcluster import LocalCluster


async def main():
    async with LocalCluster(gpus="amdsmi", n_gpus=1, relist_period=0.5, with_controllers=False) as lc:
        await lc.wait_gpus(1, 60)
        c = lc.client
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "burner", "namespace": "default"},
                        "spec": {"restartPolicy": "Never", "containers": [{"name": "burn", "image": "amdkube/gpu-burn",
                                                                           "args": ["--ms", "8000"],
                                                                           "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "plain", "namespace": "default"},
                        "spec": {"restartPolicy": "Never", "containers": [{"name": "plain", "image": "busybox",
                                                                           "command": ["sleep", "20"]}]}})
        t0 = time.time()
        for _ in range(24):
            for nm in ("burner", "plain"):
                p = await c.get("pods", nm, "default")
                st = p.get("status") or {}
                print(round(time.time() - t0, 2), nm, st.get("phase"), json.dumps([x.get("state") for x in st.get("containerStatuses") or []])[:300], flush=True)
            await asyncio.sleep(0.5)
        print("LOGS burner:", (await c.logs("default", "burner"))[-800:], flush=True)
        print("LOGS plain:", (await c.logs("default", "plain"))[-800:], flush=True)
        print("shim:", lc.shim.isolation, [(x.name, x.state, x.exit_code, x.reason) for x in lc.shim.containers.values()], flush=True)

asyncio.run(main())
