"""Static pods from --pod-manifest-path and their mirror pods (reference
pkg/kubelet/config/file_test.go, pkg/kubelet/pod/mirror_client_test.go,
test/e2e_node/mirror_pod_test.go: a mirror pod appears, is recreated when deleted, follows
manifest updates, and goes away with the manifest)."""
from __future__ import annotations

import asyncio
import os

import yaml

from amdkube.api import meta as m
from amdkube.localcluster import LocalCluster


async def until(fn, timeout=20.0, every=0.05):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    last = None
    while loop.time() < end:
        last = await fn()
        if last:
            return last
        await asyncio.sleep(every)
    raise TimeoutError(f"condition not met (last={last!r})")


def write_manifest(d, name, image="amdkube/pause:3.1", args=None):
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "kube-system", "labels": {"tier": "control"}},
           "spec": {"containers": [{"name": "c", "image": image, **({"args": args} if args else {})}]}}
    p = os.path.join(d, f"{name}.yaml")
    with open(p + ".tmp", "w") as f:
        yaml.safe_dump(pod, f)
    os.replace(p + ".tmp", p)
    return p


async def test_static_pod_mirror_lifecycle(tmp_path):
    mdir = tmp_path / "manifests"
    mdir.mkdir()
    write_manifest(str(mdir), "etcd-lite")
    async with LocalCluster(gpus="none", relist_period=0.2,
                            kubelet_kw={"pod_manifest_path": str(mdir), "file_check_frequency": 0.2}) as lc:
        c = lc.client
        name = f"etcd-lite-{lc.node_name}"

        async def mirror_running():
            p = await c.get_or_none("pods", name, "kube-system")
            return p if p and (p.get("status") or {}).get("phase") == "Running" else None
        mp = await until(mirror_running)
        ann = m.annotations_of(mp)
        assert ann["kubernetes.io/config.source"] == "file" and ann["kubernetes.io/config.mirror"] == ann["kubernetes.io/config.hash"]
        assert mp["spec"]["nodeName"] == lc.node_name
        static_uid = next(iter(lc.kubelet.static))
        assert m.uid_of(mp) != static_uid    # the mirror is an API object standing for the static pod
        running = [cont for cont in lc.shim.containers.values() if cont.state == 1]
        assert len(running) == 1

        # deleting the mirror pod does not stop the static pod; the mirror comes back
        await c.delete("pods", name, "kube-system", grace=0)
        mp2 = await until(mirror_running)
        assert m.uid_of(mp2) != m.uid_of(mp)
        assert [cont.id for cont in lc.shim.containers.values() if cont.state == 1] == [running[0].id]

        # a manifest change replaces the static pod (new hash) and its mirror
        write_manifest(str(mdir), "etcd-lite", image="busybox", args=["-c", "sleep 60"])

        async def updated():
            p = await mirror_running()
            return p if p and p["spec"]["containers"][0]["image"] == "busybox" else None
        await until(updated)

        # removing the manifest removes the static pod and its mirror
        os.unlink(mdir / "etcd-lite.yaml")
        await until(lambda: _gone(c, name))

        async def stopped():
            return not any(cont.state == 1 for cont in lc.shim.containers.values())
        await until(stopped)


async def _gone(c, name):
    return await c.get_or_none("pods", name, "kube-system") is None


async def test_restarted_kubelet_adopts_running_static_pod(tmp_path):
    """a static pod's creationTimestamp is re-stamped on every manifest read, so a
    restarted kubelet must decide from runtime state (its startup ListPodSandbox), not from
    timestamps, whether the runtime already holds the pod: the running sandbox is adopted,
    never duplicated — even when the manifest is read long after the kubelet started."""
    from amdkube.client import Client
    from amdkube.kubelet.kubelet import Kubelet

    mdir = tmp_path / "manifests"
    mdir.mkdir()
    write_manifest(str(mdir), "ctl", image="busybox", args=["-c", "sleep 60"])
    async with LocalCluster(gpus="none", relist_period=0.2,
                            kubelet_kw={"pod_manifest_path": str(mdir), "file_check_frequency": 0.2}) as lc:
        async def one_running():
            run = [x for x in lc.shim.containers.values() if x.state == 1]
            return run if len(run) == 1 else None
        first = await until(one_running)
        sandboxes = set(lc.shim.sandboxes)
        cfg = lc.kubelet.cfg
        await lc.kubelet.stop()
        await lc.kubelet.client.close()
        k = Kubelet(Client(lc.api.url), cfg, smi_backend=lc.backend)
        k.started_at -= 30.0          # the old timestamp heuristic would now call the static pod fresh
        loop_fn = k._static_pods_loop

        async def late_loop():   # the manifest is first read once the runtime's event stream is up
            await asyncio.sleep(0.8)
            await loop_fn()
        k._static_pods_loop = late_loop
        lc.kubelet = await k.start()
        await asyncio.sleep(2.0)
        assert set(lc.shim.sandboxes) == sandboxes
        assert [x.id for x in lc.shim.containers.values() if x.state == 1] == [first[0].id]
