"""rkt as the container runtime (reference pkg/kubelet/rkt rkt_test.go, the rktshim
stubs, and the rktlet CRI mapping): the kubelet's CRI client drives rktshim, which drives the
`rkt` command line — here the scripted rkt of tests/fake_rkt.py (no rkt exists offline, so parity
with a real rkt binary is unpinned)."""
import asyncio
import json
import os
import sys

from amdkube.grpcdesc.cri import CRI as C
from amdkube.kubelet.cri_client import CRIClient
from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.runtime.rktshim import RktShim, _normalize, app_name
from tests.conftest import run

FAKE = [sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "fake_rkt.py")]


def _shim_kw(tmp_path):
    return {"rkt": FAKE, "rkt_env": {"FAKE_RKT_DIR": str(tmp_path / "rkt")}}


def test_cri_over_rkt(tmp_path):
    async def go():
        shim = await RktShim(str(tmp_path / "rkt.sock"), str(tmp_path / "state"), **_shim_kw(tmp_path)).start()
        cri = await CRIClient(str(tmp_path / "rkt.sock")).connect()
        try:
            v = await cri.version()
            assert v.runtime_name == "rkt" and v.runtime_version == "1.30.0"
            ref = await cri.pull_image("busybox")
            assert ref.startswith("sha512-")
            assert (await cri.image_status("docker.io/library/busybox:latest")).id == ref
            cfg = C.PodSandboxConfig(metadata=C.PodSandboxMetadata(name="p", uid="u1", namespace="default"),
                                     hostname="p", log_directory=str(tmp_path / "logs"), labels={"app": "x"})
            sid = await cri.run_pod_sandbox(cfg)
            s = shim.sandboxes[sid]
            pod = json.load(open(tmp_path / "rkt" / "pods" / s.uuid / "pod.json"))
            assert pod["annotations"]["coreos.com/rkt/experiment/logmode"] == "k8s"
            cc = C.ContainerConfig(metadata=C.ContainerMetadata(name="Main_App", attempt=0), image=C.ImageSpec(image="busybox"),
                                   command=["/bin/sh", "-c", "echo hello $GREETING; echo rocr=$ROCR_VISIBLE_DEVICES; exit 3"],
                                   envs=[C.KeyValue(key="GREETING", value="from-rkt"), C.KeyValue(key="ROCR_VISIBLE_DEVICES", value="0")],
                                   devices=[C.Device(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")],
                                   mounts=[C.Mount(container_path="/data", host_path=str(tmp_path), readonly=True)],
                                   log_path="main/0.log")
            cid = await cri.create_container(sid, cc, cfg)
            app = json.load(open(tmp_path / "rkt" / "pods" / s.uuid / "apps" / f"{app_name('Main_App')}.json"))
            assert app["name"] == "main-app" and app["argv"][:2] == ["/bin/sh", "-c"]
            assert {"name": "dev-0", "kind": "host", "source": "/dev/kfd", "target": "/dev/kfd", "readOnly": "false"} in app["volumes"]
            assert any(v["target"] == "/data" and v["readOnly"] == "true" for v in app["volumes"])
            await cri.start_container(cid)
            for _ in range(200):
                st, _ = await cri.container_status(cid)
                if st.state == C.CONTAINER_EXITED:
                    break
                await asyncio.sleep(0.02)
            assert st.state == C.CONTAINER_EXITED and st.exit_code == 3 and st.reason == "Error"
            logs = open(st.log_path).read()
            assert "hello from-rkt" in logs and "rocr=0" in logs and st.log_path == str(tmp_path / "logs" / "main" / "0.log")
            # a long-running app: exec into it, then stop it
            cc2 = C.ContainerConfig(metadata=C.ContainerMetadata(name="sleeper"), image=C.ImageSpec(image="busybox"),
                                    command=["/bin/sh", "-c", "sleep 30"], envs=[C.KeyValue(key="WHO", value="rkt-app")])
            cid2 = await cri.create_container(sid, cc2, cfg)
            await cri.start_container(cid2)
            st2, _ = await cri.container_status(cid2)
            assert st2.state == C.CONTAINER_RUNNING
            out, err, rc = await cri.exec_sync(cid2, ["/bin/sh", "-c", "echo $WHO; echo $HIP_VISIBLE_DEVICES"], 10)
            assert rc == 0 and out.split() == [b"rkt-app", b"-1"], (out, err)   # a non-GPU app sees no GPU
            listed = {c.id: c.state for c in await cri.list_containers()}
            assert listed == {cid: C.CONTAINER_EXITED, cid2: C.CONTAINER_RUNNING}
            await cri.stop_container(cid2, 5)
            assert (await cri.container_status(cid2))[0].state == C.CONTAINER_EXITED
            await cri.remove_container(cid2)
            await cri.stop_pod_sandbox(sid)
            assert (await cri.pod_sandbox_status(sid)).state == C.SANDBOX_NOTREADY
            await cri.remove_pod_sandbox(sid)
            assert not (tmp_path / "rkt" / "pods" / s.uuid).exists()
            await cri.remove_image("busybox")
            assert await cri.list_images() == []
        finally:
            await cri.close()
            await shim.stop(kill_pods=True)
    run(go(), 60)
    assert _normalize("docker.io/library/busybox") == "busybox:latest" == _normalize("busybox")


def test_gpu_pod_through_rkt(tmp_path):
    """A GPU pod on a node whose runtime is rkt: the device plugin's devices and visibility env
    reach the rkt app; the pod runs to completion and its logs come back through the kubelet."""
    async def go():
        async with LocalCluster(gpus="fake", n_gpus=2, relist_period=0.2, runtime="rkt", shim_kw=_shim_kw(tmp_path),
                                kubelet_kw={"evented_pleg": False}) as lc:
            await lc.wait_gpus(2, 30)
            await lc.client.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "g", "namespace": "default"},
                                    "spec": {"restartPolicy": "Never", "containers": [{
                                        "name": "c", "image": "busybox", "imagePullPolicy": "IfNotPresent",
                                        "command": ["/bin/sh", "-c", "echo visible=$ROCR_VISIBLE_DEVICES"],
                                        "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
            p = await wait_pod(lc.client, "default", "g", ("Succeeded", "Failed"), 60)
            logs = await lc.client.logs("default", "g")
            assert p["status"]["phase"] == "Succeeded", (p["status"], logs)
            assert logs.startswith("visible=") and logs.strip() != "visible=", logs
            pods = os.listdir(tmp_path / "rkt" / "pods")
            apps = [json.load(open(tmp_path / "rkt" / "pods" / u / "apps" / a)) for u in pods
                    for a in os.listdir(tmp_path / "rkt" / "pods" / u / "apps") if not a.endswith(".status.json")]
            gpu_app = next(a for a in apps if a["name"] == "c")
            assert any(v["target"].endswith("kfd") for v in gpu_app["volumes"]), gpu_app["volumes"]
    run(go(), 90)
