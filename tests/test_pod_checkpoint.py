"""pkg/kubelet/checkpoint (--bootstrap-checkpoint-path): annotated pods are checkpointed while
the API server knows them, run again by a restarted kubelet with no API server, and dropped
once the API server (reachable again) no longer has them."""
import asyncio
import os

from amdkube.kubelet.checkpoint import BOOTSTRAP_CHECKPOINT_ANNOTATION, PodCheckpointManager
from amdkube.kubelet.kubelet import Kubelet, KubeletConfig
from amdkube.client import Client
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


def test_manager_only_keeps_annotated_pods(tmp_path):
    mgr = PodCheckpointManager(str(tmp_path / "ck"))
    pod = {"metadata": {"name": "a", "uid": "u1", "annotations": {BOOTSTRAP_CHECKPOINT_ANNOTATION: "true"}},
           "spec": {"containers": []}, "status": {"phase": "Running"}}
    assert mgr.write_pod(pod)
    assert not mgr.write_pod({"metadata": {"name": "b", "uid": "u2"}, "spec": {}})
    (tmp_path / "ck" / "Pod_bad.yaml").write_text("{not json")
    loaded = mgr.load_pods()
    assert [p["metadata"]["uid"] for p in loaded] == ["u1"] and "status" not in loaded[0]
    mgr.delete_pod(pod)
    mgr.delete_pod(pod)
    assert mgr.load_pods() == []


def test_checkpointed_pod_restarts_without_api_server(tmp_path):
    ck = str(tmp_path / "ck")

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"bootstrap_checkpoint_path": ck}) as lc:
            c = lc.client
            for name, ann in (("selfhosted", {BOOTSTRAP_CHECKPOINT_ANNOTATION: "true"}), ("plain", {})):
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "annotations": ann},
                                "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"]}]}},
                               "default")
                await wait_pod(c, "default", name, ("Running",), 20)
            files = os.listdir(ck)
            assert len(files) == 1 and files[0].startswith("Pod_")
            node_name, root, sock = lc.node_name, lc.kubelet.cfg.root_dir, lc.kubelet.cfg.cri_socket
            uid = (await c.get("pods", "selfhosted", "default"))["metadata"]["uid"]
            await lc.kubelet.stop()
            # a kubelet whose API server is unreachable still runs the checkpointed pod
            cfg = KubeletConfig(node_name=node_name, root_dir=root, plugins_dir=str(tmp_path / "plugins2"), cri_socket=sock,
                                port=0, relist_period=0.2, bootstrap_checkpoint_path=ck)
            k2 = await Kubelet(Client("http://127.0.0.1:9"), cfg).start()
            try:
                assert uid in k2.pods and uid in k2.restored
                for _ in range(100):
                    if any(cs.metadata.name == "c" for cs in await k2.cri.list_containers()
                           if cs.labels.get("io.kubernetes.pod.uid") == uid):
                        break
                    await asyncio.sleep(0.1)
                else:
                    raise AssertionError("checkpointed pod has no container")
                st = k2.status.get(uid) or {}
                for _ in range(100):
                    st = k2.status.get(uid) or {}
                    if st.get("phase") == "Running":
                        break
                    await asyncio.sleep(0.1)
                assert st.get("phase") == "Running", st
                assert not k2.informer    # never reached the API server
            finally:
                await k2.stop()
    run(go(), 90)


def test_restored_pod_deleted_from_the_api_is_dropped(tmp_path):
    ck = str(tmp_path / "ck")
    mgr = PodCheckpointManager(ck)
    mgr.write_pod({"apiVersion": "v1", "kind": "Pod",
                   "metadata": {"name": "ghost", "namespace": "default", "uid": "ghost-uid",
                                "annotations": {BOOTSTRAP_CHECKPOINT_ANNOTATION: "true"}},
                   "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"]}]}})

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False,
                                kubelet_kw={"bootstrap_checkpoint_path": ck}) as lc:
            k = lc.kubelet
            for _ in range(100):
                if "ghost-uid" not in k.pods:
                    break
                await asyncio.sleep(0.05)
            assert "ghost-uid" not in k.pods and not k.restored
            assert mgr.load_pods() == []
    run(go(), 60)
