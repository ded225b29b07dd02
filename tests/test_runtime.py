"""rocshim (CRI runtime) and the hooks.d service.

Hook-selection semantics ported from pkg/kubelet/dockershim/docker_hooks_test.go:80-225
(add → reload, remove → reload, hooks naming a runtime the runtime does not provide are
invalid, first hook with ANY matching annotation or image prefix wins)."""
import asyncio
import json
import os
import tempfile

import pytest

from amdkube.grpcdesc.cri import CRI as C
from amdkube.kubelet.cri_client import CRIClient
from amdkube.runtime import HookService, RocShim
from tests.conftest import run, log_text


def sandbox_cfg(name="p", uid="u1"):
    return C.PodSandboxConfig(metadata=C.PodSandboxMetadata(name=name, uid=uid, namespace="default"),
                              labels={"io.kubernetes.pod.uid": uid})


def ctr_cfg(name, cmd, envs=None, devices=None, annotations=None, image="busybox"):
    return C.ContainerConfig(metadata=C.ContainerMetadata(name=name), image=C.ImageSpec(image=image), command=cmd,
                             envs=[C.KeyValue(key=k, value=v) for k, v in (envs or {}).items()],
                             devices=[C.Device(container_path=d, host_path=d, permissions="rw") for d in devices or []],
                             annotations=annotations or {})


def test_hooks_selection_and_reload(tmp_path):
    async def go():
        hs = HookService(str(tmp_path / "hooks.d"), {"rocm", "default"}, poll_interval=0.05)
        await hs.start()
        assert oct(os.stat(hs.dir).st_mode & 0o777) == "0o755"  # fix #16
        assert hs.get_runtime(["rocm/vector-add:latest"], {}) == ""
        (tmp_path / "hooks.d" / "a.json").write_text(json.dumps({"runtime": "rocm", "annotations": {"gpu": "yes"}, "images": ["rocm/"]}))
        (tmp_path / "hooks.d" / "b.json").write_text(json.dumps({"runtime": "nvidia", "images": [""]}))  # invalid runtime
        for _ in range(100):
            if hs.hooks:
                break
            await asyncio.sleep(0.02)
        assert [h.runtime for h in hs.hooks] == ["rocm"]
        assert hs.get_runtime(["rocm/vector-add:latest"], {}) == "rocm"
        assert hs.get_runtime(["busybox:latest"], {"gpu": "yes"}) == "rocm"
        assert hs.get_runtime(["busybox:latest"], {"gpu": "no"}) == ""
        os.unlink(tmp_path / "hooks.d" / "a.json")
        for _ in range(100):
            if not hs.hooks:
                break
            await asyncio.sleep(0.02)
        assert hs.hooks == []
        await hs.stop()
    run(go())


async def _shim(base):
    shim = await RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"), hooks_dir=os.path.join(base, "hooks")).start()
    cri = await CRIClient(os.path.join(base, "s.sock")).connect()
    return shim, cri


def test_container_lifecycle_logs_exit_codes_and_env_scrub():
    async def go():
        base = tempfile.mkdtemp(prefix="rs", dir="/tmp")
        os.environ["HIP_VISIBLE_DEVICES"] = "3"
        shim, cri = await _shim(base)
        try:
            v = await cri.version()
            assert v.runtime_name == "rocshim"
            sc = sandbox_cfg()
            sid = await cri.run_pod_sandbox(sc)
            [sb] = await cri.list_pod_sandbox("u1")
            assert sb.state == C.SANDBOX_READY
            cid = await cri.create_container(sid, ctr_cfg("a", ["sh", "-c", "echo HIP=$HIP_VISIBLE_DEVICES ROCR=${ROCR_VISIBLE_DEVICES:-unset}; exit 3"]), sc)
            await cri.start_container(cid)
            for _ in range(200):
                st, _ = await cri.container_status(cid)
                if st.state == C.CONTAINER_EXITED:
                    break
                await asyncio.sleep(0.01)
            assert st.exit_code == 3 and st.reason == "Error"
            assert log_text(st.log_path).strip() == "HIP=-1 ROCR=unset"  # non-GPU container sees no GPU
            gid = await cri.create_container(sid, ctr_cfg("g", ["sh", "-c", "echo ROCR=$ROCR_VISIBLE_DEVICES HIP=${HIP_VISIBLE_DEVICES:-unset}"],
                                                          envs={"ROCR_VISIBLE_DEVICES": "GPU-abc"}, devices=["/dev/kfd"]), sc)
            await cri.start_container(gid)
            for _ in range(200):
                st, info = await cri.container_status(gid, verbose=True)
                if st.state == C.CONTAINER_EXITED:
                    break
                await asyncio.sleep(0.01)
            assert st.exit_code == 0
            assert log_text(st.log_path).strip() == "ROCR=GPU-abc HIP=unset"
            assert info["handler"] == "rocm"
            lid = await cri.create_container(sid, ctr_cfg("long", ["sleep", "30"]), sc)
            await cri.start_container(lid)
            out, err, rc = await cri.exec_sync(lid, ["sh", "-c", "echo hello"], 5)
            assert out.strip() == b"hello" and rc == 0
            await cri.stop_container(lid, 1)
            st, _ = await cri.container_status(lid)
            assert st.state == C.CONTAINER_EXITED
            await cri.stop_pod_sandbox(sid)
            await cri.remove_pod_sandbox(sid)
            assert await cri.list_pod_sandbox() == [] and await cri.list_containers() == []
        finally:
            os.environ.pop("HIP_VISIBLE_DEVICES", None)
            await cri.close()
            await shim.stop(kill_pods=True)
    run(go())


def test_runtime_restart_readopts_running_containers():
    async def go():
        base = tempfile.mkdtemp(prefix="rs", dir="/tmp")
        shim, cri = await _shim(base)
        sc = sandbox_cfg()
        sid = await cri.run_pod_sandbox(sc)
        cid = await cri.create_container(sid, ctr_cfg("a", ["sh", "-c", "sleep 0.8; exit 7"]), sc)
        await cri.start_container(cid)
        await cri.close()
        await shim.stop(kill_pods=False)     # runtime crash/restart: the pod keeps running
        shim2, cri2 = await _shim(base)
        try:
            st, _ = await cri2.container_status(cid)
            assert st.state == C.CONTAINER_RUNNING
            for _ in range(300):
                st, _ = await cri2.container_status(cid)
                if st.state == C.CONTAINER_EXITED:
                    break
                await asyncio.sleep(0.02)
            assert st.state == C.CONTAINER_EXITED and st.exit_code == 7  # recovered from the exit file
        finally:
            await cri2.close()
            await shim2.stop(kill_pods=True)
    run(go(), 60)


def test_images_pull_and_unknown_image():
    async def go():
        base = tempfile.mkdtemp(prefix="rs", dir="/tmp")
        shim, cri = await _shim(base)
        try:
            assert await cri.image_status("rocm/vector-add") is not None
            assert await cri.image_status("nope/x") is None
            import grpc
            with pytest.raises(grpc.RpcError):
                await cri.pull_image("registry.example.com/nope:1")
            script = os.path.join(base, "tool.sh")
            open(script, "w").write("#!/bin/sh\necho tool\n")
            os.chmod(script, 0o755)
            await cri.pull_image("file://" + script)
            assert await cri.image_status("file://" + script) is not None
        finally:
            await cri.close()
            await shim.stop()
    run(go())


def test_launches_in_flight_at_stop_do_not_outlive_the_runtime():
    """Sandbox and container processes are launched from worker threads; a launch that lands
    after stop(kill_pods=True) began is killed instead of being left behind untracked."""
    async def go():
        base = tempfile.mkdtemp(prefix="rs", dir="/tmp")
        shim = await RocShim(os.path.join(base, "s.sock"), os.path.join(base, "state"),
                             hooks_dir=os.path.join(base, "hooks")).start()
        import amdkube.runtime.rocshim as rs
        pids = []
        real_spawn = rs.spawn

        async def slow_spawn(argv, **kw):
            proc = await real_spawn(argv, **kw)       # the process exists ...
            pids.append(proc.pid)
            await asyncio.sleep(0.2)                  # ... and its launch is still in flight at stop()
            return proc
        rs.spawn = slow_spawn
        try:
            t = asyncio.create_task(shim.run_sandbox(sandbox_cfg("late", "u-late")))
            await asyncio.sleep(0.1)
            await shim.stop(kill_pods=True)
            with pytest.raises(RuntimeError, match="shutting down"):
                await t
        finally:
            rs.spawn = real_spawn
        assert not shim.sandboxes and len(pids) == 1
        assert not os.path.exists(f"/proc/{pids[0]}") or open(f"/proc/{pids[0]}/stat").read().split()[2] == "Z"
        with pytest.raises(RuntimeError, match="shutting down"):
            await shim._launch(["/bin/true"])
    run(go())
