"""Kubelet run-once mode (pkg/kubelet/runonce_test.go): static pods from the manifest directory
are run without any API server until running; a pod that can never run is reported after the
retries; the `--runonce` command exits with the overall result."""
import json
import os
import subprocess
import sys

from amdkube.kubelet.kubelet import Kubelet, KubeletConfig
from amdkube.kubelet.runonce import NullClient, run_once, start_standalone
from amdkube.runtime import RocShim
from tests.conftest import ROOT, run


def _manifests(d):
    d.mkdir()
    (d / "web.yaml").write_text("apiVersion: v1\nkind: Pod\nmetadata: {name: web}\nspec:\n  containers:\n"
                                "  - {name: c, image: busybox, command: [sleep, '30']}\n")
    (d / "broken.yaml").write_text("apiVersion: v1\nkind: Pod\nmetadata: {name: broken}\nspec:\n  containers:\n"
                                   "  - {name: c, image: no-such-image:latest, command: [sleep, '30']}\n")


def test_run_once_runs_static_pods_without_api(tmp_path):
    _manifests(tmp_path / "manifests")

    async def go():
        shim = await RocShim(str(tmp_path / "cri.sock"), str(tmp_path / "shim")).start()
        try:
            cfg = KubeletConfig(node_name="lonely", root_dir=str(tmp_path / "kubelet"), plugins_dir=str(tmp_path / "plugins"),
                                cri_socket=str(tmp_path / "cri.sock"), pod_manifest_path=str(tmp_path / "manifests"),
                                volume_mounter="none")
            k = await start_standalone(Kubelet(NullClient(), cfg))
            res = {r["pod"]: r["error"] for r in await run_once(k, retries=3, delay=0.05)}
            await k.volume_manager.stop()
            assert res["web-lonely"] is None
            assert res["broken-lonely"] and "timeout after 3 attempts" in res["broken-lonely"]
            running = [c for c in shim.containers.values() if c.state == 1]
            assert [c.name for c in running] == ["c"] and running[0].labels.get("io.kubernetes.pod.name") == "web-lonely"
        finally:
            await shim.stop(kill_pods=True)
    run(go(), 60)


def test_runonce_command_exit_status(tmp_path):
    _manifests(tmp_path / "manifests")
    shim = subprocess.Popen([sys.executable, "-m", "amdkube", "rocshim", "--listen", str(tmp_path / "cri.sock"),
                             "--state-dir", str(tmp_path / "shim")], cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        for _ in range(200):
            if os.path.exists(tmp_path / "cri.sock"):
                break
            import time
            time.sleep(0.05)
        os.remove(tmp_path / "manifests" / "broken.yaml")
        r = subprocess.run([sys.executable, "-m", "amdkube", "kubelet", "--runonce", "--pod-manifest-path",
                            str(tmp_path / "manifests"), "--root-dir", str(tmp_path / "kubelet"), "--container-runtime-endpoint",
                            str(tmp_path / "cri.sock"), "--hostname-override", "n1", "--port", "0"],
                           cwd=ROOT, capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr[-2000:]
        assert [json.loads(x) for x in r.stdout.split("\n") if x.startswith("{")] == [{"pod": "web-n1", "error": None}]
    finally:
        shim.terminate()
        shim.wait(10)
        _kill_runtime_leftovers(tmp_path / "shim")


def _kill_runtime_leftovers(state_dir):
    """A --runonce kubelet leaves its pods running (that is the point of runonce), and a
    runtime keeps its sandboxes across its own restart: kill what the runtime recorded."""
    import glob
    import signal
    for f in glob.glob(os.path.join(str(state_dir), "*", "*.json")):
        try:
            pid = int(json.load(open(f)).get("pid") or 0)
        except (OSError, ValueError, AttributeError):
            continue
        if pid > 1:
            try:
                os.killpg(pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                try:
                    os.kill(pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass

