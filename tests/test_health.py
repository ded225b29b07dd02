"""Device health judged on NEW faults (smi/health.py), published as a device attribute, with
the reference's consequences: the kubelet refuses new pods on an Unhealthy device and leaves
running ones alone (pkg/kubelet/cm/devicemanager/device_store.go:103-110,
manager_store.go:116-118; test/e2e_node/gpu_device_plugin.go keeps running pods untouched)."""
import asyncio

from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.smi import FakeBackend
from amdkube.smi.health import HEALTH_REASON_ATTR, HealthMonitor
from tests.conftest import run


def test_historical_errors_do_not_mark_a_part_unhealthy():
    fb = FakeBackend(n=2)
    fb.inject_ecc(0, uncorrectable=5)          # last year's errors
    fb.inject_bad_page(0, pending=0, retired=3)
    hm = HealthMonitor(fb, ecc_threshold=0)
    hm.snapshot(0)
    assert hm.check(0) == (True, "")
    fb.inject_ecc(0)                           # a fresh one on a part already above the threshold
    ok, why = hm.check(0)
    assert not ok and "+1 since the plugin started" in why and "lifetime 6" in why
    fb.samples[0]["ecc_uncorrectable"] = 5     # stays out of service until a new baseline
    assert hm.check(0)[0] is False


def test_xgmi_and_bad_page_faults():
    fb = FakeBackend(n=3)
    hm = HealthMonitor(fb)
    for i in range(3):
        hm.snapshot(i)
    fb.inject_xgmi_error(0)
    fb.inject_bad_page(1, pending=2)
    fb.ras_state.setdefault(2, fb.ras(2))
    fb.ras_state[2].update(bad_pages=512, bad_pages_retired=512)
    assert hm.check(0) == (False, "xGMI link error")
    assert hm.check(1) == (False, "2 new bad page(s) pending retirement")
    ok, why = hm.check(2)
    assert not ok and "threshold 512" in why


def test_xgmi_block_errors_when_the_status_file_is_unreadable():
    fb = FakeBackend(n=1)
    hm = HealthMonitor(fb)
    fb.ras(0)
    fb.ras_state[0].pop("xgmi_error")
    fb.ras_state[0]["xgmi_ecc_uncorrectable"] = 4      # historical
    hm.snapshot(0)
    assert hm.check(0)[0]
    fb.ras_state[0]["xgmi_ecc_uncorrectable"] = 5
    assert hm.check(0) == (False, "xGMI link uncorrectable errors: +1 since the plugin started")


def test_ecc_threshold_allows_a_budget():
    fb = FakeBackend(n=1)
    hm = HealthMonitor(fb, ecc_threshold=2)
    hm.snapshot(0)
    fb.inject_ecc(0, 2)
    assert hm.check(0)[0]
    fb.inject_ecc(0, 1)
    assert not hm.check(0)[0]


def test_fault_flips_device_publishes_reason_and_spares_the_running_pod():
    async def go():
        async with LocalCluster(gpus="fake", n_gpus=2, relist_period=0.2, node_status_update_frequency=0.2,
                                with_controllers=False) as lc:
            lc.plugin.health_interval = 0.1
            fb = lc.backend
            await lc.wait_gpus(2, 30)
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "runner", "namespace": "default"},
                   "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "busybox",
                            "command": ["sleep", "30"], "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
            await lc.client.create(pod)
            p = await wait_pod(lc.client, "default", "runner", ("Running",), 30)
            [did] = p["spec"]["extendedResources"][0]["assigned"]
            idx = lc.plugin.by_id[did]["index"]
            fb.inject_xgmi_error(idx)
            dev = None
            for _ in range(200):
                node = await lc.client.get("nodes", lc.node_name)
                dev = node["status"]["extendedResources"]["amd.com/gpu"]["resources"][did]
                if dev["health"] == "Unhealthy":
                    break
                await asyncio.sleep(0.05)
            assert dev["health"] == "Unhealthy", dev
            assert dev["attributes"][HEALTH_REASON_ATTR] == "xGMI_link_error"
            # the running pod is left alone
            p = await lc.client.get("pods", "runner", "default")
            assert p["status"]["phase"] == "Running"
            # a new 1-GPU pod lands on the healthy GPU, never the flagged one
            pod["metadata"]["name"] = "next"
            await lc.client.create(pod)
            p2 = await wait_pod(lc.client, "default", "next", ("Running",), 30)
            assert p2["spec"]["extendedResources"][0]["assigned"] != [did]
    run(go(), 90)


def test_fault_survives_a_plugin_restart_until_an_operator_reset(tmp_path):
    """Round-3 review: the baseline and sticky faults lived only in memory, so a restarted plugin
    re-baselined and re-advertised a faulted GPU Healthy. With the checkpoint the restarted
    plugin keeps the GPU Unhealthy with its reason, and judges against the ORIGINAL baseline
    (errors that happened while it was down still count) until `amdkube gpu-health reset`."""
    import subprocess
    import sys
    from amdkube.deviceplugin.amd import AMDGPUPlugin
    from amdkube.smi import device_id
    state = str(tmp_path / "health.json")
    fb = FakeBackend(n=2)

    async def plugin():
        p = AMDGPUPlugin(fb, plugins_dir=str(tmp_path / "plugins"), health_interval=0.05, health_state=state)
        await p.start()
        return p

    async def go():
        p = await plugin()
        ids = [device_id(g) for g in fb.gpus()]
        fb.inject_xgmi_error(0)
        for _ in range(100):
            if p.devices[0]["health"] == "Unhealthy":
                break
            await asyncio.sleep(0.02)
        assert p.devices[0]["health"] == "Unhealthy" and p.devices[1]["health"] == "Healthy"
        await p.stop()
        # the fault clears at the source (driver reload), and GPU 1 takes ECC errors while the
        # plugin is down: the restart must not re-baseline either
        fb.ras_state[0]["xgmi_error"] = 0
        fb.inject_ecc(1, uncorrectable=3)
        p = await plugin()
        h = {d["ID"]: (d["health"], d["Attributes"].get(HEALTH_REASON_ATTR)) for d in p.devices}
        assert h[ids[0]] == ("Unhealthy", "xGMI_link_error"), h
        assert h[ids[1]][0] == "Unhealthy" and "ECC" in h[ids[1]][1], h
        # the operator puts GPU 0 back; GPU 1 stays out
        r = subprocess.run([sys.executable, "-m", "amdkube", "gpu-health", "reset", ids[0], "--state-file", state],
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        for _ in range(100):
            if p.devices[0]["health"] == "Healthy":
                break
            await asyncio.sleep(0.02)
        assert p.devices[0]["health"] == "Healthy" and p.devices[1]["health"] == "Unhealthy"
        show = subprocess.run([sys.executable, "-m", "amdkube", "gpu-health", "show", "--state-file", state],
                              capture_output=True, text=True, timeout=60).stdout
        assert f"{ids[0]}\tHealthy" in show and f"{ids[1]}\tUnhealthy" in show
        await p.stop()
    run(go())


def test_checkpoint_from_another_boot_is_rebaselined_but_faults_stay(tmp_path):
    """ECC/xGMI counters restart at 0 after a reboot or driver reload while the state
    file survives. A checkpoint from another boot/driver instance is re-baselined (else the
    subtraction would hide new errors until the old count is exceeded), keeping sticky faults."""
    state = str(tmp_path / "health.json")
    fb = FakeBackend(n=2)
    fb.inject_ecc(0, uncorrectable=7)
    hm = HealthMonitor(fb, state_file=state, instance="boot-A/1")
    hm.snapshot(0)
    hm.snapshot(1)
    hm.fault(1, "operator: bad HBM stack")
    # reboot: the counters restart at 0, then one new uncorrectable error
    fb2 = FakeBackend(n=2)
    hm2 = HealthMonitor(fb2, state_file=state, instance="boot-B/1")
    hm2.snapshot(0)
    hm2.snapshot(1)
    assert hm2.baseline[0].get("ecc_uncorrectable", 0) == 0
    fb2.inject_ecc(0)
    ok, why = hm2.check(0)
    assert not ok and "+1 since the plugin started" in why
    assert hm2.check(1) == (False, "operator: bad HBM stack")
    # the same instance keeps the original baseline (a plain plugin restart)
    hm3 = HealthMonitor(fb2, state_file=state, instance="boot-B/1")
    hm3.snapshot(1)
    assert hm3.check(1)[0] is False


def test_counters_going_down_under_a_live_monitor_rebaseline():
    fb = FakeBackend(n=1)
    fb.inject_ecc(0, uncorrectable=4)
    hm = HealthMonitor(fb, instance="x")
    hm.snapshot(0)
    fb.samples[0]["ecc_uncorrectable"] = 0        # driver reload under the plugin
    assert hm.check(0) == (True, "")
    fb.inject_ecc(0)
    ok, why = hm.check(0)
    assert not ok and "+1" in why


def test_reset_requests_are_taken_atomically(tmp_path):
    """A reset appended while the plugin collects requests lands in a new file and is read on
    the next tick instead of being unlinked unread."""
    from amdkube.smi.health import request_reset
    state = str(tmp_path / "h.json")
    hm = HealthMonitor(FakeBackend(n=1), state_file=state, instance="x")
    request_reset(state, ["GPU-a"])
    import os
    real_replace = os.replace

    def replace_then_append(src, dst):
        real_replace(src, dst)
        request_reset(state, ["GPU-b"])            # arrives between the take and the read
    os.replace = replace_then_append
    try:
        assert hm.pending_resets() == {"GPU-a"}
    finally:
        os.replace = real_replace
    assert hm.pending_resets() == {"GPU-b"}
