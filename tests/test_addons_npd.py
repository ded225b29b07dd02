"""Cluster addon manager (cluster/addons/addon-manager/kube-addons.sh) and node-problem-detector
(test/e2e_node/node_problem_detector_linux.go's table, plus the amdgpu rule set feeding the
device plugin's health)."""
import asyncio
import json
import os
import time

import pytest
import yaml

from amdkube.api import meta as m
from amdkube.localcluster import LocalCluster
from amdkube.monitoring.problemdetector import (KernelMonitor, LogEntry, MonitorConfig, NodeProblemDetector,
                                                go_layout_to_strptime, parse_kmsg_record)
from tests.conftest import run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NPD_DIR = os.path.join(ROOT, "deploy", "node-problem-detector")


# ============================================================ node-problem-detector
def _ref_config(log_file: str, lookback: str) -> dict:
    """The reference e2e's monitor config (node_problem_detector_linux.go:112-146)."""
    return {"plugin": "filelog",
            "pluginConfig": {"timestamp": "^.{15}", "message": "kernel: \\[.*\\] (.*)", "timestampFormat": "Jan _2 15:04:05"},
            "logPath": log_file, "lookback": lookback, "bufferSize": 10, "source": "kernel-monitor-test",
            "conditions": [{"type": "TestCondition", "reason": "Default", "message": "default message"}],
            "rules": [{"type": "temporary", "reason": "Temporary", "pattern": "temporary error"},
                      {"type": "permanent", "condition": "TestCondition", "reason": "Permanent1", "pattern": "permanent error 1.*"},
                      {"type": "permanent", "condition": "TestCondition", "reason": "Permanent2", "pattern": "permanent error 2.*"}]}


def _inject(path: str, ts: float, msg: str, n: int):
    with open(path, "a") as f:
        for _ in range(n):
            f.write(f"{time.strftime('%b %e %H:%M:%S', time.localtime(ts))} kernel: [0.000000] {msg}\n")


def test_go_layouts():
    assert go_layout_to_strptime("Jan _2 15:04:05") == "%b %d %H:%M:%S"
    assert go_layout_to_strptime("2006-01-02T15:04:05.000000-07:00") == "%Y-%m-%dT%H:%M:%S.%f%z"
    e = parse_kmsg_record("3,1234,5000000,-;amdgpu 0000:05:00.0: amdgpu: GPU reset begin!\n SUBSYSTEM=pci", 1000.0)
    assert e.ts == 1005.0 and e.message == "amdgpu 0000:05:00.0: amdgpu: GPU reset begin!"


def test_node_problem_detector_reference_table(tmp_path):
    """Each row of the reference's SystemLogMonitor table, in order, against a live apiserver:
    default condition; too-old logs ignored; old logs within lookback counted; new logs; a
    repeat of the same permanent reason leaves the condition; a new reason replaces it."""
    log_file = str(tmp_path / "test.log")
    open(log_file, "w").close()
    boot = time.time() - 3600            # the "node" booted an hour ago
    now = time.time()

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n1"},
                            "status": {"conditions": [{"type": "Ready", "status": "True", "reason": "KubeletReady"}]}})
            cfg = MonitorConfig.parse(_ref_config(log_file, f"{int(now - boot) + 3600}s"))
            npd = NodeProblemDetector(c, "n1", [cfg], boot=boot, poll=0.05, resync=60)
            await npd.start()

            async def state():
                for _ in range(100):          # the recorder writes asynchronously
                    await asyncio.sleep(0.02)
                    if npd.recorders["kernel-monitor-test"].queue.empty():
                        break
                await asyncio.sleep(0.1)
                evs, _ = await c.list("events", "default")
                mine = [e for e in evs if (e.get("source") or {}).get("component") == "kernel-monitor-test"]
                assert all(e["reason"] == "Temporary" and e["message"] == "temporary error" for e in mine), mine
                node = await c.get("nodes", "n1")
                conds = {x["type"]: x for x in node["status"]["conditions"]}
                assert conds["Ready"]["status"] == "True"      # the kubelet's condition is untouched
                tc = conds["TestCondition"]
                return sum(e.get("count", 1) for e in mine), (tc["status"], tc["reason"], tc["message"])

            rows = [  # (timestamp, message, n, events, condition)
                (None, None, 0, 0, ("False", "Default", "default message")),
                (boot - 60, "temporary error", 3, 0, ("False", "Default", "default message")),
                (boot - 60, "permanent error 1", 1, 0, ("False", "Default", "default message")),
                (now, "temporary error", 3, 3, ("False", "Default", "default message")),
                (now, "permanent error 1", 1, 3, ("True", "Permanent1", "permanent error 1")),
                (now + 300, "temporary error", 3, 6, ("True", "Permanent1", "permanent error 1")),
                (now + 300, "permanent error 1different message", 1, 6, ("True", "Permanent1", "permanent error 1")),
                (now + 300, "permanent error 2", 1, 6, ("True", "Permanent2", "permanent error 2")),
            ]
            for ts, msg, n, want_events, want_cond in rows:
                if n:
                    _inject(log_file, ts, msg, n)
                for _ in range(50):
                    got = await state()
                    if got == (want_events, want_cond):
                        break
                    await asyncio.sleep(0.05)
                assert got == (want_events, want_cond), (msg, got)
            await npd.stop()
    run(go())


def _amdgpu_monitor(tmp_path, lines: list[str], boot: float):
    cfg = json.load(open(os.path.join(NPD_DIR, "amdgpu-monitor.json")))
    path = tmp_path / "kmsg"
    path.write_text("".join(f"3,{i},{int((time.time() - boot) * 1e6) + i},-;{ln}\n" for i, ln in enumerate(lines)))
    cfg["logPath"] = str(path)
    return MonitorConfig.parse(cfg)


def test_amdgpu_rules_events_conditions_and_faults():
    cfg = MonitorConfig.parse(json.load(open(os.path.join(NPD_DIR, "amdgpu-monitor.json"))))
    for f in ("kernel-monitor.json", "kernel-monitor-filelog.json"):
        MonitorConfig.load(os.path.join(NPD_DIR, f))            # the shipped configs all parse
    mon = KernelMonitor(cfg, boot=time.time() - 100)
    t = time.time()

    def feed(msg):
        return mon.process(LogEntry(t, msg))
    st = feed("[drm:amdgpu_job_timedout [amdgpu]] *ERROR* ring comp_1.0.0 timeout, signaled seq=1234, emitted seq=1236")
    assert [r for r, _ in st.events] == ["AMDGPURingTimeout"] and not st.conditions and not st.gpu_faults
    st = feed("amdgpu 0000:05:00.0: amdgpu: GPU reset begin!")
    assert [r for r, _ in st.events] == ["AMDGPUReset"]
    st = feed("amdgpu 0000:05:00.0: amdgpu: GPU reset(2) succeeded!")
    assert [r for r, _ in st.events] == ["AMDGPUResetSucceeded"] and not st.gpu_faults
    st = feed("amdgpu 0000:15:00.0: amdgpu: [gfxhub] page fault (src_id:0 ring:24 vmid:8 pasid:32770)")
    assert [r for r, _ in st.events] == ["AMDGPUPageFault"] and not st.gpu_faults   # a workload bug, not a GPU fault
    st = feed("amdgpu 0000:15:00.0: amdgpu: 2 uncorrectable hardware errors detected in umc block")
    assert st.conditions["AMDGPUProblem"]["reason"] == "AMDGPUUncorrectableError"
    assert st.gpu_faults and st.gpu_faults[0][0] == "0000:15:00.0"
    st = feed("amdgpu 0000:05:00.0: amdgpu: GPU reset(3) failed")
    assert st.conditions["AMDGPUProblem"]["reason"] == "AMDGPUResetFailed"
    assert [b for b, _ in st.gpu_faults] == ["0000:05:00.0"]
    st = feed("amdgpu 0000:25:00.0: amdgpu: xGMI link down detected on link 3")
    assert st.conditions["XGMILinkProblem"]["reason"] == "XGMILinkDown"
    assert not feed("usb 1-1: new high-speed USB device number 2").events


def test_multiline_pattern_matches_only_at_the_newest_entry():
    cfg = MonitorConfig.parse({"plugin": "kmsg", "logPath": "/dev/null", "bufferSize": 3, "source": "s",
                               "conditions": [], "rules": [{"type": "temporary", "reason": "Hung",
                                                            "pattern": "INFO: task \\S+ blocked\\nCall Trace:"}]})
    mon = KernelMonitor(cfg, boot=0)
    t = time.time()
    assert not mon.process(LogEntry(t, "INFO: task x blocked")).events
    st = mon.process(LogEntry(t, "Call Trace:"))
    assert st.events == [("Hung", "INFO: task x blocked\nCall Trace:")]
    assert not mon.process(LogEntry(t, "something else")).events       # an old match does not re-fire


def test_kernel_log_gpu_fault_takes_the_gpu_out_of_service(tmp_path):
    """npd amdgpu rule (kmsg) → <health-state>.faults → the device plugin marks exactly that GPU
    Unhealthy with the kernel's words, sticky across a plugin restart; the node gets the
    AMDGPUProblem condition."""
    from amdkube.deviceplugin.amd import AMDGPUPlugin
    from amdkube.smi import FakeBackend, device_id
    from amdkube.smi.health import HEALTH_REASON_ATTR
    state = str(tmp_path / "dp" / "health.json")
    fb = FakeBackend(n=2)
    bdf1 = fb.gpus()[1]["bdf"]
    boot = time.time() - 50
    cfg = _amdgpu_monitor(tmp_path, [f"amdgpu {bdf1}: amdgpu: poison is consumed by client 12, kick off gpu reset flow"], boot)

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            await lc.client.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "gpu-node"}})
            p = AMDGPUPlugin(fb, plugins_dir=str(tmp_path / "dp" / "plugins"), health_interval=0.05, health_state=state)
            await p.start()
            npd = NodeProblemDetector(lc.client, "gpu-node", [cfg], health_state=state, boot=boot, poll=0.05)
            await npd.start()
            ids = [device_id(g) for g in fb.gpus()]
            for _ in range(200):
                if p.devices[1]["health"] == "Unhealthy":
                    break
                await asyncio.sleep(0.02)
            assert p.devices[0]["health"] == "Healthy"
            assert p.devices[1]["health"] == "Unhealthy"
            assert "AMDGPUPoisonConsumed" in p.devices[1]["Attributes"][HEALTH_REASON_ATTR]
            await asyncio.sleep(0.2)
            node = await lc.client.get("nodes", "gpu-node")
            cond = {x["type"]: x for x in node["status"]["conditions"]}
            assert cond["AMDGPUProblem"]["status"] == "True" and cond["AMDGPUProblem"]["reason"] == "AMDGPUPoisonConsumed"
            assert cond["XGMILinkProblem"]["status"] == "False"
            await npd.stop()
            await p.stop()
            p2 = AMDGPUPlugin(fb, plugins_dir=str(tmp_path / "dp" / "plugins"), health_interval=0.05, health_state=state)
            await p2.start()
            h = {d["ID"]: d["health"] for d in p2.devices}
            assert h == {ids[0]: "Healthy", ids[1]: "Unhealthy"}
            await p2.stop()
    run(go())


# ============================================================ addon manager
def _addon(kind, name, mode=None, cluster_service=False, **extra):
    labels = {}
    if mode:
        labels["addonmanager.kubernetes.io/mode"] = mode
    if cluster_service:
        labels["kubernetes.io/cluster-service"] = "true"
    api = {"ConfigMap": "v1", "ServiceAccount": "v1", "Service": "v1"}.get(kind, "v1")
    doc = {"apiVersion": api, "kind": kind, "metadata": {"name": name, "namespace": "kube-system", "labels": labels}}
    doc.update(extra)
    return doc


def test_addon_manager_reconcile_ensure_exists_and_prune(tmp_path):
    from amdkube.addons import AddonManager
    d = tmp_path / "addons"
    (d / "sub").mkdir(parents=True)

    def write(name, docs):
        (d / name).write_text(yaml.safe_dump_all(docs))

    write("rec.yaml", [_addon("ConfigMap", "rec", "Reconcile", data={"a": "1"}),
                       _addon("ConfigMap", "gone-later", "Reconcile", data={"x": "1"})])
    write("sub/ensure.yaml", [_addon("ConfigMap", "ens", "EnsureExists", data={"a": "1"})])
    write("sub/legacy.json", [_addon("ConfigMap", "legacy", cluster_service=True, data={"l": "1"})])
    (d / "sub" / "legacy.json").write_text(json.dumps(_addon("ConfigMap", "legacy", cluster_service=True, data={"l": "1"})))
    write("unlabelled.yaml", [_addon("ConfigMap", "ignored", data={"i": "1"})])
    write("notes.txt", [])

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "default", "namespace": "kube-system"}})
            mgr = AddonManager(c, str(d), admission_controls=None, interval=3600, leader_election=True, identity="me")
            await mgr.bootstrap(5)
            assert await mgr.sync_once()
            get = lambda n: c.get_or_none("configmaps", n, "kube-system")   # noqa: E731
            assert (await get("rec"))["data"] == {"a": "1"}
            assert (await get("ens"))["data"] == {"a": "1"}
            assert (await get("legacy"))["data"] == {"l": "1"}           # the deprecated label is reconciled
            assert await get("ignored") is None
            # users edit both; the Reconcile one is put back, the EnsureExists one is left alone
            await c.patch("configmaps", "rec", {"data": {"a": "user"}}, "kube-system")
            await c.patch("configmaps", "ens", {"data": {"a": "user"}}, "kube-system")
            # an unrelated object with the label but never applied is not pruned
            await c.create(_addon("ConfigMap", "hand-made", "Reconcile", data={}))
            write("rec.yaml", [_addon("ConfigMap", "rec", "Reconcile", data={"a": "2"})])   # gone-later left
            assert await mgr.sync_once()
            assert (await get("rec"))["data"] == {"a": "2"}
            assert (await get("ens"))["data"] == {"a": "user"}
            assert await get("gone-later") is None                        # pruned
            assert await get("hand-made") is not None                     # no last-applied: kept
            # removing the LAST Reconcile manifest still prunes (kubectl alone would refuse)
            os.unlink(d / "rec.yaml")
            assert await mgr.sync_once()
            assert await get("rec") is None and await get("legacy") is not None
            # deleting an EnsureExists object re-creates it on the next pass
            await c.delete("configmaps", "ens", "kube-system")
            assert await mgr.sync_once()
            assert (await get("ens"))["data"] == {"a": "1"}
            # another holder of the controller-manager lease: this manager stands by
            await c.create({"apiVersion": "v1", "kind": "Endpoints", "metadata": {
                "name": "kube-controller-manager", "namespace": "kube-system",
                "annotations": {"control-plane.alpha.kubernetes.io/leader": json.dumps({"holderIdentity": "other_1234"})}}})
            assert not await mgr.sync_once()
            mgr.identity = "other"
            assert await mgr.sync_once()
    run(go())


def test_kubectl_apply_selector_filters_manifests_and_recursive(tmp_path, capsys):
    from tests.test_rollout import kubectl
    d = tmp_path / "m"
    (d / "deep").mkdir(parents=True)
    (d / "a.yaml").write_text(yaml.safe_dump({"apiVersion": "v1", "kind": "ConfigMap",
                                              "metadata": {"name": "a", "labels": {"t": "x"}}, "data": {}}))
    (d / "deep" / "b.yaml").write_text(yaml.safe_dump({"apiVersion": "v1", "kind": "ConfigMap",
                                                       "metadata": {"name": "b", "labels": {"t": "y"}}, "data": {}}))

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            await kubectl(c, "apply", "-f", str(d), "-l", "t=x")
            assert await c.get_or_none("configmaps", "a", "default") is not None
            assert await c.get_or_none("configmaps", "b", "default") is None      # not recursive
            await kubectl(c, "apply", "-f", str(d), "--recursive", "-l", "t=y")
            assert await c.get_or_none("configmaps", "b", "default") is not None
            with pytest.raises(SystemExit, match="no objects passed to apply"):
                await kubectl(c, "apply", "-f", str(d), "-l", "t=none")
    run(go())


def test_deploy_addons_parse_and_carry_the_mode_label():
    from amdkube.kubectl.main import _read_files
    docs = _read_files([os.path.join(ROOT, "deploy", "addons")], recursive=True)
    kinds = {(d["kind"], m.name_of(d)) for d in docs}
    assert ("DaemonSet", "node-problem-detector") in kinds and ("DaemonSet", "amd-gpu-device-plugin") in kinds
    for doc in docs:
        assert m.labels_of(doc).get("addonmanager.kubernetes.io/mode") in ("Reconcile", "EnsureExists"), doc["metadata"]


def test_filelog_follows_rotation_and_truncation(tmp_path):
    from amdkube.monitoring.problemdetector import LogWatcher
    log_file = tmp_path / "kern.log"
    log_file.write_text("")
    cfg = MonitorConfig.parse(_ref_config(str(log_file), "1h"))
    w = LogWatcher(cfg, boot=0)
    assert w.open()
    now = time.time()
    _inject(str(log_file), now, "first", 1)
    assert [e.message for e in w.read()] == ["first"]
    os.rename(log_file, tmp_path / "kern.log.1")            # logrotate: move away, new file
    log_file.write_text("")
    _inject(str(log_file), now, "after rotation", 1)
    assert [e.message for e in w.read()] == ["after rotation"]
    log_file.write_text("")                                   # copytruncate
    _inject(str(log_file), now, "after truncation", 1)
    assert [e.message for e in w.read()] == ["after truncation"]
    w.close()
