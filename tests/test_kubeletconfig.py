"""KubeletConfiguration files and dynamic kubelet config (pkg/kubelet/kubeletconfig:
checkpoint/download_test.go, configsync, rollback; status messages)."""
import asyncio
import json

import pytest
import yaml

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.kubelet import kubeletconfig as kc
from amdkube.kubelet.kubelet import Kubelet, KubeletConfig
from amdkube.localcluster import LocalCluster
from tests.conftest import run


def test_apply_maps_fields_and_validates(tmp_path):
    cfg = KubeletConfig(node_name="n")
    new = kc.apply(cfg, {"kind": "KubeletConfiguration", "apiVersion": "kubeletconfig/v1alpha1", "maxPods": 42,
                         "evictionHard": {"memory.available": "200Mi"}, "kubeReserved": {"cpu": "500m"},
                         "featureGates": {"CPUManager": True}, "nodeStatusUpdateFrequency": "4s", "cgroupDriver": "systemd"})
    assert (new.max_pods, new.eviction_hard, new.kube_reserved, new.node_status_update_frequency) == \
        (42, "memory.available<200Mi", "cpu=500m", 4.0)
    assert new.feature_gates == "CPUManager=true" and cfg.max_pods == 110
    for bad in ({"bogusField": 1}, {"imageGCHighThresholdPercent": 50, "imageGCLowThresholdPercent": 60},
                {"evictionHard": {"disk.weird": "1"}}, {"kind": "Pod"}, {"cpuManagerPolicy": "dynamic"}):
        with pytest.raises(ValueError):
            kc.apply(cfg, bad)
    f = tmp_path / "kubelet.yaml"
    f.write_text(yaml.safe_dump({"kind": "KubeletConfiguration", "maxPods": 7}))
    k = Kubelet(Client("http://127.0.0.1:1"), KubeletConfig(node_name="n", root_dir=str(tmp_path / "root"), config_file=str(f)))
    assert k.cfg.max_pods == 7


class FakeClient:
    def __init__(self, cms):
        self.cms = cms

    async def get(self, res, name, ns):
        if (ns, name) not in self.cms:
            raise m.not_found(res, name)
        return self.cms[(ns, name)]


def _cm(uid, body):
    return {"metadata": {"name": "kcfg", "namespace": "kube-system", "uid": uid}, "data": {"kubelet": body}}


def _node(uid):
    return {"spec": {"configSource": {"configMapRef": {"namespace": "kube-system", "name": "kcfg", "uid": uid}}}}


def test_dynamic_config_checkpoint_trial_and_rollback(tmp_path):
    async def go():
        base = KubeletConfig(node_name="n")
        clock = [1000.0]
        d = kc.DynamicConfig(str(tmp_path), trial=60, crash_loop_threshold=3, clock=lambda: clock[0])
        good = FakeClient({("kube-system", "kcfg"): _cm("u1", "kind: KubeletConfiguration\nmaxPods: 50\n")})
        assert await d.sync(good, _node("u1")) is True                   # new current → restart
        assert await d.sync(good, _node("u1")) is False
        cfg = kc.DynamicConfig(str(tmp_path), trial=60, clock=lambda: clock[0]).bootstrap(base)
        assert cfg.max_pods == 50
        # UID mismatch and partial references do not change anything
        assert await d.sync(good, _node("u-other")) is False and "does not match UID" in d.condition["reason"]
        assert await d.sync(good, {"spec": {"configSource": {"configMapRef": {"name": "kcfg"}}}}) is False
        # after the trial period current becomes last-known-good
        import os
        os.utime(str(tmp_path / "meta" / "current"), (clock[0] - 120, clock[0] - 120))
        d2 = kc.DynamicConfig(str(tmp_path), trial=60, clock=lambda: clock[0])
        d2.bootstrap(base)
        assert json.loads((tmp_path / "meta" / "last-known-good").read_text())["uid"] == "u1"
        # a broken config: rollback to last-known-good with ConfigOK=False
        bad = FakeClient({("kube-system", "kcfg"): _cm("u2", "kind: KubeletConfiguration\nmaxPods: -3\n")})
        assert await d2.sync(bad, _node("u2")) is True
        d3 = kc.DynamicConfig(str(tmp_path), trial=60, clock=lambda: clock[0])
        cfg = d3.bootstrap(base)
        assert cfg.max_pods == 50 and d3.condition["status"] == "False"
        assert d3.condition["message"] == "using last-known-good (UID: 'u1')" and "u2" in d3.condition["reason"]
        # crash loop: too many start-ups of a good current within its trial → last-known-good
        ok2 = FakeClient({("kube-system", "kcfg"): _cm("u3", "kind: KubeletConfiguration\nmaxPods: 60\n")})
        await d3.sync(ok2, _node("u3"))
        for i in range(3):
            assert kc.DynamicConfig(str(tmp_path), trial=60, crash_loop_threshold=3,
                                    clock=lambda: clock[0]).bootstrap(base).max_pods == 60
        d4 = kc.DynamicConfig(str(tmp_path), trial=60, crash_loop_threshold=3, clock=lambda: clock[0])
        assert d4.bootstrap(base).max_pods == 50 and "crash loop" in d4.condition["reason"]
        # configSource removed → back to the local configuration
        assert await d4.sync(ok2, {"spec": {}}) is True
        assert kc.DynamicConfig(str(tmp_path)).bootstrap(base).max_pods == 110
    run(go(), 30)


def test_dynamic_config_end_to_end_restart(tmp_path):
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False, node_status_update_frequency=0.2,
                                kubelet_kw={"dynamic_config_dir": str(tmp_path / "dyn"),
                                            "feature_gates": "DynamicKubeletConfig=true"}) as lc:
            c = lc.client
            cm = await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "kcfg", "namespace": "kube-system"},
                                 "data": {"kubelet": "kind: KubeletConfiguration\nmaxPods: 33\n"}})
            await c.patch("nodes", lc.node_name, {"spec": {"configSource": {"configMapRef": {
                "namespace": "kube-system", "name": "kcfg", "uid": m.uid_of(cm)}}}})
            await asyncio.wait_for(lc.kubelet.restart_requested.wait(), 10)
            cfg = lc.kubelet.cfg
            await lc.kubelet.stop()
            await lc.kubelet.client.close()
            lc.kubelet = await Kubelet(Client(lc.api.url), cfg, smi_backend=lc.backend).start()
            assert lc.kubelet.cfg.max_pods == 33
            for _ in range(50):
                node = await c.get("nodes", lc.node_name)
                conds = {x["type"]: x for x in node["status"]["conditions"]}
                if node["status"]["capacity"]["pods"] == "33" and "ConfigOK" in conds:
                    break
                await asyncio.sleep(0.1)
            assert node["status"]["capacity"]["pods"] == "33"
            assert conds["ConfigOK"]["status"] == "True" and m.uid_of(cm) in conds["ConfigOK"]["message"]
    run(go(), 60)
