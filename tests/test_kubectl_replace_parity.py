"""kubectl replace against pkg/kubectl/cmd/replace.go (RunReplace, forceReplace) and
replace_test.go (TestReplaceObject, TestReplaceMultipleObject, TestForceReplaceObjectNotFound),
on a live apiserver."""
from __future__ import annotations

import json

import yaml

from tests.conftest import run
from tests.test_kubectl_commands_parity import _kubectl


def test_replace_through_the_cluster(tmp_path):
    from amdkube.localcluster import LocalCluster

    async def body():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cfg"}, "data": {"a": "1"}}
            svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web"},
                   "spec": {"ports": [{"port": 80}], "selector": {"app": "web"}}}
            await c.create(cm, "default")
            await c.create(svc, "default")
            f = tmp_path / "cfg.json"
            f.write_text(json.dumps({**cm, "data": {"a": "2"}}))
            rc, out, err = await _kubectl(c, "replace", "-f", str(f))              # no resourceVersion: unconditional
            assert (rc, out) == (0, 'configmap "cfg" replaced\n'), err
            assert (await c.get("configmaps", "cfg", "default"))["data"] == {"a": "2"}
            both = tmp_path / "both.yaml"
            both.write_text(yaml.safe_dump({**cm, "data": {"a": "3"}}) + "---\n" + yaml.safe_dump(svc))
            rc, out, err = await _kubectl(c, "replace", "-f", str(both), "-o", "name")
            assert (rc, out) == (0, "configmap/cfg\nservice/web\n"), err
            stale = tmp_path / "stale.json"
            stale.write_text(json.dumps({**cm, "metadata": {"name": "cfg", "resourceVersion": "1"}, "data": {"a": "9"}}))
            rc, out, err = await _kubectl(c, "replace", "-f", str(stale))
            assert rc == 1 and f'error when replacing "{stale}"' in err
            for argv, msg in (([], "Must specify --filename to replace"),
                              (["-f", str(f), "--grace-period", "0"], "--grace-period must have --force specified"),
                              (["-f", str(f), "--timeout", "5s"], "--timeout must have --force specified")):
                rc, out, err = await _kubectl(c, "replace", *argv)
                assert rc == 1 and msg in err, (argv, err)
            uid = (await c.get("configmaps", "cfg", "default"))["metadata"]["uid"]
            rc, out, err = await _kubectl(c, "replace", "--force", "-f", str(f), "--save-config")
            assert (rc, out) == (0, 'configmap "cfg" deleted\nconfigmap "cfg" replaced\n'), err
            now = await c.get("configmaps", "cfg", "default")
            assert now["metadata"]["uid"] != uid and "kubectl.kubernetes.io/last-applied-configuration" in now["metadata"]["annotations"]
            gone = tmp_path / "gone.json"
            gone.write_text(json.dumps({**cm, "metadata": {"name": "newcfg"}}))
            rc, out, err = await _kubectl(c, "replace", "--force", "-f", str(gone))    # TestForceReplaceObjectNotFound
            assert (rc, out) == (0, 'configmap "newcfg" replaced\n'), err
    run(body())
