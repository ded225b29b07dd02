"""kubectl patch against pkg/kubectl/cmd/patch.go RunPatch and patch_test.go (TestPatchObject,
TestPatchObjectFromFile, TestPatchNoop, TestPatchObjectFromFileOutput), run on a live apiserver."""
from __future__ import annotations

import json

from tests.conftest import run
from tests.test_kubectl_commands_parity import _kubectl


def test_patch_through_the_cluster(tmp_path):
    from amdkube.localcluster import LocalCluster

    async def body():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "frontend", "labels": {"app": "x"}},
                   "spec": {"ports": [{"port": 80}], "selector": {"app": "x"}}}
            await c.create(svc, "default")
            # TestPatchObject: TYPE NAME and TYPE/NAME, strategic by default
            rc, out, err = await _kubectl(c, "patch", "services", "frontend", "-p", '{"spec":{"type":"NodePort"}}')
            assert (rc, out) == (0, 'service "frontend" patched\n'), err
            assert (await c.get("services", "frontend", "default"))["spec"]["type"] == "NodePort"
            # TestPatchNoop: nothing changed
            rc, out, err = await _kubectl(c, "patch", "service/frontend", "-p", '{"spec":{"type":"NodePort"}}')
            assert (rc, out) == (1, 'service "frontend" not patched\n')
            # YAML patches, merge type, -o name
            rc, out, err = await _kubectl(c, "patch", "service/frontend", "--type", "merge", "-p", "metadata: {labels: {tier: web}}",
                                          "-o", "name")
            assert (rc, out) == (0, "service/frontend\n"), err
            assert (await c.get("services", "frontend", "default"))["metadata"]["labels"] == {"app": "x", "tier": "web"}
            # json patch, -o json prints the object
            rc, out, err = await _kubectl(c, "patch", "service/frontend", "--type", "JSON", "-p",
                                          '[{"op":"replace","path":"/metadata/labels/tier","value":"api"}]', "-o", "json")
            assert rc == 0 and json.loads(out)["metadata"]["labels"]["tier"] == "api", err
            # TestPatchObjectFromFile
            f = tmp_path / "svc.json"
            f.write_text(json.dumps(svc))
            rc, out, err = await _kubectl(c, "patch", "-f", str(f), "-p", '{"metadata":{"annotations":{"a":"b"}}}')
            assert (rc, out) == (0, 'service "frontend" patched\n'), err
            # --local never reaches the server (TestPatchObjectFromFileOutput)
            rc, out, err = await _kubectl(c, "patch", "--local", "-f", str(f), "-p", '{"spec":{"type":"NodePort"}}', "-o", "json")
            assert rc == 0 and json.loads(out)["spec"]["type"] == "NodePort" and "annotations" not in json.loads(out)["metadata"]
            for argv, msg in ((["--local", "service/frontend", "-p", "{}"], "cannot specify --local and server resources"),
                              (["service/frontend", "--type", "apply", "-p", "{}"],
                               '--type must be one of [json merge strategic], not "apply"'),
                              (["service/frontend"], "Must specify -p to patch"),
                              (["service/frontend", "-p", "{bad"], "unable to parse")):
                rc, out, err = await _kubectl(c, "patch", *argv)
                assert rc == 1 and msg in err, (argv, err)
            rc, out, err = await _kubectl(c, "patch", "service/missing", "-p", "{}")
            assert rc == 1 and 'services "missing" not found' in err
    run(body())
