"""CustomResourceDefinitions (reference staging/src/k8s.io/apiextensions-apiserver:
test/integration/basic_test.go (serve, list/watch, delete), validation_test.go (openAPIV3Schema
on create/update), finalization_test.go (instances removed before the definition),
registration_test.go (namespaced and cluster scope, discovery))."""
import asyncio

from amdkube.api import meta as m
from amdkube.apiserver.crd import validate_crd, validate_schema
from amdkube.localcluster import LocalCluster


def crd(scope="Namespaced", schema=None):
    spec = {"group": "amd.com", "version": "v1alpha1", "scope": scope,
            "names": {"plural": "gpujobs", "singular": "gpujob", "kind": "GPUJob", "shortNames": ["gj"]},
            "subresources": {"status": {}}}
    if schema:
        spec["validation"] = {"openAPIV3Schema": schema}
    return {"apiVersion": "apiextensions.k8s.io/v1beta1", "kind": "CustomResourceDefinition",
            "metadata": {"name": "gpujobs.amd.com"}, "spec": spec}


SCHEMA = {"properties": {"spec": {"type": "object", "required": ["gpus", "image"],
                                  "properties": {"gpus": {"type": "integer", "minimum": 1, "maximum": 8},
                                                 "image": {"type": "string", "pattern": "^[a-z0-9./:-]+$"},
                                                 "topology": {"type": "string", "enum": ["xgmi", "any"]},
                                                 "args": {"type": "array", "items": {"type": "string"}, "maxItems": 4}}}}}


def test_crd_and_schema_validation_rules():
    assert validate_crd(crd()) == []
    bad = crd()
    bad["metadata"]["name"] = "jobs.amd.com"
    bad["spec"]["group"] = "amd"
    bad["spec"]["scope"] = "Global"
    errs = validate_crd(bad)
    assert any("spec.group" in e for e in errs) and any("metadata.name" in e for e in errs) and any("spec.scope" in e for e in errs)
    s = SCHEMA["properties"]["spec"]
    assert validate_schema({"gpus": 2, "image": "rocm/vector-add"}, s) == []
    errs = validate_schema({"gpus": 9, "image": "Bad Image", "topology": "nvlink", "args": ["a"] * 5}, s)
    assert len(errs) == 4
    assert "gpus: Invalid value: must be of type integer" in validate_schema({"gpus": "2"}, s)
    assert validate_schema({"a": 1}, {"type": "object", "additionalProperties": False})
    assert validate_schema(3, {"oneOf": [{"type": "integer"}, {"type": "number"}]})   # both match → not exactly one


async def test_custom_resources_served_validated_and_finalized():
    async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
        c = lc.client
        await c.create(crd(schema=SCHEMA))

        async def established():
            for _ in range(100):
                o = await c.get("customresourcedefinitions.apiextensions.k8s.io", "gpujobs.amd.com")
                conds = {x["type"]: x["status"] for x in (o.get("status") or {}).get("conditions") or []}
                if conds.get("Established") == "True":
                    return o
                await asyncio.sleep(0.05)
            raise AssertionError(o)
        o = await established()
        assert o["status"]["acceptedNames"]["kind"] == "GPUJob"
        assert "customresourcecleanup.apiextensions.k8s.io" in o["metadata"]["finalizers"]
        # discovery lists the new group/version and resource
        res = await c.request("GET", "/apis/amd.com/v1alpha1")
        assert [r["name"] for r in res["resources"] if r["name"] == "gpujobs"]
        job = {"apiVersion": "amd.com/v1alpha1", "kind": "GPUJob", "metadata": {"name": "train"},
               "spec": {"gpus": 8, "image": "rocm/pytorch", "topology": "xgmi"}}
        created = await c.create(job, "default")
        assert created["metadata"]["uid"] and created["spec"]["gpus"] == 8
        bad = {**job, "metadata": {"name": "bad"}, "spec": {"gpus": 16, "image": "x"}}
        try:
            await c.create(bad, "default")
            raise AssertionError("schema violation must be rejected")
        except m.StatusError as e:
            assert e.code == 422 and "gpus" in e.message
        items, rv = await c.list("gpujobs.amd.com", "default")
        assert [m.name_of(i) for i in items] == ["train"]
        # watch + status subresource
        seen = []

        async def watch():
            async for typ, obj in c.watch("gpujobs.amd.com", "default", rv):
                seen.append((typ, (obj.get("status") or {}).get("phase")))
                if typ == "MODIFIED":
                    return
        t = asyncio.create_task(watch())
        await asyncio.sleep(0.1)
        await c.patch("gpujobs.amd.com", "train", {"status": {"phase": "Running"}}, "default", sub="status")
        await asyncio.wait_for(t, 10)
        assert seen[-1] == ("MODIFIED", "Running")
        # a custom resource named like a built-in one does not collide with it
        assert (await c.list("pods", "default"))[0] == []
        # deleting the definition removes every instance first (finalizer), then the API
        await c.delete("customresourcedefinitions.apiextensions.k8s.io", "gpujobs.amd.com")
        for _ in range(100):
            if await c.get_or_none("customresourcedefinitions.apiextensions.k8s.io", "gpujobs.amd.com") is None:
                break
            await asyncio.sleep(0.05)
        assert await c.get_or_none("customresourcedefinitions.apiextensions.k8s.io", "gpujobs.amd.com") is None
        assert not lc.api.store.range("/registry/crd/amd.com/gpujobs/")[0]
        try:
            await c.request("GET", "/apis/amd.com/v1alpha1/namespaces/default/gpujobs")
            raise AssertionError("the resource must be gone")
        except m.StatusError as e:
            assert e.code == 404


def test_kubectl_discovers_custom_resources(tmp_path, capsys):
    """kubectl in its own process knows only built-in kinds: a custom resource name is resolved
    through the server's discovery documents."""
    import subprocess
    import sys

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            await lc.client.create(crd(schema=SCHEMA))
            for _ in range(100):
                if "gpujobs.amd.com" in lc.api.crds.installed:
                    break
                await asyncio.sleep(0.05)
            f = tmp_path / "job.yaml"
            f.write_text("apiVersion: amd.com/v1alpha1\nkind: GPUJob\nmetadata:\n  name: train\nspec:\n  gpus: 4\n  image: rocm/pytorch\n")
            env = {"PYTHONPATH": "/root/repo", "PATH": "/usr/bin:/bin", "AMDKUBE_SERVER": lc.api.url}
            tok = ["--token", lc.api.loopback_token]
            run = lambda *args: asyncio.get_running_loop().run_in_executor(None, lambda: subprocess.run(
                [sys.executable, "-m", "amdkube", "kubectl", *tok, *args], capture_output=True, text=True, env=env, timeout=60))
            r = await run("apply", "-f", str(f))
            assert r.returncode == 0 and "gpujob/train created" in r.stdout, r.stderr
            r = await run("get", "gj", "-o", "jsonpath={.items[0].spec.gpus}")
            assert r.stdout.strip() == "4", r.stderr
            r = await run("delete", "gpujobs", "train")
            assert r.returncode == 0 and 'deleted' in r.stdout, r.stderr
    from tests.conftest import run as run_async
    run_async(go(), 120)
