"""OpenAPI document, kubectl explain and client-side --validate
(pkg/kubectl/explain/*_test.go, pkg/kubectl/cmd/util/openapi/validation/validation_test.go,
staging/src/k8s.io/apiserver/pkg/server/routes/openapi.go)."""
import glob

import aiohttp

from amdkube.api import openapi as oa
from amdkube.api.scheme import SCHEME, load_manifests
from amdkube.kubectl.main import main as kubectl_main
from amdkube.localcluster import LocalCluster
from tests.conftest import ROOT, run


def _refs(node, out):
    if isinstance(node, dict):
        if isinstance(node.get("$ref"), str):       # (JSONSchemaProps has a *property* named $ref)
            out.add(node["$ref"].rsplit("/", 1)[1])
        for v in node.values():
            _refs(v, out)
    elif isinstance(node, list):
        for v in node:
            _refs(v, out)


def test_document_is_closed_and_covers_every_served_kind():
    doc = oa.document()
    defs = doc["definitions"]
    assert doc["swagger"] == "2.0"
    refs = set()
    _refs(doc, refs)
    assert refs <= set(defs), refs - set(defs)
    for ri in SCHEME.by_kind.values():
        if "." in ri.group and not ri.group.endswith("k8s.io"):
            continue        # custom resources other tests registered in this process
        assert oa.kind_definition(ri.api_version, ri.kind), ri
        base = ri.api_prefix() + ("/namespaces/{namespace}" if ri.namespaced else "") + f"/{ri.plural}"
        assert base in doc["paths"] and base + "/{name}" in doc["paths"], base
    # served-only versions share their storage kind's definition unless their shape differs
    assert oa.kind_definition("apps/v1beta2", "Deployment") == "io.k8s.api.apps.v1.Deployment"
    gvks = defs["io.k8s.api.apps.v1.Deployment"]["x-kubernetes-group-version-kind"]
    assert {"group": "apps", "version": "v1beta2", "kind": "Deployment"} in gvks
    assert oa.kind_definition("extensions/v1beta1", "Deployment") == "io.k8s.api.extensions.v1beta1.Deployment"
    assert "rollbackTo" in defs["io.k8s.api.extensions.v1beta1.DeploymentSpec"]["properties"]
    assert "rollbackTo" not in defs["io.k8s.api.apps.v1.DeploymentSpec"]["properties"]
    # the fork's device-granular fields
    assert defs["io.k8s.api.core.v1.Container"]["properties"]["extendedResourceRequests"]["items"] == {"type": "string"}
    assert defs["io.k8s.api.core.v1.PodSpec"]["properties"]["extendedResources"]["items"]["$ref"].endswith("PodExtendedResource")
    assert "extendedResourceBinding" in defs["io.k8s.api.core.v1.ObjectReference"]["properties"]
    assert "extendedResources" in defs["io.k8s.api.core.v1.NodeStatus"]["properties"]
    assert defs["io.k8s.api.core.v1.PodList"]["properties"]["items"]["items"]["$ref"].endswith("core.v1.Pod")


def test_validation_messages():
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "x", "labels": {"a": 1}},
           "spec": {"contaners": [], "containers": [{"image": "rocm/vector-add", "ports": [{"containerPort": "80"}],
                                                    "resources": {"limits": {"amd.com/gpu": 2, "memory": "1Gi"}},
                                                    "livenessProbe": {"httpGet": {"port": "http"}}}],
                    "tolerations": {"key": "x"}}}
    errs = oa.validate(pod)
    assert 'ValidationError(Pod.spec): unknown field "contaners" in io.k8s.api.core.v1.PodSpec' in errs
    assert 'ValidationError(Pod.spec.containers[0]): missing required field "name" in io.k8s.api.core.v1.Container' in errs
    assert ('ValidationError(Pod.spec.containers[0].ports[0].containerPort): invalid type for '
            'io.k8s.api.core.v1.ContainerPort.containerPort: got "string", expected "integer"') in errs
    assert ('ValidationError(Pod.metadata.labels.a): invalid type for io.k8s.apimachinery.pkg.apis.meta.v1.ObjectMeta.labels: '
            'got "integer", expected "string"') in errs
    assert any("Pod.spec.tolerations" in e and 'expected "array"' in e for e in errs)
    assert len(errs) == 5, errs     # quantities accept numbers, int-or-string accepts names
    # unknown kinds (custom resources) are not validated; a v1 List validates its items
    assert oa.validate({"apiVersion": "example.com/v1", "kind": "Widget", "spec": {"anything": 1}}) == []
    lst = {"apiVersion": "v1", "kind": "List", "items": [{"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c"},
                                                          "data": {"k": "v"}, "bogus": 1}]}
    assert oa.validate(lst) == ['ValidationError(List.items[0].ConfigMap): unknown field "bogus" in io.k8s.api.core.v1.ConfigMap']
    # extensions/v1beta1 defaults its selector, so it is not required in that version
    dep = {"apiVersion": "extensions/v1beta1", "kind": "Deployment", "metadata": {"name": "d"},
           "spec": {"template": {"metadata": {"labels": {"a": "b"}}, "spec": {"containers": [{"name": "c", "image": "i"}]}}}}
    assert oa.validate(dep) == []
    assert oa.validate(dict(dep, apiVersion="apps/v1")) == [
        'ValidationError(Deployment.spec): missing required field "selector" in io.k8s.api.apps.v1.DeploymentSpec']


def test_shipped_manifests_validate():
    for f in sorted(glob.glob(f"{ROOT}/deploy/**/*.yaml", recursive=True)):
        for d in load_manifests(open(f).read()):
            assert oa.validate(d) == [], (f, oa.validate(d))


def test_explain_rendering():
    defs = oa.definitions()
    top = oa.explain(defs, "v1", "Pod", [])
    assert top.startswith("KIND:     Pod\nVERSION:  v1\n\nDESCRIPTION:\n")
    assert "   spec\t<Object>\n" in top and "   apiVersion\t<string>\n" in top
    res = oa.explain(defs, "v1", "Pod", ["spec", "containers"])
    assert "RESOURCE: containers <[]Object>" in res and "   name\t<string> -required-" in res
    assert "   extendedResourceRequests\t<[]string>" in res
    leaf = oa.explain(defs, "v1", "Node", ["status", "extendedResources"])
    assert "RESOURCE: extendedResources <map[string]Object>" in leaf and "   resources\t<map[string]Object>" in leaf
    prim = oa.explain(defs, "apps/v1", "Deployment", ["spec", "replicas"])
    assert "FIELD:    replicas <integer>" in prim
    rec = oa.explain(defs, "v1", "Pod", ["spec", "affinity"], recursive=True)
    assert "      requiredDuringSchedulingIgnoredDuringExecution\t<Object>\n         nodeSelectorTerms\t<[]Object>" in rec
    try:
        oa.explain(defs, "v1", "Pod", ["spec", "nope"])
        raise AssertionError("no error")
    except KeyError as e:
        assert 'field "nope" does not exist' in e.args[0]


def test_served_document_explain_and_validate_through_kubectl(tmp_path, capsys):
    bad = tmp_path / "bad.yaml"
    bad.write_text("apiVersion: v1\nkind: Pod\nmetadata: {name: typo}\nspec:\n  containers:\n"
                   "  - {name: c, image: busybox, command: [sleep, '60'], imagePulPolicy: Always}\n")

    async def go():
        async with LocalCluster(gpus="none", with_controllers=False, with_kubelet=False) as lc:
            url = lc.api.url
            async with aiohttp.ClientSession() as s:
                async with s.get(url + "/openapi/v2") as r:
                    assert r.status == 200
                    doc = await r.json()
                    etag = r.headers["ETag"]
                async with s.get(url + "/swagger.json", headers={"If-None-Match": etag}) as r:
                    assert r.status == 304
            assert doc["definitions"]["io.k8s.api.core.v1.Pod"]["x-kubernetes-group-version-kind"] == [
                {"group": "", "version": "v1", "kind": "Pod"}]
            return url

    url = run(go(), 60)
    capsys.readouterr()
    # the server has gone; explain falls back to this build's document and validation to it too
    assert kubectl_main(["-s", url, "explain", "pods.spec.tolerations"]) == 0
    out = capsys.readouterr().out
    assert "RESOURCE: tolerations <[]Object>" in out and "tolerationSeconds\t<integer>" in out

    async def go2():
        async with LocalCluster(gpus="none", with_controllers=False, with_kubelet=False) as lc:
            def k(*argv):
                import asyncio
                return asyncio.get_running_loop().run_in_executor(None, kubectl_main, ["-s", lc.api.url, *argv])
            assert await k("explain", "deployments.apps.spec.strategy.rollingUpdate") == 0
            assert await k("create", "-f", str(bad)) == 1
            assert await lc.client.get_or_none("pods", "typo", "default") is None
            assert await k("create", "-f", str(bad), "--validate=false") == 0
            assert await lc.client.get_or_none("pods", "typo", "default") is not None
    run(go2(), 60)
    cap = capsys.readouterr()
    assert "RESOURCE: rollingUpdate <Object>" in cap.out and "maxSurge\t<string>" in cap.out
    assert (f'error: error validating "{bad}": error validating data: [ValidationError(Pod.spec.containers[0]): '
            'unknown field "imagePulPolicy" in io.k8s.api.core.v1.Container]; if you choose to ignore these errors, '
            'turn validation off with --validate=false') in cap.err
    assert "pod/typo created" in cap.out


def test_kubectl_alpha_diff(tmp_path, capsys):
    """diff.go: LOCAL vs LIVE by default; MERGED is what apply would leave; LAST the annotation."""
    f = tmp_path / "cm.yaml"

    async def go():
        async with LocalCluster(gpus="none", with_controllers=False, with_kubelet=False) as lc:
            import asyncio

            def k(*argv):
                return asyncio.get_running_loop().run_in_executor(None, kubectl_main, ["-s", lc.api.url, *argv])
            f.write_text("apiVersion: v1\nkind: ConfigMap\nmetadata: {name: gpu-cfg}\ndata: {arch: gfx950, cus: '256'}\n")
            assert await k("alpha", "diff", "-f", str(f)) == 0     # not on the server: everything is added
            assert await k("apply", "-f", str(f)) == 0
            # a change made on the server outside apply, then an edit of the file
            cm = await lc.client.get("configmaps", "gpu-cfg", "default")
            cm["data"]["owner"] = "ops"
            await lc.client.update(cm)
            f.write_text("apiVersion: v1\nkind: ConfigMap\nmetadata: {name: gpu-cfg}\ndata: {arch: gfx950, cus: '304'}\n")
            capsys.readouterr()
            assert await k("alpha", "diff", "-f", str(f), "LAST", "LOCAL") == 0
            last_local = capsys.readouterr().out
            assert await k("alpha", "diff", "-f", str(f), "MERGED") == 0
            merged_live = capsys.readouterr().out
            try:
                await k("alpha", "diff", "-f", str(f), "LOCAL", "NOPE")
                raise AssertionError("accepted a bad version keyword")
            except SystemExit as e:
                assert 'Invalid parameter "NOPE"' in str(e)
            return last_local, merged_live
    last_local, merged_live = run(go(), 60)
    # LAST → LOCAL: only the edited key
    assert "-  cus: '256'" in last_local and "+  cus: '304'" in last_local and "owner" not in last_local
    assert "--- LAST/v1.ConfigMap.default.gpu-cfg" in last_local
    # MERGED vs LIVE: apply changes cus and keeps the server-side key
    assert "-  cus: '304'" in merged_live and "+  cus: '256'" in merged_live
    assert "owner" not in [ln for ln in merged_live.splitlines() if ln.startswith(("+ ", "- "))]
