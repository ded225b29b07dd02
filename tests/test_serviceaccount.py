"""ServiceAccount admission (plugin/pkg/admission/serviceaccount/admission.go) and the in-cluster
client config a pod's amdkube component uses (client-go rest.InClusterConfig)."""
import os

import pytest

from amdkube.api import meta as m
from amdkube.client import Client
from amdkube.client.rest import ConfigError
from amdkube.localcluster import LocalCluster
from tests.conftest import run

MOUNT = "/var/run/secrets/kubernetes.io/serviceaccount"


def _pod(name, sa=None, **spec):
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "team"},
         "spec": {"containers": [{"name": "c", "image": "busybox"}], "initContainers": [{"name": "i", "image": "busybox"}]}}
    if sa:
        p["spec"]["serviceAccountName"] = sa
    p["spec"].update(spec)
    return p


def test_serviceaccount_admission_mounts_tokens_and_enforces_references():
    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
            await c.create({"apiVersion": "v1", "kind": "Secret", "metadata": {
                "name": "builder-token-abcde", "namespace": "team",
                "annotations": {"kubernetes.io/service-account.name": "builder"}},
                "type": "kubernetes.io/service-account-token", "data": {"token": "dG9r"}})
            await c.create({"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "other", "namespace": "team"},
                            "data": {"x": "eQ=="}})
            await c.create({"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "builder", "namespace": "team"},
                            "secrets": [{"name": "builder-token-abcde"}], "imagePullSecrets": [{"name": "regcred"}]})
            # the token is mounted in every container, init containers too, as a secret volume
            p = await c.create(_pod("a", "builder"))
            vols = {v["name"]: v for v in p["spec"]["volumes"]}
            assert vols["builder-token-abcde"]["secret"]["secretName"] == "builder-token-abcde"
            for ct in p["spec"]["containers"] + p["spec"]["initContainers"]:
                assert {"name": "builder-token-abcde", "readOnly": True, "mountPath": MOUNT} in ct["volumeMounts"]
            assert p["spec"]["imagePullSecrets"] == [{"name": "regcred"}]
            # automountServiceAccountToken: false on the pod wins; a container's own mount there wins
            p = await c.create(_pod("b", "builder", automountServiceAccountToken=False))
            assert not p["spec"].get("volumes")
            own = _pod("c", "builder")
            own["spec"]["containers"][0]["volumeMounts"] = [{"name": "mine", "mountPath": MOUNT}]
            own["spec"]["volumes"] = [{"name": "mine", "emptyDir": {}}]
            p = await c.create(own)
            assert [vm["name"] for vm in p["spec"]["containers"][0]["volumeMounts"]] == ["mine"]
            assert p["spec"]["initContainers"][0]["volumeMounts"][0]["name"] == "builder-token-abcde"
            # a named account that does not exist: 403; the default account missing: no token, no error
            with pytest.raises(m.StatusError) as ei:
                await c.create(_pod("d", "ghost"))
            assert ei.value.code == 403 and 'serviceaccount "ghost" not found' in ei.value.message
            p = await c.create(_pod("e"))
            assert p["spec"]["serviceAccountName"] == "default" and not p["spec"].get("volumes")
            # enforce-mountable-secrets: only the account's secrets
            await c.patch("serviceaccounts", "builder", {"metadata": {"annotations": {
                "kubernetes.io/enforce-mountable-secrets": "true"}}}, "team")
            bad = _pod("f", "builder")
            bad["spec"]["volumes"] = [{"name": "o", "secret": {"secretName": "other"}}]
            with pytest.raises(m.StatusError) as ei:
                await c.create(bad)
            assert ei.value.code == 403 and 'secret.secretName="other" is not allowed' in ei.value.message
            # mirror pods may reference neither accounts nor secrets
            mirror = _pod("g", "builder")
            mirror["metadata"]["annotations"] = {"kubernetes.io/config.mirror": "x"}
            with pytest.raises(m.StatusError) as ei:
                await c.create(mirror)
            assert "mirror pod may not reference service accounts" in ei.value.message
    run(go())


def test_in_cluster_config(tmp_path, monkeypatch):
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    with pytest.raises(ConfigError):
        Client.in_cluster()
    root = tmp_path / "rootfs"
    d = root / MOUNT.lstrip("/")
    d.mkdir(parents=True)
    (d / "token").write_text("sa-jwt\n")
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "10.0.0.1")
    monkeypatch.setenv("KUBERNETES_SERVICE_PORT", "443")
    monkeypatch.setenv("AMDKUBE_ROOTFS", str(root))       # no mount namespace: the volume sits under the rootfs

    async def go():
        c = Client.in_cluster()
        try:
            assert c.server == "https://10.0.0.1:443" and c.headers["Authorization"] == "Bearer sa-jwt"
        finally:
            await c.close()
    run(go())
    import argparse
    from amdkube.cmd.components import _client

    async def go2():
        c = _client(argparse.Namespace(server="http://127.0.0.1:8080", kubeconfig=None, token=None))
        try:
            assert c.server == "https://10.0.0.1:443"
        finally:
            await c.close()
        c = _client(argparse.Namespace(server="http://10.1.1.1:8080", kubeconfig=None, token=None))
        try:
            assert c.server == "http://10.1.1.1:8080"                  # an explicit --server wins
        finally:
            await c.close()
    run(go2())
