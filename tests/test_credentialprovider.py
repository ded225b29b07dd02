"""Registry credentials (pkg/credentialprovider: config.go, keyring.go, secrets.go) and the
kubelet's use of them, plus the waiting reasons of a container that cannot start
(reason_cache.go: ErrImagePull, ImagePullBackOff, ErrImageNeverPull)."""
import asyncio
import base64
import hashlib
import json
import os

from amdkube.kubelet.credentialprovider import (AuthConfig, DockerKeyring, UnionKeyring, key_matches, node_keyring,
                                                parse_docker_config, secrets_keyring, split_image)
from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


def _b64(s: str) -> str:
    return base64.b64encode(s.encode()).decode()


def test_docker_config_formats():
    cfg = parse_docker_config({"auths": {"reg.example.com": {"auth": _b64("alice:s3cret"), "email": "a@x"}}})
    a = cfg["reg.example.com"]
    assert (a.username, a.password, a.email) == ("alice", "s3cret", "a@x")
    old = parse_docker_config(json.dumps({"https://index.docker.io/v1/": {"username": "bob", "password": "pw"}}))
    b = old["https://index.docker.io/v1/"]
    assert b.auth == _b64("bob:pw") and b.server_address == "https://index.docker.io/v1/"


def test_image_reference_parsing():
    assert split_image("busybox") == ("index.docker.io", "", "library/busybox")
    assert split_image("docker.io/team/app:1") == ("index.docker.io", "", "team/app")
    assert split_image("reg.example.com:5000/team/app:v1") == ("reg.example.com", "5000", "team/app")
    assert split_image("localhost/app@sha256:abc") == ("localhost", "", "app")


def test_keyring_matching_rules():
    # keyring.go urlsMatch: globbed host parts, equal ports, key path is a repository prefix
    assert key_matches("*.example.com", "reg.example.com/app")
    assert not key_matches("*.example.com", "a.b.example.com/app")
    assert key_matches("reg.example.com:5000", "reg.example.com:5000/x/y:1")
    assert not key_matches("reg.example.com:5000", "reg.example.com/x/y")
    assert key_matches("reg.example.com/team", "reg.example.com/team/app:1")
    assert not key_matches("reg.example.com/team", "reg.example.com/teamx/app")
    assert key_matches("https://index.docker.io/v1/", "busybox")
    assert key_matches("docker.io", "library/nginx:1")
    ring = DockerKeyring({"reg.example.com": AuthConfig("generic"), "reg.example.com/team": AuthConfig("team"),
                          "*.example.com": AuthConfig("glob"), "other.io": AuthConfig("other")})
    assert [a.username for a in ring.lookup("reg.example.com/team/app")] == ["team", "generic", "glob"]
    assert ring.lookup("quay.io/x") == []


def test_pod_secrets_before_node_config(tmp_path):
    (tmp_path / "config.json").write_text(json.dumps({"auths": {"reg.example.com": {"auth": _b64("node:n")}}}))
    node = node_keyring(str(tmp_path))
    assert [a.username for a in node.lookup("reg.example.com/app")] == ["node"]
    secrets = [
        {"type": "kubernetes.io/dockerconfigjson", "metadata": {"name": "s1"},
         "data": {".dockerconfigjson": _b64(json.dumps({"auths": {"reg.example.com": {"auth": _b64("pod:p")}}}))}},
        {"type": "kubernetes.io/dockercfg", "metadata": {"name": "s2"},
         "data": {".dockercfg": _b64(json.dumps({"reg2.example.com": {"username": "old", "password": "o"}}))}},
        {"type": "Opaque", "data": {".dockerconfigjson": _b64("{}")}},
        {"type": "kubernetes.io/dockerconfigjson", "metadata": {"name": "bad"}, "data": {".dockerconfigjson": _b64("not json")}},
    ]
    ring = UnionKeyring(secrets_keyring(secrets), node)
    assert [a.username for a in ring.lookup("reg.example.com/app")] == ["pod", "node"]
    assert [a.username for a in ring.lookup("reg2.example.com/app")] == ["old"]


def _registry(tmp_path):
    reg = tmp_path / "registry"
    img = reg / "registry.amd.local:5000" / "team" / "app" / "v1"
    img.mkdir(parents=True)
    run_ = img / "run"
    run_.write_text("#!/bin/sh\necho hello-from-private-registry\n")
    run_.chmod(0o755)
    (reg / "registry.amd.local:5000" / "auth.json").write_text(
        json.dumps({"users": {"alice": hashlib.sha256(b"s3cret").hexdigest()}}))
    return str(reg)


def _pod(name, secret=None, image="registry.amd.local:5000/team/app:v1", policy="IfNotPresent"):
    spec = {"restartPolicy": "Never", "containers": [{"name": "c", "image": image, "imagePullPolicy": policy}]}
    if secret:
        spec["imagePullSecrets"] = [{"name": secret}]
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"}, "spec": spec}


async def _waiting(c, name, want, timeout=15.0):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while True:
        p = await c.get("pods", name, "default")
        for cs in (p.get("status") or {}).get("containerStatuses") or []:
            w = (cs.get("state") or {}).get("waiting") or {}
            if w.get("reason") in want:
                return w
        assert loop.time() < end, p.get("status")
        await asyncio.sleep(0.1)


def test_private_registry_needs_the_pods_pull_secret(tmp_path):
    reg = _registry(tmp_path)

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, shim_kw={"registry_dir": reg}) as lc:
            c = lc.client
            # no credentials: the pull is refused and the container waits with the reason
            await c.create(_pod("anon"))
            w = await _waiting(c, "anon", ("ErrImagePull", "ImagePullBackOff"))
            assert "unauthorized" in w["message"] or "Back-off pulling image" in w["message"], w
            # a never-pull policy on an absent image
            await c.create(_pod("never", policy="Never", image="registry.amd.local:5000/team/other:v9"))
            w = await _waiting(c, "never", ("ErrImageNeverPull",))
            assert "not present with pull policy of Never" in w["message"]
            # the wrong password is refused too
            bad = {"auths": {"registry.amd.local:5000": {"auth": _b64("alice:wrong")}}}
            await c.create({"apiVersion": "v1", "kind": "Secret", "type": "kubernetes.io/dockerconfigjson",
                            "metadata": {"name": "bad", "namespace": "default"},
                            "data": {".dockerconfigjson": _b64(json.dumps(bad))}})
            await c.create(_pod("wrong", secret="bad"))
            await _waiting(c, "wrong", ("ErrImagePull", "ImagePullBackOff"))
            # the right credentials from the pod's imagePullSecrets
            good = {"auths": {"registry.amd.local:5000": {"auth": _b64("alice:s3cret")}}}
            await c.create({"apiVersion": "v1", "kind": "Secret", "type": "kubernetes.io/dockerconfigjson",
                            "metadata": {"name": "regcred", "namespace": "default"},
                            "data": {".dockerconfigjson": _b64(json.dumps(good))}})
            await c.create(_pod("authed", secret="regcred"))
            p = await wait_pod(c, "default", "authed", ("Succeeded", "Failed"), 30)
            assert p["status"]["phase"] == "Succeeded", p["status"]
            assert "hello-from-private-registry" in await c.logs("default", "authed")
            assert any(n.startswith("registry.amd.local:5000/team/app") for n, _, _ in lc.shim.images.list())
    run(go(), 90)


def test_image_store_registry_auth(tmp_path):
    from amdkube.runtime.images import ImageStore
    st = ImageStore(str(tmp_path / "state"), _registry(tmp_path))
    import pytest
    with pytest.raises(PermissionError):
        st.pull("registry.amd.local:5000/team/app:v1")
    with pytest.raises(PermissionError):
        st.pull("registry.amd.local:5000/team/app:v1", {"username": "alice", "password": "nope"})
    ref = st.pull("registry.amd.local:5000/team/app:v1", {"auth": _b64("alice:s3cret")})
    assert ref.startswith("sha256:") and st.size("registry.amd.local:5000/team/app:v1") > 0
    # present images are still re-checked against the registry's credentials (pull policy Always)
    with pytest.raises(PermissionError):
        st.pull("registry.amd.local:5000/team/app:v1")
    with pytest.raises(KeyError):
        st.pull("registry.amd.local:5000/team/missing:v1", {"auth": _b64("alice:s3cret")})
    assert os.path.isdir(st.blob_root)
