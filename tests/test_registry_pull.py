"""Image pull from a registry over the Docker Registry HTTP API v2 (runtime/registry.py), against
an in-repo fake registry (tests/fake_registry.py): token auth with the CRI AuthConfig,
manifest lists, digest references, digest-verified blobs, redirects without credentials, and a
pod whose image comes from a private registry through its imagePullSecrets.

Reference: kubeGenericRuntimeManager.PullImage (pkg/kubelet/kuberuntime/kuberuntime_image.go:31)
behind imageManager.EnsureImageExists (pkg/kubelet/images/image_manager.go:86) →
dockerService.PullImage (pkg/kubelet/dockershim/docker_image.go:73). Parity is unpinned: no
real registry is reachable here, the fake speaks the published protocol.
"""
import asyncio
import base64
import json
import os

import pytest

from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.runtime.oci import ImageFormatError
from amdkube.runtime.registry import RegistryClient, Unauthorized, is_remote, parse_reference, pull_image
from tests.conftest import run
from tests.fake_registry import FakeRegistry
from tests.test_images_rootfs import host_closure

BASE = [("etc", None, 0o755, None), ("etc/motd", b"base", 0o644, None), ("old", b"x", 0o644, None)]
TOP = [(".wh.old", b"", 0o644, None), ("etc/motd", b"from-registry", 0o644, None), ("new", b"n", 0o644, None)]


def test_reference_parsing():
    assert parse_reference("registry.local:5000/rocm/app:1") == ("registry.local:5000", "rocm/app", "1")
    assert parse_reference("localhost/app") == ("localhost", "app", "latest")
    assert parse_reference("busybox") == ("registry-1.docker.io", "library/busybox", "latest")
    d = "sha256:" + "a" * 64
    assert parse_reference(f"r.io/x/y@{d}") == ("r.io", "x/y", d)
    assert is_remote("127.0.0.1:5000/a:1") and is_remote("gcr.io/x") and not is_remote("rocm/vector-add")
    assert not is_remote("file:///tmp/x.tar") and not is_remote("busybox:latest")


def test_pull_multilayer_image_behind_token_auth(tmp_path):
    with FakeRegistry(users={"ci": "s3cret"}, redirect_blobs=True) as reg:
        digest = reg.push("team/app", "1", [BASE, TOP], {"Cmd": ["cat", "/etc/motd"]})
        cl = RegistryClient()
        rec = pull_image(f"{reg.host}/team/app:1", str(tmp_path / "store"), {"username": "ci", "password": "s3cret"}, cl)
        root = rec["rootfs"]
        assert open(os.path.join(root, "etc/motd")).read() == "from-registry"
        assert os.path.exists(os.path.join(root, "new")) and not os.path.exists(os.path.join(root, "old"))
        assert rec["cmd"] == ["cat", "/etc/motd"] and len(rec["layers"]) == 2
        assert rec["repo_digests"] == [f"{reg.host}/team/app@{digest}"]
        # the token came from the realm with the pull scope; blob-store redirects carried no credentials
        assert any(p.startswith("/token?") and "repository%3Ateam%2Fapp%3Apull" in p for _, p, _ in reg.log)
        assert all(a is None for _, p, a in reg.log if p.startswith("/blobstore/"))
        assert all(a and a.startswith("Bearer ") for _, p, a in reg.log[2:] if p.startswith("/v2/team/app/manifests"))
        # by digest, the same content
        rec2 = pull_image(f"{reg.host}/team/app@{digest}", str(tmp_path / "store2"), {"username": "ci", "password": "s3cret"})
        assert rec2["id"] == rec["id"]


def test_wrong_credentials_and_tampered_blobs_are_refused(tmp_path):
    with FakeRegistry(users={"ci": "s3cret"}) as reg:
        reg.push("team/app", "1", [BASE], {})
        for creds in (None, {"username": "ci", "password": "wrong"}):
            with pytest.raises(Unauthorized):
                pull_image(f"{reg.host}/team/app:1", str(tmp_path / "s"), creds)
        # docker config `auth` form
        auth = {"auth": base64.b64encode(b"ci:s3cret").decode()}
        assert pull_image(f"{reg.host}/team/app:1", str(tmp_path / "ok"), auth)["rootfs"]
        layer = json.loads(reg.manifests[("team/app", "1")][1])["layers"][0]["digest"]
        reg.tamper(layer)
        with pytest.raises(ImageFormatError, match="does not match its digest"):
            pull_image(f"{reg.host}/team/app:1", str(tmp_path / "t"), auth)
        with pytest.raises(KeyError):
            pull_image(f"{reg.host}/team/missing:1", str(tmp_path / "m"), auth)


def test_manifest_list_resolves_linux_amd64_and_basic_auth(tmp_path):
    with FakeRegistry(users={"u": "p"}, auth="basic") as reg:
        amd = reg.push("multi", "amd64", [[("arch", b"amd64", 0o644, None)]], {})
        arm = reg.push("multi", "arm64", [[("arch", b"arm64", 0o644, None)]], {}, arch="arm64")
        reg.push_list("multi", "v1", {"arm64": arm, "amd64": amd})
        rec = pull_image(f"{reg.host}/multi:v1", str(tmp_path / "s"), {"username": "u", "password": "p"})
        assert open(os.path.join(rec["rootfs"], "arch")).read() == "amd64"
        assert all(a and a.startswith("Basic ") for _, p, a in reg.log[1:])


def test_pod_runs_an_image_from_a_private_registry(tmp_path):
    """kubelet → CRI PullImage with the AuthConfig from the pod's imagePullSecrets → rocshim
    pulls over the v2 API, unpacks and runs it. Bad credentials surface as ErrImagePull."""
    layer = host_closure("/bin/sh", "/bin/cat") + [("etc", None, 0o755, None), ("etc/msg", b"hello-from-registry", 0o644, None)]

    async def go():
        with FakeRegistry(users={"ci": "s3cret"}) as reg:
            # WorkingDir "/" and a relative path: on an unprivileged node (no mount namespace) the
            # container runs the image's own loader from the rootfs with the rootfs as its cwd
            reg.push("team/app", "1", [layer], {"Entrypoint": ["/bin/sh", "-c"], "Cmd": ["cat etc/msg"],
                                                "Env": ["PATH=/usr/bin:/bin"], "WorkingDir": "/"})
            async with LocalCluster(gpus="none", with_controllers=False, relist_period=0.2) as lc:
                c = lc.client

                def secret(name, pw):
                    cfg = {"auths": {reg.host: {"username": "ci", "password": pw,
                                                "auth": base64.b64encode(f"ci:{pw}".encode()).decode()}}}
                    return {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": name},
                            "type": "kubernetes.io/dockerconfigjson",
                            "data": {".dockerconfigjson": base64.b64encode(json.dumps(cfg).encode()).decode()}}
                await c.create(secret("good", "s3cret"), "default")
                await c.create(secret("bad", "nope"), "default")

                def pod(name, sec):
                    # Always: the node already holds the image after the first pod; a re-pull
                    # checks the registry's manifest with this pod's credentials (dockerd's pull)
                    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
                            "spec": {"restartPolicy": "Never", "imagePullSecrets": [{"name": sec}],
                                     "containers": [{"name": "app", "image": f"{reg.host}/team/app:1",
                                                     "imagePullPolicy": "Always"}]}}
                await c.create(pod("good", "good"), "default")
                p = await wait_pod(c, "default", "good", ("Succeeded", "Failed"), 60)
                assert p["status"]["phase"] == "Succeeded", p["status"]
                assert (await c.logs("default", "good")).strip() == "hello-from-registry"
                await c.create(pod("bad", "bad"), "default")
                for _ in range(200):
                    p = await c.get("pods", "bad", "default")
                    waiting = [(cs.get("state") or {}).get("waiting") or {} for cs in (p.get("status") or {}).get("containerStatuses") or []]
                    if any(w.get("reason") in ("ErrImagePull", "ImagePullBackOff") for w in waiting):
                        break
                    await asyncio.sleep(0.1)
                else:
                    raise AssertionError(p.get("status"))
    run(go(), 120)
