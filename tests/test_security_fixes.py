"""Round-2 advisor findings, each pinned by a test.

* volume item paths (validation.go validateLocalDescendingPath / IsConfigMapKey, and the
  kubelet's own check before it writes as root);
* ABAC subjectMatches (pkg/auth/authorizer/abac/abac.go): user AND group when both are set;
* OIDC (plugin/pkg/auth/authenticator/token/oidc/oidc.go:255-270): exp required, email
  usernames need email_verified == true;
* bootstrap checkpoints follow the annotation (pkg/kubelet/checkpoint).
(Front-proxy certificates must be signed by the requestheader CA:
tests/test_metrics_server.py::test_requestheader_authenticator.)
"""
import asyncio
import base64
import json
import os
import subprocess
import time

import pytest

from amdkube.api.validation import validate_pod, validate_config_data
from amdkube.apiserver.auth import Attributes
from amdkube.apiserver.authx import ABACAuthorizer, OIDCAuthenticator
from amdkube.kubelet.checkpoint import PodCheckpointManager
from amdkube.kubelet.podcontext import volume_file


def _pod(vol):
    from amdkube.api.scheme import SCHEME
    return SCHEME.default({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default"},
                           "spec": {"containers": [{"name": "c", "image": "busybox"}], "volumes": [vol]}})


@pytest.mark.parametrize("path", ["../../../../etc/cron.d/x", "/etc/passwd", "a/../../b", ".."])
def test_volume_item_paths_must_stay_inside(path):
    for vol in ({"name": "v", "secret": {"secretName": "s", "items": [{"key": "k", "path": path}]}},
                {"name": "v", "configMap": {"name": "c", "items": [{"key": "k", "path": path}]}},
                {"name": "v", "downwardAPI": {"items": [{"path": path, "fieldRef": {"fieldPath": "metadata.name"}}]}},
                {"name": "v", "projected": {"sources": [{"secret": {"name": "s", "items": [{"key": "k", "path": path}]}}]}}):
        errs = validate_pod(_pod(vol))
        assert any(".path" in e for e in errs), (vol, errs)
    ok = {"name": "v", "secret": {"secretName": "s", "items": [{"key": "k", "path": "dir/..data/file"}]}}
    assert not validate_pod(_pod(ok))


def test_config_keys_are_file_names():
    for bad in ("../x", "a/b", "..hidden", ".", "sp ace"):
        assert validate_config_data({"metadata": {"name": "c", "namespace": "d"}, "data": {bad: "v"}}), bad
    assert not validate_config_data({"metadata": {"name": "c", "namespace": "d"}, "data": {"tls.crt": "v", "a-b_c": "v"}})


def test_kubelet_refuses_escaping_volume_files(tmp_path):
    d = tmp_path / "vol"
    d.mkdir()
    assert volume_file(str(d), "a/b.txt") == str(d / "a" / "b.txt")
    for bad in ("../x", "/abs", "a/../../x", ""):
        with pytest.raises(ValueError):
            volume_file(str(d), bad)
    os.symlink("/etc", d / "link")          # a symlink already inside the volume cannot lead out
    with pytest.raises(ValueError):
        volume_file(str(d), "link/passwd")


def _attrs(user, groups):
    return Attributes({"name": user, "groups": groups}, "get", "", "pods", namespace="ns")


def test_abac_subject_needs_user_and_group(tmp_path):
    f = tmp_path / "policy.jsonl"
    f.write_text(json.dumps({"apiVersion": "abac.authorization.kubernetes.io/v1beta1", "kind": "Policy",
                             "spec": {"user": "alice", "group": "admins", "namespace": "*", "resource": "*"}}) + "\n")
    a = ABACAuthorizer(str(f))
    assert a.authorize(_attrs("alice", ["admins"]))[0]
    assert not a.authorize(_attrs("alice", ["devs"]))[0]      # alice outside admins: no
    assert not a.authorize(_attrs("bob", ["admins"]))[0]      # another admin: no
    f.write_text(json.dumps({"spec": {"group": "admins", "namespace": "*", "resource": "*"}}) + "\n")
    assert ABACAuthorizer(str(f)).authorize(_attrs("bob", ["admins"]))[0]
    f.write_text(json.dumps({"spec": {"user": "*", "group": "admins", "namespace": "*", "resource": "*"}}) + "\n")
    assert not ABACAuthorizer(str(f)).authorize(_attrs("bob", ["devs"]))[0]


def _b64u(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def test_oidc_requires_exp_and_verified_email(tmp_path):
    from amdkube.utils.crypto import rsa_spki
    key = tmp_path / "k.pem"
    subprocess.run(["openssl", "genrsa", "-out", str(key), "2048"], check=True, capture_output=True)
    mod = subprocess.run(["openssl", "rsa", "-in", str(key), "-noout", "-modulus"], capture_output=True, text=True,
                         check=True).stdout.strip().split("=")[1]

    def sign(claims):
        h = _b64u(json.dumps({"alg": "RS256", "kid": "k1"}).encode())
        p = _b64u(json.dumps(claims).encode())
        (tmp_path / "d").write_bytes(f"{h}.{p}".encode())
        subprocess.run(["openssl", "dgst", "-sha256", "-sign", str(key), "-out", str(tmp_path / "s"), str(tmp_path / "d")],
                       check=True, capture_output=True)
        return f"{h}.{p}.{_b64u((tmp_path / 's').read_bytes())}"
    iss = "https://issuer.example"

    def authn(claim):
        a = OIDCAuthenticator(iss, "amdkube", username_claim=claim)
        a.keys, a._fetched = {"k1": rsa_spki(int(mod, 16), 65537)}, time.monotonic()
        return a
    now = int(time.time())
    base = {"iss": iss, "aud": "amdkube", "sub": "1234", "email": "a@x.io"}
    run = lambda a, c: asyncio.run(a.authenticate(sign(c)))   # noqa: E731
    assert run(authn("sub"), {**base, "exp": now + 60})["name"] == f"{iss}#1234"
    assert run(authn("sub"), base) is None                                # no exp: refused
    assert run(authn("sub"), {**base, "exp": now - 5}) is None            # expired
    assert run(authn("sub"), {**base, "exp": "never"}) is None
    e = authn("email")
    assert run(e, {**base, "exp": now + 60, "email_verified": True})["name"] == "a@x.io"
    assert run(e, {**base, "exp": now + 60}) is None                      # email_verified missing
    assert run(e, {**base, "exp": now + 60, "email_verified": "true"}) is None   # not a boolean


def test_checkpoint_removed_when_annotation_dropped(tmp_path):
    cm = PodCheckpointManager(str(tmp_path))
    pod = {"metadata": {"name": "apiserver", "uid": "u1",
                        "annotations": {"node.kubernetes.io/bootstrap-checkpoint": "true"}}, "spec": {}}
    assert cm.write_pod(pod) and len(cm.load_pods()) == 1
    pod["metadata"]["annotations"] = {}
    assert not cm.write_pod(pod)
    assert cm.load_pods() == []
    os.chmod(tmp_path, 0o500)              # unwritable: logged, not raised
    try:
        pod["metadata"]["annotations"] = {"node.kubernetes.io/bootstrap-checkpoint": "true"}
        if os.geteuid() != 0:
            assert cm.write_pod(pod) is False
    finally:
        os.chmod(tmp_path, 0o700)
