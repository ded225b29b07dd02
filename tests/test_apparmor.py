"""AppArmor pod profiles (SURVEY §2.3 "runc apparmor" row; reference
pkg/security/apparmor/validate_test.go, helpers.go; kubelet admit handler
pkg/kubelet/lifecycle/handlers.go:142-165; validation.go:3198 ValidateAppArmorPodAnnotations)."""
from __future__ import annotations

import os
import subprocess

from amdkube.api import meta as m
from amdkube.api.validation import validate_pod
from amdkube.localcluster import LocalCluster, wait_pod
from amdkube.runtime.images import NATIVE_BIN
from amdkube.security import apparmor as aa

KEY = aa.CONTAINER_ANNOTATION_PREFIX


def _pod(name, ann):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "annotations": ann},
            "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "busybox", "args": ["-c", "echo ok"]}]}}


def _fs(tmp_path):
    d = tmp_path / "apparmor"
    d.mkdir()
    (d / "profiles").write_text("amdkube-gpu (enforce)\nns://other (complain)\n/usr/bin/foo (enforce)\nbogus line\n")
    return str(d)


def test_profile_parsing_and_format():
    assert aa.parse_profiles("a (enforce)\nns://b (complain)\nnoparen\n") == {"a", "ns://b"}
    for ok in ("", "runtime/default", "unconfined", "localhost/x"):
        assert aa.validate_profile_format(ok) is None
    assert aa.validate_profile_format("docker-default")
    assert not aa.is_required(_pod("p", {KEY + "c": "unconfined"}))
    assert aa.is_required(_pod("p", {KEY + "c": "runtime/default"}))


def test_api_validation_of_annotations():
    assert not [e for e in validate_pod(_pod("p", {KEY + "c": "localhost/amdkube-gpu"})) if "apparmor" in e]
    errs = validate_pod(_pod("p", {KEY + "nope": "localhost/x", KEY + "c": "badformat"}))
    assert any("container not found" in e for e in errs) and any("invalid AppArmor profile" in e for e in errs)
    errs = validate_pod(_pod("p", {"seccomp.security.alpha.kubernetes.io/pod": "bogus"}))
    assert any("valid seccomp profile" in e for e in errs)
    assert any("'..'" in e for e in validate_pod(_pod("p", {"container.seccomp.security.alpha.kubernetes.io/c": "localhost/../x"})))


def test_validator_host_and_loaded_profiles(tmp_path):
    v = aa.Validator(apparmor_fs=_fs(tmp_path))
    assert v.validate(_pod("p", {KEY + "c": "localhost/amdkube-gpu"})) is None
    assert v.validate(_pod("p", {KEY + "c": "localhost/ns://other"})) is None
    assert "not loaded" in v.validate(_pod("p", {KEY + "c": "localhost/missing"}))
    assert v.validate(_pod("p", {})) is None
    assert "feature-gate" in aa.Validator(gate_enabled=False).validate(_pod("p", {KEY + "c": "runtime/default"}))
    off = aa.Validator(host_check=lambda: False)
    assert "not enabled on the host" in off.validate(_pod("p", {KEY + "c": "runtime/default"}))
    assert off.validate(_pod("p", {KEY + "c": "unconfined"})) is None      # unconfined never needs the host


def test_nsexec_apparmor_transition_is_fatal_without_lsm():
    if os.path.isdir("/sys/kernel/security/apparmor"):
        return  # host has AppArmor: the negative case below does not apply
    r = subprocess.run([os.path.join(NATIVE_BIN, "amdkube-nsexec"), "--no-namespaces", "--apparmor", "amdkube-gpu", "--",
                        "true"], capture_output=True, text=True)
    assert r.returncode == 126 and "AppArmor profile amdkube-gpu" in r.stderr


async def test_kubelet_rejects_unloaded_profile(tmp_path):
    async with LocalCluster(gpus="none", relist_period=0.2, kubelet_kw={"apparmor_fs": _fs(tmp_path)}) as lc:
        c = lc.client
        await c.create(_pod("missing", {KEY + "c": "localhost/not-there"}), "default")
        await c.create(_pod("unconfined", {KEY + "c": "unconfined"}), "default")
        p = await wait_pod(c, "default", "missing", ("Failed",), 20)
        assert p["status"]["reason"] == "AppArmor" and "not loaded" in p["status"]["message"]
        await wait_pod(c, "default", "unconfined", ("Succeeded",), 20)
        try:
            await c.create(_pod("bad", {KEY + "c": "docker-default"}), "default")
            raise AssertionError("malformed profile must be rejected by the apiserver")
        except m.StatusError as e:
            assert e.code == 422
