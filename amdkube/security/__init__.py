"""Pod security profiles: AppArmor (apparmor.py) and seccomp annotation validation.

Reference: pkg/apis/core/validation/validation.go:3171-3196 (ValidateSeccompProfile,
ValidateSeccompPodAnnotations). The seccomp compiler/applier itself is native
(native/seccomp_bpf.h, run by amdkube-nsexec); the kubelet resolves the annotations into the
CRI seccomp_profile_path (kubelet/kuberuntime.py::seccomp_profile).
"""
from __future__ import annotations

from ..api.field import go_value

SECCOMP_POD_ANNOTATION = "seccomp.security.alpha.kubernetes.io/pod"
SECCOMP_CONTAINER_PREFIX = "container.seccomp.security.alpha.kubernetes.io/"


def validate_seccomp_profile(p: str) -> str | None:
    if p in ("docker/default", "runtime/default", "unconfined"):
        return None
    if p.startswith("localhost/"):
        rel = p[len("localhost/"):]
        if not rel or ".." in rel.split("/"):
            return "must be a valid seccomp profile: localhost path must not contain '..'"
        return None
    return "must be a valid seccomp profile"


def validate_seccomp_annotations(annotations: dict) -> list[str]:
    errs = []
    for k, v in (annotations or {}).items():
        if k == SECCOMP_POD_ANNOTATION or k.startswith(SECCOMP_CONTAINER_PREFIX):
            e = validate_seccomp_profile(v)
            if e:
                errs.append(f"metadata.annotations[{k}]: Invalid value: {go_value(v)}: {e}")
    return errs
