"""AppArmor for pod containers: annotation helpers, API validation and the kubelet admit check.

Reference: pkg/security/apparmor/helpers.go:25-80 (annotation keys, runtime/default,
localhost/<name>, unconfined), validate.go:45-230 (NewValidator: gate + kernel + runtime check;
Validate: every container's profile format is valid and every localhost/ profile is loaded,
read from <securityfs>/apparmor/profiles), pkg/apis/core/validation/validation.go:3198-3234
(ValidateAppArmorPodAnnotations), pkg/kubelet/lifecycle/handlers.go:142-165 (AppArmor admit
handler, reason "AppArmor"), pkg/kubelet/kuberuntime/security_context.go:40 (profile into
the CRI security context).

The enforcement end is native: rocshim hands a localhost/<name> profile to amdkube-nsexec
`--apparmor <name>`, which writes `exec <name>` to /proc/self/attr/apparmor/exec (falling
back to /proc/self/attr/exec) right before execve, so the container's first instruction runs
confined; a failed transition is fatal (exit 126).
"""
from __future__ import annotations

import os

from ..api.field import go_value

CONTAINER_ANNOTATION_PREFIX = "container.apparmor.security.beta.kubernetes.io/"
DEFAULT_PROFILE_ANNOTATION = "apparmor.security.beta.kubernetes.io/defaultProfileName"
ALLOWED_PROFILES_ANNOTATION = "apparmor.security.beta.kubernetes.io/allowedProfileNames"
RUNTIME_DEFAULT = "runtime/default"
LOCALHOST = "localhost/"
UNCONFINED = "unconfined"


def profile_name(pod: dict, container: str) -> str:
    return ((pod.get("metadata") or {}).get("annotations") or {}).get(CONTAINER_ANNOTATION_PREFIX + container, "")


def is_required(pod: dict) -> bool:
    """True when any container asks for a profile other than unconfined (helpers.go:44)."""
    for k, v in ((pod.get("metadata") or {}).get("annotations") or {}).items():
        if k.startswith(CONTAINER_ANNOTATION_PREFIX) and v != UNCONFINED:
            return True
    return False


def validate_profile_format(profile: str) -> str | None:
    if profile in ("", RUNTIME_DEFAULT, UNCONFINED) or profile.startswith(LOCALHOST):
        return None
    return f"invalid AppArmor profile name: {profile!r}"


def validate_pod_annotations(pod: dict, gate_enabled: bool = True) -> list[str]:
    """API-side check: the container must exist and the profile name must be well formed."""
    spec = pod.get("spec") or {}
    names = {c.get("name") for c in (spec.get("containers") or []) + (spec.get("initContainers") or [])}
    errs = []
    for k, v in ((pod.get("metadata") or {}).get("annotations") or {}).items():
        if not k.startswith(CONTAINER_ANNOTATION_PREFIX):
            continue
        path = f"metadata.annotations[{k}]"
        if not gate_enabled:
            errs.append(f"{path}: Forbidden: AppArmor is disabled by feature-gate")
            continue
        if k[len(CONTAINER_ANNOTATION_PREFIX):] not in names:
            errs.append(f"{path}: Invalid value: {go_value(k[len(CONTAINER_ANNOTATION_PREFIX):])}: container not found")
        e = validate_profile_format(v)
        if e:
            errs.append(f"{path}: Invalid value: {go_value(v)}: {e}")
    return errs


def parse_profiles(text: str) -> set[str]:
    """<securityfs>/apparmor/profiles: `name (mode)` or `ns://name (mode)` per line."""
    out = set()
    for line in text.splitlines():
        i = line.find("(")
        if i >= 0 and line[:i].strip():
            out.add(line[:i].strip())
    return out


def find_apparmor_fs(mounts: str = "/proc/mounts") -> str:
    with open(mounts) as f:
        for line in f:
            fields = line.split()
            if len(fields) >= 3 and fields[2] == "securityfs":
                p = os.path.join(fields[1], "apparmor")
                if os.path.exists(p):
                    return p
                raise LookupError(f"path {p} does not exist")
    raise LookupError("securityfs not found")


def host_enabled(sys_root: str = "/sys") -> bool:
    """Kernel support (validate.go:221): apparmor securityfs present and module parameter `Y`."""
    if os.environ.get("container"):
        return False
    try:
        with open(os.path.join(sys_root, "module/apparmor/parameters/enabled")) as f:
            return f.read(1) == "Y" and os.path.isdir(os.path.join(sys_root, "kernel/security/apparmor"))
    except OSError:
        return False


class Validator:
    """Kubelet-side: computed once at startup, consulted for every pod admission."""

    def __init__(self, gate_enabled: bool = True, runtime: str = "remote", apparmor_fs: str | None = None,
                 host_check=host_enabled):
        self.fs, self.host_err = apparmor_fs, None
        if not gate_enabled:
            self.host_err = "AppArmor disabled by feature-gate"
        elif runtime not in ("remote", "docker"):
            self.host_err = f"AppArmor is only enabled for 'docker' and 'remote' runtimes. Found: {runtime!r}."
        elif apparmor_fs is None:
            if not host_check():
                self.host_err = "AppArmor is not enabled on the host"
            else:
                try:
                    self.fs = find_apparmor_fs()
                except (OSError, LookupError) as e:
                    self.host_err = f"error finding AppArmor FS: {e}"

    def loaded_profiles(self) -> set[str]:
        with open(os.path.join(self.fs, "profiles")) as f:
            return parse_profiles(f.read())

    def validate(self, pod: dict) -> str | None:
        if not is_required(pod):
            return None
        if self.host_err:
            return self.host_err
        try:
            loaded = self.loaded_profiles()
        except OSError as e:
            return f"could not read loaded profiles: {e}"
        spec = pod.get("spec") or {}
        for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
            prof = profile_name(pod, c["name"])
            err = validate_profile_format(prof)
            if err:
                return err
            if prof.startswith(LOCALHOST) and prof[len(LOCALHOST):] not in loaded:
                return f"profile {prof[len(LOCALHOST):]!r} is not loaded"
        return None
