"""Pod sysctls (alpha in the reference release).

Reference: pkg/apis/core/annotation_key_constants.go (`security.alpha.kubernetes.io/sysctls`
and `security.alpha.kubernetes.io/unsafe-sysctls`, comma-separated `name=value`),
pkg/apis/core/validation/validation.go:127-147,3250-3268 (name syntax, ≤253 chars, not both safe
and unsafe), pkg/kubelet/sysctl/whitelist.go (safe whitelist kernel.shm_rmid_forced,
net.ipv4.ip_local_port_range, net.ipv4.tcp_syncookies; --experimental-allowed-unsafe-sysctls
patterns ending in `*` must be namespaced; Admit rejects with SysctlForbidden, also for net
sysctls with hostNetwork and ipc sysctls with hostIPC) and namespace.go (kernel.sem,
kernel.shm*, kernel.msg*, fs.mqueue.* → ipc; net.* → net). The admitted sysctls go to the
runtime in LinuxPodSandboxConfig.sysctls.
"""
from __future__ import annotations

import re

from ..api.field import go_value

SAFE_ANNOTATION = "security.alpha.kubernetes.io/sysctls"
UNSAFE_ANNOTATION = "security.alpha.kubernetes.io/unsafe-sysctls"
MAX_LEN = 253
_SEG = r"[a-z0-9]([-_a-z0-9]*[a-z0-9])?"
SYSCTL_RE = re.compile(rf"^({_SEG}\.)*{_SEG}$")
PATTERN_RE = re.compile(rf"^({_SEG}\.)*({_SEG}|\*)$")
SAFE = ("kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range", "net.ipv4.tcp_syncookies")
FORBIDDEN_REASON = "SysctlForbidden"
INVALID_REASON = "InvalidSysctlAnnotation"


def namespaced_by(name: str) -> str:
    if name == "kernel.sem":
        return "ipc"
    for p, ns in (("kernel.shm", "ipc"), ("kernel.msg", "ipc"), ("fs.mqueue.", "ipc"), ("net.", "net")):
        if name.startswith(p):
            return ns
    return ""


def parse_annotation(value: str | None) -> list[tuple[str, str]]:
    """helper.SysctlsFromPodAnnotation: `a=1,b=2` → [(a, 1), (b, 2)]."""
    if not value:
        return []
    out = []
    for kv in value.split(","):
        k, sep, v = kv.partition("=")
        if not sep or not k:
            raise ValueError(f"sysctl {kv!r} not of the format sysctl_name=value")
        out.append((k, v))
    return out


def validate_annotations(annotations: dict | None, path: str = "metadata.annotations") -> list[str]:
    ann = annotations or {}
    errs, names = [], {}
    for key in (SAFE_ANNOTATION, UNSAFE_ANNOTATION):
        try:
            pairs = parse_annotation(ann.get(key))
        except ValueError as e:
            errs.append(f"{path}[{key}]: Invalid value: {go_value(ann.get(key))}: {e}")
            continue
        for i, (k, _v) in enumerate(pairs):
            if len(k) > MAX_LEN or not SYSCTL_RE.match(k):
                errs.append(f"{path}[{key}][{i}].name: Invalid value: {go_value(k)}: must have at most {MAX_LEN} characters "
                            f"and match regex {SYSCTL_RE.pattern}")
        names[key] = {k for k, _ in pairs}
    both = sorted(names.get(SAFE_ANNOTATION, set()) & names.get(UNSAFE_ANNOTATION, set()))
    if both:
        errs.append(f"{path}[{UNSAFE_ANNOTATION}]: Invalid value: {go_value(', '.join(both))}: can not be safe and unsafe")
    return errs


class Whitelist:
    """patternWhitelist for one annotation key."""

    def __init__(self, patterns, annotation: str):
        self.annotation = annotation
        self.exact: dict[str, str] = {}
        self.prefixes: dict[str, str] = {}
        for p in patterns:
            if len(p) > MAX_LEN or not PATTERN_RE.match(p):
                raise ValueError(f"sysctl {p!r} must have at most {MAX_LEN} characters and match regex {PATTERN_RE.pattern}")
            if p.endswith("*"):
                prefix = p[:-1]
                ns = namespaced_by(prefix)
                if not ns:
                    raise ValueError(f"the sysctls {p!r} are not known to be namespaced")
                self.prefixes[prefix] = ns
            else:
                ns = namespaced_by(p)
                if not ns:
                    raise ValueError(f"the sysctl {p!r} are not known to be namespaced")
                self.exact[p] = ns

    def _check(self, name: str, host_net: bool, host_ipc: bool) -> str:
        ns = self.exact.get(name)
        if ns is None:
            ns = next((v for p, v in self.prefixes.items() if name.startswith(p)), None)
        if ns is None:
            return f"{name!r} not whitelisted"
        if (ns == "ipc" and host_ipc) or (ns == "net" and host_net):
            return f"{name!r} not allowed with host {ns} enabled"
        return ""

    def admit(self, pod: dict) -> tuple[bool, str, str]:
        ann = ((pod.get("metadata") or {}).get("annotations") or {}).get(self.annotation)
        if not ann:
            return True, "", ""
        try:
            pairs = parse_annotation(ann)
        except ValueError as e:
            return False, INVALID_REASON, f"invalid {self.annotation} annotation: {e}"
        spec = pod.get("spec") or {}
        for k, _v in pairs:
            err = self._check(k, bool(spec.get("hostNetwork")), bool(spec.get("hostIPC")))
            if err:
                return False, FORBIDDEN_REASON, f"forbidden sysctl: {err}"
        return True, "", ""


def pod_sysctls(pod: dict) -> dict[str, str]:
    """Both annotations merged: what the runtime is asked to set in the sandbox."""
    ann = (pod.get("metadata") or {}).get("annotations") or {}
    out = {}
    for key in (SAFE_ANNOTATION, UNSAFE_ANNOTATION):
        try:
            out.update(parse_annotation(ann.get(key)))
        except ValueError:
            pass
    return out
