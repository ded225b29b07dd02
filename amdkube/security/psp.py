"""PodSecurityPolicy: strategies, provider and the admission decision.

Reference: pkg/security/podsecuritypolicy/ — factory.go (one strategy per field of the policy),
user/{mustrunas,nonroot,runasany}.go, group/{mustrunas,runasany}.go (fsGroup and
supplementalGroups), selinux/{mustrunas,runasany}.go, capabilities/mustrunas.go (default add,
required drop, allowed), apparmor/strategy.go and seccomp/strategy.go (annotations of the
policy: default profile, allowed list), sysctl/mustmatchpatterns.go (the policy's
security.alpha.kubernetes.io/sysctls patterns), util/util.go (volume fs types, host path
prefixes), provider.go (CreatePod/ContainerSecurityContext default only what is unset,
Validate* check the result); plugin/pkg/admission/security/podsecuritypolicy/admission.go
(computeSecurityContext: every policy in name order is tried on a copy of the pod; a policy
that validates without changing the pod wins at once, else the first one that validates with
changes (create only); the requester or the pod's service account must be authorized to
`use` it; errors are reported only for policies the requester may use).

Errors are `FieldError`s rendered like apimachinery's field.Error ("path: Invalid value: v:
detail").
"""
from __future__ import annotations

import copy

from ..api.field import FieldError, forbidden, go_slice, invalid, required  # noqa: F401  (FieldError re-exported)

SECCOMP_POD_ANNOTATION = "seccomp.security.alpha.kubernetes.io/pod"
SECCOMP_CONTAINER_PREFIX = "container.seccomp.security.alpha.kubernetes.io/"
SECCOMP_DEFAULT_PROFILE = "seccomp.security.alpha.kubernetes.io/defaultProfileName"
SECCOMP_ALLOWED_PROFILES = "seccomp.security.alpha.kubernetes.io/allowedProfileNames"
SECCOMP_ALLOW_ANY = "*"
APPARMOR_CONTAINER_PREFIX = "container.apparmor.security.beta.kubernetes.io/"
APPARMOR_DEFAULT_PROFILE = "apparmor.security.beta.kubernetes.io/defaultProfileName"
APPARMOR_ALLOWED_PROFILES = "apparmor.security.beta.kubernetes.io/allowedProfileNames"
SYSCTLS_POD_ANNOTATION = "security.alpha.kubernetes.io/sysctls"
UNSAFE_SYSCTLS_POD_ANNOTATION = "security.alpha.kubernetes.io/unsafe-sysctls"
SYSCTLS_PSP_ANNOTATION = "security.alpha.kubernetes.io/sysctls"
VALIDATED_PSP_ANNOTATION = "kubernetes.io/psp"
ALLOW_ALL_CAPABILITIES = "*"

FS_TYPES = ("hostPath", "azureFile", "flocker", "flexVolume", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore",
            "gitRepo", "secret", "nfs", "iscsi", "glusterfs", "persistentVolumeClaim", "rbd", "cinder", "cephFS",
            "downwardAPI", "fc", "configMap", "vsphereVolume", "quobyte", "azureDisk", "photonPersistentDisk",
            "storageos", "projected", "portworxVolume", "scaleIO", "csi")
# the pod volume source key for each fs type (GetVolumeFSType: csi has no inline source in 1.9)
_VOLUME_KEYS = (("hostPath", "hostPath"), ("emptyDir", "emptyDir"), ("gcePersistentDisk", "gcePersistentDisk"),
                ("awsElasticBlockStore", "awsElasticBlockStore"), ("gitRepo", "gitRepo"), ("secret", "secret"),
                ("nfs", "nfs"), ("iscsi", "iscsi"), ("glusterfs", "glusterfs"),
                ("persistentVolumeClaim", "persistentVolumeClaim"), ("rbd", "rbd"), ("flexVolume", "flexVolume"),
                ("cinder", "cinder"), ("cephfs", "cephFS"), ("flocker", "flocker"), ("downwardAPI", "downwardAPI"),
                ("fc", "fc"), ("azureFile", "azureFile"), ("configMap", "configMap"),
                ("vsphereVolume", "vsphereVolume"), ("quobyte", "quobyte"), ("azureDisk", "azureDisk"),
                ("photonPersistentDisk", "photonPersistentDisk"), ("storageos", "storageos"),
                ("projected", "projected"), ("portworxVolume", "portworxVolume"), ("scaleIO", "scaleIO"))


def _key(path: str, key: str) -> str:
    return f"{path}[{key}]"


def _child(path: str, name: str) -> str:
    return f"{path}.{name}" if path else name


# ============================================================================ util
def volume_fs_type(v: dict) -> str:
    for key, fs in _VOLUME_KEYS:
        if v.get(key) is not None:
            return fs
    raise ValueError(f"unknown volume type for volume: {v!r}")


def psp_allows_fs_type(psp, fs: str) -> bool:
    return any(x in (fs, "*") for x in (psp.get("spec") or {}).get("volumes") or [])


def has_path_prefix(s: str, prefix: str) -> bool:
    """hasPathPrefix: a prefix in path segments ("/foo" covers "/foo/bar", not "/foobar")."""
    s, prefix = _trim(s), _trim(prefix)
    if not s.startswith(prefix):
        return False
    return len(s) == len(prefix) or s[len(prefix):len(prefix) + 1] == "/"


def _trim(x: str) -> str:
    return x[:-1] if x.endswith("/") else x


def allows_host_volume_path(psp, host_path: str) -> bool:
    allowed = (psp.get("spec") or {}).get("allowedHostPaths") or []
    if not allowed:
        return True
    return any(has_path_prefix(host_path, a.get("pathPrefix", "")) for a in allowed)


def _in(v, rng) -> bool:
    return int(rng.get("min", 0)) <= v <= int(rng.get("max", 0))


def sysctls_from_annotation(value: str):
    """SysctlsFromPodAnnotation: `name=value,...`."""
    if not value:
        return []
    out = []
    for kv in value.split(","):
        cs = kv.split("=")
        if len(cs) != 2 or not cs[0]:
            raise ValueError(f'sysctl "{kv}" not of the format sysctl_name=value')
        out.append((cs[0], cs[1]))
    return out


# ============================================================================ strategies
class UserMustRunAs:
    def __init__(self, opts):
        if not (opts or {}).get("ranges"):
            raise ValueError("MustRunAsRange requires at least one range")
        self.ranges = opts["ranges"]

    def generate(self, pod, container):
        return int(self.ranges[0].get("min", 0))

    def validate(self, path, pod, container, run_as_non_root, run_as_user):
        if run_as_user is None:
            return [required(_child(path, "runAsUser"))]
        if not any(_in(run_as_user, r) for r in self.ranges):
            return [invalid(_child(path, "runAsUser"), run_as_user, f"must be in the ranges: {_ranges_str(self.ranges)}")]
        return []


def _ranges_str(ranges) -> str:
    return "[" + " ".join("{%d %d}" % (int(r.get("min", 0)), int(r.get("max", 0))) for r in ranges) + "]"


class UserNonRoot:
    def generate(self, pod, container):
        return None

    def validate(self, path, pod, container, run_as_non_root, run_as_user):
        if run_as_non_root is None and run_as_user is None:
            return [required(_child(path, "runAsNonRoot"), "must be true")]
        if run_as_non_root is False:
            return [invalid(_child(path, "runAsNonRoot"), False, "must be true")]
        if run_as_user == 0:
            return [invalid(_child(path, "runAsUser"), 0, "running with the root UID is forbidden")]
        return []


class UserRunAsAny:
    def generate(self, pod, container):
        return None

    def validate(self, path, pod, container, run_as_non_root, run_as_user):
        return []


class GroupMustRunAs:
    def __init__(self, ranges, field):
        if not ranges:
            raise ValueError("ranges must be supplied for MustRunAs")
        self.ranges, self.field = ranges, field

    def generate(self, pod):
        return [int(self.ranges[0].get("min", 0))]

    def generate_single(self, pod):
        return int(self.ranges[0].get("min", 0))

    def validate(self, pod, groups):
        errs = []
        if not groups:
            errs.append(invalid(self.field, go_slice("int64", groups), "unable to validate empty groups against required ranges"))
        for g in groups or []:
            if not any(_in(g, r) for r in self.ranges):
                errs.append(invalid(self.field, go_slice("int64", groups), f"{g} is not an allowed group"))
        return errs


class GroupRunAsAny:
    def generate(self, pod):
        return None

    def generate_single(self, pod):
        return None

    def validate(self, pod, groups):
        return []


class SELinuxMustRunAs:
    def __init__(self, opts):
        if (opts or {}).get("seLinuxOptions") is None:
            raise ValueError("MustRunAs requires SELinuxOptions")
        self.options = opts["seLinuxOptions"]

    def generate(self, pod, container):
        return dict(self.options)

    def validate(self, path, pod, container, options):
        if options is None:
            return [required(path)]
        errs = []
        for k in ("level", "role", "type", "user"):
            want = self.options.get(k, "")
            if options.get(k, "") != want:
                errs.append(invalid(_child(path, k), options.get(k, ""), f"must be {want}"))
        return errs


class SELinuxRunAsAny:
    def generate(self, pod, container):
        return None

    def validate(self, path, pod, container, options):
        return []


class AppArmorStrategy:
    def __init__(self, psp_annotations: dict):
        allowed = psp_annotations.get(APPARMOR_ALLOWED_PROFILES)
        self.allowed = None if allowed is None else set(allowed.split(","))
        self.allowed_str = allowed or ""
        self.default = psp_annotations.get(APPARMOR_DEFAULT_PROFILE, "")

    def generate(self, annotations, container):
        out = dict(annotations) if annotations is not None else None
        name = container.get("name", "")
        if (annotations or {}).get(APPARMOR_CONTAINER_PREFIX + name):
            return out
        if not self.default:
            return out
        out = out if out is not None else {}
        out[APPARMOR_CONTAINER_PREFIX + name] = self.default
        return out

    def validate(self, pod, container):
        if self.allowed is None:
            return []
        name = container.get("name", "")
        path = _key("pod.metadata.annotations", APPARMOR_CONTAINER_PREFIX + name)
        profile = _annotations(pod).get(APPARMOR_CONTAINER_PREFIX + name, "")
        if not profile:
            return [forbidden(path, "AppArmor profile must be set")] if self.allowed else []
        if profile not in self.allowed:
            return [forbidden(path, f'{profile} is not an allowed profile. Allowed values: "{self.allowed_str}"')]
        return []


def _annotations(pod) -> dict:
    return (pod.get("metadata") or {}).get("annotations") or {}


class SeccompStrategy:
    def __init__(self, psp_annotations: dict):
        self.allow_any = False
        self.allowed = None
        self.allowed_str = psp_annotations.get(SECCOMP_ALLOWED_PROFILES, "")
        if SECCOMP_ALLOWED_PROFILES in psp_annotations:
            self.allowed = set()
            for p in psp_annotations[SECCOMP_ALLOWED_PROFILES].split(","):
                if p == SECCOMP_ALLOW_ANY:
                    self.allow_any = True
                    continue
                self.allowed.add(p)
        self.default = psp_annotations.get(SECCOMP_DEFAULT_PROFILE, "")

    def generate(self, annotations, pod) -> str:
        if (annotations or {}).get(SECCOMP_POD_ANNOTATION):
            return annotations[SECCOMP_POD_ANNOTATION]
        return self.default

    def _allowed(self, profile: str) -> bool:
        if not self.allowed and profile == "":
            return True
        return self.allow_any or profile in (self.allowed or ())

    def _check(self, path, profile):
        if not self.allow_any and not self.allowed and profile != "":
            return [forbidden(path, "seccomp may not be set")]
        if not self._allowed(profile):
            return [forbidden(path, f"{profile} is not an allowed seccomp profile. Valid values are {self.allowed_str}")]
        return []

    def validate_pod(self, pod):
        return self._check(_key("pod.metadata.annotations", SECCOMP_POD_ANNOTATION),
                           _annotations(pod).get(SECCOMP_POD_ANNOTATION, ""))

    def validate_container(self, pod, container):
        name = container.get("name", "")
        ann = _annotations(pod)
        profile = ann[SECCOMP_CONTAINER_PREFIX + name] if SECCOMP_CONTAINER_PREFIX + name in ann else \
            ann.get(SECCOMP_POD_ANNOTATION, "")
        return self._check(_key("pod.metadata.annotations", SECCOMP_CONTAINER_PREFIX + name), profile)


class Capabilities:
    def __init__(self, default_add, required_drop, allowed):
        self.default_add, self.required_drop, self.allowed = list(default_add or []), list(required_drop or []), \
            list(allowed or [])

    def generate(self, pod, container):
        caps = ((container.get("securityContext") or {}).get("capabilities"))
        c_add = set((caps or {}).get("add") or [])
        c_drop = set((caps or {}).get("drop") or [])
        default_add = set(self.default_add) - c_drop
        combined_add = default_add | c_add
        combined_drop = set(self.required_drop) | c_drop
        if len(combined_add) == len(c_add) and len(combined_drop) == len(c_drop):
            return caps
        out = {}
        if combined_add:
            out["add"] = sorted(combined_add)
        if combined_drop:
            out["drop"] = sorted(combined_drop)
        return out

    def validate(self, pod, container, caps):
        if caps is None:
            if not self.default_add and not self.required_drop:
                return []
            return [invalid("capabilities", None, "required capabilities are not set on the securityContext")]
        if ALLOW_ALL_CAPABILITIES in self.allowed:
            return []
        errs = []
        for c in caps.get("add") or []:
            if c not in self.default_add and c not in self.allowed:
                errs.append(invalid("capabilities.add", c, "capability may not be added"))
        drops = set(caps.get("drop") or [])
        for d in self.required_drop:
            if d not in drops:
                errs.append(invalid("capabilities.drop", go_slice("core.Capability", caps.get("drop")),
                                    f"{d} is required to be dropped but was not found"))
        return errs


class SysctlMustMatchPatterns:
    def __init__(self, patterns):
        self.patterns = ["*"] if patterns is None else list(patterns)

    def validate(self, pod):
        return self._validate(pod, SYSCTLS_POD_ANNOTATION) + self._validate(pod, UNSAFE_SYSCTLS_POD_ANNOTATION)

    def _validate(self, pod, key):
        path = _key("pod.metadata.annotations", key)
        value = _annotations(pod).get(key, "")
        errs = []
        try:
            sysctls = sysctls_from_annotation(value)
        except ValueError as e:
            return [invalid(path, value, str(e))]
        if sysctls:
            if not self.patterns:
                errs.append(invalid(path, value, "sysctls are not allowed"))
            else:
                for i, (name, _) in enumerate(sysctls):
                    errs += self.validate_sysctl(name, f"{path}[{i}]")
        return errs

    def validate_sysctl(self, name: str, path: str):
        for p in self.patterns:
            if p.endswith("*"):
                if name.startswith(p[:-1]):
                    return []
            elif name == p:
                return []
        return [forbidden(path, f'sysctl "{name}" is not allowed')]


def create_strategies(psp: dict) -> dict:
    """StrategyFactory.CreateStrategies: every misconfiguration is collected."""
    spec = psp.get("spec") or {}
    ann = (psp.get("metadata") or {}).get("annotations") or {}
    errs, out = [], {}
    ru = spec.get("runAsUser") or {}
    try:
        out["user"] = {"MustRunAs": lambda: UserMustRunAs(ru), "MustRunAsNonRoot": UserNonRoot,
                       "RunAsAny": UserRunAsAny}[ru.get("rule")]()
    except KeyError:
        errs.append(f"Unrecognized RunAsUser strategy type {ru.get('rule', '')}")
    except ValueError as e:
        errs.append(str(e))
    se = spec.get("seLinux") or {}
    try:
        out["selinux"] = {"MustRunAs": lambda: SELinuxMustRunAs(se), "RunAsAny": SELinuxRunAsAny}[se.get("rule")]()
    except KeyError:
        errs.append(f"Unrecognized SELinuxContext strategy type {se.get('rule', '')}")
    except ValueError as e:
        errs.append(str(e))
    out["apparmor"] = AppArmorStrategy(ann)
    out["seccomp"] = SeccompStrategy(ann)
    for key, field, label in (("fsGroup", "fsGroup", "FSGroup"), ("supplementalGroups", "supplementalGroups",
                                                                   "SupplementalGroups")):
        g = spec.get(key) or {}
        try:
            out[key] = {"MustRunAs": lambda: GroupMustRunAs(g.get("ranges"), field),
                        "RunAsAny": GroupRunAsAny}[g.get("rule")]()
        except KeyError:
            errs.append(f"Unrecognized {label} strategy type {g.get('rule', '')}")
        except ValueError as e:
            errs.append(str(e))
    out["capabilities"] = Capabilities(spec.get("defaultAddCapabilities"), spec.get("requiredDropCapabilities"),
                                       spec.get("allowedCapabilities"))
    patterns = None
    if SYSCTLS_PSP_ANNOTATION in ann:
        patterns = ann[SYSCTLS_PSP_ANNOTATION].split(",") if ann[SYSCTLS_PSP_ANNOTATION] else []
    out["sysctls"] = SysctlMustMatchPatterns(patterns)
    if errs:
        raise ValueError("[" + ", ".join(errs) + "]" if len(errs) > 1 else errs[0])
    return out


# ============================================================================ security context access
def _set(d: dict | None, key: str, v):
    """The wrappers' setters: no struct is allocated to hold a nil."""
    if d is None:
        if v is None:
            return None
        d = {}
    if v is None:
        d.pop(key, None)
    else:
        d[key] = v
    return d


class Provider:
    """provider.go simpleProvider."""

    def __init__(self, psp: dict, namespace: str = ""):
        if psp is None:
            raise ValueError("NewSimpleProvider requires a PodSecurityPolicy")
        self.psp, self.spec, self.name = psp, psp.get("spec") or {}, (psp.get("metadata") or {}).get("name", "")
        self.s = create_strategies(psp)

    @property
    def allow_escalation(self) -> bool:
        """The API defaults allowPrivilegeEscalation to true (extensions/v1beta1 defaults.go)."""
        return bool(self.spec.get("allowPrivilegeEscalation", True))

    # ------------------------------------------------------------------ create
    def create_pod_security_context(self, pod: dict):
        spec = pod.get("spec") or {}
        psc = copy.deepcopy(spec.get("securityContext"))
        annotations = dict(_annotations(pod)) if (pod.get("metadata") or {}).get("annotations") is not None else None
        if (psc or {}).get("supplementalGroups") is None:
            sg = self.s["supplementalGroups"].generate(pod)
            # SetSupplementalGroups: nothing allocated, nothing replaced, for an empty value
            if sg or (psc is not None and psc.get("supplementalGroups")):
                psc = _set(psc, "supplementalGroups", sg or None)
        if (psc or {}).get("fsGroup") is None:
            psc = _set(psc, "fsGroup", self.s["fsGroup"].generate_single(pod))
        if (psc or {}).get("seLinuxOptions") is None:
            psc = _set(psc, "seLinuxOptions", self.s["selinux"].generate(pod, None))
        profile = self.s["seccomp"].generate(annotations, pod)
        if profile:
            annotations = annotations if annotations is not None else {}
            annotations[SECCOMP_POD_ANNOTATION] = profile
        return psc, annotations

    def create_container_security_context(self, pod: dict, container: dict):
        psc = (pod.get("spec") or {}).get("securityContext") or {}
        sc = copy.deepcopy(container.get("securityContext"))
        annotations = dict(_annotations(pod)) if (pod.get("metadata") or {}).get("annotations") is not None else None

        def eff(k):
            v = (sc or {}).get(k)
            return v if v is not None else psc.get(k)

        def set_eff(k, v):                 # the effective mutator: only a value that differs lands
            nonlocal sc
            if eff(k) != v:
                sc = _set(sc, k, v)

        def set_own(k, v):
            nonlocal sc
            if (sc or {}).get(k) != v:
                sc = _set(sc, k, v)

        if eff("runAsUser") is None:
            set_eff("runAsUser", self.s["user"].generate(pod, container))
        if eff("seLinuxOptions") is None:
            set_eff("seLinuxOptions", self.s["selinux"].generate(pod, container))
        annotations = self.s["apparmor"].generate(annotations, container)
        if eff("runAsNonRoot") is None and eff("runAsUser") is None and \
                (self.spec.get("runAsUser") or {}).get("rule") == "MustRunAsNonRoot":
            set_eff("runAsNonRoot", True)
        set_own("capabilities", self.s["capabilities"].generate(pod, dict(container, securityContext=sc)))
        if self.spec.get("readOnlyRootFilesystem") and (sc or {}).get("readOnlyRootFilesystem") is None:
            set_own("readOnlyRootFilesystem", True)
        if self.spec.get("defaultAllowPrivilegeEscalation") is not None and \
                (sc or {}).get("allowPrivilegeEscalation") is None:
            set_own("allowPrivilegeEscalation", bool(self.spec["defaultAllowPrivilegeEscalation"]))
        if not self.allow_escalation and (sc or {}).get("allowPrivilegeEscalation") is None:
            set_own("allowPrivilegeEscalation", False)
        return sc, annotations

    # ------------------------------------------------------------------ validate
    def validate_pod_security_context(self, pod: dict, path: str = "spec.securityContext") -> list:
        spec = pod.get("spec") or {}
        psc = spec.get("securityContext") or {}
        errs = []
        fs = [psc["fsGroup"]] if psc.get("fsGroup") is not None else []
        errs += self.s["fsGroup"].validate(pod, fs)
        errs += self.s["supplementalGroups"].validate(pod, psc.get("supplementalGroups") or [])
        errs += self.s["seccomp"].validate_pod(pod)
        errs += self.s["selinux"].validate(f"{path}.seLinuxOptions", pod, None, psc.get("seLinuxOptions"))
        for k, what in (("hostNetwork", "Host network"), ("hostPID", "Host PID"), ("hostIPC", "Host IPC")):
            if not self.spec.get(k) and spec.get(k):      # v1 keeps the host namespaces on the pod spec
                errs.append(invalid(f"{path}.{k}", True, f"{what} is not allowed to be used"))
        errs += self.s["sysctls"].validate(pod)
        if spec.get("volumes"):
            allow_all = psp_allows_fs_type(self.psp, "*")
            allowed = set(self.spec.get("volumes") or [])
            for i, v in enumerate(spec["volumes"]):
                try:
                    fs = volume_fs_type(v)
                except ValueError as e:
                    errs.append(invalid(f"spec.volumes[{i}]", "", str(e)))
                    continue
                if not allow_all and fs not in allowed:
                    errs.append(invalid(f"spec.volumes[{i}]", fs, f"{fs} volumes are not allowed to be used"))
                    continue
                if fs == "hostPath" and not allows_host_volume_path(self.psp, (v.get("hostPath") or {}).get("path", "")):
                    errs.append(invalid(f"spec.volumes[{i}].hostPath.pathPrefix",
                                        (v.get("hostPath") or {}).get("path", ""), "is not allowed to be used"))
                if fs == "flexVolume" and self.spec.get("allowedFlexVolumes"):
                    driver = (v.get("flexVolume") or {}).get("driver", "")
                    if driver not in [f.get("driver") for f in self.spec["allowedFlexVolumes"]]:
                        errs.append(invalid(f"{path}.volumes[{i}].driver", driver,
                                            "Flexvolume driver is not allowed to be used"))
        return errs

    def validate_container_security_context(self, pod: dict, container: dict, path: str) -> list:
        spec = pod.get("spec") or {}
        psc = spec.get("securityContext") or {}
        sc = container.get("securityContext") or {}

        def eff(k):
            v = sc.get(k)
            return v if v is not None else psc.get(k)
        errs = []
        errs += self.s["user"].validate(f"{path}.securityContext", pod, container, eff("runAsNonRoot"), eff("runAsUser"))
        errs += self.s["selinux"].validate(f"{path}.seLinuxOptions", pod, container, eff("seLinuxOptions"))
        errs += self.s["apparmor"].validate(pod, container)
        errs += self.s["seccomp"].validate_container(pod, container)
        if not self.spec.get("privileged") and sc.get("privileged"):
            errs.append(invalid(f"{path}.privileged", True, "Privileged containers are not allowed"))
        errs += self.s["capabilities"].validate(pod, container, sc.get("capabilities"))
        if not self.spec.get("hostNetwork") and spec.get("hostNetwork"):
            errs.append(invalid(f"{path}.hostNetwork", True, "Host network is not allowed to be used"))
        for kind in ("containers", "initContainers"):
            for idx, c in enumerate(spec.get(kind) or []):
                errs += self._invalid_host_ports(c, f"{path}.{kind}[{idx}]")
        if not self.spec.get("hostPID") and spec.get("hostPID"):
            errs.append(invalid(f"{path}.hostPID", True, "Host PID is not allowed to be used"))
        if not self.spec.get("hostIPC") and spec.get("hostIPC"):
            errs.append(invalid(f"{path}.hostIPC", True, "Host IPC is not allowed to be used"))
        if self.spec.get("readOnlyRootFilesystem"):
            ro = sc.get("readOnlyRootFilesystem")
            if ro is None:
                errs.append(invalid(f"{path}.readOnlyRootFilesystem", None,
                                    "ReadOnlyRootFilesystem may not be nil and must be set to true"))
            elif not ro:
                errs.append(invalid(f"{path}.readOnlyRootFilesystem", False, "ReadOnlyRootFilesystem must be set to true"))
        esc = sc.get("allowPrivilegeEscalation")
        if not self.allow_escalation and (esc is None or esc):
            errs.append(invalid(f"{path}.allowPrivilegeEscalation", esc,
                                "Allowing privilege escalation for containers is not allowed"))
        return errs

    def _invalid_host_ports(self, c, path):
        errs = []
        for p in c.get("ports") or []:
            hp = int(p.get("hostPort") or 0)
            if hp > 0 and not any(int(r.get("min", 0)) <= hp <= int(r.get("max", 0)) for r in self.spec.get("hostPorts") or []):
                errs.append(invalid(f"{path}.hostPort", hp, f"Host port {hp} is not allowed to be used. Allowed ports: "
                                                           f"[{host_port_ranges_to_string(self.spec.get('hostPorts'))}]"))
        return errs


def host_port_ranges_to_string(ranges) -> str:
    out = []
    for r in ranges or []:
        lo, hi = int(r.get("min", 0)), int(r.get("max", 0))
        out.append(str(lo) if lo == hi else f"{lo}-{hi}")
    return ",".join(out)


# ============================================================================ admission
def assign_security_context(provider: Provider, pod: dict) -> list:
    """assignSecurityContext: default then validate the pod and each (init) container in place."""
    errs = []
    spec = pod.setdefault("spec", {})
    md = pod.setdefault("metadata", {})
    try:
        psc, ann = provider.create_pod_security_context(pod)
    except Exception as e:                                # noqa: BLE001
        errs.append(invalid("spec.securityContext", spec.get("securityContext"), str(e)))
        psc, ann = spec.get("securityContext"), md.get("annotations")
    _put(spec, "securityContext", psc)
    _put(md, "annotations", ann)
    errs += provider.validate_pod_security_context(pod, "spec.securityContext")
    for kind in ("initContainers", "containers"):
        for i, c in enumerate(spec.get(kind) or []):
            path = f"spec.{kind}[{i}].securityContext"
            try:
                sc, ann = provider.create_container_security_context(pod, c)
            except Exception as e:                        # noqa: BLE001
                errs.append(invalid(path, "", str(e)))
                continue
            _put(c, "securityContext", sc)
            _put(md, "annotations", ann)
            errs += provider.validate_container_security_context(pod, c, path)
    return errs


def _put(d: dict, k: str, v):
    if v is None:
        d.pop(k, None)
    else:
        d[k] = v


def compute_security_context(policies: list, pod: dict, authorized, mutation_allowed: bool,
                             fail_on_no_policies: bool = True):
    """computeSecurityContext -> (pod to admit | None, policy name, errors). `authorized(name)`
    tells whether the requester or the pod's service account may `use` the policy."""
    if not policies and not fail_on_no_policies:
        return pod, "", []
    providers = []
    for p in sorted(policies, key=lambda x: (x.get("metadata") or {}).get("name", "")):
        try:
            providers.append(Provider(p, (pod.get("metadata") or {}).get("namespace", "")))
        except ValueError:
            continue                                      # a misconfigured policy offers nothing
    if not providers:
        raise PermissionError("no providers available to validate pod request")
    mutated_pod, mutated_name = None, ""
    validation_errs: dict[str, list] = {}
    for pr in providers:
        cand = copy.deepcopy(pod)
        errs = assign_security_context(pr, cand)
        if errs:
            validation_errs[pr.name] = errs
            continue
        mutated = not _semantic_equal(pod, cand)
        if mutated and not mutation_allowed:
            continue
        if not authorized(pr.name):
            continue
        if not mutated:
            return cand, pr.name, []
        if mutation_allowed and mutated_pod is None:
            mutated_pod, mutated_name = cand, pr.name
    if mutated_pod is not None:
        return mutated_pod, mutated_name, []
    agg = []
    for name, errs in validation_errs.items():
        if authorized(name):
            agg += errs
    return None, "", agg


def _semantic_equal(a, b) -> bool:
    return _norm(a) == _norm(b)


_MAP_KEYS = {"annotations", "labels", "nodeSelector"}


def _norm(v, key=None):
    """apiequality.Semantic: nil and empty slices alike, nil and empty maps alike (a nil
    struct pointer still differs from an empty struct)."""
    if isinstance(v, dict):
        out = {}
        for k, x in v.items():
            if x is None or x == []:
                continue
            if x == {} and k in _MAP_KEYS:
                continue
            out[k] = _norm(x, k)
        return out
    if isinstance(v, list):
        return [_norm(x) for x in v]
    return v
