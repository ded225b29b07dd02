"""PodSecurityPolicy held to the reference's tests.

Transcribed, cited by file (pkg/security/podsecuritypolicy/ and
plugin/pkg/admission/security/podsecuritypolicy/):
* user/{mustrunas,nonroot,runasany}_test.go, group/{mustrunas,runasany}_test.go,
  selinux/{mustrunas,runasany}_test.go, capabilities/mustrunas_test.go (every table, exact
  error strings), apparmor/strategy_test.go, seccomp/strategy_test.go,
  sysctl/mustmatchpatterns_test.go, util/util_test.go (PSPAllowsFSType, AllowsHostVolumePath,
  the volume-source drift check over amdkube's volume keys).
* provider_test.go — Create*SecurityContextNonmutating, Validate{Pod,Container}SecurityContext
  {Failures,Success}, GenerateContainerSecurityContextReadOnlyRootFS, ValidateAllowedVolumes,
  Validate(Default)AllowPrivilegeEscalation.
* admission_test.go — TestAdmitSeccomp, Privileged, PreferNonmutating, Caps (containers and init
  containers), Volumes, HostNetwork, HostPorts, HostPID, HostIPC, SELinux, AppArmor, RunAsUser,
  SupplementalGroups, FSGroup, ReadOnlyRootFilesystem, Sysctls, AssignSecurityContext,
  CreateProvidersFromConstraints, PolicyAuthorization, PolicyAuthorizationErrors.
The reference's tests build internal-API pods (host namespaces inside the pod security context);
here pods are v1 JSON, so hostNetwork / hostPID / hostIPC sit on the pod spec. Its fixture
policies are unconverted internal structs, so `allowPrivilegeEscalation` absent there means
false; here it is spelled out (the API itself defaults it to true, api/defaults.py).
"""
from __future__ import annotations

import copy
import json

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import admission_ext as X
from amdkube.apiserver.admission import CREATE, UPDATE, Attributes
from amdkube.security import psp as P

CONTAINER = "test-c"


def _c(o):
    return json.loads(json.dumps(o))


# ------------------------------------------------------------------ user
def test_user_must_run_as_options():
    for opts, ok in ((None, False), ({}, False), ({"ranges": [{"min": 1, "max": 1}]}, True)):
        if ok:
            P.UserMustRunAs(opts)
        else:
            with pytest.raises(ValueError):
                P.UserMustRunAs(opts)


def test_user_must_run_as_generate_and_validate():
    s = P.UserMustRunAs({"ranges": [{"min": 1, "max": 1}]})
    assert s.generate(None, None) == 1
    s = P.UserMustRunAs({"ranges": [{"min": 1, "max": 1}, {"min": 10, "max": 20}]})
    assert s.validate("", None, None, None, 15) == []
    errs = s.validate("", None, None, None, None)
    assert len(errs) == 1 and "runAsUser: Required" in str(errs[0])
    errs = s.validate("", None, None, None, 21)
    assert len(errs) == 1 and "runAsUser: Invalid" in str(errs[0])


@pytest.mark.parametrize("non_root,uid,err", [
    (None, 0, True), (None, 1, False), (False, None, True), (True, 1, False), (None, None, True),
])
def test_user_non_root(non_root, uid, err):
    s = P.UserNonRoot()
    assert s.generate(None, None) is None
    assert bool(s.validate("", None, None, non_root, uid)) == err


def test_user_run_as_any():
    s = P.UserRunAsAny()
    assert s.generate(None, None) is None and s.validate("", None, None, None, 0) == []


# ------------------------------------------------------------------ group
def test_group_must_run_as_options():
    with pytest.raises(ValueError):
        P.GroupMustRunAs([], "")
    P.GroupMustRunAs([{"min": 1, "max": 1}], "")


@pytest.mark.parametrize("ranges", [[{"min": 1, "max": 2}], [{"min": 1, "max": 1}], [{"min": 1, "max": 1}, {"min": 2, "max": 500}]])
def test_group_generate(ranges):
    s = P.GroupMustRunAs(ranges, "")
    assert s.generate(None) == [1] and s.generate_single(None) == 1


@pytest.mark.parametrize("ranges,groups,ok", [
    ([{"min": 1, "max": 3}], None, False), ([{"min": 1, "max": 3}], [], False),
    ([{"min": 1, "max": 3}, {"min": 4, "max": 4}], [5], False), ([{"min": 1, "max": 3}], [2], True),
    ([{"min": 1, "max": 3}], [1], True), ([{"min": 1, "max": 3}], [3], True), ([{"min": 4, "max": 4}], [4], True),
])
def test_group_validate(ranges, groups, ok):
    assert (P.GroupMustRunAs(ranges, "").validate(None, groups) == []) == ok


def test_group_run_as_any():
    s = P.GroupRunAsAny()
    assert s.generate(None) is None and s.generate_single(None) is None and s.validate(None, [1]) == []


# ------------------------------------------------------------------ selinux
def test_selinux_must_run_as():
    with pytest.raises(ValueError):
        P.SELinuxMustRunAs({})
    P.SELinuxMustRunAs({"seLinuxOptions": {}})
    opts = {"user": "user", "role": "role", "type": "type", "level": "level"}
    s = P.SELinuxMustRunAs({"seLinuxOptions": opts})
    assert s.generate(None, None) == opts
    for k in ("role", "user", "level", "type"):
        bad = dict(opts, **{k: "invalid"})
        errs = s.validate("", None, None, bad)
        assert len(errs) == 1 and f"{k}: Invalid value" in str(errs[0])
    assert s.validate("", None, None, dict(opts)) == []


def test_selinux_run_as_any():
    s = P.SELinuxRunAsAny()
    assert s.generate(None, None) is None and s.validate("", None, None, {"user": "x"}) == []


# ------------------------------------------------------------------ capabilities
def _cap_container(caps):
    return {"securityContext": {"capabilities": caps}}


@pytest.mark.parametrize("default_add,container_caps,expected", [
    (None, None, None),
    (None, {}, {}),
    (["foo"], None, {"add": ["foo"]}),
    (["foo"], {"add": ["foo"]}, {"add": ["foo"]}),
    (["foo", "bar", "baz"], {"add": ["foo"]}, {"add": ["bar", "baz", "foo"]}),
    (["foo"], {"add": ["bar"]}, {"add": ["bar", "foo"]}),
    (["foo", "bar"], {"add": ["foo", "foo", "bar", "baz"]}, {"add": ["foo", "foo", "bar", "baz"]}),
    (["foo", "bar"], {"add": ["foo", "baz"]}, {"add": ["bar", "baz", "foo"]}),
    (["foo"], {"add": ["FOO"]}, {"add": ["FOO", "foo"]}),
], ids=["no required, no container requests", "no required, no container requests, non-nil",
        "required, no container requests", "required, container requests add required",
        "multiple required, container requests add required", "required, container requests add non-required",
        "generation does not mutate unnecessarily", "generation dedupes", "generation is case sensitive"])
def test_capabilities_generate_adds(default_add, container_caps, expected):
    assert P.Capabilities(default_add, None, None).generate(None, _cap_container(container_caps)) == expected


@pytest.mark.parametrize("default_add,required_drop,container_caps,expected", [
    (None, None, None, None),
    (None, None, {}, {}),
    (None, ["foo"], None, {"drop": ["foo"]}),
    (None, ["baz"], {"drop": ["foo", "bar"]}, {"drop": ["bar", "baz", "foo"]}),
    (None, ["baz"], {"drop": ["foo", "bar", "baz"]}, {"drop": ["foo", "bar", "baz"]}),
    (["foo"], None, {"drop": ["foo"]}, {"drop": ["foo"]}),
    (["foo"], None, {"drop": ["bar"]}, {"add": ["foo"], "drop": ["bar"]}),
    (["foo", "bar", "baz"], ["abc"], {"drop": ["foo"]}, {"add": ["bar", "baz"], "drop": ["abc", "foo"]}),
    (None, ["baz", "foo"], {"drop": ["bar", "foo"]}, {"drop": ["bar", "baz", "foo"]}),
    (None, ["bar"], {"drop": ["BAR"]}, {"drop": ["BAR", "bar"]}),
])
def test_capabilities_generate_drops(default_add, required_drop, container_caps, expected):
    assert P.Capabilities(default_add, required_drop, None).generate(None, _cap_container(container_caps)) == expected


@pytest.mark.parametrize("default_add,allowed,caps,expected", [
    (None, None, None, ""),
    (None, ["foo"], None, ""),
    (["foo"], None, None, 'capabilities: Invalid value: "null": required capabilities are not set on the securityContext'),
    (["foo"], None, {"add": ["foo"]}, ""),
    (["foo"], None, {"add": ["bar"]}, 'capabilities.add: Invalid value: "bar": capability may not be added'),
    (None, ["foo"], {"add": ["foo"]}, ""),
    (None, ["*"], {"add": ["foo"]}, ""),
    (None, ["foo"], {"add": ["bar"]}, 'capabilities.add: Invalid value: "bar": capability may not be added'),
    (["foo"], ["bar"], {"add": ["foo"]}, ""),
    (["foo"], ["bar"], {"add": ["bar"]}, ""),
    (["foo"], ["bar"], {"add": ["baz"]}, 'capabilities.add: Invalid value: "baz": capability may not be added'),
    (["foo"], None, {"add": ["FOO"]}, 'capabilities.add: Invalid value: "FOO": capability may not be added'),
])
def test_capabilities_validate_adds(default_add, allowed, caps, expected):
    errs = P.Capabilities(default_add, None, allowed).validate(None, None, caps)
    assert [str(e) for e in errs] == ([expected] if expected else [])


@pytest.mark.parametrize("required_drop,caps,expected", [
    (None, None, ""),
    (["foo"], None, 'capabilities: Invalid value: "null": required capabilities are not set on the securityContext'),
    (["foo"], {"drop": ["foo"]}, ""),
    (["foo"], {"drop": ["bar"]},
     'capabilities.drop: Invalid value: []core.Capability{"bar"}: foo is required to be dropped but was not found'),
    (["foo"], {"drop": ["FOO"]},
     'capabilities.drop: Invalid value: []core.Capability{"FOO"}: foo is required to be dropped but was not found'),
])
def test_capabilities_validate_drops(required_drop, caps, expected):
    errs = P.Capabilities(None, required_drop, None).validate(None, None, caps)
    assert [str(e) for e in errs] == ([expected] if expected else [])


# ------------------------------------------------------------------ apparmor
AA_KEY = P.APPARMOR_CONTAINER_PREFIX + CONTAINER
WITHOUT_AA = {"foo": "bar"}
WITH_DEFAULT = {"foo": "bar", AA_KEY: "runtime/default"}
WITH_LOCAL = {"foo": "bar", AA_KEY: "localhost/foo"}
WITH_DISALLOWED = {"foo": "bar", AA_KEY: "localhost/bad"}
NO_AA = {"foo": "bar"}
UNCONSTRAINED_DEFAULT = {P.APPARMOR_DEFAULT_PROFILE: "runtime/default"}
CONSTRAINED = {P.APPARMOR_ALLOWED_PROFILES: "runtime/default,localhost/foo"}
CONSTRAINED_DEFAULT = {P.APPARMOR_DEFAULT_PROFILE: "runtime/default",
                       P.APPARMOR_ALLOWED_PROFILES: "runtime/default,localhost/foo"}
AA_PSPS = [NO_AA, UNCONSTRAINED_DEFAULT, CONSTRAINED, CONSTRAINED_DEFAULT]


def _aa_generate_cases():
    cases = [(NO_AA, WITHOUT_AA, WITHOUT_AA), (UNCONSTRAINED_DEFAULT, WITHOUT_AA, WITH_DEFAULT),
             (CONSTRAINED, WITHOUT_AA, WITHOUT_AA), (CONSTRAINED_DEFAULT, WITHOUT_AA, WITH_DEFAULT)]
    cases += [(psp, pod, pod) for pod in (WITH_DEFAULT, WITH_LOCAL) for psp in AA_PSPS]
    return cases


@pytest.mark.parametrize("psp_ann,pod_ann,expected", _aa_generate_cases())
def test_apparmor_generate(psp_ann, pod_ann, expected):
    assert P.AppArmorStrategy(psp_ann).generate(pod_ann, {"name": CONTAINER, "image": "busybox"}) == expected


def _aa_validate_cases():
    cases = [(psp, pod, False) for pod in (WITH_DEFAULT, WITH_LOCAL) for psp in AA_PSPS]
    cases += [(psp, pod, False) for pod in (WITHOUT_AA, WITH_DISALLOWED) for psp in (NO_AA, UNCONSTRAINED_DEFAULT)]
    cases += [(psp, pod, True) for pod in (WITHOUT_AA, WITH_DISALLOWED) for psp in (CONSTRAINED, CONSTRAINED_DEFAULT)]
    return cases


@pytest.mark.parametrize("psp_ann,pod_ann,err", _aa_validate_cases())
def test_apparmor_validate(psp_ann, pod_ann, err):
    c = {"name": CONTAINER, "image": "busybox"}
    pod = {"metadata": {"name": "test-pod", "annotations": dict(pod_ann)}, "spec": {"containers": [c]}}
    assert len(P.AppArmorStrategy(psp_ann).validate(pod, c)) == (1 if err else 0)


# ------------------------------------------------------------------ seccomp
WITHOUT_SECCOMP = {"foo": "bar"}
ALLOW_ANY_NO_DEFAULT = {P.SECCOMP_ALLOWED_PROFILES: "*"}
ALLOW_ANY_DEFAULT = {P.SECCOMP_ALLOWED_PROFILES: "*", P.SECCOMP_DEFAULT_PROFILE: "foo"}
ALLOW_ANY_AND_SPECIFIC_DEFAULT = {P.SECCOMP_ALLOWED_PROFILES: "*,bar", P.SECCOMP_DEFAULT_PROFILE: "foo"}
ALLOW_SPECIFIC = {P.SECCOMP_ALLOWED_PROFILES: "foo"}


@pytest.mark.parametrize("ann,allow_any,allowed_str,allowed,default", [
    (WITHOUT_SECCOMP, False, "", None, ""), (ALLOW_ANY_NO_DEFAULT, True, "*", set(), ""),
    (ALLOW_ANY_DEFAULT, True, "*", set(), "foo"), (ALLOW_ANY_AND_SPECIFIC_DEFAULT, True, "*,bar", {"bar"}, "foo"),
])
def test_seccomp_new_strategy(ann, allow_any, allowed_str, allowed, default):
    s = P.SeccompStrategy(ann)
    assert (s.allow_any, s.allowed_str, s.allowed, s.default) == (allow_any, allowed_str, allowed, default)


@pytest.mark.parametrize("psp_ann,pod_ann,expected", [
    (WITHOUT_SECCOMP, None, ""), (WITHOUT_SECCOMP, {P.SECCOMP_POD_ANNOTATION: "foo"}, "foo"),
    (ALLOW_ANY_NO_DEFAULT, None, ""), (ALLOW_ANY_NO_DEFAULT, {P.SECCOMP_POD_ANNOTATION: "foo"}, "foo"),
    (ALLOW_ANY_DEFAULT, None, "foo"), (ALLOW_ANY_DEFAULT, {P.SECCOMP_POD_ANNOTATION: "bar"}, "bar"),
])
def test_seccomp_generate(psp_ann, pod_ann, expected):
    assert P.SeccompStrategy(psp_ann).generate(pod_ann, None) == expected


@pytest.mark.parametrize("psp_ann,pod_ann,expected", [
    (ALLOW_SPECIFIC, None, "Forbidden:  is not an allowed seccomp profile. Valid values are foo"),
    (WITHOUT_SECCOMP, None, ""),
    (ALLOW_SPECIFIC, {P.SECCOMP_POD_ANNOTATION: "foo"}, ""),
    (ALLOW_SPECIFIC, {P.SECCOMP_POD_ANNOTATION: "bar"}, "Forbidden: bar is not an allowed seccomp profile. Valid values are foo"),
    (WITHOUT_SECCOMP, {P.SECCOMP_POD_ANNOTATION: "foo"}, "Forbidden: seccomp may not be set"),
    (ALLOW_ANY_NO_DEFAULT, {P.SECCOMP_POD_ANNOTATION: "foo"}, ""),
    (ALLOW_ANY_NO_DEFAULT, None, ""),
])
def test_seccomp_validate_pod(psp_ann, pod_ann, expected):
    errs = P.SeccompStrategy(psp_ann).validate_pod({"metadata": {"annotations": pod_ann}})
    assert len(errs) == (1 if expected else 0)
    if expected:
        assert expected in str(errs[0])


SC_CKEY = P.SECCOMP_CONTAINER_PREFIX + "container"


@pytest.mark.parametrize("psp_ann,pod_ann,expected", [
    (ALLOW_SPECIFIC, None, "Forbidden:  is not an allowed seccomp profile. Valid values are foo"),
    (WITHOUT_SECCOMP, None, ""),
    (ALLOW_SPECIFIC, {SC_CKEY: "foo"}, ""),
    (ALLOW_SPECIFIC, {SC_CKEY: "bar"}, "Forbidden: bar is not an allowed seccomp profile. Valid values are foo"),
    (WITHOUT_SECCOMP, {SC_CKEY: "foo"}, "Forbidden: seccomp may not be set"),
    (ALLOW_ANY_NO_DEFAULT, {SC_CKEY: "foo"}, ""),
    (ALLOW_ANY_NO_DEFAULT, None, ""),
    (ALLOW_SPECIFIC, {P.SECCOMP_POD_ANNOTATION: "foo"}, ""),
    (ALLOW_SPECIFIC, {P.SECCOMP_POD_ANNOTATION: "bar"}, "Forbidden: bar is not an allowed seccomp profile. Valid values are foo"),
])
def test_seccomp_validate_container(psp_ann, pod_ann, expected):
    errs = P.SeccompStrategy(psp_ann).validate_container({"metadata": {"annotations": pod_ann}}, {"name": "container"})
    assert len(errs) == (1 if expected else 0)
    if expected:
        assert expected in str(errs[0])


# ------------------------------------------------------------------ sysctl
@pytest.mark.parametrize("patterns,allowed,disallowed", [
    (None, ["foo"], []), ([], [], ["foo"]), (["a", "a.b"], ["a", "a.b"], ["b"]), (["*"], ["a", "a.b"], []),
    (["a.b.c", "*"], ["a", "a.b", "a.b.c", "b"], []),
    (["a.*", "b.*", "c.d.e", "d.e.f.*"], ["a.b", "b.c", "c.d.e", "d.e.f.g.h"], ["a", "b", "c", "c.d", "d.e", "d.e.f"]),
], ids=["nil", "empty", "without wildcard", "with catch-all wildcard", "with catch-all wildcard and non-wildcard",
        "without catch-all wildcard"])
def test_sysctl_must_match_patterns(patterns, allowed, disallowed):
    s = P.SysctlMustMatchPatterns(patterns)
    assert s.validate({"metadata": {}}) == []
    for key in (P.SYSCTLS_POD_ANNOTATION, P.UNSAFE_SYSCTLS_POD_ANNOTATION):
        pod = {"metadata": {"annotations": {key: ",".join(f"{n}=dummy" for n in allowed)}}}
        assert s.validate(pod) == []
        for n in disallowed:
            assert s.validate({"metadata": {"annotations": {key: f"{n}=dummy"}}})


# ------------------------------------------------------------------ util
VOLUME_SOURCES = ["hostPath", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "secret", "nfs", "iscsi",
                  "glusterfs", "persistentVolumeClaim", "rbd", "flexVolume", "cinder", "cephfs", "flocker", "downwardAPI",
                  "fc", "azureFile", "configMap", "vsphereVolume", "quobyte", "azureDisk", "photonPersistentDisk",
                  "projected", "portworxVolume", "scaleIO", "storageos"]


@pytest.mark.parametrize("source", VOLUME_SOURCES)
def test_volume_source_fs_type_drift(source):
    assert P.volume_fs_type({"name": "v", source: {}}) in P.FS_TYPES


@pytest.mark.parametrize("psp,fs,allows", [
    ({}, "hostPath", False), ({"spec": {"volumes": ["awsElasticBlockStore"]}}, "hostPath", False),
    ({"spec": {"volumes": ["*"]}}, "hostPath", True), ({"spec": {"volumes": ["hostPath"]}}, "hostPath", True),
])
def test_psp_allows_fs_type(psp, fs, allows):
    assert P.psp_allows_fs_type(psp, fs) == allows


def _hp(prefix):
    return {"spec": {"allowedHostPaths": [{"pathPrefix": prefix}]}}


@pytest.mark.parametrize("psp,path,allows", [
    ({}, "/test", True), (_hp("/foo"), "/foobar", False), (_hp("/foo"), "/foo", True), (_hp("/foo"), "/foo/", True),
    (_hp("/foo/"), "/foo", True), (_hp("/foo/"), "/foo/bar", True), (_hp("/foo/bar"), "/foo", False),
], ids=["empty allowed paths", "non-matching", "direct match", "trailing slash on host path",
        "trailing slash on allowed path", "child directory", "non-matching parent directory"])
def test_allows_host_volume_path(psp, path, allows):
    assert P.allows_host_volume_path(psp, path) == allows


# ------------------------------------------------------------------ provider_test.go
def default_psp(**spec):
    s = {"runAsUser": {"rule": "RunAsAny"}, "seLinux": {"rule": "RunAsAny"}, "fsGroup": {"rule": "RunAsAny"},
         "supplementalGroups": {"rule": "RunAsAny"}, "allowPrivilegeEscalation": True}
    s.update(spec)
    return {"metadata": {"name": "psp-sa", "annotations": {}}, "spec": s}


def default_pod():
    return {"metadata": {"annotations": {}},
            "spec": {"securityContext": {}, "containers": [{"name": CONTAINER, "securityContext": {"privileged": False}}]}}


def test_create_pod_security_context_nonmutating():
    pod, psp = {"spec": {"securityContext": {}}}, default_psp()
    psp["metadata"]["annotations"] = {P.SECCOMP_ALLOWED_PROFILES: "*"}
    before_pod, before_psp = _c(pod), _c(psp)
    P.Provider(psp, "namespace").create_pod_security_context(pod)
    assert pod == before_pod and psp == before_psp


@pytest.mark.parametrize("sc", [None, {"runAsNonRoot": False}])
def test_create_container_security_context_nonmutating(sc):
    pod = {"spec": {"containers": [{} if sc is None else {"securityContext": sc}]}}
    psp = default_psp()
    psp["metadata"]["annotations"] = {P.SECCOMP_ALLOWED_PROFILES: "*", P.SECCOMP_DEFAULT_PROFILE: "foo"}
    before_pod, before_psp = _c(pod), _c(psp)
    P.Provider(psp, "namespace").create_container_security_context(pod, pod["spec"]["containers"][0])
    assert pod == before_pod and psp == before_psp


def _with(pod, fn):
    fn(pod)
    return pod


def _flex_psp(allow_all_flex, allow_all_volumes):
    return default_psp(allowedFlexVolumes=[] if allow_all_flex else [{"driver": "example/foo"}, {"driver": "example/bar"}],
                       volumes=["*" if allow_all_volumes else "flexVolume"])


SG_PSP = default_psp(supplementalGroups={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]})
FS_PSP = default_psp(fsGroup={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]})
SEL_PSP = default_psp(seLinux={"rule": "MustRunAs", "seLinuxOptions": {"level": "foo"}})
NO_SYSCTL_PSP = _with(default_psp(), lambda p: p["metadata"]["annotations"].__setitem__(P.SYSCTLS_PSP_ANNOTATION, ""))
OTHER_SYSCTL_PSP = _with(default_psp(), lambda p: p["metadata"]["annotations"].__setitem__(P.SYSCTLS_PSP_ANNOTATION, "bar,abc"))
SAFE_FOO = _with(default_pod(), lambda p: p["metadata"]["annotations"].__setitem__(P.SYSCTLS_POD_ANNOTATION, "foo=1"))
UNSAFE_FOO = _with(default_pod(), lambda p: p["metadata"]["annotations"].__setitem__(P.UNSAFE_SYSCTLS_POD_ANNOTATION, "foo=1"))
FLEX_POD = _with(default_pod(), lambda p: p["spec"].__setitem__(
    "volumes", [{"name": "flex-volume", "flexVolume": {"driver": "example/unknown"}}]))

POD_FAILURES = {
    "failHostNetwork": (_with(default_pod(), lambda p: p["spec"].__setitem__("hostNetwork", True)), default_psp(),
                        "Host network is not allowed to be used"),
    "failHostPID": (_with(default_pod(), lambda p: p["spec"].__setitem__("hostPID", True)), default_psp(),
                    "Host PID is not allowed to be used"),
    "failHostIPC": (_with(default_pod(), lambda p: p["spec"].__setitem__("hostIPC", True)), default_psp(),
                    "Host IPC is not allowed to be used"),
    "failSupplementalGroupOutOfRange": (_with(default_pod(), lambda p: p["spec"]["securityContext"].__setitem__(
        "supplementalGroups", [999])), SG_PSP, "999 is not an allowed group"),
    "failSupplementalGroupEmpty": (default_pod(), SG_PSP, "unable to validate empty groups against required ranges"),
    "failFSGroupOutOfRange": (_with(default_pod(), lambda p: p["spec"]["securityContext"].__setitem__("fsGroup", 999)),
                              FS_PSP, "999 is not an allowed group"),
    "failFSGroupEmpty": (default_pod(), FS_PSP, "unable to validate empty groups against required ranges"),
    "failNilSELinux": (default_pod(), SEL_PSP, "seLinuxOptions: Required"),
    "failInvalidSELinux": (_with(default_pod(), lambda p: p["spec"]["securityContext"].__setitem__(
        "seLinuxOptions", {"level": "bar"})), SEL_PSP, "seLinuxOptions.level: Invalid value"),
    "failHostDirPSP": (_with(default_pod(), lambda p: p["spec"].__setitem__("volumes", [{"name": "bad volume", "hostPath": {}}])),
                       default_psp(), "hostPath volumes are not allowed to be used"),
    "failHostPathDirPSP": (_with(default_pod(), lambda p: p["spec"].__setitem__(
        "volumes", [{"name": "bad volume", "hostPath": {"path": "/fail"}}])),
        default_psp(volumes=["hostPath"], allowedHostPaths=[{"pathPrefix": "/foo/bar"}]), "is not allowed to be used"),
    "failSafeSysctlFooPod with failNoSysctlAllowedSCC": (SAFE_FOO, NO_SYSCTL_PSP, "sysctls are not allowed"),
    "failUnsafeSysctlFooPod with failNoSysctlAllowedSCC": (UNSAFE_FOO, NO_SYSCTL_PSP, "sysctls are not allowed"),
    "failSafeSysctlFooPod with failOtherSysctlsAllowedSCC": (SAFE_FOO, OTHER_SYSCTL_PSP, 'sysctl "foo" is not allowed'),
    "failUnsafeSysctlFooPod with failOtherSysctlsAllowedSCC": (UNSAFE_FOO, OTHER_SYSCTL_PSP, 'sysctl "foo" is not allowed'),
    "failInvalidSeccomp": (_with(default_pod(), lambda p: p["metadata"].__setitem__(
        "annotations", {P.SECCOMP_POD_ANNOTATION: "foo"})), default_psp(), "Forbidden: seccomp may not be set"),
    "fail pod with disallowed flexVolume when flex volumes are allowed": (FLEX_POD, _flex_psp(False, False),
                                                                         "Flexvolume driver is not allowed to be used"),
    "fail pod with disallowed flexVolume when all volumes are allowed": (FLEX_POD, _flex_psp(False, True),
                                                                        "Flexvolume driver is not allowed to be used"),
}


@pytest.mark.parametrize("name", list(POD_FAILURES))
def test_validate_pod_security_context_failures(name):
    pod, psp, expected = POD_FAILURES[name]
    errs = P.Provider(_c(psp), "namespace").validate_pod_security_context(_c(pod), "")
    assert errs and expected in str(errs[0]), errs


def _csc(p, **kv):
    p["spec"]["containers"][0]["securityContext"].update(kv)
    return p


AA_PSP = _with(default_psp(), lambda p: p["metadata"].__setitem__(
    "annotations", {P.APPARMOR_ALLOWED_PROFILES: "runtime/default"}))
RO_PSP = default_psp(readOnlyRootFilesystem=True)

CONTAINER_FAILURES = {
    "failUserPSP": (_csc(default_pod(), runAsUser=1), default_psp(runAsUser={"rule": "MustRunAs", "ranges": [{"min": 999, "max": 999}]}),
                    "runAsUser: Invalid value"),
    "failSELinuxPSP": (_csc(default_pod(), seLinuxOptions={"level": "bar"}), SEL_PSP, "seLinuxOptions.level: Invalid value"),
    "failNilAppArmor": (default_pod(), AA_PSP, "AppArmor profile must be set"),
    "failInvalidAppArmor": (_with(default_pod(), lambda p: p["metadata"]["annotations"].__setitem__(
        P.APPARMOR_CONTAINER_PREFIX + CONTAINER, "localhost/foo")), AA_PSP,
        'localhost/foo is not an allowed profile. Allowed values: "runtime/default"'),
    "failPrivPSP": (_csc(default_pod(), privileged=True), default_psp(), "Privileged containers are not allowed"),
    "failCapsPSP": (_csc(default_pod(), capabilities={"add": ["foo"]}), default_psp(), "capability may not be added"),
    "failHostPortPSP": (_with(default_pod(), lambda p: p["spec"]["containers"][0].__setitem__("ports", [{"hostPort": 1}])),
                        default_psp(), "Host port 1 is not allowed to be used. Allowed ports: []"),
    "failReadOnlyRootFS - nil": (default_pod(), RO_PSP, "ReadOnlyRootFilesystem may not be nil and must be set to true"),
    "failReadOnlyRootFS - false": (_csc(default_pod(), readOnlyRootFilesystem=False), RO_PSP,
                                   "ReadOnlyRootFilesystem must be set to true"),
    "failSeccompContainerAnnotation": (_with(default_pod(), lambda p: p["metadata"].__setitem__(
        "annotations", {P.SECCOMP_CONTAINER_PREFIX + CONTAINER: "foo"})), default_psp(), "Forbidden: seccomp may not be set"),
    "failSeccompContainerPodAnnotation": (_with(default_pod(), lambda p: p["metadata"].__setitem__(
        "annotations", {P.SECCOMP_POD_ANNOTATION: "foo"})), default_psp(), "Forbidden: seccomp may not be set"),
}


@pytest.mark.parametrize("name", list(CONTAINER_FAILURES))
def test_validate_container_security_context_failures(name):
    pod, psp, expected = CONTAINER_FAILURES[name]
    pod = _c(pod)
    errs = P.Provider(_c(psp), "namespace").validate_container_security_context(pod, pod["spec"]["containers"][0], "")
    assert errs and expected in str(errs[0]), errs


SEL_OPTS = {"user": "user", "role": "role", "type": "type", "level": "level"}
POD_SUCCESSES = {
    "pass hostNetwork validating PSP": (_with(default_pod(), lambda p: p["spec"].__setitem__("hostNetwork", True)),
                                        default_psp(hostNetwork=True)),
    "pass hostPID validating PSP": (_with(default_pod(), lambda p: p["spec"].__setitem__("hostPID", True)), default_psp(hostPID=True)),
    "pass hostIPC validating PSP": (_with(default_pod(), lambda p: p["spec"].__setitem__("hostIPC", True)), default_psp(hostIPC=True)),
    "pass supplemental group validating PSP": (_with(default_pod(), lambda p: p["spec"]["securityContext"].__setitem__(
        "supplementalGroups", [3])), default_psp(supplementalGroups={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 5}]})),
    "pass fs group validating PSP": (_with(default_pod(), lambda p: p["spec"]["securityContext"].__setitem__("fsGroup", 3)),
                                     default_psp(fsGroup={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 5}]})),
    "pass selinux validating PSP": (_with(default_pod(), lambda p: p["spec"]["securityContext"].__setitem__(
        "seLinuxOptions", dict(SEL_OPTS))), default_psp(seLinux={"rule": "MustRunAs", "seLinuxOptions": dict(SEL_OPTS)})),
    "pass sysctl specific profile with safe sysctl": (SAFE_FOO, _with(default_psp(), lambda p: p["metadata"]["annotations"].__setitem__(
        P.SYSCTLS_PSP_ANNOTATION, "foo"))),
    "pass sysctl specific profile with unsafe sysctl": (UNSAFE_FOO, _with(default_psp(), lambda p: p["metadata"]["annotations"].__setitem__(
        P.SYSCTLS_PSP_ANNOTATION, "foo"))),
    "pass empty profile with safe sysctl": (SAFE_FOO, default_psp()),
    "pass empty profile with unsafe sysctl": (UNSAFE_FOO, default_psp()),
    "pass hostDir allowed directory validating PSP": (
        _with(default_pod(), lambda p: p["spec"].__setitem__("volumes", [{"name": "good volume", "hostPath": {"path": "/foo/bar/baz"}}])),
        default_psp(volumes=["hostPath"], allowedHostPaths=[{"pathPrefix": "/foo/bar"}])),
    "pass hostDir all volumes allowed validating PSP": (
        _with(default_pod(), lambda p: p["spec"].__setitem__("volumes", [{"name": "good volume", "hostPath": {"path": "/foo/bar/baz"}}])),
        default_psp(volumes=["*"], allowedHostPaths=[{"pathPrefix": "/foo/bar"}])),
    "pass seccomp validating PSP": (_with(default_pod(), lambda p: p["metadata"].__setitem__(
        "annotations", {P.SECCOMP_POD_ANNOTATION: "foo"})), _with(default_psp(), lambda p: p["metadata"].__setitem__(
            "annotations", {P.SECCOMP_ALLOWED_PROFILES: "foo"}))),
}
_FLEX_OK = _with(default_pod(), lambda p: p["spec"].__setitem__("volumes", [{"name": "flex-volume", "flexVolume": {"driver": "example/bar"}}]))
for _a, _b in ((False, True), (True, True), (False, False), (True, False)):
    POD_SUCCESSES[f"flex volume driver allowFlex={_a} allowAll={_b}"] = (_FLEX_OK, _flex_psp(_a, _b))


@pytest.mark.parametrize("name", list(POD_SUCCESSES))
def test_validate_pod_security_context_success(name):
    pod, psp = POD_SUCCESSES[name]
    assert P.Provider(_c(psp), "namespace").validate_pod_security_context(_c(pod), "") == []


CONTAINER_SUCCESSES = {
    "pass user must run as PSP": (_csc(default_pod(), runAsUser=999),
                                  default_psp(runAsUser={"rule": "MustRunAs", "ranges": [{"min": 999, "max": 999}]})),
    "pass seLinux must run as PSP": (_csc(default_pod(), seLinuxOptions={"level": "foo"}), SEL_PSP),
    "pass AppArmor allowed profiles": (_with(default_pod(), lambda p: p["metadata"]["annotations"].__setitem__(
        P.APPARMOR_CONTAINER_PREFIX + CONTAINER, "runtime/default")), AA_PSP),
    "pass priv validating PSP": (_csc(default_pod(), privileged=True), default_psp(privileged=True)),
    "pass allowed caps validating PSP": (_csc(default_pod(), capabilities={"add": ["foo"]}), default_psp(allowedCapabilities=["foo"])),
    "pass required caps validating PSP": (_csc(default_pod(), capabilities={"add": ["foo"]}), default_psp(defaultAddCapabilities=["foo"])),
    "pass hostDir validating PSP": (_with(default_pod(), lambda p: p["spec"].__setitem__("volumes", [{"name": "bad volume", "hostPath": {}}])),
                                    default_psp(volumes=["hostPath"])),
    "pass hostPort validating PSP": (_with(default_pod(), lambda p: p["spec"]["containers"][0].__setitem__("ports", [{"hostPort": 1}])),
                                     default_psp(hostPorts=[{"min": 1, "max": 1}])),
    "pass read only root fs - nil": (default_pod(), default_psp()),
    "pass read only root fs - false": (_csc(default_pod(), readOnlyRootFilesystem=False), default_psp()),
    "pass read only root fs - true": (_csc(default_pod(), readOnlyRootFilesystem=True), default_psp()),
    "pass seccomp container annotation": (_with(default_pod(), lambda p: p["metadata"].__setitem__(
        "annotations", {P.SECCOMP_CONTAINER_PREFIX + CONTAINER: "foo"})), _with(default_psp(), lambda p: p["metadata"].__setitem__(
            "annotations", {P.SECCOMP_ALLOWED_PROFILES: "foo"}))),
    "pass seccomp inherit pod annotation": (_with(default_pod(), lambda p: p["metadata"].__setitem__(
        "annotations", {P.SECCOMP_POD_ANNOTATION: "foo"})), _with(default_psp(), lambda p: p["metadata"].__setitem__(
            "annotations", {P.SECCOMP_ALLOWED_PROFILES: "foo"}))),
}


@pytest.mark.parametrize("name", list(CONTAINER_SUCCESSES))
def test_validate_container_security_context_success(name):
    pod, psp = CONTAINER_SUCCESSES[name]
    pod = _c(pod)
    assert P.Provider(_c(psp), "namespace").validate_container_security_context(pod, pod["spec"]["containers"][0], "") == []


@pytest.mark.parametrize("psp_ro,pod_ro,expected", [
    (False, None, None), (False, False, False), (False, True, True), (True, None, True), (True, False, False), (True, True, True),
])
def test_generate_container_security_context_read_only_root_fs(psp_ro, pod_ro, expected):
    pod = default_pod() if pod_ro is None else _csc(default_pod(), readOnlyRootFilesystem=pod_ro)
    psp = default_psp(readOnlyRootFilesystem=psp_ro)
    sc, _ = P.Provider(psp, "namespace").create_container_security_context(pod, pod["spec"]["containers"][0])
    assert (sc or {}).get("readOnlyRootFilesystem") == expected


@pytest.mark.parametrize("source,fs", [(s, P.volume_fs_type({s: {}})) for s in VOLUME_SOURCES])
def test_validate_allowed_volumes(source, fs):
    pod = default_pod()
    pod["spec"]["volumes"] = [{source: {}}]
    psp = default_psp()
    provider = P.Provider(psp, "namespace")
    errs = provider.validate_pod_security_context(pod, "")
    assert len(errs) == 1 and f"{fs} volumes are not allowed to be used" in str(errs[0])
    psp["spec"]["volumes"] = [fs]
    assert provider.validate_pod_security_context(pod, "") == []
    psp["spec"]["volumes"] = ["*"]
    assert provider.validate_pod_security_context(pod, "") == []


def test_validate_allow_privilege_escalation():
    pod = _csc(default_pod(), allowPrivilegeEscalation=True)
    psp = default_psp(allowPrivilegeEscalation=False)
    provider = P.Provider(psp, "namespace")
    errs = provider.validate_container_security_context(pod, pod["spec"]["containers"][0], "")
    assert len(errs) == 1 and "Allowing privilege escalation for containers is not allowed" in str(errs[0])
    psp["spec"]["allowPrivilegeEscalation"] = True
    assert provider.validate_container_security_context(pod, pod["spec"]["containers"][0], "") == []


def test_validate_default_allow_privilege_escalation():
    pod = _csc(default_pod(), allowPrivilegeEscalation=True)
    psp = default_psp(defaultAllowPrivilegeEscalation=False, allowPrivilegeEscalation=False)
    provider = P.Provider(psp, "namespace")
    c = pod["spec"]["containers"][0]
    msg = "Allowing privilege escalation for containers is not allowed"
    errs = provider.validate_container_security_context(pod, c, "")
    assert len(errs) == 1 and msg in str(errs[0])
    psp["spec"]["defaultAllowPrivilegeEscalation"] = True
    errs = provider.validate_container_security_context(pod, c, "")
    assert len(errs) == 1 and msg in str(errs[0])
    psp["spec"]["allowPrivilegeEscalation"] = True
    assert provider.validate_container_security_context(pod, c, "") == []
    psp["spec"]["allowPrivilegeEscalation"] = False
    del c["securityContext"]["allowPrivilegeEscalation"]
    errs = provider.validate_container_security_context(pod, c, "")
    assert len(errs) == 1 and msg in str(errs[0])
    psp["spec"]["allowPrivilegeEscalation"] = True
    assert provider.validate_container_security_context(pod, c, "") == []


# ------------------------------------------------------------------ admission_test.go
def restrictive_psp(name="restrictive", **spec):
    s = {"runAsUser": {"rule": "MustRunAs", "ranges": [{"min": 999, "max": 999}]},
         "seLinux": {"rule": "MustRunAs", "seLinuxOptions": {"level": "s9:z0,z1"}},
         "fsGroup": {"rule": "MustRunAs", "ranges": [{"min": 999, "max": 999}]},
         "supplementalGroups": {"rule": "MustRunAs", "ranges": [{"min": 999, "max": 999}]},
         "allowPrivilegeEscalation": False}
    s.update(spec)
    return {"apiVersion": "extensions/v1beta1", "kind": "PodSecurityPolicy",
            "metadata": {"name": name, "annotations": {}}, "spec": s}


def permissive_psp(name="privileged", **spec):
    s = {"allowPrivilegeEscalation": True, "hostIPC": True, "hostNetwork": True, "hostPID": True,
         "hostPorts": [{"min": 0, "max": 65536}], "volumes": ["*"], "allowedCapabilities": ["*"],
         "runAsUser": {"rule": "RunAsAny"}, "seLinux": {"rule": "RunAsAny"}, "fsGroup": {"rule": "RunAsAny"},
         "supplementalGroups": {"rule": "RunAsAny"}}
    s.update(spec)
    return {"apiVersion": "extensions/v1beta1", "kind": "PodSecurityPolicy",
            "metadata": {"name": name, "annotations": {}}, "spec": s}


def good_pod():
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": "pod", "namespace": "namespace", "annotations": {}},
            "spec": {"serviceAccountName": "default", "securityContext": {},
                     "containers": [{"name": CONTAINER, "securityContext": {}}]}}


class Ctx:
    """The admission context: a PSP lister and the TestAuthorizer (user -> namespace -> PSPs;
    None allows everything)."""

    def __init__(self, psps, allowed=None):
        self.psps, self.allowed = psps, allowed

    def list_objects(self, plural, ns, group=""):
        return [_c(p) for p in self.psps] if plural == "podsecuritypolicies" else []

    def authorize(self, user, verb, group, resource, sub="", ns="", name=""):
        if self.allowed is None:
            return True
        by_ns = self.allowed.get((user or {}).get("name", ""), {})
        return bool(by_ns.get(ns, {}).get(name) or by_ns.get("", {}).get(name))


def admit_and_validate(psps, pod, should_admit, should_validate, expected_psp, op=CREATE, old=None, allowed=None,
                       user=None, can_mutate=True):
    plugin = X.PodSecurityPolicy()
    original = _c(pod)
    a = Attributes(op, "pods", "", m.namespace_of(pod), m.name_of(pod), pod, old,
                   {"name": "", "groups": []} if user is None else user)
    ctx = Ctx(psps, allowed)
    err = None
    try:
        plugin.admit(a, ctx)
    except m.StatusError as e:
        err = e
    assert (err is None) == should_admit, err
    if should_admit:
        assert ((pod.get("metadata") or {}).get("annotations") or {}).get(P.VALIDATED_PSP_ANNOTATION, "") == expected_psp
        if not can_mutate:
            assert P._semantic_equal(original["spec"], pod["spec"])
    err = None
    try:
        plugin.validate(a, ctx)
    except m.StatusError as e:
        err = e
    assert (err is None) == should_validate, err


SECCOMP_CASES = [
    (None, None, True), (None, {P.SECCOMP_POD_ANNOTATION: "foo"}, False), (None, {P.SECCOMP_CONTAINER_PREFIX + "container": "foo"}, False),
    ({P.SECCOMP_ALLOWED_PROFILES: "*"}, None, True), ({P.SECCOMP_ALLOWED_PROFILES: "*"}, {P.SECCOMP_POD_ANNOTATION: "foo"}, True),
    ({P.SECCOMP_ALLOWED_PROFILES: "*"}, {P.SECCOMP_CONTAINER_PREFIX + "container": "foo"}, True),
    ({P.SECCOMP_ALLOWED_PROFILES: "foo"}, {P.SECCOMP_POD_ANNOTATION: "bar"}, False),
    ({P.SECCOMP_DEFAULT_PROFILE: "foo", P.SECCOMP_ALLOWED_PROFILES: "foo"}, {P.SECCOMP_CONTAINER_PREFIX + "container": "bar"}, False),
    ({P.SECCOMP_ALLOWED_PROFILES: "foo"}, {P.SECCOMP_POD_ANNOTATION: "foo"}, True),
    ({P.SECCOMP_DEFAULT_PROFILE: "foo", P.SECCOMP_ALLOWED_PROFILES: "foo,bar"}, {P.SECCOMP_CONTAINER_PREFIX + "container": "bar"}, True),
]


@pytest.mark.parametrize("psp_ann,pod_ann,ok", SECCOMP_CASES)
def test_admit_seccomp(psp_ann, pod_ann, ok):
    psp = restrictive_psp()
    psp["metadata"]["annotations"] = psp_ann
    pod = {"metadata": {"annotations": pod_ann}, "spec": {"containers": [{"name": "container"}]}}
    admit_and_validate([psp], pod, ok, ok, psp["metadata"]["name"])


def _priv_pod(priv):
    p = good_pod()
    p["spec"]["containers"][0]["securityContext"]["privileged"] = priv
    return p


NON_PRIV, PRIV = restrictive_psp("non-priv", privileged=False), restrictive_psp("priv", privileged=True)


@pytest.mark.parametrize("pod,psps,ok,expected_priv,expected_psp", [
    (good_pod(), [NON_PRIV], True, None, "non-priv"), (good_pod(), [PRIV], True, None, "priv"),
    (_priv_pod(False), [NON_PRIV], True, False, "non-priv"), (_priv_pod(False), [PRIV], True, False, "priv"),
    (_priv_pod(True), [NON_PRIV], False, None, ""), (_priv_pod(True), [NON_PRIV, PRIV], True, True, "priv"),
])
def test_admit_privileged(pod, psps, ok, expected_priv, expected_psp):
    pod = _c(pod)
    admit_and_validate(psps, pod, ok, ok, expected_psp)
    if ok:
        assert pod["spec"]["containers"][0]["securityContext"].get("privileged") == expected_priv


def _unpriv_runasany_pod():
    """defaultPod(): the v1 defaults the reference applies to its test pod."""
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {},
            "spec": {"serviceAccountName": "default", "restartPolicy": "Always", "terminationGracePeriodSeconds": 30,
                     "dnsPolicy": "ClusterFirst", "securityContext": {}, "schedulerName": "default-scheduler",
                     "containers": [{"name": "mycontainer", "image": "myimage", "terminationMessagePath": "/dev/termination-log",
                                     "terminationMessagePolicy": "File", "imagePullPolicy": "Always"}]}}


def test_admit_prefer_nonmutating():
    mutating1 = restrictive_psp("mutating1", runAsUser={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]})
    mutating2 = restrictive_psp("mutating2", runAsUser={"rule": "MustRunAs", "ranges": [{"min": 2, "max": 2}]})
    privileged = permissive_psp("privileged")
    base = _unpriv_runasany_pod()
    changed = _c(base)
    changed["spec"]["containers"][0]["image"] = "myimage2"
    with_sc = _c(base)
    with_sc["metadata"]["annotations"] = {P.VALIDATED_PSP_ANNOTATION: "privileged"}
    changed_with_sc = _c(changed)
    changed_with_sc["metadata"]["annotations"] = {P.VALIDATED_PSP_ANNOTATION: "privileged"}
    gc_changed = _c(base)
    gc_changed["metadata"]["ownerReferences"] = [{"kind": "Foo", "name": "bar"}]
    gc_changed["metadata"]["finalizers"] = ["foo"]
    cases = [
        ("pod should not be mutated by allow-all strategies", CREATE, _c(base), None, [privileged], True, True, False,
         None, "privileged"),
        ("pod should prefer non-mutating PSP on create", CREATE, _c(base), None, [mutating2, mutating1, privileged],
         True, True, False, None, "privileged"),
        ("pod should use deterministic mutating PSP on create", CREATE, _c(base), None, [mutating2, mutating1],
         True, True, True, 1, "mutating1"),
        ("pod should prefer non-mutating PSP on update", UPDATE, _c(changed_with_sc), _c(with_sc),
         [mutating2, mutating1, privileged], True, True, False, None, "privileged"),
        ("pod should not mutate on update, but fail validation", UPDATE, _c(changed), _c(base), [mutating2, mutating1],
         True, False, False, None, ""),
        ("pod should be allowed if completely unchanged on update", UPDATE, _c(base), _c(base), [mutating2, mutating1],
         True, True, False, None, ""),
        ("pod should be allowed if unchanged on update except finalizers,ownerrefs", UPDATE, _c(gc_changed), _c(base),
         [mutating2, mutating1], True, True, False, None, ""),
    ]
    for name, op, pod, old, psps, admit_ok, validate_ok, mutation, container_user, expected in cases:
        admit_and_validate(psps, pod, admit_ok, validate_ok, expected, op=op, old=old, can_mutate=mutation)
        assert (pod["spec"].get("securityContext") or {}).get("runAsUser") is None, name
        assert (pod["spec"]["containers"][0].get("securityContext") or {}).get("runAsUser") == container_user, name


def _caps_pod(caps):
    p = good_pod()
    p["spec"]["containers"][0]["securityContext"]["capabilities"] = caps
    return p


RESTRICTED = restrictive_psp()
ALLOW_FOO = restrictive_psp("allowCapInAllowed", allowedCapabilities=["foo"])
REQUIRE_FOO = restrictive_psp("allowCapInRequired", defaultAddCapabilities=["foo"])
DROP_FOO = restrictive_psp("requireDrop", requiredDropCapabilities=["foo"])
ALLOW_ALL = restrictive_psp("allowAllCapsInAllowed", allowedCapabilities=["*"])
CAPS_CASES = {
    "should reject cap add when not allowed or required": (_caps_pod({"add": ["foo"]}), [RESTRICTED], False, None, ""),
    "should accept cap add when in allowed": (_caps_pod({"add": ["foo"]}), [RESTRICTED, ALLOW_FOO], True, None, "allowCapInAllowed"),
    "should accept cap add when in required": (_caps_pod({"add": ["foo"]}), [RESTRICTED, REQUIRE_FOO], True, None, "allowCapInRequired"),
    "should reject cap add when requested cap is required to be dropped": (_caps_pod({"add": ["foo"]}), [RESTRICTED, DROP_FOO], False, None, ""),
    "should accept cap drop when cap is required to be dropped": (_caps_pod({"drop": ["foo"]}), [DROP_FOO], True, None, "requireDrop"),
    "required add is defaulted": (good_pod(), [REQUIRE_FOO], True, {"add": ["foo"]}, "allowCapInRequired"),
    "required drop is defaulted": (good_pod(), [DROP_FOO], True, {"drop": ["foo"]}, "requireDrop"),
    "should accept cap add when all caps are allowed": (_caps_pod({"add": ["foo"]}), [RESTRICTED, ALLOW_ALL], True, None, "allowAllCapsInAllowed"),
}


def _use_init_containers(pod):
    pod["spec"]["initContainers"] = pod["spec"]["containers"]
    pod["spec"]["containers"] = []
    return pod


@pytest.mark.parametrize("init", [False, True], ids=["containers", "initContainers"])
@pytest.mark.parametrize("name", list(CAPS_CASES))
def test_admit_caps(name, init):
    pod, psps, ok, expected_caps, expected_psp = CAPS_CASES[name]
    pod = _c(pod)
    if init:
        _use_init_containers(pod)
    admit_and_validate(psps, pod, ok, ok, expected_psp)
    if expected_caps is not None:
        c = pod["spec"]["initContainers" if init else "containers"][0]
        assert c["securityContext"]["capabilities"] == expected_caps


@pytest.mark.parametrize("source", VOLUME_SOURCES)
def test_admit_volumes(source):
    fs = P.volume_fs_type({source: {}})
    pod = good_pod()
    pod["spec"]["volumes"] = [{"name": "v", source: {}}]
    psp = restrictive_psp()
    admit_and_validate([psp], _c(pod), False, False, "")
    _use_init_containers(pod)
    admit_and_validate([psp], _c(pod), False, False, "")
    psp["spec"]["volumes"] = [fs]
    admit_and_validate([psp], _c(pod), True, True, "restrictive")
    psp["spec"]["volumes"] = ["*"]
    admit_and_validate([psp], _c(pod), True, True, "restrictive")


def _host_pod(field, value):
    p = good_pod()
    p["spec"][field] = value
    return p


@pytest.mark.parametrize("field", ["hostNetwork", "hostPID", "hostIPC"])
@pytest.mark.parametrize("init", [False, True], ids=["containers", "initContainers"])
def test_admit_host_namespaces(field, init):
    deny, allow = restrictive_psp(f"no-{field}", **{field: False}), restrictive_psp(field, **{field: True})
    cases = [(good_pod(), [deny], True, False, deny), (good_pod(), [allow], True, False, allow),
             (_host_pod(field, True), [deny], False, None, None), (_host_pod(field, True), [deny, allow], True, True, allow)]
    for pod, psps, ok, expected, expected_psp in cases:
        pod = _c(pod)
        if init:
            _use_init_containers(pod)
        admit_and_validate(psps, pod, ok, ok, m.name_of(expected_psp) if expected_psp else "")
        if ok:
            assert bool(pod["spec"].get(field)) == expected


def _port_pod(port):
    p = good_pod()
    p["spec"]["containers"][0]["ports"] = [{"hostPort": port}]
    return p


@pytest.mark.parametrize("swap", [True, False], ids=["initContainers", "containers"])
@pytest.mark.parametrize("pod,psp,ok", [
    (_port_pod(11), restrictive_psp("hostPorts", hostPorts=[{"min": 1, "max": 10}]), False),
    (_port_pod(5), restrictive_psp("hostPorts", hostPorts=[{"min": 1, "max": 10}]), True),
    (good_pod(), restrictive_psp("hostPorts", hostPorts=[{"min": 1, "max": 10}]), True),
    (good_pod(), restrictive_psp("noHostPorts"), True),
    (_port_pod(5), restrictive_psp("noHostPorts"), False),
], ids=["host port out of range", "host port in range", "no host ports with range", "no host ports without range",
        "host ports without range"])
def test_admit_host_ports(pod, psp, ok, swap):
    pod = _c(pod)
    if swap:
        pod["spec"]["containers"], pod["spec"]["initContainers"] = [], pod["spec"]["containers"]
    admit_and_validate([psp], pod, ok, ok, m.name_of(psp) if ok else "")


def _sc_pod(pod_sc, container_sc):
    p = good_pod()
    if pod_sc is None:
        del p["spec"]["securityContext"]
    else:
        p["spec"]["securityContext"] = pod_sc
    if container_sc is None:
        del p["spec"]["containers"][0]["securityContext"]
    else:
        p["spec"]["containers"][0]["securityContext"] = container_sc
    return p


SEL = {"level": "level", "role": "role", "type": "type", "user": "user"}
RUN_AS_ANY_SEL = permissive_psp("runAsAny", seLinux={"rule": "RunAsAny"})
MUST_SEL = permissive_psp("mustRunAs", seLinux={"rule": "MustRunAs", "seLinuxOptions": dict(SEL)})


@pytest.mark.parametrize("pod_sc,c_sc,psp,ok,exp_pod,exp_c", [
    (None, None, RUN_AS_ANY_SEL, True, None, None),
    ({}, None, RUN_AS_ANY_SEL, True, {}, None),
    (None, {}, RUN_AS_ANY_SEL, True, None, {}),
    ({"seLinuxOptions": {"user": "foo"}}, None, RUN_AS_ANY_SEL, True, {"seLinuxOptions": {"user": "foo"}}, None),
    (None, {"seLinuxOptions": {"user": "foo"}}, RUN_AS_ANY_SEL, True, None, {"seLinuxOptions": {"user": "foo"}}),
    ({"seLinuxOptions": {"user": "bar"}}, {"seLinuxOptions": {"user": "foo"}}, RUN_AS_ANY_SEL, True,
     {"seLinuxOptions": {"user": "bar"}}, {"seLinuxOptions": {"user": "foo"}}),
    ({"seLinuxOptions": {"user": "foo"}}, None, MUST_SEL, False, None, None),
    (None, {"seLinuxOptions": {"user": "foo"}}, MUST_SEL, False, None, None),
    (None, None, MUST_SEL, True, {"seLinuxOptions": SEL}, None),
    ({"seLinuxOptions": dict(SEL)}, None, MUST_SEL, True, {"seLinuxOptions": SEL}, None),
], ids=["runAsAny with no request", "runAsAny with empty pod request", "runAsAny with empty container request",
        "runAsAny with pod request", "runAsAny with container request", "runAsAny with pod and container request",
        "mustRunAs with bad pod request", "mustRunAs with bad container request", "mustRunAs with no request",
        "mustRunAs with good pod request"])
def test_admit_selinux(pod_sc, c_sc, psp, ok, exp_pod, exp_c):
    pod = _sc_pod(_c(pod_sc), _c(c_sc))
    admit_and_validate([psp], pod, ok, ok, m.name_of(psp) if ok else "")
    if ok:
        assert pod["spec"].get("securityContext") == exp_pod
        assert pod["spec"]["containers"][0].get("securityContext") == exp_c


def _aa_pod(profile):
    p = good_pod()
    p["metadata"]["annotations"][P.APPARMOR_CONTAINER_PREFIX + CONTAINER] = profile
    return p


def _aa_psp(ann):
    p = restrictive_psp()
    p["metadata"]["annotations"] = ann
    return p


@pytest.mark.parametrize("pod,psp,ok,expected", [
    (good_pod(), _aa_psp({}), True, ""), (_aa_pod("runtime/default"), _aa_psp({}), True, "runtime/default"),
    (good_pod(), _aa_psp({P.APPARMOR_DEFAULT_PROFILE: "runtime/default"}), True, "runtime/default"),
    (good_pod(), _aa_psp({P.APPARMOR_ALLOWED_PROFILES: "runtime/default"}), False, None),
    (good_pod(), _aa_psp(CONSTRAINED_DEFAULT), True, "runtime/default"),
    (_aa_pod("localhost/foo"), _aa_psp(CONSTRAINED_DEFAULT), True, "localhost/foo"),
    (_aa_pod("localhost/bar"), _aa_psp({P.APPARMOR_ALLOWED_PROFILES: "runtime/default"}), False, None),
], ids=["unconstrained with no profile", "unconstrained with profile", "unconstrained with default profile",
        "AppArmor enforced with no profile", "AppArmor enforced with default profile", "AppArmor enforced with good profile",
        "AppArmor enforced with local profile"])
def test_admit_apparmor(pod, psp, ok, expected):
    pod = _c(pod)
    admit_and_validate([psp], pod, ok, ok, m.name_of(psp))
    if ok:
        assert pod["metadata"]["annotations"].get(P.APPARMOR_CONTAINER_PREFIX + CONTAINER, "") == expected


RUN_AS_ANY_U = permissive_psp("runAsAny")
MUST_U = permissive_psp("mustRunAs", runAsUser={"rule": "MustRunAs", "ranges": [{"min": 999, "max": 1000}]})
NON_ROOT_U = permissive_psp("runAsNonRoot", runAsUser={"rule": "MustRunAsNonRoot"})


def _u(uid):
    return {"runAsUser": uid}


@pytest.mark.parametrize("pod_sc,c_sc,psp,ok,exp_pod,exp_c", [
    (None, None, RUN_AS_ANY_U, True, None, None),
    (_u(1), None, RUN_AS_ANY_U, True, _u(1), None),
    (None, _u(1), RUN_AS_ANY_U, True, None, _u(1)),
    (_u(1), None, MUST_U, False, None, None),
    (_u(999), _u(1), MUST_U, False, None, None),
    (_u(999), None, MUST_U, True, _u(999), None),
    (None, _u(999), MUST_U, True, None, _u(999)),
    (_u(999), _u(1000), MUST_U, True, _u(999), _u(1000)),
    (None, None, MUST_U, True, None, _u(999)),
    (None, None, NON_ROOT_U, True, None, {"runAsNonRoot": True}),
    (_u(0), None, NON_ROOT_U, False, None, None),
    (_u(1), None, NON_ROOT_U, True, _u(1), None),
    (_u(1), _u(0), NON_ROOT_U, False, None, None),
    (_u(1), _u(2), NON_ROOT_U, True, _u(1), _u(2)),
], ids=["runAsAny no pod request", "runAsAny pod request", "runAsAny container request",
        "mustRunAs pod request out of range", "mustRunAs container request out of range", "mustRunAs pod request in range",
        "mustRunAs container request in range", "mustRunAs pod and container request in range", "mustRunAs no request",
        "runAsNonRoot no request", "runAsNonRoot pod request root", "runAsNonRoot pod request non-root",
        "runAsNonRoot container request root", "runAsNonRoot container request non-root"])
def test_admit_run_as_user(pod_sc, c_sc, psp, ok, exp_pod, exp_c):
    pod = _sc_pod(_c(pod_sc), _c(c_sc))
    admit_and_validate([psp], pod, ok, ok, m.name_of(psp) if ok else "")
    if ok:
        assert pod["spec"].get("securityContext") == exp_pod
        assert pod["spec"]["containers"][0].get("securityContext") == exp_c


RUN_AS_ANY_G = permissive_psp("runAsAny")
MUST_G = permissive_psp("mustRunAs", supplementalGroups={"rule": "MustRunAs", "ranges": [{"min": 999, "max": 1000}]})


@pytest.mark.parametrize("pod_sc,psp,ok,expected", [
    (None, RUN_AS_ANY_G, True, None), ({}, RUN_AS_ANY_G, True, {}),
    ({"supplementalGroups": []}, RUN_AS_ANY_G, True, {"supplementalGroups": []}),
    ({"supplementalGroups": [1]}, RUN_AS_ANY_G, True, {"supplementalGroups": [1]}),
    (None, MUST_G, True, {"supplementalGroups": [999]}), ({"supplementalGroups": [1]}, MUST_G, False, None),
    ({"supplementalGroups": [999]}, MUST_G, True, {"supplementalGroups": [999]}),
], ids=["runAsAny no pod request", "runAsAny empty pod request", "runAsAny empty pod request empty supplemental groups",
        "runAsAny pod request", "mustRunAs no pod request", "mustRunAs bad pod request", "mustRunAs good pod request"])
def test_admit_supplemental_groups(pod_sc, psp, ok, expected):
    pod = _sc_pod(_c(pod_sc), None)
    admit_and_validate([psp], pod, ok, ok, m.name_of(psp) if ok else "")
    if ok:
        assert pod["spec"].get("securityContext") == expected


def _fs_pod(group):
    p = good_pod()
    p["spec"]["securityContext"]["fsGroup"] = group
    return p


@pytest.mark.parametrize("pod,psp,ok,expected", [
    (good_pod(), restrictive_psp("runAsAny", fsGroup={"rule": "RunAsAny"}), True, None),
    (_fs_pod(1), restrictive_psp("runAsAny", fsGroup={"rule": "RunAsAny"}), True, 1),
    (good_pod(), restrictive_psp("mustRunAs"), True, 999),
    (_fs_pod(1), restrictive_psp("mustRunAs"), False, None),
    (_fs_pod(999), restrictive_psp("mustRunAs"), True, 999),
])
def test_admit_fs_group(pod, psp, ok, expected):
    pod = _c(pod)
    admit_and_validate([psp], pod, ok, ok, m.name_of(psp) if ok else "")
    if ok:
        assert pod["spec"]["securityContext"].get("fsGroup") == expected


def _ro_pod(ro):
    p = good_pod()
    p["spec"]["containers"][0]["securityContext"]["readOnlyRootFilesystem"] = ro
    return p


@pytest.mark.parametrize("pod,psp,ok,expected", [
    (_ro_pod(True), restrictive_psp("no-rorfs", readOnlyRootFilesystem=False), True, True),
    (_ro_pod(False), restrictive_psp("no-rorfs", readOnlyRootFilesystem=False), True, False),
    (_ro_pod(False), restrictive_psp("rorfs", readOnlyRootFilesystem=True), False, None),
    (good_pod(), restrictive_psp("rorfs", readOnlyRootFilesystem=True), True, True),
    (_ro_pod(True), restrictive_psp("rorfs", readOnlyRootFilesystem=True), True, True),
])
def test_admit_read_only_root_filesystem(pod, psp, ok, expected):
    pod = _c(pod)
    admit_and_validate([psp], pod, ok, ok, m.name_of(psp) if ok else "")
    if ok:
        assert pod["spec"]["containers"][0]["securityContext"].get("readOnlyRootFilesystem") is expected


def _sysctl_pod(safe, unsafe):
    p = good_pod()
    p["metadata"]["annotations"][P.SYSCTLS_POD_ANNOTATION] = ",".join(f"{n}=dummy" for n in safe)
    p["metadata"]["annotations"][P.UNSAFE_SYSCTLS_POD_ANNOTATION] = ",".join(f"{n}=dummy" for n in unsafe)
    return p


def _sysctl_psp(name, patterns):
    p = restrictive_psp(name)
    if patterns is not None:
        p["metadata"]["annotations"][P.SYSCTLS_PSP_ANNOTATION] = patterns
    return p


NO_S, EMPTY_S = _sysctl_psp("no sysctls", None), _sysctl_psp("empty sysctls", "")
MIXED_S = _sysctl_psp("wildcard sysctls", "a.*,b.*,c,d.e.f")
A_S, B_S, C_S = _sysctl_psp("a sysctl", "a"), _sysctl_psp("b sysctl", "b"), _sysctl_psp("c sysctl", "c")
ALL_S = _sysctl_psp("catchall sysctl", "*")


@pytest.mark.parametrize("pod,psps,expected", [
    (good_pod(), [NO_S], "no sysctls"), (good_pod(), [EMPTY_S], "empty sysctls"),
    (_sysctl_pod(["a", "b"], []), [NO_S], "no sysctls"), (_sysctl_pod([], ["a", "b"]), [NO_S], "no sysctls"),
    (_sysctl_pod(["a", "b"], []), [EMPTY_S], None), (_sysctl_pod([], ["a", "b"]), [A_S], None),
    (_sysctl_pod([], ["b"]), [A_S], None), (_sysctl_pod([], ["a"]), [A_S], "a sysctl"),
    (_sysctl_pod(["a", "b"], []), [A_S], None), (_sysctl_pod(["b"], []), [A_S], None),
    (_sysctl_pod(["a"], []), [A_S], "a sysctl"), (_sysctl_pod([], ["a", "b"]), [EMPTY_S], None),
    (_sysctl_pod(["a.b", "b.c"], ["c", "d.e.f"]), [MIXED_S], "wildcard sysctls"),
    (_sysctl_pod(["a.b", "b.c", "c", "d.e.f"], ["e"]), [MIXED_S], None),
    (_sysctl_pod(["a.b", "b.c", "c", "d.e.f", "e"], []), [MIXED_S], None),
    (_sysctl_pod(["e"], ["f"]), [ALL_S], "catchall sysctl"),
    (_sysctl_pod(["e"], ["f"]), [MIXED_S, ALL_S, EMPTY_S], "catchall sysctl"),
    (_sysctl_pod([], ["c"]), [A_S, B_S, C_S], "c sysctl"), (_sysctl_pod(["c"], []), [A_S, B_S, C_S], "c sysctl"),
])
def test_admit_sysctls(pod, psps, expected):
    pod = _c(pod)
    before = {k: v for k, v in pod["metadata"]["annotations"].items() if "sysctl" in k}
    admit_and_validate(psps, pod, expected is not None, expected is not None, expected or "")
    if expected is not None:
        assert {k: v for k, v in pod["metadata"]["annotations"].items() if "sysctl" in k} == before


@pytest.mark.parametrize("privs,ok", [([True], False), ([False, True], False), ([False], True)],
                         ids=["pod and container SC is not changed when invalid", "must validate all containers", "pod validates"])
def test_assign_security_context(privs, ok):
    provider = P.Provider(restrictive_psp(), "namespace")
    pod = {"spec": {"securityContext": {}, "containers": [{"securityContext": {"privileged": p}} for p in privs]}}
    assert (P.assign_security_context(provider, pod) == []) == ok


def test_create_providers_from_constraints():
    valid = {"metadata": {"name": "valid psp"}, "spec": {
        "seLinux": {"rule": "RunAsAny"}, "runAsUser": {"rule": "RunAsAny"}, "fsGroup": {"rule": "RunAsAny"},
        "supplementalGroups": {"rule": "RunAsAny"}}}
    bad = _c(valid)
    bad["metadata"]["name"] = "bad psp user options"
    bad["spec"]["runAsUser"] = {"rule": "MustRunAs"}
    before = _c(valid)
    P.Provider(valid)
    assert valid == before
    with pytest.raises(ValueError, match="MustRunAsRange requires at least one range"):
        P.Provider(bad)


SA_USER = "system:serviceaccount:test:sa"


@pytest.mark.parametrize("user,sa,allowed,policies,expected", [
    ("user", "sa", {"user": {"test": {"policy": True}}}, ["policy"], "policy"),
    ("user", "sa", {SA_USER: {"test": {"policy": True}}}, ["policy"], "policy"),
    ("user", "sa", {}, ["policy"], ""),
    ("user", "sa", {SA_USER: {"test": {"policy1": True}, "": {"policy4": True}, "other": {"policy6": True}},
                    "user": {"test": {"policy2": True}, "": {"policy5": True}, "other": {"policy7": True}}},
     ["a_policy1", "a_policy2", "policy2", "policy3", "policy4", "policy5", "policy6"], "policy2"),
    (None, "sa", {SA_USER: {"test": {"policy1": True}}, "user": {"test": {"policy2": True}}},
     ["policy1", "policy2", "policy3"], "policy1"),
    ("user", "", {SA_USER: {"test": {"policy1": True}}, "user": {"test": {"policy2": True}}},
     ["policy1", "policy2", "policy3"], "policy2"),
    (None, "", {SA_USER: {"test": {"policy1": True}}, "user": {"test": {"policy2": True}}},
     ["policy1", "policy2", "policy3"], ""),
], ids=["policy allowed by user", "policy allowed by sa", "no policies allowed", "multiple policies allowed",
        "policies are not allowed for nil user info", "policies are not allowed for nil sa info",
        "policies are not allowed for nil sa and user info"])
def test_policy_authorization(user, sa, allowed, policies, expected):
    pod = good_pod()
    pod["metadata"]["namespace"] = "test"
    pod["spec"]["serviceAccountName"] = sa
    admit_and_validate([permissive_psp(n) for n in policies], pod, bool(expected), bool(expected), expected,
                       allowed=allowed, user={"name": user, "groups": []} if user else {})


@pytest.mark.parametrize("allowed,n_errs", [
    ({}, 0), ({"user": {"test": {"policy1": True}}}, 1), ({SA_USER: {"test": {"policy2": True}}}, 1),
    ({"user": {"test": {"policy1": True}}, SA_USER: {"test": {"policy2": True}}}, 2),
], ids=["policies not allowed", "policy allowed by user", "policy allowed by service account", "multiple policies allowed"])
def test_policy_authorization_errors(allowed, n_errs):
    pod = good_pod()
    pod["metadata"]["namespace"] = "test"
    pod["spec"]["serviceAccountName"] = "sa"
    pod["spec"]["containers"][0]["securityContext"]["privileged"] = True
    ctx = Ctx([restrictive_psp("policy1"), restrictive_psp("policy2")], allowed)
    a = Attributes(CREATE, "pods", "", "test", "pod", pod, None, {"name": "user", "groups": []})
    plugin = X.PodSecurityPolicy()
    allowed_pod, _, errs = P.compute_security_context(ctx.list_objects("podsecuritypolicies", ""), pod,
                                                      plugin._authorized(a, ctx, pod), True)
    assert allowed_pod is None and len(errs) == n_errs


def test_validate_never_selects_a_mutating_policy():
    """computeSecurityContext with mutation disallowed (the validate phase): a policy that would
    change the pod is skipped before authorization is consulted, so only non-mutating policies can
    admit; with none, the pod is rejected even though a mutating policy validates it."""
    mutating = restrictive_psp("mutating", runAsUser={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]})
    pod = _unpriv_runasany_pod()
    asked = []

    def authorized(name):
        asked.append(name)
        return True
    admitted, name, errs = P.compute_security_context([mutating], _c(pod), authorized, False)
    assert (admitted, name, errs) == (None, "", []) and asked == []
    admitted, name, _ = P.compute_security_context([mutating], _c(pod), authorized, True)
    assert name == "mutating" and admitted["spec"]["containers"][0]["securityContext"]["runAsUser"] == 1
    privileged = permissive_psp("privileged")
    asked.clear()
    admitted, name, _ = P.compute_security_context([mutating, privileged], _c(pod), authorized, False)
    assert name == "privileged" and asked == ["privileged"] and P._semantic_equal(admitted, pod)
