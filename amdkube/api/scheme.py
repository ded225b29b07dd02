"""The type registry (runtime.Scheme analogue) and codecs.

Reference: staging/src/k8s.io/apimachinery/pkg/runtime/scheme.go:160 (AddKnownTypes),
:392 (Default), :404 (Convert); codecs in .../runtime/serializer (json/yaml/protobuf).

amdkube keeps objects as JSON dicts, so the scheme is a table of ResourceInfo records
(group/version/kind/plural/scope/short names) plus per-kind defaulting and validation
hooks that the registry and kubectl look up. Only the external version exists (no
internal<->v1 conversion round trip), which removes a whole copy per request.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Callable

import yaml


@dataclass
class ResourceInfo:
    group: str
    version: str
    kind: str
    plural: str
    namespaced: bool
    short_names: tuple = ()
    subresources: tuple = ()
    list_kind: str = ""
    verbs: tuple = ("create", "delete", "deletecollection", "get", "list", "patch", "update", "watch")
    defaulter: Callable | None = field(default=None, repr=False)
    validator: Callable | None = field(default=None, repr=False)
    # served-only version: (group, plural) of the canonical resource whose storage it shares
    # (extensions/v1beta1 deployments → apps deployments); None for a storage version
    storage: tuple | None = None
    to_storage: Callable | None = field(default=None, repr=False)     # request body → canonical (version defaults)
    from_storage: Callable | None = field(default=None, repr=False)   # stored object → this version's shape

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    @property
    def group_resource(self) -> str:
        return f"{self.plural}.{self.group}" if self.group else self.plural

    def api_prefix(self) -> str:
        return f"/apis/{self.group}/{self.version}" if self.group else f"/api/{self.version}"


class Scheme:
    def __init__(self):
        self.by_kind: dict[tuple[str, str], ResourceInfo] = {}
        self.by_plural: dict[tuple[str, str], ResourceInfo] = {}
        self.by_name: dict[str, ResourceInfo] = {}
        self.by_gvr: dict[tuple[str, str, str], ResourceInfo] = {}

    def add(self, ri: ResourceInfo):
        ri.list_kind = ri.list_kind or ri.kind + "List"
        self.by_kind[(ri.api_version, ri.kind)] = ri
        self.by_gvr[(ri.group, ri.version, ri.plural)] = ri
        if ri.storage is None or (ri.group, ri.plural) not in self.by_plural:
            self.by_plural[(ri.group, ri.plural)] = ri
        for n in (ri.plural, ri.kind.lower(), *ri.short_names, ri.group_resource):
            self.by_name.setdefault(n, ri)

    def add_alias(self, group: str, version: str, of: tuple, kind: str | None = None, to_storage=None,
                  from_storage=None) -> ResourceInfo:
        """Serve an existing resource under another group/version (the apiserver's multi-version
        serving: same storage, objects rewritten to the requested apiVersion on the way out)."""
        canon = self.by_plural[of]
        ri = ResourceInfo(group, version, kind or canon.kind, canon.plural, canon.namespaced, canon.short_names,
                          canon.subresources, storage=of, to_storage=to_storage, from_storage=from_storage)
        self.add(ri)
        return ri

    def storage_of(self, ri: ResourceInfo) -> ResourceInfo:
        return self.by_plural[ri.storage] if ri.storage else ri

    def served(self, group: str, version: str, plural: str) -> ResourceInfo | None:
        return self.by_gvr.get((group, version, plural))

    def storage_versions(self):
        return [ri for ri in self.by_kind.values() if ri.storage is None]

    def preferred_version(self, group: str) -> str | None:
        vs = [ri.version for ri in self.by_kind.values() if ri.group == group and ri.storage is None]
        if not vs:
            vs = [ri.version for ri in self.by_kind.values() if ri.group == group]
        return _version_sort(vs)[0] if vs else None

    def for_kind(self, api_version: str, kind: str) -> ResourceInfo | None:
        return self.by_kind.get((api_version, kind))

    def for_plural(self, group: str, plural: str) -> ResourceInfo | None:
        return self.by_plural.get((group, plural))

    def for_object(self, obj: dict) -> ResourceInfo | None:
        return self.for_kind(obj.get("apiVersion", ""), obj.get("kind", ""))

    def resolve(self, name: str) -> ResourceInfo | None:
        """kubectl-style lookup: 'po', 'pods', 'pod', 'daemonsets.apps', 'ds'."""
        return self.by_name.get(name.lower())

    def groups(self) -> dict[str, list[ResourceInfo]]:
        out: dict[str, list[ResourceInfo]] = {}
        for ri in self.by_kind.values():
            out.setdefault(ri.api_version, []).append(ri)
        return out

    def to_storage(self, obj: dict) -> dict:
        """A body in a served-only version → its storage version (apiVersion and the version's
        defaults); storage-version bodies are returned as they are."""
        ri = self.for_object(obj)
        if ri is None or ri.storage is None:
            return obj
        if ri.to_storage:
            ri.to_storage(obj)
        canon = self.by_plural[ri.storage]
        obj["apiVersion"], obj["kind"] = canon.api_version, canon.kind
        return obj

    def default(self, obj: dict) -> dict:
        ri = self.for_object(obj)
        if ri and ri.defaulter:
            ri.defaulter(obj)
        return obj

    def validate(self, obj: dict, old: dict | None = None) -> list[str]:
        ri = self.for_object(obj)
        if ri and ri.validator:
            return ri.validator(obj, old)
        return []


SCHEME = Scheme()

_CORE = [
    ("Pod", "pods", True, ("po",), ("status", "binding", "eviction", "log", "exec", "attach", "portforward", "proxy")),
    ("Node", "nodes", False, ("no",), ("status", "proxy")),
    ("Binding", "bindings", True, (), ()),
    ("Event", "events", True, ("ev",), ()),
    ("Namespace", "namespaces", False, ("ns",), ("status", "finalize")),
    ("Service", "services", True, ("svc",), ("status", "proxy")),
    ("Endpoints", "endpoints", True, ("ep",), ()),
    ("ConfigMap", "configmaps", True, ("cm",), ()),
    ("Secret", "secrets", True, (), ()),
    ("ServiceAccount", "serviceaccounts", True, ("sa",), ()),
    ("LimitRange", "limitranges", True, ("limits",), ()),
    ("ResourceQuota", "resourcequotas", True, ("quota",), ("status",)),
    ("PersistentVolume", "persistentvolumes", False, ("pv",), ("status",)),
    ("PersistentVolumeClaim", "persistentvolumeclaims", True, ("pvc",), ("status",)),
    ("ReplicationController", "replicationcontrollers", True, ("rc",), ("status", "scale")),
    ("PodTemplate", "podtemplates", True, (), ()),
]
_APPS = [
    ("DaemonSet", "daemonsets", True, ("ds",), ("status",)),
    ("ReplicaSet", "replicasets", True, ("rs",), ("status", "scale")),
    ("Deployment", "deployments", True, ("deploy",), ("status", "scale", "rollback")),
    ("StatefulSet", "statefulsets", True, ("sts",), ("status", "scale")),
    ("ControllerRevision", "controllerrevisions", True, (), ()),
]
_BATCH = [("Job", "jobs", True, (), ("status",))]
_BATCH_BETA = [("CronJob", "cronjobs", True, ("cj",), ("status",))]
_COORD = [("Lease", "leases", True, (), ())]
_SCHED = [("PriorityClass", "priorityclasses", False, ("pc",), ())]
_AUTOSCALING = [("HorizontalPodAutoscaler", "horizontalpodautoscalers", True, ("hpa",), ("status",))]
_POLICY = [("PodDisruptionBudget", "poddisruptionbudgets", True, ("pdb",), ("status",))]
_CERTS = [("CertificateSigningRequest", "certificatesigningrequests", False, ("csr",), ("status", "approval"))]
_RBAC = [("Role", "roles", True, (), ()), ("ClusterRole", "clusterroles", False, (), ()),
         ("RoleBinding", "rolebindings", True, (), ()), ("ClusterRoleBinding", "clusterrolebindings", False, (), ())]
_STORAGE = [("StorageClass", "storageclasses", False, ("sc",), ())]
_STORAGE_BETA = [("VolumeAttachment", "volumeattachments", False, (), ("status",))]
_AUTHZ = [("SubjectAccessReview", "subjectaccessreviews", False, (), ()),
          ("SelfSubjectAccessReview", "selfsubjectaccessreviews", False, (), ()),
          ("LocalSubjectAccessReview", "localsubjectaccessreviews", True, (), ())]
_AUTHN = [("TokenReview", "tokenreviews", False, (), ())]
_ADMREG = [("MutatingWebhookConfiguration", "mutatingwebhookconfigurations", False, (), ()),
           ("ValidatingWebhookConfiguration", "validatingwebhookconfigurations", False, (), ())]
_APIEXT = [("CustomResourceDefinition", "customresourcedefinitions", False, ("crd", "crds"), ("status",))]

_EXTENSIONS = [("Ingress", "ingresses", True, ("ing",), ("status",)),
               ("PodSecurityPolicy", "podsecuritypolicies", False, ("psp",), ())]
_NETWORKING = [("NetworkPolicy", "networkpolicies", True, ("netpol",), ())]
_SETTINGS = [("PodPreset", "podpresets", True, (), ())]
_ADMREG_ALPHA = [("InitializerConfiguration", "initializerconfigurations", False, (), ())]
_APIREG = [("APIService", "apiservices", False, (), ("status",))]

for group, version, table in (("", "v1", _CORE), ("apps", "v1", _APPS), ("batch", "v1", _BATCH),
                              ("batch", "v1beta1", _BATCH_BETA), ("coordination.k8s.io", "v1", _COORD),
                              ("scheduling.k8s.io", "v1", _SCHED), ("autoscaling", "v1", _AUTOSCALING),
                              ("policy", "v1beta1", _POLICY), ("certificates.k8s.io", "v1beta1", _CERTS),
                              ("rbac.authorization.k8s.io", "v1", _RBAC), ("storage.k8s.io", "v1", _STORAGE),
                              ("storage.k8s.io", "v1beta1", _STORAGE_BETA),
                              ("authorization.k8s.io", "v1", _AUTHZ), ("authentication.k8s.io", "v1", _AUTHN),
                              ("apiextensions.k8s.io", "v1beta1", _APIEXT),
                              ("admissionregistration.k8s.io", "v1beta1", _ADMREG),
                              ("extensions", "v1beta1", _EXTENSIONS), ("networking.k8s.io", "v1", _NETWORKING),
                              ("settings.k8s.io", "v1alpha1", _SETTINGS),
                              ("admissionregistration.k8s.io", "v1alpha1", _ADMREG_ALPHA),
                              ("apiregistration.k8s.io", "v1beta1", _APIREG)):
    for kind, plural, ns, short, subs in table:
        SCHEME.add(ResourceInfo(group, version, kind, plural, ns, short, subs))


def _v1beta_selector_default(obj: dict):
    """extensions/v1beta1, apps/v1beta1 defaulting: a missing spec.selector is the template's
    labels (apps/v1 requires it, so it is filled before the object is converted)."""
    spec = obj.setdefault("spec", {})
    if not spec.get("selector"):
        labels = ((spec.get("template") or {}).get("metadata") or {}).get("labels") or {}
        if labels:
            spec["selector"] = {"matchLabels": dict(labels)}


# the reference release's other served versions (pkg/master/master.go DefaultAPIResourceConfigSource
# + each group's install): same storage, rewritten apiVersion
for _g, _v, _of, _conv in (
        ("extensions", "v1beta1", ("apps", "deployments"), _v1beta_selector_default),
        ("extensions", "v1beta1", ("apps", "daemonsets"), _v1beta_selector_default),
        ("extensions", "v1beta1", ("apps", "replicasets"), _v1beta_selector_default),
        ("extensions", "v1beta1", ("networking.k8s.io", "networkpolicies"), None),
        ("apps", "v1beta1", ("apps", "deployments"), _v1beta_selector_default),
        ("apps", "v1beta1", ("apps", "statefulsets"), _v1beta_selector_default),
        ("apps", "v1beta1", ("apps", "controllerrevisions"), None),
        ("apps", "v1beta2", ("apps", "deployments"), None), ("apps", "v1beta2", ("apps", "daemonsets"), None),
        ("apps", "v1beta2", ("apps", "replicasets"), None), ("apps", "v1beta2", ("apps", "statefulsets"), None),
        ("apps", "v1beta2", ("apps", "controllerrevisions"), None),
        ("batch", "v2alpha1", ("batch", "cronjobs"), None),
        ("rbac.authorization.k8s.io", "v1beta1", ("rbac.authorization.k8s.io", "roles"), None),
        ("rbac.authorization.k8s.io", "v1beta1", ("rbac.authorization.k8s.io", "clusterroles"), None),
        ("rbac.authorization.k8s.io", "v1beta1", ("rbac.authorization.k8s.io", "rolebindings"), None),
        ("rbac.authorization.k8s.io", "v1beta1", ("rbac.authorization.k8s.io", "clusterrolebindings"), None),
        ("rbac.authorization.k8s.io", "v1alpha1", ("rbac.authorization.k8s.io", "roles"), None),
        ("rbac.authorization.k8s.io", "v1alpha1", ("rbac.authorization.k8s.io", "clusterroles"), None),
        ("rbac.authorization.k8s.io", "v1alpha1", ("rbac.authorization.k8s.io", "rolebindings"), None),
        ("rbac.authorization.k8s.io", "v1alpha1", ("rbac.authorization.k8s.io", "clusterrolebindings"), None),
        ("storage.k8s.io", "v1beta1", ("storage.k8s.io", "storageclasses"), None),
        ("scheduling.k8s.io", "v1alpha1", ("scheduling.k8s.io", "priorityclasses"), None),
        ("authorization.k8s.io", "v1beta1", ("authorization.k8s.io", "subjectaccessreviews"), None),
        ("authorization.k8s.io", "v1beta1", ("authorization.k8s.io", "selfsubjectaccessreviews"), None),
        ("authorization.k8s.io", "v1beta1", ("authorization.k8s.io", "localsubjectaccessreviews"), None),
        ("authentication.k8s.io", "v1beta1", ("authentication.k8s.io", "tokenreviews"), None)):
    SCHEME.add_alias(_g, _v, _of, to_storage=_conv)

# autoscaling/v2beta1 HPAs: multiple metrics, kept in annotations on the v1 storage object
from . import autoscaling as _as   # noqa: E402
SCHEME.add_alias("autoscaling", "v2beta1", ("autoscaling", "horizontalpodautoscalers"),
                 to_storage=_as.v2_to_v1, from_storage=_as.v1_to_v2)


def _version_sort(vs):
    """Kubernetes version priority: GA > beta > alpha, then higher numbers first."""
    import re as _re

    def key(v):
        mt = _re.match(r"^v(\d+)(?:(alpha|beta)(\d+))?$", v)
        if not mt:
            return (3, 0, 0, v)
        major, stage, minor = int(mt.group(1)), mt.group(2), int(mt.group(3) or 0)
        return ({None: 0, "beta": 1, "alpha": 2}[stage], -major, -minor, v)
    return sorted(set(vs), key=key)


def register_hooks(kind: str, api_version: str = "v1", defaulter=None, validator=None):
    ri = SCHEME.for_kind(api_version, kind)
    if ri is None:
        raise KeyError(kind)
    if defaulter:
        ri.defaulter = defaulter
    if validator:
        ri.validator = validator


# ------------------------------------------------------------------------ codecs
def encode(obj) -> bytes:
    return json.dumps(obj, separators=(",", ":")).encode()


def decode(data: bytes | str):
    return json.loads(data)


def load_manifests(text: str) -> list[dict]:
    """YAML or JSON, multi-document; `kind: List` is flattened (kubectl create -f)."""
    text = text.strip()
    docs = []
    if text.startswith("{") or text.startswith("["):
        d = json.loads(text)
        docs = d if isinstance(d, list) else [d]
    else:
        docs = [d for d in yaml.safe_load_all(text) if d]
    out = []
    for d in docs:
        if isinstance(d, dict) and d.get("kind", "").endswith("List") and "items" in d:
            out.extend(d["items"])
        else:
            out.append(d)
    return out


def dump_yaml(obj) -> str:
    return yaml.safe_dump(obj, default_flow_style=False, sort_keys=False)


# Protobuf envelope (`k8s\x00` + runtime.Unknown). amdkube serves JSON; the envelope is
# implemented for content negotiation parity (reference serializer/protobuf/protobuf.go:42,88)
# with the JSON object as the raw payload and contentType application/json.
PROTO_MAGIC = b"k8s\x00"


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, payload: bytes) -> bytes:
    return _varint(num << 3 | 2) + _varint(len(payload)) + payload


def encode_envelope(obj: dict) -> bytes:
    tm = _field(1, obj.get("apiVersion", "").encode()) + _field(2, obj.get("kind", "").encode())
    return PROTO_MAGIC + _field(1, tm) + _field(2, encode(obj)) + _field(4, b"application/json")


def decode_envelope(data: bytes) -> dict:
    if not data.startswith(PROTO_MAGIC):
        raise ValueError("missing k8s protobuf magic")
    buf, i, fields = data[4:], 0, {}
    while i < len(buf):
        key, shift = 0, 0
        while True:
            b = buf[i]; i += 1
            key |= (b & 0x7F) << shift; shift += 7
            if not b & 0x80:
                break
        ln, shift = 0, 0
        while True:
            b = buf[i]; i += 1
            ln |= (b & 0x7F) << shift; shift += 7
            if not b & 0x80:
                break
        fields[key >> 3] = buf[i:i + ln]
        i += ln
    return decode(fields[2])
