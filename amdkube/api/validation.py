"""Validation for the served kinds.

Reference: pkg/apis/core/validation/validation.go — ValidatePod/ValidatePodSpec,
fork ValidateExtendedResources (:2950-2987) and validateContainersExtendedResources
(:2457-2483, applied to Containers at :2883-2888), ValidatePodBinding (:3416-3429),
ValidateNode. Deliberate fixes: #9 init containers' extendedResourceRequests
are validated too; #10 the binding's extendedResourceBinding is validated (statically
here, against node state in the registry).
"""
from __future__ import annotations

import json
import re

from .field import go_value as gv
from .helpers import HEALTHY, UNHEALTHY, is_extended_resource_name, is_native_resource
from .labels import (SelectorError, is_dns1123_label, is_dns1123_subdomain, is_qualified_name,
                     is_valid_label_value, node_requirements_as_selector, selector_from_label_selector)
from .quantity import Quantity, QuantityError
from .scheme import register_hooks

RESTART_POLICIES = ("Always", "OnFailure", "Never")


def validate_object_meta(obj: dict, namespaced: bool, name_fn=is_dns1123_subdomain) -> list[str]:
    errs = []
    md = obj.get("metadata") or {}
    name = md.get("name") or ""
    if not name and not md.get("generateName"):
        errs.append("metadata.name: Required value: name or generateName is required")
    elif name:
        errs += [f"metadata.name: Invalid value: {gv(name)}: {e}" for e in name_fn(name)]
    ns = md.get("namespace") or ""
    if namespaced and not ns:
        errs.append("metadata.namespace: Required value")
    if not namespaced and ns:
        errs.append("metadata.namespace: Forbidden: not allowed on this type")
    if ns:
        errs += [f"metadata.namespace: Invalid value: {gv(ns)}: {e}" for e in is_dns1123_label(ns)]
    for k, v in (md.get("labels") or {}).items():
        errs += [f"metadata.labels: Invalid value: {gv(k)}: {e}" for e in is_qualified_name(k)]
        errs += [f"metadata.labels: Invalid value: {gv(v)}: {e}" for e in is_valid_label_value(str(v))]
    ann = md.get("annotations") or {}
    for k in ann:
        errs += [f"metadata.annotations: Invalid value: {gv(k)}: {e}" for e in is_qualified_name(k.lower())]
    if sum(len(k) + len(str(v)) for k, v in ann.items()) > 256 * 1024:
        errs.append("metadata.annotations: Too long: must have at most 262144 characters")
    return errs


def _validate_resource_list(rl: dict | None, path: str) -> list[str]:
    errs = []
    for k, v in (rl or {}).items():
        if is_qualified_name(k):
            errs.append(f"{path}[{k}]: Invalid value: {gv(k)}: must be a standard resource name or fully qualified")
        try:
            q = Quantity(v)
            if q.as_fraction() < 0:
                errs.append(f"{path}[{k}]: Invalid value: {gv(v)}: must be greater than or equal to 0")
            if not is_native_resource(k) and q.as_fraction().denominator != 1:
                errs.append(f"{path}[{k}]: Invalid value: {gv(v)}: must be an integer")
        except QuantityError as e:
            errs.append(f"{path}[{k}]: Invalid value: {gv(v)}: {e}")
    return errs


def validate_resource_requirements(res: dict | None, path: str) -> list[str]:
    res = res or {}
    lim, req = res.get("limits") or {}, res.get("requests") or {}
    errs = _validate_resource_list(lim, path + ".limits") + _validate_resource_list(req, path + ".requests")
    if errs:
        return errs
    for k, v in req.items():
        if k in lim:
            if Quantity(v) > Quantity(lim[k]):
                errs.append(f"{path}.requests[{k}]: Invalid value: {gv(v)}: must be less than or equal to {k} limit")
            if (is_extended_resource_name(k) or k == "alpha.kubernetes.io/amd-gpu") and Quantity(v) != Quantity(lim[k]):
                # extended resources and the legacy GPU resource (validation.go:4448-4449) cannot overcommit
                errs.append(f"{path}.requests[{k}]: Invalid value: {gv(v)}: must be equal to {k} limit")
        elif is_extended_resource_name(k):
            errs.append(f"{path}.limits[{k}]: Required value: Limit must be set for non overcommitable resources")
    return errs


def validate_extended_resources(pres_list: list[dict] | None, path="spec.extendedResources") -> tuple[dict, list[str]]:
    """Port of the fork's ValidateExtendedResources semantics (validation.go:2950-2987)."""
    coll: dict[str, int] = {}
    errs: list[str] = []
    for i, r in enumerate(pres_list or []):
        p = f"{path}[{i}]"
        name = r.get("name") or ""
        if not name:
            errs.append(f"{p}.name: Invalid value: Extended resource name can't be empty")
        if name in coll:
            errs.append(f"{p}.name: Invalid value: {gv(name)}: Extended resource name should be unique")
        coll[name] = 0
        res = r.get("resources") or {}
        lim, req = res.get("limits") or {}, res.get("requests") or {}
        if len(lim) != 1:
            errs.append(f"{p}.resources.limits: Invalid value: unexpected limits length {len(lim)} != 1")
        if len(req) != 1:
            errs.append(f"{p}.resources.requests: Invalid value: unexpected requests length {len(req)} != 1")
        for rname, lval in lim.items():
            try:
                if rname not in req or Quantity(req[rname]) != Quantity(lval):
                    errs.append(f"{p}.resources: Invalid value: Invalid Requests, Limits and Requests should be equal")
                elif Quantity(lval).as_fraction() <= 0 or Quantity(lval).as_fraction().denominator != 1:
                    errs.append(f"{p}.resources.limits[{rname}]: Invalid value: must be a positive integer")
            except QuantityError as e:
                errs.append(f"{p}.resources: Invalid value: {e}")
            if not is_extended_resource_name(rname):
                errs.append(f"{p}.resources.limits[{rname}]: Invalid value: must be an extended resource name")
        try:
            node_requirements_as_selector((r.get("affinity") or {}).get("required"))
        except SelectorError as e:
            errs.append(f"{p}.affinity.required: Invalid value: {e}")
        for j, did in enumerate(r.get("assigned") or []):
            if not isinstance(did, str) or not did:
                errs.append(f"{p}.assigned[{j}]: Invalid value: device IDs must be non-empty strings")
    return coll, errs


def validate_containers_extended_resources(containers, names: dict, path: str) -> list[str]:
    """validation.go:2457-2483 — each reference must exist and be used at most once."""
    errs = []
    for ci, c in enumerate(containers or []):
        for ref in c.get("extendedResourceRequests") or []:
            if ref not in names:
                errs.append(f"{path}[{ci}].extendedResourceRequests: Invalid value: {gv(ref)}: Reference to unknown extended resource")
                continue
            if names[ref] != 0:
                errs.append(f"{path}[{ci}].extendedResourceRequests: Invalid value: {gv(ref)}: Multiple reference to extended resource (sharing is not allowed)")
                continue
            names[ref] += 1
    return errs


# pkg/capabilities: cluster-wide switches the apiserver sets from its flags (--allow-privileged)
CAPABILITIES = {"allow_privileged": True}


_ENV_NAME_RE = re.compile(r"^[-._a-zA-Z][-._a-zA-Z0-9]*$")
ENV_FIELD_PATHS = ("metadata.name", "metadata.namespace", "metadata.uid", "spec.nodeName", "spec.serviceAccountName",
                   "status.hostIP", "status.podIP")
VOLUME_FIELD_PATHS = ("metadata.name", "metadata.namespace", "metadata.labels", "metadata.annotations", "metadata.uid")
ENV_RESOURCE_FIELDS = ("limits.cpu", "limits.memory", "limits.ephemeral-storage", "requests.cpu", "requests.memory",
                       "requests.ephemeral-storage")


def is_env_var_name(v: str) -> list[str]:
    """apimachinery validation.go IsEnvVarName (:305-319) with hasChDirPrefix (:380-391)."""
    errs = []
    if not _ENV_NAME_RE.match(v):
        errs.append("a valid environment variable name must consist of alphabetic characters, digits, '_', '-', or '.', "
                    "and must not start with a digit (e.g. 'my.env-name',  or 'MY_ENV.NAME',  or 'MyEnvName1', regex used "
                    "for validation is '[-._a-zA-Z][-._a-zA-Z0-9]*')")
    if v == ".":
        errs.append("must not be '.'")
    elif v == "..":
        errs.append("must not be '..'")
    elif v.startswith(".."):
        errs.append("must not start with '..'")
    return errs


def _validate_ref_name(name: str, path: str) -> list[str]:
    """ValidateConfigMapName / ValidateSecretName: a DNS-1123 subdomain."""
    if not name:
        return [f"{path}: Required value"]
    return [f"{path}: Invalid value: {gv(name)}: {msg}" for msg in is_dns1123_subdomain(name)]


def _split_subscript(fp: str):
    """fieldpath.SplitMaybeSubscriptedPath: "metadata.labels['k']" -> ("metadata.labels", "k")."""
    if not fp.endswith("']"):
        return fp, None
    base, sep, sub = fp[:-2].partition("['")
    if not sep or not base:
        return fp, None
    return base, sub


_DOWNWARD_LABELS = ("metadata.annotations", "metadata.labels", "metadata.name", "metadata.namespace", "metadata.uid",
                    "spec.nodeName", "spec.restartPolicy", "spec.serviceAccountName", "spec.schedulerName",
                    "status.phase", "status.hostIP", "status.podIP")


def validate_object_field_selector(fs: dict, expressions, path: str) -> list[str]:
    """validateObjectFieldSelector (validation.go:1948-1985) with ConvertDownwardAPIFieldLabel
    (pods/helpers.go:29-62): apiVersion v1, a convertible label, a subscript only on labels /
    annotations (the key a qualified name), otherwise one of `expressions`."""
    version, fp = fs.get("apiVersion") or "", fs.get("fieldPath") or ""
    if not version:
        return [f"{path}.apiVersion: Required value"]
    if not fp:
        return [f"{path}.fieldPath: Required value"]
    base, sub = _split_subscript(fp)
    conv_err = None
    if version != "v1":
        conv_err = f"unsupported pod version: {version}"
    elif sub is not None and base not in ("metadata.annotations", "metadata.labels"):
        conv_err = f"field label does not support subscript: {fp}"
    elif sub is None and fp not in _DOWNWARD_LABELS and fp != "spec.host":
        conv_err = f"field label not supported: {fp}"
    if conv_err:
        return [f"{path}.fieldPath: Invalid value: {gv(fp)}: error converting fieldPath: {conv_err}"]
    if fp == "spec.host":
        fp = "spec.nodeName"
    if sub is not None:
        key = sub.lower() if base == "metadata.annotations" else sub
        return [f"{path}: Invalid value: {gv(sub)}: {msg}" for msg in is_qualified_name(key)]
    if fp not in expressions:
        return [f"{path}.fieldPath: Unsupported value: {gv(fp)}: supported values: "
                + ", ".join(f'"{x}"' for x in sorted(expressions))]
    return []


def validate_env(env: list, path: str) -> list[str]:
    """core/validation ValidateEnv + validateEnvVarValueFrom (validation.go:1879-1940)."""
    errs = []
    for i, e in enumerate(env):
        p = f"{path}[{i}]"
        name = e.get("name") or ""
        if not name:
            errs.append(f"{p}.name: Required value")
        else:
            errs += [f"{p}.name: Invalid value: {gv(name)}: {msg}" for msg in is_env_var_name(name)]
        vf = e.get("valueFrom")
        if vf is None:
            continue
        vp = f"{p}.valueFrom"
        n = 0
        fr = vf.get("fieldRef")
        if fr is not None:
            n += 1
            errs += validate_object_field_selector(fr, ENV_FIELD_PATHS, vp + ".fieldRef")
        rf = vf.get("resourceFieldRef")
        if rf is not None:
            n += 1
            res = rf.get("resource") or ""
            if not res:
                errs.append(f"{vp}.resourceFieldRef.resource: Required value")
            elif res not in ENV_RESOURCE_FIELDS:
                errs.append(f"{vp}.resourceFieldRef.resource: Unsupported value: {gv(res)}")
        for kind in ("configMapKeyRef", "secretKeyRef"):
            ref = vf.get(kind)
            if ref is None:
                continue
            n += 1
            errs += _validate_ref_name(ref.get("name") or "", f"{vp}.{kind}.name")
            key = ref.get("key") or ""
            if not key:
                errs.append(f"{vp}.{kind}.key: Required value")
            else:
                errs += [f"{vp}.{kind}.key: Invalid value: {gv(key)}: {msg}" for msg in is_config_map_key(key)]
        if n == 0:
            errs.append(f"{vp}: Invalid value: \"\": must specify one of: `fieldRef`, `resourceFieldRef`, "
                        "`configMapKeyRef` or `secretKeyRef`")
        elif e.get("value"):
            errs.append(f"{vp}: Invalid value: \"\": may not be specified when `value` is not empty")
        elif n > 1:
            errs.append(f"{vp}: Invalid value: \"\": may not have more than one field specified at a time")
    return errs


def validate_env_from(env_from: list, path: str) -> list[str]:
    """ValidateEnvFrom (validation.go:2007-2035): prefix is an env var name; one source."""
    errs = []
    for i, e in enumerate(env_from):
        p = f"{path}[{i}]"
        prefix = e.get("prefix") or ""
        if prefix:
            errs += [f"{p}.prefix: Invalid value: {gv(prefix)}: {msg}" for msg in is_env_var_name(prefix)]
        srcs = [k for k in ("configMapRef", "secretRef") if e.get(k) is not None]
        for k in srcs:
            errs += _validate_ref_name((e.get(k) or {}).get("name") or "", f"{p}.{k}.name")
        if not srcs:
            errs.append(f"{path}: Invalid value: \"\": must specify one of: `configMapRef` or `secretRef`")
        elif len(srcs) > 1:
            errs.append(f"{path}: Invalid value: \"\": may not have more than one field specified at a time")
    return errs


def _validate_node_selector_terms(terms, path) -> list[str]:
    errs = []
    for i, t in enumerate(terms or []):
        try:
            node_requirements_as_selector(t.get("matchExpressions"))
        except SelectorError as e:
            errs.append(f"{path}[{i}].matchExpressions: Invalid value: {e}")
    return errs


_CONFIG_KEY_RE = re.compile(r"^[-._a-zA-Z0-9]+$")


def is_config_map_key(k: str) -> list[str]:
    """validation.go IsConfigMapKey: a plain file name, never '.', '..' or '..'-prefixed."""
    if not k or len(k) > 253:
        return ["must be no more than 253 characters and non-empty"]
    if not _CONFIG_KEY_RE.match(k):
        return ["a valid config key must consist of alphanumeric characters, '-', '_' or '.'"]
    if k in (".", "..") or k.startswith(".."):
        return ["must not be '.' or '..' and must not start with '..'"]
    return []


def validate_local_descending_path(p: str, path: str) -> list[str]:
    """validation.go validateLocalDescendingPath: relative, and no '..' element."""
    if not p:
        return [f"{path}: Required value"]
    errs = []
    if p.startswith("/"):
        errs.append(f"{path}: Invalid value: {gv(p)}: must be a relative path")
    if ".." in p.split("/"):
        errs.append(f"{path}: Invalid value: {gv(p)}: must not contain '..'")
    return errs


def _validate_volume_items(v: dict, path: str) -> list[str]:
    """validateKeyToPath / validateDownwardAPIVolumeFile / validateProjectionSources: every file
    a secret, configMap, downwardAPI or projected volume writes stays inside the volume."""
    errs = []
    for src_key in ("secret", "configMap"):
        for i, it in enumerate((v.get(src_key) or {}).get("items") or []):
            if not it.get("key"):
                errs.append(f"{path}.{src_key}.items[{i}].key: Required value")
            errs += validate_local_descending_path(it.get("path") or "", f"{path}.{src_key}.items[{i}].path")
    for i, it in enumerate((v.get("downwardAPI") or {}).get("items") or []):
        errs += validate_local_descending_path(it.get("path") or "", f"{path}.downwardAPI.items[{i}].path")
        if it.get("fieldRef") is not None:       # validateDownwardAPIVolumeFile
            errs += validate_object_field_selector(it["fieldRef"], VOLUME_FIELD_PATHS,
                                                   f"{path}.downwardAPI.items[{i}].fieldRef")
    for j, srcs in enumerate((v.get("projected") or {}).get("sources") or []):
        for src_key in ("secret", "configMap", "downwardAPI"):
            for i, it in enumerate((srcs.get(src_key) or {}).get("items") or []):
                errs += validate_local_descending_path(it.get("path") or "",
                                                       f"{path}.projected.sources[{j}].{src_key}.items[{i}].path")
    return errs


def validate_pod_spec(spec: dict, path="spec") -> list[str]:
    """ValidatePodSpec — corevalidation.validate_pod_spec (validation.go:2879)."""
    from .corevalidation import validate_pod_spec as _v
    return _v(spec, path)


def validate_pod(pod: dict, old: dict | None = None) -> list[str]:
    """ValidatePod (+ ValidatePodUpdate when `old`) — corevalidation.validate_pod."""
    from .corevalidation import validate_pod as _v
    return _v(pod, old)


def validate_node(node: dict, old: dict | None = None) -> list[str]:
    errs = validate_object_meta(node, False)
    st = node.get("status") or {}
    errs += _validate_resource_list(st.get("capacity"), "status.capacity")
    errs += _validate_resource_list(st.get("allocatable"), "status.allocatable")
    for rname, dom in (st.get("extendedResources") or {}).items():
        if not is_extended_resource_name(rname):
            errs.append(f"status.extendedResources[{rname}]: Invalid value: must be an extended resource name")
        for did, dev in ((dom or {}).get("resources") or {}).items():
            p = f"status.extendedResources[{rname}].resources[{did}]"
            if dev.get("id", did) != did:
                errs.append(f"{p}.id: Invalid value: must equal the map key")
            if dev.get("health", HEALTHY) not in (HEALTHY, UNHEALTHY):
                errs.append(f"{p}.health: Unsupported value: {gv(dev.get('health'))}")
            for k, v in (dev.get("attributes") or {}).items():
                errs += [f"{p}.attributes: Invalid value: {gv(k)}: {e}" for e in is_qualified_name(k)]
                errs += [f"{p}.attributes: Invalid value: {gv(v)}: {e}" for e in is_valid_label_value(str(v))]
    for i, t in enumerate((node.get("spec") or {}).get("taints") or []):
        if t.get("effect") not in ("NoSchedule", "PreferNoSchedule", "NoExecute"):
            errs.append(f"spec.taints[{i}].effect: Unsupported value: {gv(t.get('effect'))}")
        errs += [f"spec.taints[{i}].key: Invalid value: {e}" for e in is_qualified_name(t.get("key") or "")]
    return errs


def validate_binding(b: dict) -> list[str]:
    """Static half of fix #10 (node-state half: apiserver pods/binding registry)."""
    errs = []
    tgt = b.get("target") or {}
    if tgt.get("kind") not in (None, "", "Node"):
        errs.append("target.kind: Invalid value: must be empty or 'Node'")
    if not tgt.get("name"):
        errs.append("target.name: Required value")
    for k, v in (tgt.get("extendedResourceBinding") or {}).items():
        ids = (v or {}).get("resources")
        if not isinstance(ids, list) or not all(isinstance(x, str) and x for x in ids):
            errs.append(f"target.extendedResourceBinding[{k}].resources: Invalid value: must be a list of device IDs")
        elif len(set(ids)) != len(ids):
            errs.append(f"target.extendedResourceBinding[{k}].resources: Duplicate value: device IDs must be unique")
    return errs


def validate_generic_namespaced(obj, old=None):
    return validate_object_meta(obj, True)


def validate_config_data(obj, old=None):
    """ValidateConfigMap / ValidateSecret: every data key is a valid config key (it becomes a
    file name in configMap and secret volumes)."""
    errs = validate_object_meta(obj, True)
    for field in ("data", "binaryData", "stringData"):
        for k in (obj.get(field) or {}):
            errs += [f"{field}[{k}]: Invalid value: {gv(k)}: {e}" for e in is_config_map_key(k)]
    return errs


def validate_event(ev, old=None):
    errs = validate_object_meta(ev, True)
    if not (ev.get("involvedObject") or {}).get("kind"):
        errs.append("involvedObject.kind: Required value")
    return errs


from . import corevalidation as _cv  # noqa: E402
from . import groupvalidation as _gv  # noqa: E402

validate_namespace = _cv.validate_namespace
register_hooks("Pod", validator=_cv.validate_pod)
register_hooks("Node", validator=validate_node)
register_hooks("Namespace", validator=_cv.validate_namespace)
register_hooks("Event", validator=validate_event)
from .networking import default_service, validate_service  # noqa: E402


def _validate_crd(obj, old=None):
    from ..apiserver.crd import validate_crd
    return validate_object_meta(obj, False) + validate_crd(obj, old)


register_hooks("CustomResourceDefinition", "apiextensions.k8s.io/v1beta1", validator=_validate_crd)
register_hooks("Service", defaulter=default_service, validator=validate_service)
for _k, _fn in (("ConfigMap", _cv.validate_config_map), ("Secret", _cv.validate_secret),
                ("ServiceAccount", _cv.validate_service_account), ("Endpoints", _cv.validate_endpoints),
                ("LimitRange", _cv.validate_limit_range), ("ResourceQuota", _cv.validate_resource_quota),
                ("PersistentVolume", _cv.validate_persistent_volume),
                ("PersistentVolumeClaim", _cv.validate_persistent_volume_claim),
                ("ReplicationController", _cv.validate_replication_controller),
                ("PodTemplate", _cv.validate_pod_template)):
    register_hooks(_k, validator=_fn)
_gv.register()
