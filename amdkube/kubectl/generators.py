"""The configmap/v1 and secret/v1 generators of `kubectl create configmap|secret generic`.

Reference: pkg/kubectl/configmap.go and secret.go (StructuredGenerate, validate, the
from-file/from-literal/from-env-file handlers), pkg/kubectl/util/util.go ParseFileSource /
ParseLiteralSource, pkg/kubectl/env_file.go (addFromEnvFile: BOM on the first line, leading
whitespace and #-comments skipped, IsEnvVarName keys, `KEY` alone takes the value from the
environment) and pkg/kubectl/util/hash (--append-hash: the first 10 hex digits of the SHA-256 of
{"data","kind","name"[,"type"]} with 0,1,3,a,e mapped to g,h,k,m,t).
"""
from __future__ import annotations

import base64
import hashlib
import json
import os

from ..api.validation import is_config_map_key, is_env_var_name


class GenerateError(Exception):
    pass


def parse_file_source(source: str) -> tuple[str, str]:
    n = source.count("=")
    if n == 0:
        return os.path.basename(source.rstrip("/")) or source, source
    if n == 1 and source.startswith("="):
        raise GenerateError(f"key name for file path {source[1:]} missing.")
    if n == 1 and source.endswith("="):
        raise GenerateError(f"file path for key name {source[:-1]} missing.")
    if n > 1:
        raise GenerateError("Key names or file paths cannot contain '='.")
    k, p = source.split("=")
    return k, p


def parse_literal_source(source: str) -> tuple[str, str]:
    if source.startswith("=") or "=" not in source:
        raise GenerateError(f"invalid literal source {source}, expected key=value")
    k, v = source.split("=", 1)
    return k, v


def env_file_pairs(path: str) -> list[tuple[str, str]]:
    out = []
    with open(path, "rb") as f:
        for i, raw in enumerate(f.read().split(b"\n")):
            raw = raw.rstrip(b"\r")
            try:
                line = raw.decode("utf-8")
            except UnicodeDecodeError:
                raise GenerateError(f"env file {path} contains invalid utf8 bytes at line {i + 1}: {list(raw)}") from None
            if i == 0 and line.startswith("﻿"):
                line = line[1:]
            line = line.lstrip()
            if not line or line.startswith("#"):
                continue
            key, sep, value = line.partition("=")
            errs = is_env_var_name(key)
            if errs:
                raise GenerateError(f'"{key}" is not a valid key name: {";".join(errs)}')
            out.append((key, value if sep else os.environ.get(key, "")))
    return out


def _go_map(d: dict, secret: bool) -> str:
    def val(v):
        return "[" + " ".join(str(b) for b in v) + "]" if secret else v
    return "map[" + " ".join(f"{k}:{val(d[k])}" for k in sorted(d)) + "]"


def _add(data: dict, key: str, value, what: str):
    errs = is_config_map_key(key)
    if errs:
        raise GenerateError(f'"{key}" is not a valid key name for a {what}: {";".join(errs)}')
    if key in data:
        raise GenerateError(f"cannot add key {key}, another key by that name already exists: {_go_map(data, what == 'Secret')}.")
    data[key] = value


def _collect(what: str, file_sources, literal_sources, env_file, to_value):
    data: dict = {}
    for src in file_sources or []:
        key, path = parse_file_source(src)
        if not os.path.exists(path):
            raise GenerateError(f"error reading {path}: no such file or directory")
        if os.path.isdir(path):
            if "=" in src:
                raise GenerateError("cannot give a key name for a directory path.")
            for item in sorted(os.listdir(path)):
                p = os.path.join(path, item)
                if os.path.isfile(p) and not os.path.islink(p):
                    with open(p, "rb") as f:
                        _add(data, item, to_value(f.read()), what)
        else:
            with open(path, "rb") as f:
                _add(data, key, to_value(f.read()), what)
    for src in literal_sources or []:
        k, v = parse_literal_source(src)
        _add(data, k, to_value(v.encode()), what)
    if env_file:
        if not os.path.exists(env_file):
            raise GenerateError(f"error reading {env_file}: no such file or directory")
        if os.path.isdir(env_file):
            raise GenerateError("env config file cannot be a directory")
        for k, v in env_file_pairs(env_file):
            _add(data, k, to_value(v.encode()), what)
    return data


def _encode_hash(hexdigest: str) -> str:
    return hexdigest[:10].translate(str.maketrans({"0": "g", "1": "h", "3": "k", "a": "m", "e": "t"}))


def _go_json(obj) -> str:
    return json.dumps(obj, sort_keys=True, separators=(",", ":"), ensure_ascii=False)


def encode_config_map(cm: dict) -> str:
    return _go_json({"kind": "ConfigMap", "name": (cm.get("metadata") or {}).get("name", ""), "data": cm.get("data") or {}})


def encode_secret(sec: dict) -> str:
    return _go_json({"kind": "Secret", "type": sec.get("type", ""), "name": (sec.get("metadata") or {}).get("name", ""),
                     "data": sec.get("data") or {}})


def config_map_hash(cm: dict) -> str:
    return _encode_hash(hashlib.sha256(encode_config_map(cm).encode()).hexdigest())


def secret_hash(sec: dict) -> str:
    return _encode_hash(hashlib.sha256(encode_secret(sec).encode()).hexdigest())


def _validate(name, file_sources, literal_sources, env_file):
    if not name:
        raise GenerateError("name must be specified")
    if env_file and (file_sources or literal_sources):
        raise GenerateError("from-env-file cannot be combined with from-file or from-literal")


def generate_config_map(name: str, file_sources=(), literal_sources=(), env_file: str = "", append_hash=False) -> dict:
    _validate(name, file_sources, literal_sources, env_file)
    data = _collect("ConfigMap", file_sources, literal_sources, env_file, lambda b: b.decode("utf-8", "replace"))
    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name}, "data": data}
    if append_hash:
        cm["metadata"]["name"] = f"{name}-{config_map_hash(cm)}"
    return cm


def generate_secret(name: str, type_: str = "", file_sources=(), literal_sources=(), env_file: str = "",
                    append_hash=False) -> dict:
    _validate(name, file_sources, literal_sources, env_file)
    data = _collect("Secret", file_sources, literal_sources, env_file, lambda b: base64.b64encode(b).decode())
    sec = {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": name}, "data": data}
    if type_:
        sec["type"] = type_
    if append_hash:
        sec["metadata"]["name"] = f"{name}-{secret_hash(sec)}"
    return sec


# ---------------------------------------------------------------- service/v2 basic generators
SERVICE_TYPES = {"clusterip": "ClusterIP", "nodeport": "NodePort", "loadbalancer": "LoadBalancer", "externalname": "ExternalName"}


def _atoi(s: str) -> int:
    try:
        return int(s, 10)
    except ValueError:
        raise GenerateError(f'strconv.Atoi: parsing "{s}": invalid syntax') from None


def parse_ports(spec: str) -> tuple[int, int | str]:
    """service_basic.go parsePorts: `port[:targetPort]`, the target a number or a port name."""
    from ..api.corevalidation import is_valid_port_name, is_valid_port_num
    parts = spec.split(":")
    port = _atoi(parts[0])
    errs = is_valid_port_num(port)
    if errs:
        raise GenerateError(",".join(errs))
    if len(parts) == 1:
        return port, port
    try:
        target: int | str = int(parts[1], 10)
    except ValueError:
        errs = is_valid_port_name(parts[1])
        if errs:
            raise GenerateError(",".join(errs)) from None
        return port, parts[1]
    errs = is_valid_port_num(target)
    if errs:
        raise GenerateError(",".join(errs))
    return port, target


def generate_service(name: str, type_: str, tcp=(), cluster_ip: str = "", external_name: str = "", node_port: int = 0) -> dict:
    """ServiceCommonGeneratorV1 (validate + StructuredGenerate): ports named after their
    specifier with ':' turned into '-', label and selector app=<name>."""
    from ..api.labels import is_dns1123_subdomain
    if not name:
        raise GenerateError("name must be specified")
    if not type_:
        raise GenerateError("type must be specified")
    if cluster_ip == "None" and type_ != "ClusterIP":
        raise GenerateError("ClusterIP=None can only be used with ClusterIP service type")
    if cluster_ip != "None" and not tcp and type_ != "ExternalName":
        raise GenerateError("at least one tcp port specifier must be provided")
    if type_ == "ExternalName" and is_dns1123_subdomain(external_name):
        raise GenerateError(f"invalid service external name {external_name}")
    ports = []
    for t in tcp or []:
        port, target = parse_ports(t)
        p = {"name": t.replace(":", "-"), "protocol": "TCP", "port": port, "targetPort": target}
        if node_port:
            p["nodePort"] = node_port
        ports.append(p)
    spec = {"type": type_, "selector": {"app": name}, "ports": ports}
    if external_name:
        spec["externalName"] = external_name
    if cluster_ip:
        spec["clusterIP"] = cluster_ip
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "labels": {"app": name}}, "spec": spec}


# ------------------------------------------------------ resourcequotas/v1 and poddisruptionbudget/v1beta1/v2
def populate_resource_list(spec: str) -> dict | None:
    """quota.go populateResourceListV1: `resource=quantity,...`."""
    from ..api.quantity import Quantity
    if not spec:
        return None
    out = {}
    for stmt in spec.split(","):
        parts = stmt.split("=")
        if len(parts) != 2:
            raise GenerateError(f"Invalid argument syntax {stmt}, expected <resource>=<value>")
        try:
            Quantity(parts[1])
        except (ValueError, TypeError):
            raise GenerateError("quantities must match the regular expression "
                                "'^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$'") from None
        out[parts[0]] = parts[1]
    return out


def parse_scopes(spec: str) -> list | None:
    if not spec:
        return None
    out = []
    for s in spec.split(","):
        if not s:
            raise GenerateError('invalid resource quota scope ""')
        out.append(s)
    return out


def generate_quota(name: str, hard: str = "", scopes: str = "") -> dict:
    if not name:
        raise GenerateError("name must be specified")
    spec = {}
    rl = populate_resource_list(hard)
    if rl is not None:
        spec["hard"] = rl
    sc = parse_scopes(scopes)
    if sc is not None:
        spec["scopes"] = sc
    return {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": name}, "spec": spec}


def parse_to_label_selector(selector: str) -> dict:
    """metav1.ParseToLabelSelector: equality terms become matchLabels, set terms
    matchExpressions; `!=`, `>` and `<` cannot be expressed."""
    from ..api.labels import SelectorError, parse_selector
    try:
        sel = parse_selector(selector)
    except SelectorError as e:
        raise GenerateError(f'couldn\'t parse the selector string "{selector}": {e}') from None
    ops = {"in": "In", "notin": "NotIn", "exists": "Exists", "!": "DoesNotExist"}
    out = {"matchLabels": {}, "matchExpressions": []}
    for r in getattr(sel, "reqs", []):
        if r.op in ("=", "=="):
            out["matchLabels"][r.key] = r.values[0]
        elif r.op in ops:
            e = {"key": r.key, "operator": ops[r.op]}
            if r.values:
                e["values"] = sorted(r.values)
            out["matchExpressions"].append(e)
        elif r.op in (">", "<", "gt", "lt"):
            raise GenerateError(f'"{r.op}" isn\'t supported in label selectors')
        else:
            raise GenerateError(f'"{r.op}" is not a valid label selector operator')
    return out


def _int_or_string(s: str):
    try:
        return int(s, 10)
    except ValueError:
        return s


def generate_pdb(name: str, selector: str = "", min_available: str = "", max_unavailable: str = "") -> dict:
    """PodDisruptionBudgetV2Generator."""
    if not name:
        raise GenerateError("name must be specified")
    if not selector:
        raise GenerateError("a selector must be specified")
    if not max_unavailable and not min_available:
        raise GenerateError("one of min-available or max-unavailable must be specified")
    if max_unavailable and min_available:
        raise GenerateError("min-available and max-unavailable cannot be both specified")
    spec = {"selector": parse_to_label_selector(selector)}
    if max_unavailable:
        spec["maxUnavailable"] = _int_or_string(max_unavailable)
    else:
        spec["minAvailable"] = _int_or_string(min_available)
    return {"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget", "metadata": {"name": name}, "spec": spec}


# ---------------------------------------------------- rolebinding.rbac.authorization.k8s.io/v1alpha1
RBAC_GROUP = "rbac.authorization.k8s.io"


def generate_role_binding(kind: str, name: str, role: str = "", cluster_role: str = "", users=(), groups=(),
                          service_accounts=()) -> dict:
    """RoleBindingGeneratorV1 / ClusterRoleBindingGeneratorV1: one role reference (a RoleBinding
    takes exactly one of --role/--clusterrole), subjects de-duplicated and sorted per kind,
    service accounts as <namespace>:<name>."""
    if not name:
        raise GenerateError("name must be specified")
    if kind == "ClusterRoleBinding":
        if not cluster_role:
            raise GenerateError("clusterrole must be specified")
        ref = {"apiGroup": RBAC_GROUP, "kind": "ClusterRole", "name": cluster_role}
    else:
        if bool(cluster_role) == bool(role):
            raise GenerateError("exactly one of clusterrole or role must be specified")
        ref = {"apiGroup": RBAC_GROUP, "kind": "Role", "name": role} if role else \
            {"apiGroup": RBAC_GROUP, "kind": "ClusterRole", "name": cluster_role}
    subjects = [{"kind": "User", "apiGroup": RBAC_GROUP, "name": u} for u in sorted(set(users or []))]
    subjects += [{"kind": "Group", "apiGroup": RBAC_GROUP, "name": g} for g in sorted(set(groups or []))]
    for sa in sorted(set(service_accounts or [])):
        tokens = sa.split(":")
        if len(tokens) != 2 or not tokens[1]:
            raise GenerateError("serviceaccount must be <namespace>:<name>")
        subjects.append({"kind": "ServiceAccount", "namespace": tokens[0], "name": tokens[1]})
    obj = {"apiVersion": f"{RBAC_GROUP}/v1", "kind": kind, "metadata": {"name": name}, "roleRef": ref}
    if subjects:
        obj["subjects"] = subjects
    return obj


# ----------------------------------------------------------------- create role / clusterrole
VALID_RESOURCE_VERBS = ("*", "get", "delete", "list", "create", "update", "patch", "watch", "proxy", "deletecollection", "use",
                        "bind", "impersonate")
SPECIAL_VERBS = {"use": {("extensions", "podsecuritypolicies")},
                 "bind": {(RBAC_GROUP, "roles"), (RBAC_GROUP, "clusterroles")},
                 "impersonate": {("", "users"), ("", "serviceaccounts"), ("", "groups"), ("authentication.k8s.io", "userextras")}}


def _dedup(xs):
    out = []
    for x in xs or []:
        if x not in out:
            out.append(x)
    return out


def _resource_for(resource: str, group: str) -> tuple[str, str]:
    """RESTMapper.ResourceFor: the plural and group the server serves (short and singular names
    resolve); unknown resources keep what was given."""
    from ..api.scheme import SCHEME
    ri = SCHEME.resolve(f"{resource}.{group}" if group else resource)
    return (ri.plural, ri.group) if ri is not None else (resource, group)


def generate_role(kind: str, name: str, verbs=(), resources=(), resource_names=(), non_resource_urls=()) -> dict:
    """create_role.go Complete/Validate/RunCreateRole (and create_clusterrole.go): verbs
    de-duplicated ("*" alone wins) and checked, `resource[.group][/subresource]` specifiers mapped
    to served groups, special verbs only on their resources, one rule per API group (sorted)
    carrying every verb and resource name."""
    if not name:
        raise GenerateError("name must be specified")
    vs = ["*"] if "*" in (verbs or []) else _dedup(verbs)
    if not vs:
        raise GenerateError("at least one verb must be specified")
    for v in vs:
        if v not in VALID_RESOURCE_VERBS:
            raise GenerateError(f"invalid verb: '{v}'")
    if not resources and not non_resource_urls:
        raise GenerateError("at least one resource must be specified")
    by_group: dict[str, list[str]] = {}
    for spec in resources or []:
        base, _, sub = spec.partition("/")
        res, _, group = base.partition(".")
        if not res:
            raise GenerateError("resource must be specified if apiGroup/subresource specified")
        res, group = _resource_for(res, group)
        for v in vs:
            if v in SPECIAL_VERBS and (group, res) not in SPECIAL_VERBS[v]:
                raise GenerateError(f"can not perform '{v}' on '{res}' in group '{group}'")
        full = f"{res}/{sub}" if sub else res
        if full not in by_group.setdefault(group, []):
            by_group[group].append(full)
    rules = []
    names = _dedup(resource_names)
    for g in sorted(by_group):
        rule = {"verbs": vs, "apiGroups": [g], "resources": by_group[g]}
        if names:
            rule["resourceNames"] = names
        rules.append(rule)
    if non_resource_urls:
        rules.append({"verbs": vs, "nonResourceURLs": list(non_resource_urls)})
    return {"apiVersion": f"{RBAC_GROUP}/v1", "kind": kind, "metadata": {"name": name}, "rules": rules}
