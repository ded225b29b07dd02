"""Validation for the API types of the reference release's other groups.

* networking.k8s.io/v1 NetworkPolicy — pkg/apis/networking/validation/validation.go
  (ValidateNetworkPolicySpec: pod selector, ports TCP/UDP + 1-65535 or IANA name, peers with
  exactly one of podSelector/namespaceSelector/ipBlock, ipBlock.except strictly inside cidr,
  policyTypes ⊆ {Ingress, Egress}).
* extensions/v1beta1 Ingress — pkg/apis/extensions/validation/validation.go ValidateIngress
  (backend or rules; host a DNS-1123 subdomain, not an IP, optional leading `*.`; HTTP paths
  absolute and valid regexes; backend serviceName DNS-1035 label + servicePort).
* extensions/v1beta1 PodSecurityPolicy — ValidatePodSecurityPolicySpec (runAsUser /
  seLinux / supplementalGroups / fsGroup strategies and ranges, volumes, host ports,
  capabilities not both allowed and required-drop, allowedHostPaths).
* settings.k8s.io/v1alpha1 PodPreset — pkg/apis/settings/validation (selector, env, envFrom,
  volumes, volumeMounts).
* admissionregistration.k8s.io/v1alpha1 InitializerConfiguration — pkg/apis/admissionregistration/
  validation (initializer names with ≥ 3 dot-separated segments, unique; rule groups/versions/
  resources non-empty, `*` alone).
* apiregistration.k8s.io/v1beta1 APIService — staging/src/k8s.io/kube-aggregator/pkg/apis/
  apiregistration/validation (name = <version>.<group>, priorities, service or local, caBundle
  unless insecureSkipTLSVerify).
"""
from __future__ import annotations

import ipaddress
import re

from .labels import SelectorError, is_dns1123_label, is_dns1123_subdomain, selector_from_label_selector
from .scheme import register_hooks
from .field import go_slice, go_value

_IANA_SVC = re.compile(r"^[a-z0-9]([a-z0-9-]*[a-z0-9])?$")


def _meta(obj, namespaced):
    from .validation import validate_object_meta
    return validate_object_meta(obj, namespaced)


def _selector(sel, path):
    try:
        selector_from_label_selector(sel or {})
        return []
    except (SelectorError, ValueError) as e:
        return [f"{path}: Invalid value: {e}"]


def _port(p, path, allow_name=True):
    if isinstance(p, int):
        return [] if 1 <= p <= 65535 else [f"{path}: Invalid value: {p}: must be between 1 and 65535, inclusive"]
    if isinstance(p, str) and allow_name:
        if p.isdigit():
            return _port(int(p), path)
        if len(p) > 15 or not _IANA_SVC.match(p) or "--" in p or not re.search("[a-z]", p):
            return [f"{path}: Invalid value: {go_value(p)}: must be a valid IANA service name"]
        return []
    return [f"{path}: Invalid value: {go_value(p)}"]


def _cidr(s, path):
    try:
        return ipaddress.ip_network(s, strict=False), []
    except ValueError:
        return None, [f"{path}: Invalid value: {go_value(s)}: must be a valid CIDR"]


# ----------------------------------------------------------------- NetworkPolicy
def _peers(peers, path):
    errs = []
    for i, p in enumerate(peers or []):
        pp = f"{path}[{i}]"
        n = sum(1 for k in ("podSelector", "namespaceSelector", "ipBlock") if p.get(k) is not None)
        if n != 1:
            errs.append(f"{pp}: Required value: must specify exactly one of podSelector, namespaceSelector or ipBlock")
            continue
        if p.get("podSelector") is not None:
            errs += _selector(p["podSelector"], f"{pp}.podSelector")
        if p.get("namespaceSelector") is not None:
            errs += _selector(p["namespaceSelector"], f"{pp}.namespaceSelector")
        if p.get("ipBlock") is not None:
            ib = p["ipBlock"]
            net, e = _cidr(ib.get("cidr", ""), f"{pp}.ipBlock.cidr")
            errs += e
            for j, ex in enumerate(ib.get("except") or []):
                sub, e = _cidr(ex, f"{pp}.ipBlock.except[{j}]")
                errs += e
                if net is not None and sub is not None and (sub.version != net.version or not sub.subnet_of(net)
                                                            or sub.prefixlen <= net.prefixlen):
                    errs.append(f"{pp}.ipBlock.except[{j}]: Invalid value: {go_value(ex)}: must be a strict subset of `cidr`")
    return errs


def _np_ports(ports, path):
    errs = []
    for i, p in enumerate(ports or []):
        if p.get("protocol", "TCP") not in ("TCP", "UDP"):
            errs.append(f"{path}[{i}].protocol: Unsupported value: {go_value(p.get('protocol'))}: supported values: \"TCP\", \"UDP\"")
        if p.get("port") is not None:
            errs += _port(p["port"], f"{path}[{i}].port")
    return errs


def validate_network_policy(np, old=None):
    errs = _meta(np, True)
    spec = np.get("spec") or {}
    errs += _selector(spec.get("podSelector") or {}, "spec.podSelector")
    for i, r in enumerate(spec.get("ingress") or []):
        errs += _np_ports(r.get("ports"), f"spec.ingress[{i}].ports") + _peers(r.get("from"), f"spec.ingress[{i}].from")
    for i, r in enumerate(spec.get("egress") or []):
        errs += _np_ports(r.get("ports"), f"spec.egress[{i}].ports") + _peers(r.get("to"), f"spec.egress[{i}].to")
    pts = spec.get("policyTypes") or []
    for i, t in enumerate(pts):
        if t not in ("Ingress", "Egress"):
            errs.append(f"spec.policyTypes[{i}]: Unsupported value: {go_value(t)}: supported values: \"Ingress\", \"Egress\"")
    if len(pts) > 2 or len(set(pts)) != len(pts):
        errs.append(f"spec.policyTypes: Invalid value: {go_slice('networking.PolicyType', pts)}: may not contain duplicates or more than 2 entries")
    return errs


def default_network_policy(np):
    """networking/v1 defaults: protocol TCP; policyTypes [Ingress] (+ Egress if egress rules)."""
    spec = np.setdefault("spec", {})
    for rules, k in ((spec.get("ingress") or [], "ports"), (spec.get("egress") or [], "ports")):
        for r in rules:
            for p in r.get(k) or []:
                p.setdefault("protocol", "TCP")
    if not spec.get("policyTypes"):
        spec["policyTypes"] = ["Ingress"] + (["Egress"] if spec.get("egress") else [])


# ----------------------------------------------------------------------- Ingress
def _backend(b, path):
    errs = []
    sn = b.get("serviceName", "")
    if not sn:
        errs.append(f"{path}.serviceName: Required value")
    elif not re.match(r"^[a-z]([-a-z0-9]*[a-z0-9])?$", sn) or len(sn) > 63:
        errs.append(f"{path}.serviceName: Invalid value: {go_value(sn)}: a DNS-1035 label")
    if b.get("servicePort") in (None, "", 0):
        errs.append(f"{path}.servicePort: Required value")
    else:
        errs += _port(b["servicePort"], f"{path}.servicePort")
    return errs


def validate_ingress(ing, old=None):
    errs = _meta(ing, True)
    spec = ing.get("spec") or {}
    if not spec.get("backend") and not spec.get("rules"):
        errs.append("spec: Invalid value: either `backend` or `rules` must be specified")
    if spec.get("backend"):
        errs += _backend(spec["backend"], "spec.backend")
    for i, r in enumerate(spec.get("rules") or []):
        host = r.get("host", "")
        if host:
            try:
                ipaddress.ip_address(host)
                errs.append(f"spec.rules[{i}].host: Invalid value: {go_value(host)}: must be a DNS name, not an IP address")
            except ValueError:
                h = host[2:] if host.startswith("*.") else host
                for e in is_dns1123_subdomain(h):
                    errs.append(f"spec.rules[{i}].host: Invalid value: {go_value(host)}: {e}")
        for j, p in enumerate(((r.get("http") or {}).get("paths")) or []):
            path = p.get("path", "")
            if path:
                if not path.startswith("/"):
                    errs.append(f"spec.rules[{i}].http.paths[{j}].path: Invalid value: {go_value(path)}: must be an absolute path")
                try:
                    re.compile(path)
                except re.error:
                    errs.append(f"spec.rules[{i}].http.paths[{j}].path: Invalid value: {go_value(path)}: must be a valid regex")
            errs += _backend(p.get("backend") or {}, f"spec.rules[{i}].http.paths[{j}].backend")
        if r.get("http") is not None and not (r["http"].get("paths")):
            errs.append(f"spec.rules[{i}].http.paths: Required value")
    for i, t in enumerate(spec.get("tls") or []):
        for j, h in enumerate(t.get("hosts") or []):
            for e in is_dns1123_subdomain(h[2:] if h.startswith("*.") else h):
                errs.append(f"spec.tls[{i}].hosts[{j}]: Invalid value: {go_value(h)}: {e}")
    return errs


# ------------------------------------------------------------- PodSecurityPolicy
FS_TYPES = ("*", "azureFile", "flocker", "flexVolume", "hostPath", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore",
            "gitRepo", "secret", "nfs", "iscsi", "glusterfs", "persistentVolumeClaim", "rbd", "cinder", "cephFS",
            "downwardAPI", "fc", "configMap", "vsphereVolume", "quobyte", "azureDisk", "photonPersistentDisk",
            "projected", "portworxVolume", "scaleIO", "storageos", "none")


def _id_ranges(ranges, path):
    errs = []
    for i, r in enumerate(ranges or []):
        lo, hi = r.get("min", 0), r.get("max", 0)
        if lo < 0 or hi < 0:
            errs.append(f"{path}[{i}]: Invalid value: ids must be non-negative")
        if lo > hi:
            errs.append(f"{path}[{i}]: Invalid value: min ({lo}) is greater than max ({hi})")
    return errs


def validate_psp(psp, old=None):
    errs = _meta(psp, False)
    spec = psp.get("spec") or {}
    ru = spec.get("runAsUser") or {}
    if ru.get("rule") not in ("MustRunAs", "MustRunAsNonRoot", "RunAsAny"):
        errs.append(f"spec.runAsUser.rule: Unsupported value: {go_value(ru.get('rule'))}")
    if ru.get("rule") == "MustRunAs" and not ru.get("ranges"):
        errs.append("spec.runAsUser.ranges: Invalid value: must provide at least one range")
    errs += _id_ranges(ru.get("ranges"), "spec.runAsUser.ranges")
    se = spec.get("seLinux") or {}
    if se.get("rule") not in ("MustRunAs", "RunAsAny"):
        errs.append(f"spec.seLinux.rule: Unsupported value: {go_value(se.get('rule'))}")
    for f in ("supplementalGroups", "fsGroup"):
        g = spec.get(f) or {}
        if g.get("rule") not in ("MustRunAs", "RunAsAny"):
            errs.append(f"spec.{f}.rule: Unsupported value: {go_value(g.get('rule'))}")
        errs += _id_ranges(g.get("ranges"), f"spec.{f}.ranges")
    for i, v in enumerate(spec.get("volumes") or []):
        if v not in FS_TYPES:
            errs.append(f"spec.volumes[{i}]: Unsupported value: {go_value(v)}")
    for i, hp in enumerate(spec.get("hostPorts") or []):
        if hp.get("min", 0) > hp.get("max", 0) or not (0 <= hp.get("min", 0) <= 65535) or not (0 <= hp.get("max", 0) <= 65535):
            errs.append(f"spec.hostPorts[{i}]: Invalid value: min/max must be 0-65535 with min ≤ max")
    both = set(spec.get("allowedCapabilities") or []) & set(spec.get("requiredDropCapabilities") or [])
    both |= set(spec.get("defaultAddCapabilities") or []) & set(spec.get("requiredDropCapabilities") or [])
    if both:
        errs.append(f"spec.requiredDropCapabilities: Invalid value: {go_slice('core.Capability', sorted(both))}: capability is both added and dropped")
    for i, hp in enumerate(spec.get("allowedHostPaths") or []):
        if not hp.get("pathPrefix"):
            errs.append(f"spec.allowedHostPaths[{i}].pathPrefix: Required value")
    if spec.get("allowPrivilegeEscalation") is False and spec.get("defaultAllowPrivilegeEscalation"):
        errs.append("spec.defaultAllowPrivilegeEscalation: Invalid value: cannot default to true when allowPrivilegeEscalation is false")
    return errs


# --------------------------------------------------------------------- PodPreset
def validate_pod_preset(pp, old=None):
    errs = _meta(pp, True)
    spec = pp.get("spec") or {}
    errs += _selector(spec.get("selector") or {}, "spec.selector")
    for i, e in enumerate(spec.get("env") or []):
        if not e.get("name"):
            errs.append(f"spec.env[{i}].name: Required value")
    names = set()
    for i, v in enumerate(spec.get("volumes") or []):
        n = v.get("name", "")
        errs += [f"spec.volumes[{i}].name: Invalid value: {go_value(n)}: {e}" for e in is_dns1123_label(n)]
        if n in names:
            errs.append(f"spec.volumes[{i}].name: Duplicate value: {go_value(n)}")
        names.add(n)
    for i, vm in enumerate(spec.get("volumeMounts") or []):
        if not vm.get("name") or not vm.get("mountPath"):
            errs.append(f"spec.volumeMounts[{i}]: Required value: name and mountPath")
    if not any(spec.get(k) for k in ("env", "envFrom", "volumes", "volumeMounts")):
        errs.append("spec: Required value: must specify at least one of env, envFrom, volumes or volumeMounts")
    return errs


# ---------------------------------------------------- InitializerConfiguration
def validate_initializer_configuration(ic, old=None):
    errs = _meta(ic, False)
    seen = set()
    for i, ini in enumerate(ic.get("initializers") or []):
        n = ini.get("name", "")
        if len(n.split(".")) < 3:
            errs.append(f"initializers[{i}].name: Invalid value: {go_value(n)}: should be a domain with at least three segments separated by dots")
        errs += [f"initializers[{i}].name: Invalid value: {go_value(n)}: {e}" for e in is_dns1123_subdomain(n)]
        if n in seen:
            errs.append(f"initializers[{i}].name: Duplicate value: {go_value(n)}")
        seen.add(n)
        for j, r in enumerate(ini.get("rules") or []):
            for f in ("apiGroups", "apiVersions", "resources"):
                vals = r.get(f) or []
                if not vals:
                    errs.append(f"initializers[{i}].rules[{j}].{f}: Required value")
                elif "*" in vals and len(vals) > 1:
                    errs.append(f"initializers[{i}].rules[{j}].{f}: Invalid value: if '*' is present, must not specify other values")
            if any("/" in x for x in r.get("resources") or []):
                errs.append(f"initializers[{i}].rules[{j}].resources: Invalid value: must not specify subresources")
    return errs


# --------------------------------------------------------------------- APIService
def validate_apiservice(a, old=None):
    """Names are path segments (core group: `v1.`), not DNS subdomains."""
    from .validation import validate_object_meta
    errs = validate_object_meta(a, False, name_fn=lambda n: [] if n not in (".", "..") and "/" not in n and "%" not in n
                                else ["may not contain '/' or '%' or be '.' or '..'"])
    spec = a.get("spec") or {}
    name, group, version = (a.get("metadata") or {}).get("name", ""), spec.get("group", ""), spec.get("version", "")
    want = f"{version}.{group}"
    if name != want:
        errs.append(f"metadata.name: Invalid value: {go_value(name)}: must be `spec.version+\".\"+spec.group`: {want!r}")
    if not version:
        errs.append("spec.version: Required value")
    elif is_dns1123_label(version):
        errs.append(f"spec.version: Invalid value: {go_value(version)}: a DNS-1123 label")
    if group and is_dns1123_subdomain(group):
        errs.append(f"spec.group: Invalid value: {go_value(group)}: a DNS-1123 subdomain")
    gp, vp = spec.get("groupPriorityMinimum", 0), spec.get("versionPriority", 0)
    if not (0 < gp <= 20000):
        errs.append(f"spec.groupPriorityMinimum: Invalid value: {gp}: must be positive and less than 20000")
    if not (0 < vp <= 1000):
        errs.append(f"spec.versionPriority: Invalid value: {vp}: must be positive and less than 1000")
    svc = spec.get("service")
    if svc is not None:
        if not svc.get("namespace") or not svc.get("name"):
            errs.append("spec.service: Required value: namespace and name")
        if not spec.get("insecureSkipTLSVerify") and not spec.get("caBundle"):
            errs.append("spec.caBundle: Required value: if insecureSkipTLSVerify is not true")
    elif spec.get("caBundle") or spec.get("insecureSkipTLSVerify"):
        errs.append("spec.caBundle: Invalid value: local APIServices may not have a caBundle or insecureSkipTLSVerify")
    return errs


register_hooks("NetworkPolicy", "networking.k8s.io/v1", defaulter=default_network_policy, validator=validate_network_policy)
register_hooks("Ingress", "extensions/v1beta1", validator=validate_ingress)
register_hooks("PodSecurityPolicy", "extensions/v1beta1", validator=validate_psp)
register_hooks("PodPreset", "settings.k8s.io/v1alpha1", validator=validate_pod_preset)
register_hooks("InitializerConfiguration", "admissionregistration.k8s.io/v1alpha1", validator=validate_initializer_configuration)
register_hooks("APIService", "apiregistration.k8s.io/v1beta1", validator=validate_apiservice)
