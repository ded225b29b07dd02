"""Validation of the core kinds and of the pod spec, field by field.

Reference: pkg/apis/core/validation/validation.go — ValidateVolumes / validateVolumeSource
(:368-690) and every volume source validator (:692-1441), ValidatePersistentVolume (:1453),
ValidatePersistentVolumeClaim(+Update) (:1731-1818), validateContainerPorts (:1843),
ValidateVolumeMounts / ValidateVolumeDevices (:2146-2241), validateProbe (:2243),
validateHandler and its actions (:2318-2396), validateLifecycle (:2398), validatePullPolicy
(:2411), validateInitContainers (:2426), validateContainers (:2485), validateRestartPolicy /
validateDNSPolicy / validatePodDNSConfig / validateHostNetwork / validateImagePullSecrets
(:2548-2672), validateAffinity and the node/pod (anti-)affinity term validators (:2675,
:2990-3169), ValidateTolerations (:2764), ValidateHostAliases (:2750), ValidatePod (:2844),
ValidatePodSpec (:2879), ValidatePodSecurityContext (:3271), ValidatePodUpdate (:3319),
ValidatePodTemplate (:3432), ValidateReplicationController (:3727-3827),
ValidateReadOnlyPersistentDisks (:3829), the resource name validators (:4047-4135),
ValidateLimitRange (:4138), ValidateServiceAccount (:4266), ValidateSecret (:4279),
ValidateConfigMap (:4376), ValidateResourceRequirements (:4412), ValidateResourceQuota(+Update)
(:4457-4591), ValidateNamespace (:4594), ValidateEndpoints (:4698-4795),
ValidateSecurityContext (:4806); pkg/apis/core/helper/helpers.go for the standard resource
sets; apimachinery util/validation for the name/port/IP checks.

Objects arrive as v1 JSON after defaulting (the registry defaults before it validates), so
the defaulted fields the internal types require — imagePullPolicy, terminationMessagePolicy,
restartPolicy, dnsPolicy, port protocols — are required here too. Messages are rendered the
way field.Error renders them (`<path>: <type>: <value>: <detail>`).
"""
from __future__ import annotations

import ipaddress
import json
import posixpath
import re

from .field import go_value as gv
from .labels import (SelectorError, is_dns1123_label, is_dns1123_subdomain, is_qualified_name,
                     is_valid_label_value, selector_from_label_selector)
from .quantity import Quantity, QuantityError
from ..utils.features import FeatureGate

# The apiserver's feature gates for validation. amdkube's apiserver turns on the alpha storage
# and DNS features its kubelet implements (local PVs, block volumes, mount propagation, custom pod
# DNS, volume expansion, CSI, local-storage isolation, hugepages); the reference's 1.9 defaults
# leave them off and its tests flip them per case — tests/test_validation_parity.py does the same.
GATES = FeatureGate({"PersistentLocalVolumes": True, "BlockVolume": True, "MountPropagation": True,
                     "CustomPodDNS": True, "ExpandPersistentVolumes": True, "CSIPersistentVolume": True,
                     "LocalStorageCapacityIsolation": True, "HugePages": True})

# ============================================================== field errors
NEGATIVE = "must be greater than or equal to 0"
NOT_POSITIVE = "must be greater than zero"
NOT_INTEGER = "must be an integer"
IMMUTABLE = "field is immutable"
FILE_MODE = "must be a number between 0 and 0777 (octal), both inclusive"
INVALID_QUOTA_RESOURCE = "must be a standard resource for quota"


def inclusive_range(lo, hi) -> str:
    return f"must be between {lo} and {hi}, inclusive"


PD_PARTITION = inclusive_range(1, 255)
MAX_INT32 = 2 ** 31 - 1


def required(p, d=""):
    return f"{p}: Required value" + (f": {d}" if d else "")


def invalid(p, v, d=""):
    return f"{p}: Invalid value: {gv(v)}" + (f": {d}" if d else "")


def forbidden(p, d=""):
    return f"{p}: Forbidden" + (f": {d}" if d else "")


def duplicate(p, v):
    return f"{p}: Duplicate value: {gv(v)}"


def not_found(p, v):
    return f"{p}: Not found: {gv(v)}"


def not_supported(p, v, valid):
    d = ("supported values: " + ", ".join(json.dumps(x) for x in valid)) if valid else ""
    return f"{p}: Unsupported value: {gv(v)}" + (f": {d}" if d else "")


def too_long(p, n):
    return f"{p}: Too long: must have at most {n} characters"


def _go(v) -> str:
    """A compound bad value, rendered compactly (the reference prints Go's %#v)."""
    from .field import GoRepr
    return GoRepr(json.dumps(v, sort_keys=True, separators=(",", ":")))


# ============================================================== primitive checks
_PORT_NAME_CHARS = re.compile(r"^[-a-z0-9]+$")
_HTTP_HEADER = re.compile(r"^[-A-Za-z0-9]+$")
_PERCENT = re.compile(r"^[0-9]+%$")
_DNS1035 = re.compile(r"^[a-z]([-a-z0-9]*[a-z0-9])?$")
_SYSCTL = re.compile(r"^([a-z0-9]([-_a-z0-9]*[a-z0-9])?\.)*[a-z0-9]([-_a-z0-9]*[a-z0-9])?$")
_IQN = re.compile(r"iqn\.\d{4}-\d{2}\.([A-Za-z0-9-.]+)(:[^,;*&$|\s]+)$")
_EUI = re.compile(r"^eui.[A-Za-z0-9]{16}$")
_NAA = re.compile(r"^naa.[A-Za-z0-9]{32}$")


def is_int(v) -> bool:
    return isinstance(v, int) and not isinstance(v, bool)


def is_valid_port_num(port) -> list[str]:
    return [] if is_int(port) and 1 <= port <= 65535 else [inclusive_range(1, 65535)]


def is_valid_port_name(port: str) -> list[str]:
    errs = []
    if len(port) > 15:
        errs.append("must be no more than 15 characters")
    if not _PORT_NAME_CHARS.match(port):
        errs.append("must contain only alpha-numeric characters (a-z, 0-9), and hyphens (-)")
    if not re.search(r"[a-z]", port):
        errs.append("must contain at least one letter or number (a-z, 0-9)")
    if "--" in port:
        errs.append("must not contain consecutive hyphens")
    if port and (port[0] == "-" or port[-1] == "-"):
        errs.append("must not begin or end with a hyphen")
    return errs


def is_http_header_name(v: str) -> list[str]:
    if _HTTP_HEADER.match(v or ""):
        return []
    return ["a valid HTTP header must consist of alphanumeric characters or '-' (e.g. 'X-Header-Name', "
            "regex used for validation is '[-A-Za-z0-9]+')"]


def parse_ip(v):
    try:
        return ipaddress.ip_address(v)
    except (ValueError, TypeError):
        return None


def is_valid_ip(v) -> list[str]:
    return [] if parse_ip(v) is not None else ["must be a valid IP address, (e.g. 10.9.8.7)"]


def is_valid_id(v) -> list[str]:
    return [] if is_int(v) and 0 <= v <= MAX_INT32 else [inclusive_range(0, MAX_INT32)]


def is_valid_percent(v: str) -> list[str]:
    if _PERCENT.match(v or ""):
        return []
    return ["a valid percent string must be a numeric string followed by an ending '%' (e.g. '1%',  or '93%', "
            "regex used for validation is '[0-9]+%')"]


def is_dns1035_label(v: str) -> list[str]:
    errs = []
    if len(v) > 63:
        errs.append("must be no more than 63 characters")
    if not _DNS1035.match(v or ""):
        errs.append("a DNS-1035 label must consist of lower case alphanumeric characters or '-', start with an "
                    "alphabetic character, and end with an alphanumeric character")
    return errs


def is_valid_path_segment_name(v: str) -> list[str]:
    """apimachinery api/validation/path IsValidPathSegmentName."""
    if v in (".", ".."):
        return [f"may not be '{v}'"]
    return [f"may not contain '{c}'" for c in ("/", "%") if c in v]


def nonneg(v, p) -> list[str]:
    return [invalid(p, v, NEGATIVE)] if is_int(v) and v < 0 else []


def dns_label(v, p) -> list[str]:
    return [invalid(p, v, m) for m in is_dns1123_label(v)]


def dns_subdomain(v, p) -> list[str]:
    return [invalid(p, v, m) for m in is_dns1123_subdomain(v)]


def label_name(k, p) -> list[str]:
    return [invalid(p, k, m) for m in is_qualified_name(k)]


def validate_labels(labels, p) -> list[str]:
    errs = []
    for k, v in (labels or {}).items():
        errs += label_name(k, p)
        errs += [invalid(p, v, m) for m in is_valid_label_value(str(v))]
    return errs


def validate_label_selector(sel, p) -> list[str]:
    """unversioned ValidateLabelSelector: In/NotIn need values, Exists/DoesNotExist take none."""
    if sel is None:
        return []
    errs = []
    for i, r in enumerate(sel.get("matchExpressions") or []):
        rp = f"{p}.matchExpressions[{i}]"
        op, vals = r.get("operator"), r.get("values") or []
        if op in ("In", "NotIn"):
            if not vals:
                errs.append(required(f"{rp}.values", "must be specified when `operator` is 'In' or 'NotIn'"))
        elif op in ("Exists", "DoesNotExist"):
            if vals:
                errs.append(forbidden(f"{rp}.values", "may not be specified when `operator` is 'Exists' or 'DoesNotExist'"))
        else:
            errs.append(invalid(f"{rp}.operator", op, "not a valid selector operator"))
        errs += label_name(r.get("key") or "", f"{rp}.key")
    errs += validate_labels(sel.get("matchLabels"), f"{p}.matchLabels")
    return errs


def _selector(sel):
    try:
        return selector_from_label_selector(sel)
    except SelectorError:
        return None


def _q(v):
    try:
        return Quantity(v)
    except (QuantityError, TypeError, ValueError):
        return None


# ============================================================== resources
STANDARD_CONTAINER = {"cpu", "memory", "ephemeral-storage"}
STANDARD_QUOTA = {"cpu", "memory", "ephemeral-storage", "requests.cpu", "requests.memory", "requests.storage",
                  "requests.ephemeral-storage", "limits.cpu", "limits.memory", "limits.ephemeral-storage", "pods",
                  "resourcequotas", "services", "replicationcontrollers", "secrets", "persistentvolumeclaims",
                  "configmaps", "services.nodeports", "services.loadbalancers"}
STANDARD_RESOURCES = STANDARD_QUOTA | {"storage"}
INTEGER_RESOURCES = {"pods", "resourcequotas", "services", "replicationcontrollers", "secrets", "configmaps",
                     "persistentvolumeclaims", "services.nodeports", "services.loadbalancers"}
# overcommitBlacklist: the reference's nvidia GPU plus this fork's AMD GPU resource
NO_OVERCOMMIT = {"alpha.kubernetes.io/nvidia-gpu", "alpha.kubernetes.io/amd-gpu"}
QUOTA_SCOPES = ("Terminating", "NotTerminating", "BestEffort", "NotBestEffort")
LIMIT_TYPES = ("Pod", "Container", "PersistentVolumeClaim")


def _hugepages(name: str) -> bool:
    return name.startswith("hugepages-")


def _quota_hugepages(name: str) -> bool:
    return name.startswith("hugepages-") or name.startswith("requests.hugepages-")


def is_default_namespace_resource(name: str) -> bool:
    return "/" not in name or "kubernetes.io/" in name


def is_extended_resource(name: str) -> bool:
    return not is_default_namespace_resource(name)


def is_integer_resource(name: str) -> bool:
    return name in INTEGER_RESOURCES or is_extended_resource(name)


def overcommit_allowed(name: str) -> bool:
    return is_default_namespace_resource(name) and not _hugepages(name) and name not in NO_OVERCOMMIT


def validate_resource_name(v, p) -> list[str]:
    errs = [invalid(p, v, m) for m in is_qualified_name(v)]
    if errs:
        return errs
    if "/" not in v and not (v in STANDARD_RESOURCES or _quota_hugepages(v)):
        return [invalid(p, v, "must be a standard resource type or fully qualified")]
    return []


def validate_container_resource_name(v, p) -> list[str]:
    errs = validate_resource_name(v, p)
    if "/" not in v and not (v in STANDARD_CONTAINER or _hugepages(v)):
        errs.append(invalid(p, v, "must be a standard resource for containers"))
    return errs


def validate_quota_resource_name(v, p) -> list[str]:
    errs = validate_resource_name(v, p)
    if "/" not in v and not (v in STANDARD_QUOTA or _quota_hugepages(v)):
        errs.append(invalid(p, v, INVALID_QUOTA_RESOURCE))
    return errs


def validate_quantity_value(resource, value, p) -> list[str]:
    """ValidateResourceQuantityValue: non-negative; integer resources whole."""
    q = _q(value)
    if q is None:
        return [invalid(p, value, "quantities must match the regular expression "
                                  "'^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$'")]
    errs = [invalid(p, str(q), NEGATIVE)] if q.as_fraction() < 0 else []
    if is_integer_resource(resource) and q.milli_value() % 1000 != 0:
        errs.append(invalid(p, str(q), NOT_INTEGER))
    return errs


def validate_positive_quantity(value, p) -> list[str]:
    q = _q(value)
    if q is not None and q.as_fraction() <= 0:
        return [invalid(p, str(q), NOT_POSITIVE)]
    return []


def validate_basic_resource(value, p) -> list[str]:
    q = _q(value)
    if q is not None and q.value() < 0:
        return [invalid(p, q.value(), "must be a valid resource quantity")]
    return []


def validate_resource_requirements(res, p) -> list[str]:
    errs = []
    lim, req = (res or {}).get("limits") or {}, (res or {}).get("requests") or {}
    for k, v in lim.items():
        fp = f"{p}.limits[{k}]"
        errs += validate_container_resource_name(k, fp)
        errs += validate_quantity_value(k, v, fp)
    for k, v in req.items():
        fp = f"{p}.requests[{k}]"
        errs += validate_container_resource_name(k, fp)
        errs += validate_quantity_value(k, v, fp)
        qr, ql = _q(v), _q(lim.get(k)) if k in lim else None
        if k in lim and qr is not None and ql is not None:
            if qr != ql and not overcommit_allowed(k):
                errs.append(invalid(f"{p}.requests", str(qr), f"must be equal to {k} limit"))
            elif qr.as_fraction() > ql.as_fraction():
                errs.append(invalid(f"{p}.requests", str(qr), f"must be less than or equal to {k} limit"))
        elif k == "alpha.kubernetes.io/nvidia-gpu" and qr is not None:
            errs.append(invalid(f"{p}.requests", str(qr), f"must be equal to {k} request"))
    return errs


# ============================================================== volumes
VOLUME_SOURCES = ("emptyDir", "hostPath", "gitRepo", "gcePersistentDisk", "awsElasticBlockStore", "secret", "nfs",
                  "iscsi", "glusterfs", "flocker", "persistentVolumeClaim", "rbd", "cinder", "cephfs", "quobyte",
                  "downwardAPI", "fc", "flexVolume", "configMap", "azureFile", "vsphereVolume",
                  "photonPersistentDisk", "portworxVolume", "azureDisk", "storageos", "projected", "scaleIO")
# the child name validateVolumeSource reports a second source under (its own spellings)
_DUP_NAME = {"cephfs": "cephFS", "downwardAPI": "downwarAPI"}
HOST_PATH_TYPES = ("", "DirectoryOrCreate", "Directory", "FileOrCreate", "File", "Socket", "CharDevice", "BlockDevice")


def validate_path_no_backsteps(path, p) -> list[str]:
    return [invalid(p, path, "must not contain '..'")] if ".." in str(path).split("/") else []


def validate_local_descending_path(path, p) -> list[str]:
    errs = [invalid(p, path, "must be a relative path")] if posixpath.isabs(path or "") else []
    return errs + validate_path_no_backsteps(path, p)


def validate_local_non_reserved_path(path, p) -> list[str]:
    errs = validate_local_descending_path(path, p)
    if (path or "").startswith("..") and not path.startswith("../"):
        errs.append(invalid(p, path, "must not start with '..'"))
    return errs


def _mode(m, p) -> list[str]:
    return [invalid(p, m, FILE_MODE)] if m is not None and (not is_int(m) or m > 0o777 or m < 0) else []


def validate_key_to_path(kp, p) -> list[str]:
    errs = []
    if not kp.get("key"):
        errs.append(required(f"{p}.key"))
    if not kp.get("path"):
        errs.append(required(f"{p}.path"))
    errs += validate_local_non_reserved_path(kp.get("path") or "", f"{p}.path")
    return errs + _mode(kp.get("mode"), f"{p}.mode")


VOLUME_FIELD_PATHS = ("metadata.name", "metadata.namespace", "metadata.labels", "metadata.annotations", "metadata.uid")
RESOURCE_FIELD_PATHS = ("limits.cpu", "limits.memory", "limits.ephemeral-storage", "requests.cpu", "requests.memory",
                        "requests.ephemeral-storage")


def validate_downward_api_file(f, p) -> list[str]:
    from .validation import validate_object_field_selector
    errs = []
    if not f.get("path"):
        errs.append(required(f"{p}.path"))
    errs += validate_local_non_reserved_path(f.get("path") or "", f"{p}.path")
    if f.get("fieldRef") is not None:
        errs += validate_object_field_selector(f["fieldRef"], VOLUME_FIELD_PATHS, f"{p}.fieldRef")
        if f.get("resourceFieldRef") is not None:
            errs.append(invalid(p, "resource", "fieldRef and resourceFieldRef can not be specified simultaneously"))
    elif f.get("resourceFieldRef") is not None:
        rf = f["resourceFieldRef"]
        if not rf.get("containerName"):
            errs.append(required(f"{p}.resourceFieldRef.containerName"))
        res = rf.get("resource") or ""
        if not res:
            errs.append(required(f"{p}.resourceFieldRef.resource"))
        elif res not in RESOURCE_FIELD_PATHS:
            errs.append(not_supported(f"{p}.resourceFieldRef.resource", res, sorted(RESOURCE_FIELD_PATHS)))
    else:
        errs.append(required(p, "one of fieldRef and resourceFieldRef is required"))
    return errs + _mode(f.get("mode"), f"{p}.mode")


def _iscsi(s, p, pv: bool) -> list[str]:
    errs = []
    if not s.get("targetPortal"):
        errs.append(required(f"{p}.targetPortal"))
    iqn = s.get("iqn") or ""
    if not iqn:
        errs.append(required(f"{p}.iqn"))
    elif not iqn.startswith(("iqn", "eui", "naa")):
        errs.append(invalid(f"{p}.iqn", iqn, "must be valid format" if pv else
                            "must be valid format starting with iqn, eui, or naa"))
    elif (iqn.startswith("iqn") and not _IQN.search(iqn)) or (iqn.startswith("eui") and not _EUI.search(iqn)) \
            or (iqn.startswith("naa") and not _NAA.search(iqn)):
        errs.append(invalid(f"{p}.iqn", iqn, "must be valid format"))
    lun = s.get("lun", 0)
    if not is_int(lun) or lun < 0 or lun > 255:
        errs.append(invalid(f"{p}.lun", lun, inclusive_range(0, 255)))
    if (s.get("chapAuthDiscovery") or s.get("chapAuthSession")) and s.get("secretRef") is None:
        errs.append(required(f"{p}.secretRef"))
    if pv and s.get("secretRef") is not None and not (s["secretRef"] or {}).get("name"):
        errs.append(required(f"{p}.secretRef.name"))
    ini = s.get("initiatorName")
    if ini is not None:
        if not ini.startswith(("iqn", "eui", "naa")):
            errs.append(invalid(f"{p}.initiatorname", ini, "must be valid format" if pv else
                                "must be valid format starting with iqn, eui, or naa"))
        if (ini.startswith("iqn") and not _IQN.search(ini)) or (ini.startswith("eui") and not _EUI.search(ini)) \
                or (ini.startswith("naa") and not _NAA.search(ini)):
            errs.append(invalid(f"{p}.initiatorname", ini, "must be valid format"))
    return errs


def _need(s, p, *names) -> list[str]:
    return [required(f"{p}.{n}") for n in names if not s.get(n)]


def validate_source(kind: str, s: dict, p: str, pv: bool = False) -> list[str]:
    """One volume source (the per-type validate*VolumeSource functions)."""
    s = s if isinstance(s, dict) else {}
    if kind == "emptyDir":
        lim = s.get("sizeLimit")
        if not GATES("LocalStorageCapacityIsolation"):
            if lim is not None and (_q(lim) is None or _q(lim).as_fraction() != 0):
                return [forbidden(f"{p}.sizeLimit", "SizeLimit field disabled by feature-gate for EmptyDir volumes")]
        elif lim is not None and (_q(lim) is None or _q(lim).as_fraction() < 0):
            return [forbidden(f"{p}.sizeLimit", "SizeLimit field must be a valid resource quantity")]
        if not GATES("HugePages") and s.get("medium") == "HugePages":
            return [forbidden(f"{p}.medium", "HugePages medium is disabled by feature-gate for EmptyDir volumes")]
        return []
    if kind in ("hostPath", "local"):
        if not s.get("path"):
            return [required(f"{p}.path")]
        errs = validate_path_no_backsteps(s["path"], f"{p}.path")
        if kind == "hostPath" and s.get("type") is not None and s["type"] not in HOST_PATH_TYPES:
            errs.append(not_supported(f"{p}.type", s["type"], sorted(HOST_PATH_TYPES)))
        return errs
    if kind == "gitRepo":
        return _need(s, p, "repository") + validate_local_descending_path(s.get("directory") or "", f"{p}.directory")
    if kind == "gcePersistentDisk":
        errs = _need(s, p.replace("gcePersistentDisk", "persistentDisk"), "pdName")
        part = s.get("partition", 0)
        if not is_int(part) or part < 0 or part > 255:
            errs.append(invalid(f"{p.replace('gcePersistentDisk', 'persistentDisk')}.partition", part, PD_PARTITION))
        return errs
    if kind == "awsElasticBlockStore":
        errs = _need(s, p, "volumeID")
        part = s.get("partition", 0)
        if not is_int(part) or part < 0 or part > 255:
            errs.append(invalid(f"{p}.partition", part, PD_PARTITION))
        return errs
    if kind == "secret":
        errs = _need(s, p, "secretName") + _mode(s.get("defaultMode"), f"{p}.defaultMode")
        for i, kp in enumerate(s.get("items") or []):
            errs += validate_key_to_path(kp, f"{p}.items[{i}]")
        return errs
    if kind == "configMap":
        errs = _need(s, p, "name") + _mode(s.get("defaultMode"), f"{p}.defaultMode")
        for i, kp in enumerate(s.get("items") or []):
            errs += validate_key_to_path(kp, f"{p}.items[{i}]")
        return errs
    if kind == "nfs":
        errs = _need(s, p, "server", "path")
        if not posixpath.isabs(s.get("path") or ""):
            errs.append(invalid(f"{p}.path", s.get("path") or "", "must be an absolute path"))
        return errs
    if kind == "iscsi":
        return _iscsi(s, p, pv)
    if kind == "glusterfs":
        return _need(s, p, "endpoints", "path")
    if kind == "flocker":
        n, u = s.get("datasetName") or "", s.get("datasetUUID") or ""
        errs = []
        if not n and not u:
            errs.append(required(p, "one of datasetName and datasetUUID is required"))
        if n and u:
            errs.append(invalid(p, "resource", "datasetName and datasetUUID can not be specified simultaneously"))
        if "/" in n:
            errs.append(invalid(f"{p}.datasetName", n, "must not contain '/'"))
        return errs
    if kind == "persistentVolumeClaim":
        return _need(s, p, "claimName")
    if kind == "rbd":
        return _need(s, p, "monitors", "image")
    if kind == "cinder":
        return _need(s, p, "volumeID")
    if kind == "cephfs":
        return _need(s, p, "monitors")
    if kind == "quobyte":
        errs = []
        reg = s.get("registry") or ""
        if not reg:
            errs.append(required(f"{p}.registry", "must be a host:port pair or multiple pairs separated by commas"))
        else:
            for hp in reg.split(","):
                host, sep, port = hp.rpartition(":")
                if not sep or not port.isdigit():
                    errs.append(invalid(f"{p}.registry", reg, "must be a host:port pair or multiple pairs separated by commas"))
        return errs + _need(s, p, "volume")
    if kind == "downwardAPI":
        errs = _mode(s.get("defaultMode"), f"{p}.defaultMode")
        for f in s.get("items") or []:
            errs += validate_downward_api_file(f, p)
        return errs
    if kind == "fc":
        errs = []
        wwns, wwids = s.get("targetWWNs") or [], s.get("wwids") or []
        if not wwns and not wwids:
            errs.append(required(f"{p}.targetWWNs", "must specify either targetWWNs or wwids, but not both"))
        if wwns and wwids:
            errs.append(invalid(f"{p}.targetWWNs", _go(wwns), "targetWWNs and wwids can not be specified simultaneously"))
        if wwns:
            lun = s.get("lun")
            if lun is None:
                errs.append(required(f"{p}.lun", "lun is required if targetWWNs is specified"))
            elif not is_int(lun) or lun < 0 or lun > 255:
                errs.append(invalid(f"{p}.lun", lun, inclusive_range(0, 255)))
        return errs
    if kind == "flexVolume":
        errs = _need(s, p, "driver")
        for k in s.get("options") or {}:
            ns = k.split("/", 1)[0] if "/" in k else k
            norm = "." + ns.lower()
            if norm.endswith(".kubernetes.io") or norm.endswith(".k8s.io"):
                errs.append(invalid(f"{p}.options[{k}]", k, "kubernetes.io and k8s.io namespaces are reserved"))
        return errs
    if kind == "azureFile":
        errs = _need(s, p, "secretName", "shareName")
        if pv and s.get("secretNamespace") is not None and not s["secretNamespace"]:
            errs.append(required(f"{p}.secretNamespace"))
        return errs
    if kind == "azureDisk":
        errs = _need(s, p, "diskName", "diskURI")
        cm, k, uri = s.get("cachingMode"), s.get("kind"), s.get("diskURI") or ""
        if cm is not None and cm not in ("None", "ReadOnly", "ReadWrite"):
            errs.append(not_supported(f"{p}.cachingMode", cm, ["None", "ReadOnly", "ReadWrite"]))
        if k is not None and k not in ("Shared", "Dedicated", "Managed"):
            errs.append(not_supported(f"{p}.kind", k, ["Dedicated", "Managed", "Shared"]))
        if k == "Managed" and not uri.startswith("/subscriptions/"):
            errs.append(not_supported(f"{p}.diskURI", uri, ["/subscriptions/{sub-id}/resourcegroups/{group-name}/providers/microsoft.compute/disks/{disk-id}"]))
        if k is not None and k != "Managed" and not uri.startswith("https://"):
            errs.append(not_supported(f"{p}.diskURI", uri, ["https://{account-name}.blob.core.windows.net/{container-name}/{disk-name}.vhd"]))
        return errs
    if kind == "vsphereVolume":
        return _need(s, p, "volumePath")
    if kind == "photonPersistentDisk":
        return _need(s, p, "pdID")
    if kind == "portworxVolume":
        return _need(s, p, "volumeID")
    if kind == "scaleIO":
        return _need(s, p, "gateway", "system", "volumeName")
    if kind == "storageos":
        errs = []
        if not s.get("volumeName"):
            errs.append(required(f"{p}.volumeName"))
        else:
            errs += dns_label(s["volumeName"], f"{p}.volumeName")
        if s.get("volumeNamespace"):
            errs += dns_label(s["volumeNamespace"], f"{p}.volumeNamespace")
        ref = s.get("secretRef")
        if ref is not None:
            if not ref.get("name"):
                errs.append(required(f"{p}.secretRef.name"))
            if pv and not ref.get("namespace"):
                errs.append(required(f"{p}.secretRef.namespace"))
        return errs
    if kind == "projected":
        errs = _mode(s.get("defaultMode"), f"{p}.defaultMode")
        paths: set = set()
        for src in s.get("sources") or []:
            n = 0
            for sk in ("secret", "configMap", "downwardAPI"):
                sub = src.get(sk)
                if sub is None:
                    continue
                if n:
                    errs.append(forbidden(f"{p}.{sk}", "may not specify more than 1 volume type"))
                    continue
                n += 1
                if sk == "downwardAPI":
                    for f in sub.get("items") or []:
                        errs += validate_downward_api_file(f, f"{p}.downwardAPI")
                        if f.get("path"):
                            if f["path"] in paths:
                                errs.append(invalid(p, f["path"], "conflicting duplicate paths"))
                            paths.add(f["path"])
                    continue
                if not sub.get("name"):
                    errs.append(required(f"{p}.name"))
                for i, kp in enumerate(sub.get("items") or []):
                    errs += validate_key_to_path(kp, f"{p}.items[{i}]")
                    if kp.get("path"):
                        if kp["path"] in paths:
                            errs.append(invalid(p, sub.get("name") or "", "conflicting duplicate paths"))
                        paths.add(kp["path"])
        return errs
    if kind == "csi":
        errs = [] if GATES("CSIPersistentVolume") else [forbidden(p, "CSIPersistentVolume disabled by feature-gate")]
        return errs + _need(s, p, "driver", "volumeHandle")
    return []


def validate_volume_source(v: dict, p: str, name: str) -> list[str]:
    errs, n = [], 0
    for kind in VOLUME_SOURCES:
        if v.get(kind) is None:
            continue
        if n:
            errs.append(forbidden(f"{p}.{_DUP_NAME.get(kind, kind)}", "may not specify more than 1 volume type"))
            continue
        n += 1
        errs += validate_source(kind, v[kind], f"{p}.{kind}")
        if kind == "iscsi" and (v[kind] or {}).get("initiatorName") is not None and \
                len(f"{name}:{v[kind].get('targetPortal', '')}") > 64:
            errs.append(invalid(f"{p}.name", name, "Total length of <volume name>:<iscsi.targetPortal> must be under "
                                                   "64 characters if iscsi.initiatorName is specified."))
    if n == 0:
        errs.append(required(p, "must specify a volume type"))
    return errs


def validate_volumes(volumes, p) -> tuple[dict, list[str]]:
    """(name -> volume, errors); a volume with errors is not usable by the mounts."""
    errs, vols = [], {}
    for i, v in enumerate(volumes or []):
        ip = f"{p}[{i}]"
        name = v.get("name") or ""
        el = validate_volume_source(v, ip, name)
        if not name:
            el.append(required(f"{ip}.name"))
        else:
            el += dns_label(name, f"{ip}.name")
        if name in vols:
            el.append(duplicate(f"{ip}.name", name))
        if el:
            errs += el
        else:
            vols[name] = v
    return vols, errs


def validate_volume_mounts(mounts, devices: dict, vols: dict, c: dict | None, p: str) -> list[str]:
    errs, seen = [], set()
    for i, m in enumerate(mounts or []):
        ip = f"{p}[{i}]"
        name, mp = m.get("name") or "", m.get("mountPath") or ""
        if not name:
            errs.append(required(f"{ip}.name"))
        if name not in vols:
            errs.append(not_found(f"{ip}.name", name))
        if not mp:
            errs.append(required(f"{ip}.mountPath"))
        if mp in seen:
            errs.append(invalid(f"{ip}.mountPath", mp, "must be unique"))
        seen.add(mp)
        if name in devices:
            errs.append(invalid(f"{ip}.name", name, "must not already exist in volumeDevices"))
        if mp in devices.values():
            errs.append(invalid(f"{ip}.mountPath", mp, "must not already exist as a path in volumeDevices"))
        if m.get("subPath"):
            errs += validate_local_descending_path(m["subPath"], f"{p}.subPath")
        mprop = m.get("mountPropagation")
        if mprop is not None and not GATES("MountPropagation"):
            errs.append(forbidden(f"{p}.mountPropagation", "mount propagation is disabled by feature-gate"))
        elif mprop is not None:
            if mprop not in ("Bidirectional", "HostToContainer"):
                errs.append(not_supported(f"{p}.mountPropagation", mprop, ["Bidirectional", "HostToContainer"]))
            if c is not None and mprop == "Bidirectional" and not ((c.get("securityContext") or {}).get("privileged")):
                errs.append(forbidden(f"{p}.mountPropagation", "Bidirectional mount propagation is available only to "
                                                               "privileged containers"))
    return errs


def validate_volume_devices(devs, mounts: dict, vols: dict, p: str) -> list[str]:
    errs, names, paths = [], set(), set()
    if devs is not None and not GATES("BlockVolume"):
        return [forbidden(f"{p}.volumeDevices", "Container volumeDevices is disabled by feature-gate")]
    for i, d in enumerate(devs or []):
        ip = f"{p}[{i}]"
        name, dp = d.get("name") or "", d.get("devicePath") or ""
        if not name:
            errs.append(required(f"{ip}.name"))
        if name in names:
            errs.append(invalid(f"{ip}.name", name, "must be unique"))
        if name in vols and (vols[name] or {}).get("persistentVolumeClaim") is None:
            errs.append(invalid(f"{ip}.name", name, "can only use volume source type of PersistentVolumeClaim for block mode"))
        if name not in vols:
            errs.append(not_found(f"{ip}.name", name))
        if not dp:
            errs.append(required(f"{ip}.devicePath"))
        if dp in paths:
            errs.append(invalid(f"{ip}.devicePath", dp, "must be unique"))
        if dp and validate_path_no_backsteps(dp, ""):
            errs.append(invalid(f"{ip}.devicePath", dp, "can not contain backsteps ('..')"))
        else:
            paths.add(dp)
        if name in mounts:
            errs.append(invalid(f"{ip}.name", name, "must not already exist in volumeMounts"))
        if dp in mounts.values():
            errs.append(invalid(f"{ip}.devicePath", dp, "must not already exist as a path in volumeMounts"))
        if name:
            names.add(name)
    return errs


def validate_read_only_persistent_disks(volumes, p) -> list[str]:
    errs = []
    for i, v in enumerate(volumes or []):
        if v.get("gcePersistentDisk") is not None and not v["gcePersistentDisk"].get("readOnly"):
            errs.append(invalid(f"{p}[{i}].gcePersistentDisk.readOnly", False,
                                "must be true for replicated pods > 1; GCE PD can only be mounted on multiple machines "
                                "if it is read-only"))
    return errs


# ============================================================== containers
def validate_port_num_or_name(port, p) -> list[str]:
    if is_int(port):
        return [invalid(p, port, m) for m in is_valid_port_num(port)]
    if isinstance(port, str):
        return [invalid(p, port, m) for m in is_valid_port_name(port)]
    return [f"{p}: Internal error: unknown type: {port!r}"]


def validate_handler(h: dict | None, p: str) -> list[str]:
    h = h or {}
    errs, n = [], 0
    for kind in ("exec", "httpGet", "tcpSocket"):
        a = h.get(kind)
        if a is None:
            continue
        if n:
            errs.append(forbidden(f"{p}.{kind}", "may not specify more than 1 handler type"))
            continue
        n += 1
        ap = f"{p}.{kind}"
        if kind == "exec":
            if not a.get("command"):
                errs.append(required(f"{ap}.command"))
        elif kind == "httpGet":
            if not a.get("path"):
                errs.append(required(f"{ap}.path"))
            errs += validate_port_num_or_name(a.get("port", 0), f"{ap}.port")
            sch = a.get("scheme", "HTTP")
            if sch not in ("HTTP", "HTTPS"):
                errs.append(not_supported(f"{ap}.scheme", sch, ["HTTP", "HTTPS"]))
            for hd in a.get("httpHeaders") or []:
                errs += [invalid(f"{ap}.httpHeaders", hd.get("name") or "", m) for m in is_http_header_name(hd.get("name") or "")]
        else:
            errs += validate_port_num_or_name(a.get("port", 0), f"{ap}.port")
    if n == 0:
        errs.append(required(p, "must specify a handler type"))
    return errs


def validate_probe(pr, p) -> list[str]:
    if pr is None:
        return []
    errs = validate_handler(pr, p)
    for f in ("initialDelaySeconds", "timeoutSeconds", "periodSeconds", "successThreshold", "failureThreshold"):
        errs += nonneg(pr.get(f, 0), f"{p}.{f}")
    return errs


def validate_lifecycle(lc, p) -> list[str]:
    errs = []
    for hook in ("postStart", "preStop"):
        if (lc or {}).get(hook) is not None:
            errs += validate_handler(lc[hook], f"{p}.{hook}")
    return errs


def validate_pull_policy(pol, p) -> list[str]:
    if pol in ("Always", "IfNotPresent", "Never"):
        return []
    if not pol:
        return [required(p)]
    return [not_supported(p, pol, ["Always", "IfNotPresent", "Never"])]


def validate_container_ports(ports, p) -> list[str]:
    errs, names = [], set()
    for i, port in enumerate(ports or []):
        ip = f"{p}[{i}]"
        name = port.get("name") or ""
        if name:
            msgs = is_valid_port_name(name)
            if msgs:
                errs += [invalid(f"{ip}.name", name, m) for m in msgs]
            elif name in names:
                errs.append(duplicate(f"{ip}.name", name))
            else:
                names.add(name)
        cp = port.get("containerPort", 0)
        if not cp:
            errs.append(required(f"{ip}.containerPort"))
        else:
            errs += [invalid(f"{ip}.containerPort", cp, m) for m in is_valid_port_num(cp)]
        hp = port.get("hostPort", 0)
        if hp:
            errs += [invalid(f"{ip}.hostPort", hp, m) for m in is_valid_port_num(hp)]
        proto = port.get("protocol") or ""
        if not proto:
            errs.append(required(f"{ip}.protocol"))
        elif proto not in ("TCP", "UDP"):
            errs.append(not_supported(f"{ip}.protocol", proto, ["TCP", "UDP"]))
    return errs


def check_host_port_conflicts(containers, p) -> list[str]:
    errs, seen = [], set()
    for ci, c in enumerate(containers or []):
        for pi, port in enumerate(c.get("ports") or []):
            hp = port.get("hostPort", 0)
            if not hp:
                continue
            key = f"{port.get('protocol', '')}/{port.get('hostIP', '')}/{hp}"
            if key in seen:
                errs.append(duplicate(f"{p}[{ci}].ports[{pi}].hostPort", key))
            seen.add(key)
    return errs


def validate_security_context(sc, p) -> list[str]:
    from .validation import CAPABILITIES
    if sc is None:
        return []
    errs = []
    if sc.get("privileged") and not CAPABILITIES["allow_privileged"]:
        errs.append(forbidden(f"{p}.privileged", "disallowed by cluster policy"))
    ru = sc.get("runAsUser")
    if ru is not None and is_int(ru) and ru < 0:
        errs.append(invalid(f"{p}.runAsUser", ru, NEGATIVE))
    if sc.get("allowPrivilegeEscalation") is False:
        if sc.get("privileged"):
            errs.append(invalid(p, _go(sc), "cannot set `allowPrivilegeEscalation` to false and `privileged` to true"))
        if "CAP_SYS_ADMIN" in ((sc.get("capabilities") or {}).get("add") or []):
            errs.append(invalid(p, _go(sc), "cannot set `allowPrivilegeEscalation` to false and `capabilities.Add` CAP_SYS_ADMIN"))
    return errs


def validate_containers(containers, vols: dict, p: str) -> list[str]:
    from .validation import validate_env, validate_env_from
    if not containers:
        return [required(p)]
    errs, names = [], set()
    for i, c in enumerate(containers):
        ip = f"{p}[{i}]"
        name = c.get("name") or ""
        if not name:
            errs.append(required(f"{ip}.name"))
        else:
            errs += dns_label(name, f"{ip}.name")
        if name in names:
            errs.append(duplicate(f"{ip}.name", name))
        names.add(name)
        if not c.get("image"):
            errs.append(required(f"{ip}.image"))
        if c.get("lifecycle") is not None:
            errs += validate_lifecycle(c["lifecycle"], f"{ip}.lifecycle")
        errs += validate_probe(c.get("livenessProbe"), f"{ip}.livenessProbe")
        lp = c.get("livenessProbe")
        if lp is not None and lp.get("successThreshold", 1) != 1:
            errs.append(invalid(f"{ip}.livenessProbe.successThreshold", lp.get("successThreshold"), "must be 1"))
        tmp = c.get("terminationMessagePolicy") or ""
        if not tmp:
            errs.append(required(f"{ip}.terminationMessagePolicy", "must be 'File' or 'FallbackToLogsOnError'"))
        elif tmp not in ("File", "FallbackToLogsOnError"):
            errs.append(invalid(f"{ip}.terminationMessagePolicy", tmp, "must be 'File' or 'FallbackToLogsOnError'"))
        errs += validate_probe(c.get("readinessProbe"), f"{ip}.readinessProbe")
        errs += validate_container_ports(c.get("ports"), f"{ip}.ports")
        errs += validate_env(c.get("env") or [], f"{ip}.env")
        errs += validate_env_from(c.get("envFrom") or [], f"{ip}.envFrom")
        mounts = {m.get("name"): m.get("mountPath") for m in c.get("volumeMounts") or []}
        devices = {d.get("name"): d.get("devicePath") for d in c.get("volumeDevices") or []}
        errs += validate_volume_mounts(c.get("volumeMounts"), devices, vols, c, f"{ip}.volumeMounts")
        errs += validate_volume_devices(c.get("volumeDevices"), mounts, vols, f"{ip}.volumeDevices")
        errs += validate_pull_policy(c.get("imagePullPolicy"), f"{ip}.imagePullPolicy")
        errs += validate_resource_requirements(c.get("resources"), f"{ip}.resources")
        errs += validate_security_context(c.get("securityContext"), f"{ip}.securityContext")
    return errs + check_host_port_conflicts(containers, p)


def validate_init_containers(inits, others, vols, p) -> list[str]:
    errs = validate_containers(inits, vols, p) if inits else []
    names = {c.get("name") for c in others or []}
    for i, c in enumerate(inits or []):
        ip = f"{p}[{i}]"
        if c.get("name") in names:
            errs.append(duplicate(f"{ip}.name", c.get("name")))
        if c.get("name"):
            names.add(c["name"])
        for f in ("lifecycle", "livenessProbe", "readinessProbe"):
            if c.get(f) is not None:
                errs.append(invalid(f"{ip}.{f}", _go(c[f]), "must not be set for init containers"))
    return errs


# ============================================================== pod spec
DNS_POLICIES = ("ClusterFirstWithHostNet", "ClusterFirst", "Default", "None")


def validate_restart_policy(rp, p) -> list[str]:
    if rp in ("Always", "OnFailure", "Never"):
        return []
    if not rp:
        return [required(p)]
    return [not_supported(p, rp, ["Always", "OnFailure", "Never"])]


def validate_dns_policy(dp, p) -> list[str]:
    if dp == "None" and not GATES("CustomPodDNS"):
        return [invalid(p, dp, "DNSPolicy: can not use 'None', custom pod DNS is disabled by feature gate")]
    if dp in DNS_POLICIES:
        return []
    if not dp:
        return [required(p)]
    return [not_supported(p, dp, list(DNS_POLICIES) if GATES("CustomPodDNS") else list(DNS_POLICIES[:3]))]


def validate_pod_dns_config(cfg, policy, p) -> list[str]:
    errs = []
    if policy == "None" and GATES("CustomPodDNS"):
        if cfg is None:
            return [required(p, "must provide `dnsConfig` when `dnsPolicy` is None")]
        if not cfg.get("nameservers"):
            return [required(f"{p}.nameservers", "must provide at least one DNS nameserver when `dnsPolicy` is None")]
    if cfg is None:
        return errs
    if not GATES("CustomPodDNS"):
        return [forbidden(p, "DNSConfig: custom pod DNS is disabled by feature gate")]
    ns = cfg.get("nameservers") or []
    if len(ns) > 3:
        errs.append(invalid(f"{p}.nameservers", _go(ns), "must not have more than 3 nameservers"))
    for i, n in enumerate(ns):
        if parse_ip(n) is None:
            errs.append(invalid(f"{p}.nameservers[{i}]", n, "must be valid IP address"))
    se = cfg.get("searches") or []
    if len(se) > 6:
        errs.append(invalid(f"{p}.searches", _go(se), "must not have more than 6 search paths"))
    if len(" ".join(se)) > 256:
        errs.append(invalid(f"{p}.searches", _go(se), "must not have more than 256 characters (including spaces) in the search list"))
    for i, s in enumerate(se):
        errs += dns_subdomain(s, f"{p}.searches[{i}]")
    for i, o in enumerate(cfg.get("options") or []):
        if not o.get("name"):
            errs.append(required(f"{p}.options[{i}]", "must not be empty"))
    return errs


def validate_host_network(spec, p) -> list[str]:
    errs = []
    if spec.get("hostNetwork"):
        for i, c in enumerate(spec.get("containers") or []):
            for j, port in enumerate(c.get("ports") or []):
                if port.get("hostPort", 0) != port.get("containerPort", 0):
                    errs.append(invalid(f"{p}[{i}].ports[{j}].containerPort", port.get("containerPort", 0),
                                        "must match `hostPort` when `hostNetwork` is true"))
    return errs


def validate_node_selector_requirement(r, p) -> list[str]:
    errs = []
    op, vals = r.get("operator"), r.get("values") or []
    if op in ("In", "NotIn"):
        if not vals:
            errs.append(required(f"{p}.values", "must be specified when `operator` is 'In' or 'NotIn'"))
    elif op in ("Exists", "DoesNotExist"):
        if vals:
            errs.append(forbidden(f"{p}.values", "may not be specified when `operator` is 'Exists' or 'DoesNotExist'"))
    elif op in ("Gt", "Lt"):
        if len(vals) != 1:
            errs.append(required(f"{p}.values", "must be specified single value when `operator` is 'Lt' or 'Gt'"))
    else:
        errs.append(invalid(f"{p}.operator", op, "not a valid selector operator"))
    return errs + label_name(r.get("key") or "", f"{p}.key")


def validate_node_selector_term(t, p) -> list[str]:
    exprs = (t or {}).get("matchExpressions") or []
    if not exprs:
        return [required(f"{p}.matchExpressions", "must have at least one node selector requirement")]
    errs = []
    for j, r in enumerate(exprs):
        errs += validate_node_selector_requirement(r, f"{p}.matchExpressions[{j}]")
    return errs


def validate_node_selector(ns, p) -> list[str]:
    terms = (ns or {}).get("nodeSelectorTerms") or []
    if not terms:
        return [required(f"{p}.nodeSelectorTerms", "must have at least one node selector term")]
    errs = []
    for i, t in enumerate(terms):
        errs += validate_node_selector_term(t, f"{p}.nodeSelectorTerms[{i}]")
    return errs


def validate_pod_affinity_term(t, p) -> list[str]:
    errs = validate_label_selector(t.get("labelSelector"), f"{p}.matchExpressions")
    for n in t.get("namespaces") or []:
        errs += [invalid(f"{p}.namespace", n, m) for m in is_dns1123_label(n)]
    tk = t.get("topologyKey") or ""
    if not tk:
        errs.append(required(f"{p}.topologyKey", "can not be empty"))
    return errs + label_name(tk, f"{p}.topologyKey")


def _validate_pod_affinity(pa, p) -> list[str]:
    errs = []
    for i, t in enumerate(pa.get("requiredDuringSchedulingIgnoredDuringExecution") or []):
        errs += validate_pod_affinity_term(t, f"{p}.requiredDuringSchedulingIgnoredDuringExecution[{i}]")
    for j, w in enumerate(pa.get("preferredDuringSchedulingIgnoredDuringExecution") or []):
        wp = f"{p}.preferredDuringSchedulingIgnoredDuringExecution[{j}]"
        wt = w.get("weight", 0)
        if not is_int(wt) or wt <= 0 or wt > 100:
            errs.append(invalid(f"{wp}.weight", wt, "must be in the range 1-100"))
        errs += validate_pod_affinity_term(w.get("podAffinityTerm") or {}, f"{wp}.podAffinityTerm")
    return errs


def validate_affinity(aff, p) -> list[str]:
    if not aff:
        return []
    errs = []
    na = aff.get("nodeAffinity")
    if na:
        if na.get("requiredDuringSchedulingIgnoredDuringExecution") is not None:
            errs += validate_node_selector(na["requiredDuringSchedulingIgnoredDuringExecution"],
                                           f"{p}.nodeAffinity.requiredDuringSchedulingIgnoredDuringExecution")
        for i, t in enumerate(na.get("preferredDuringSchedulingIgnoredDuringExecution") or []):
            tp = f"{p}.nodeAffinity.preferredDuringSchedulingIgnoredDuringExecution[{i}]"
            wt = t.get("weight", 0)
            if not is_int(wt) or wt <= 0 or wt > 100:
                errs.append(invalid(f"{tp}.weight", wt, "must be in the range 1-100"))
            errs += validate_node_selector_term(t.get("preference"), f"{tp}.preference")
    if aff.get("podAffinity") is not None:
        errs += _validate_pod_affinity(aff["podAffinity"], f"{p}.podAffinity")
    if aff.get("podAntiAffinity") is not None:
        errs += _validate_pod_affinity(aff["podAntiAffinity"], f"{p}.podAntiAffinity")
    return errs


def validate_taint_effect(eff, allow_empty, p) -> list[str]:
    if not allow_empty and not eff:
        return [required(p)]
    if eff not in ("NoSchedule", "PreferNoSchedule", "NoExecute"):
        return [not_supported(p, eff, ["NoSchedule", "PreferNoSchedule", "NoExecute"])]
    return []


def validate_tolerations(tols, p) -> list[str]:
    errs = []
    for i, t in enumerate(tols or []):
        ip = f"{p}[{i}]"
        key, op = t.get("key") or "", t.get("operator") or ""
        if key:
            errs += label_name(key, f"{ip}.key")
        if not key and op != "Exists":
            errs.append(invalid(f"{ip}.operator", op, "operator must be Exists when `key` is empty, which means "
                                                      "\"match all values and all keys\""))
        if t.get("tolerationSeconds") is not None and t.get("effect") != "NoExecute":
            errs.append(invalid(f"{ip}.effect", t.get("effect") or "", "effect must be 'NoExecute' when `tolerationSeconds` is set"))
        if op in ("Equal", ""):
            ms = is_valid_label_value(t.get("value") or "")
            if ms:
                errs.append(invalid(f"{ip}.operator", t.get("value") or "", ";".join(ms)))
        elif op == "Exists":
            if t.get("value"):
                errs.append(invalid(f"{ip}.operator", _go(t), "value must be empty when `operator` is 'Exists'"))
        else:
            errs.append(not_supported(f"{ip}.operator", op, ["Equal", "Exists"]))
        if t.get("effect"):
            errs += validate_taint_effect(t["effect"], True, f"{ip}.effect")
    return errs


def validate_host_aliases(aliases, p) -> list[str]:
    errs = []
    for a in aliases or []:
        if parse_ip(a.get("ip")) is None:
            errs.append(invalid(f"{p}.ip", a.get("ip") or "", "must be valid IP address"))
        for h in a.get("hostnames") or []:
            errs += dns_subdomain(h, f"{p}.hostnames")
    return errs


def validate_pod_security_context(spec, p, sp) -> list[str]:
    sc = spec.get("securityContext")
    errs = validate_host_network(spec, f"{sp}.containers")
    if sc is None:
        return errs
    if sc.get("fsGroup") is not None:
        errs += [invalid(f"{p}.fsGroup", sc["fsGroup"], m) for m in is_valid_id(sc["fsGroup"])]
    if sc.get("runAsUser") is not None:
        errs += [invalid(f"{p}.runAsUser", sc["runAsUser"], m) for m in is_valid_id(sc["runAsUser"])]
    for g, gid in enumerate(sc.get("supplementalGroups") or []):
        errs += [invalid(f"{p}.supplementalGroups[{g}]", gid, m) for m in is_valid_id(gid)]
    return errs


def validate_image_pull_secrets(secrets, p) -> list[str]:
    return [invalid(f"{p}[{i}]", _go(s), "only name may be set")
            for i, s in enumerate(secrets or []) if set(s) - {"name"}]


def validate_pod_spec(spec: dict, p: str = "spec") -> list[str]:
    """ValidatePodSpec (validation.go:2879-2948), plus the fork's extended resources."""
    from .validation import validate_containers_extended_resources, validate_extended_resources
    vols, errs = validate_volumes(spec.get("volumes"), f"{p}.volumes")
    coll, xerrs = validate_extended_resources(spec.get("extendedResources"), f"{p}.extendedResources")
    errs += xerrs
    conts, inits = spec.get("containers") or [], spec.get("initContainers") or []
    errs += validate_containers(conts, vols, f"{p}.containers")
    errs += validate_containers_extended_resources(conts, dict(coll), f"{p}.containers")
    errs += validate_containers_extended_resources(inits, dict(coll), f"{p}.initContainers")   # fix #9
    errs += validate_init_containers(inits, conts, vols, f"{p}.initContainers")
    errs += validate_restart_policy(spec.get("restartPolicy"), f"{p}.restartPolicy")
    errs += validate_dns_policy(spec.get("dnsPolicy"), f"{p}.dnsPolicy")
    errs += validate_labels(spec.get("nodeSelector"), f"{p}.nodeSelector")
    errs += validate_pod_security_context(spec, f"{p}.securityContext", p)
    errs += validate_image_pull_secrets(spec.get("imagePullSecrets"), f"{p}.imagePullSecrets")
    errs += validate_affinity(spec.get("affinity"), f"{p}.affinity")
    errs += validate_pod_dns_config(spec.get("dnsConfig"), spec.get("dnsPolicy"), f"{p}.dnsConfig")
    if spec.get("serviceAccountName"):
        errs += dns_subdomain(spec["serviceAccountName"], f"{p}.serviceAccountName")
    if spec.get("nodeName"):
        errs += dns_subdomain(spec["nodeName"], f"{p}.nodeName")
    ads = spec.get("activeDeadlineSeconds")
    if ads is not None and (not is_int(ads) or ads < 1 or ads > MAX_INT32):
        errs.append(invalid(f"{p}.activeDeadlineSeconds", ads, inclusive_range(1, MAX_INT32)))
    if spec.get("hostname"):
        errs += dns_label(spec["hostname"], f"{p}.hostname")
    if spec.get("subdomain"):
        errs += dns_label(spec["subdomain"], f"{p}.subdomain")
    if spec.get("tolerations"):
        errs += validate_tolerations(spec["tolerations"], f"{p}.tolerations")
    if spec.get("hostAliases"):
        errs += validate_host_aliases(spec["hostAliases"], f"{p}.hostAliases")
    if spec.get("priorityClassName"):
        errs += dns_subdomain(spec["priorityClassName"], f"{p}.priorityClassName")
    gp = spec.get("terminationGracePeriodSeconds")
    if gp is not None and is_int(gp) and gp < 0:
        errs.append(invalid(f"{p}.terminationGracePeriodSeconds", gp, NEGATIVE))
    return errs


def validate_pod_specific_annotations(ann, spec, p) -> list[str]:
    from ..kubelet.sysctl import validate_annotations as validate_sysctl_annotations
    from ..security import validate_seccomp_annotations
    from ..security.apparmor import validate_pod_annotations
    errs = validate_seccomp_annotations(ann)
    errs += validate_pod_annotations({"metadata": {"annotations": ann or {}}, "spec": spec})
    return errs + validate_sysctl_annotations(ann)


def validate_pod_template_spec(tpl, p) -> list[str]:
    from .validation import validate_object_meta   # noqa: F401 (template metadata: labels/annotations only)
    md = (tpl or {}).get("metadata") or {}
    errs = validate_labels(md.get("labels"), f"{p}.labels")
    errs += validate_pod_specific_annotations(md.get("annotations"), (tpl or {}).get("spec") or {}, f"{p}.annotations")
    return errs + validate_pod_spec((tpl or {}).get("spec") or {}, f"{p}.spec")


def validate_pod(pod: dict, old: dict | None = None) -> list[str]:
    from .validation import validate_object_meta
    spec = pod.get("spec") or {}
    errs = validate_object_meta(pod, True)
    errs += validate_pod_specific_annotations((pod.get("metadata") or {}).get("annotations"), spec, "metadata.annotations")
    errs += validate_pod_spec(spec)
    for kind in ("containers", "initContainers"):
        for i, c in enumerate(spec.get(kind) or []):
            img = c.get("image") or ""
            if img != img.strip():
                errs.append(invalid(f"spec.{kind}[{i}].image", img, "must not have leading or trailing whitespace"))
    huge = set()
    for c in spec.get("containers") or []:
        r = c.get("resources") or {}
        huge |= {k for k in list((r.get("limits") or {})) + list((r.get("requests") or {})) if _hugepages(k)}
    if len(huge) > 1:
        errs.append(invalid("spec", _go(sorted(huge)), "must use a single hugepage size in a pod spec"))
    if old is not None:
        errs += validate_pod_update(pod, old)
    return errs


def _strip_for_update(spec: dict, old: dict) -> dict:
    s = json.loads(json.dumps(spec))
    for kind in ("containers", "initContainers"):
        for i, c in enumerate(s.get(kind) or []):
            oc = (old.get(kind) or [])
            c["image"] = oc[i].get("image") if i < len(oc) else c.get("image")
    s.pop("activeDeadlineSeconds", None)
    if old.get("activeDeadlineSeconds") is not None:
        s["activeDeadlineSeconds"] = old["activeDeadlineSeconds"]
    s.pop("tolerations", None)
    if "tolerations" in old:
        s["tolerations"] = old["tolerations"]
    for pres in s.get("extendedResources") or []:
        pres.pop("assigned", None)      # only pods/binding writes assigned (fork)
    return s


def _norm_old(old: dict) -> dict:
    o = json.loads(json.dumps(old))
    for pres in o.get("extendedResources") or []:
        pres.pop("assigned", None)
    return o


def validate_pod_update(new: dict, old: dict) -> list[str]:
    """ValidatePodUpdate (validation.go:3319-3396): only container images, a shrinking
    activeDeadlineSeconds and added tolerations may change."""
    errs = []
    ns, os_ = new.get("spec") or {}, old.get("spec") or {}
    for kind in ("containers", "initContainers"):
        nc, oc = ns.get(kind) or [], os_.get(kind) or []
        if len(nc) != len(oc):
            return [forbidden(f"spec.{kind}", "pod updates may not add or remove containers")]
        for i, c in enumerate(nc):
            img = c.get("image") or ""
            if not img:
                errs.append(required(f"spec.{kind}[{i}].image"))
            if img.strip() != img:
                errs.append(invalid(f"spec.{kind}[{i}].image", img, "must not have leading or trailing whitespace"))
    nads, oads = ns.get("activeDeadlineSeconds"), os_.get("activeDeadlineSeconds")
    if nads is not None:
        if not is_int(nads) or nads < 0 or nads > MAX_INT32:
            return errs + [invalid("spec.activeDeadlineSeconds", nads, inclusive_range(0, MAX_INT32))]
        if oads is not None and oads < nads:
            return errs + [invalid("spec.activeDeadlineSeconds", nads, "must be less than or equal to previous value")]
    elif oads is not None:
        errs.append(invalid("spec.activeDeadlineSeconds", None, "must not update from a positive integer to nil value"))
    # tolerations: existing ones may only change their tolerationSeconds
    ntols = [{k: v for k, v in t.items() if k != "tolerationSeconds"} for t in ns.get("tolerations") or []]
    for t in os_.get("tolerations") or []:
        if {k: v for k, v in t.items() if k != "tolerationSeconds"} not in ntols:
            errs.append(forbidden("spec.tolerations", "existing toleration can not be modified except its tolerationSeconds"))
            break
    else:
        errs += validate_tolerations(ns.get("tolerations"), "spec.tolerations")
    if _strip_for_update(ns, os_) != _norm_old(os_):
        errs.append(forbidden("spec", "pod updates may not change fields other than `spec.containers[*].image`, "
                                      "`spec.initContainers[*].image`, `spec.activeDeadlineSeconds` or "
                                      "`spec.tolerations` (only additions to existing tolerations)"))
    old_nn = os_.get("nodeName")
    if old_nn and ns.get("nodeName") != old_nn:
        errs.append(forbidden("spec.nodeName", "field is immutable once set"))
    return errs


# ============================================================== core kinds
def validate_pod_template(pt, old=None) -> list[str]:
    from .validation import validate_object_meta
    return validate_object_meta(pt, True) + validate_pod_template_spec(pt.get("template"), "template")


def validate_rc_template(tpl, selector: dict, replicas, p) -> list[str]:
    if tpl is None:
        return [required(p)]
    errs = []
    labels = ((tpl.get("metadata") or {}).get("labels")) or {}
    if selector and any(labels.get(k) != v for k, v in selector.items()):
        errs.append(invalid(f"{p}.metadata.labels", _go(labels), "`selector` does not match template `labels`"))
    errs += validate_pod_template_spec(tpl, p)
    tspec = tpl.get("spec") or {}
    if is_int(replicas) and replicas > 1:
        errs += validate_read_only_persistent_disks(tspec.get("volumes"), f"{p}.spec.volumes")
    if tspec.get("restartPolicy") != "Always":
        errs.append(not_supported(f"{p}.spec.restartPolicy", tspec.get("restartPolicy") or "", ["Always"]))
    if tspec.get("activeDeadlineSeconds") is not None:
        errs.append(invalid(f"{p}.spec.activeDeadlineSeconds", tspec["activeDeadlineSeconds"], "must not be specified"))
    return errs


def validate_replication_controller(rc, old=None) -> list[str]:
    from .validation import validate_object_meta
    spec = rc.get("spec") or {}
    errs = validate_object_meta(rc, True)
    errs += nonneg(spec.get("minReadySeconds", 0), "spec.minReadySeconds")
    if not spec.get("selector"):
        errs.append(required("spec.selector"))
    errs += nonneg(spec.get("replicas", 0), "spec.replicas")
    errs += validate_rc_template(spec.get("template"), spec.get("selector") or {}, spec.get("replicas", 1), "spec.template")
    return errs


def validate_rc_status(st, p="status") -> list[str]:
    st = st or {}
    errs = []
    for f in ("replicas", "fullyLabeledReplicas", "readyReplicas", "availableReplicas", "observedGeneration"):
        errs += nonneg(st.get(f, 0), f"{p}.{f}")
    r = st.get("replicas", 0)
    for f in ("fullyLabeledReplicas", "readyReplicas", "availableReplicas"):
        if st.get(f, 0) > r:
            errs.append(invalid(f"{p}.{f}", st.get(f, 0), "cannot be greater than status.replicas"))
    if st.get("availableReplicas", 0) > st.get("readyReplicas", 0):
        errs.append(invalid(f"{p}.availableReplicas", st.get("availableReplicas", 0), "cannot be greater than readyReplicas"))
    return errs


ACCESS_MODES = ("ReadWriteOnce", "ReadOnlyMany", "ReadWriteMany")
RECLAIM_POLICIES = ("Delete", "Recycle", "Retain")
VOLUME_MODES = ("Block", "Filesystem")
PV_SOURCES = ("hostPath", "gcePersistentDisk", "awsElasticBlockStore", "glusterfs", "flocker", "nfs", "rbd", "quobyte",
              "cephfs", "iscsi", "cinder", "fc", "flexVolume", "azureFile", "vsphereVolume", "photonPersistentDisk",
              "portworxVolume", "azureDisk", "scaleIO", "local", "storageos", "csi")


def validate_persistent_volume(pv, old=None) -> list[str]:
    from .validation import validate_object_meta
    spec = pv.get("spec") or {}
    md = pv.get("metadata") or {}
    errs = validate_object_meta(pv, False)
    modes = spec.get("accessModes") or []
    if not modes:
        errs.append(required("spec.accessModes"))
    for mo in modes:
        if mo not in ACCESS_MODES:
            errs.append(not_supported("spec.accessModes", mo, sorted(ACCESS_MODES)))
    cap = spec.get("capacity") or {}
    if not cap:
        errs.append(required("spec.capacity"))
    if "storage" not in cap or len(cap) > 1:
        errs.append(not_supported("spec.capacity", _go(cap), ["storage"]))
    for r, q in cap.items():
        errs += validate_basic_resource(q, f"spec.capacity[{r}]") + validate_positive_quantity(q, f"spec.capacity[{r}]")
    rp = spec.get("persistentVolumeReclaimPolicy") or ""
    if rp and rp not in RECLAIM_POLICIES:
        errs.append(not_supported("spec.persistentVolumeReclaimPolicy", rp, sorted(RECLAIM_POLICIES)))
    n = 0
    for kind in PV_SOURCES:
        if spec.get(kind) is None:
            continue
        if n and kind != "flexVolume":
            errs.append(forbidden(f"spec.{_DUP_NAME.get(kind, kind)}", "may not specify more than 1 volume type"))
            continue
        n += 1
        errs += validate_source(kind, spec[kind], f"spec.{kind}", pv=True)
        if kind == "iscsi" and spec[kind].get("initiatorName") is not None and \
                len(f"{md.get('name', '')}:{spec[kind].get('targetPortal', '')}") > 64:
            errs.append(invalid("metadata.name", md.get("name", ""), "Total length of <volume name>:<iscsi.targetPortal> "
                                                                     "must be under 64 characters if iscsi.initiatorName is specified."))
        if kind == "local" and not GATES("PersistentLocalVolumes"):
            errs.append(forbidden("spec.local", "Local volumes are disabled by feature-gate"))
        if kind == "local" and not (md.get("annotations") or {}).get("volume.alpha.kubernetes.io/node-affinity") \
                and not spec.get("nodeAffinity"):
            errs.append(required("metadata.annotations", "Local volume requires node affinity"))
    if n == 0:
        errs.append(required("spec", "must specify a volume type"))
    hp = spec.get("hostPath")
    if hp is not None and posixpath.normpath(hp.get("path") or ".") == "/" and rp == "Recycle":
        errs.append(forbidden("spec.persistentVolumeReclaimPolicy", "may not be 'recycle' for a hostPath mount of '/'"))
    if spec.get("storageClassName"):
        errs += [invalid("spec.storageClassName", spec["storageClassName"], m) for m in is_dns1123_subdomain(spec["storageClassName"])]
    vm = spec.get("volumeMode")
    if vm is not None and not GATES("BlockVolume"):
        errs.append(forbidden("spec.volumeMode", "PersistentVolume volumeMode is disabled by feature-gate"))
    elif vm is not None and vm not in VOLUME_MODES:
        errs.append(not_supported("spec.volumeMode", vm, sorted(VOLUME_MODES)))
    if old is not None:
        src = {k: spec.get(k) for k in PV_SOURCES if spec.get(k) is not None}
        osrc = {k: (old.get("spec") or {}).get(k) for k in PV_SOURCES if (old.get("spec") or {}).get(k) is not None}
        if src != osrc:
            errs.append(forbidden("spec.persistentvolumesource", "is immutable after creation"))
        if vm != (old.get("spec") or {}).get("volumeMode"):
            errs.append(invalid("volumeMode", vm, IMMUTABLE))
    return errs


def validate_pvc_spec(spec, p) -> list[str]:
    errs = []
    modes = spec.get("accessModes") or []
    if not modes:
        errs.append(required(f"{p}.accessModes", "at least 1 access mode is required"))
    if spec.get("selector") is not None:
        errs += validate_label_selector(spec["selector"], f"{p}.selector")
    for mo in modes:
        if mo not in ACCESS_MODES:
            errs.append(not_supported(f"{p}.accessModes", mo, sorted(ACCESS_MODES)))
    req = ((spec.get("resources") or {}).get("requests")) or {}
    if "storage" not in req:
        errs.append(required(f"{p}.resources[storage]"))
    else:
        errs += validate_quantity_value("storage", req["storage"], f"{p}.resources[storage]")
        errs += validate_positive_quantity(req["storage"], f"{p}.resources[storage]")
    sc = spec.get("storageClassName")
    if sc:
        errs += [invalid(f"{p}.storageClassName", sc, m) for m in is_dns1123_subdomain(sc)]
    vm = spec.get("volumeMode")
    if vm is not None and not GATES("BlockVolume"):
        errs.append(forbidden(f"{p}.volumeMode", "PersistentVolumeClaim volumeMode is disabled by feature-gate"))
    elif vm is not None and vm not in VOLUME_MODES:
        errs.append(not_supported(f"{p}.volumeMode", vm, sorted(VOLUME_MODES)))
    return errs


def validate_persistent_volume_claim(pvc, old=None) -> list[str]:
    from .validation import validate_object_meta
    errs = validate_object_meta(pvc, True) + validate_pvc_spec(pvc.get("spec") or {}, "spec")
    if old is not None:
        new_s, old_s = json.loads(json.dumps(pvc.get("spec") or {})), json.loads(json.dumps(old.get("spec") or {}))
        if not old_s.get("volumeName"):
            old_s["volumeName"] = new_s.get("volumeName")     # binding sets volumeName once
        if GATES("ExpandPersistentVolumes") and (pvc.get("status") or {}).get("phase") == "Bound":
            # ExpandPersistentVolumes: a bound claim may grow its storage request
            nreq = (new_s.get("resources") or {}).get("requests") or {}
            oreq = (old_s.get("resources") or {}).get("requests") or {}
            if "storage" in oreq and "storage" in nreq:
                if _q(nreq["storage"]) is not None and _q(oreq["storage"]) is not None and \
                        _q(nreq["storage"]).as_fraction() < _q(oreq["storage"]).as_fraction():
                    errs.append(forbidden("spec.resources.requests.storage", "field can not be less than previous value"))
                nreq["storage"] = oreq["storage"]
            if new_s != old_s:
                errs.append(forbidden("spec", "is immutable after creation except resources.requests for bound claims"))
        elif new_s != old_s:
            errs.append(forbidden("spec", "field is immutable after creation"))
        key = "volume.beta.kubernetes.io/storage-class"
        na = ((pvc.get("metadata") or {}).get("annotations") or {}).get(key)
        oa = ((old.get("metadata") or {}).get("annotations") or {}).get(key)
        if oa != na:
            errs.append(forbidden(f"metadata.annotations[{key}]", IMMUTABLE))
    return errs


def validate_limit_range(lr, old=None) -> list[str]:
    from .validation import validate_object_meta
    errs = validate_object_meta(lr, True)
    seen = set()
    for i, item in enumerate(((lr.get("spec") or {}).get("limits")) or []):
        ip = f"spec.limits[{i}]"
        typ = item.get("type") or ""
        tm = [invalid(f"{ip}.type", typ, m) for m in is_qualified_name(typ)]
        if not tm and "/" not in typ and typ not in LIMIT_TYPES:
            tm = [invalid(f"{ip}.type", typ, "must be a standard limit type or fully qualified")]
        errs += tm
        if typ in seen:
            errs.append(duplicate(f"{ip}.type", typ))
        seen.add(typ)

        def rname(k, fp):
            if typ in ("Pod", "Container"):
                return validate_container_resource_name(k, fp)
            return validate_resource_name(k, fp)
        maps = {}
        for f in ("max", "min"):
            maps[f] = {}
            for k, q in (item.get(f) or {}).items():
                errs += rname(k, f"{ip}.{f}[{k}]")
                maps[f][k] = _q(q)
        maps["default"], maps["defaultRequest"] = {}, {}
        if typ == "Pod":
            if item.get("default"):
                errs.append(forbidden(f"{ip}.default", "may not be specified when `type` is 'Pod'"))
            if item.get("defaultRequest"):
                errs.append(forbidden(f"{ip}.defaultRequest", "may not be specified when `type` is 'Pod'"))
        else:
            for f in ("default", "defaultRequest"):
                for k, q in (item.get(f) or {}).items():
                    errs += rname(k, f"{ip}.{f}[{k}]")
                    maps[f][k] = _q(q)
        if typ == "PersistentVolumeClaim" and "storage" not in (item.get("min") or {}) and \
                "storage" not in (item.get("max") or {}):
            errs.append(required(f"{ip}.limits", "either minimum or maximum storage value is required, but neither was provided"))
        maps["ratio"] = {}
        for k, q in (item.get("maxLimitRequestRatio") or {}).items():
            errs += rname(k, f"{ip}.maxLimitRequestRatio[{k}]")
            maps["ratio"][k] = _q(q)
        keys = set().union(*(set(v) for v in maps.values()))
        for k in sorted(keys):
            mn, mx = maps["min"].get(k), maps["max"].get(k)
            df, dr, ra = maps["default"].get(k), maps["defaultRequest"].get(k), maps["ratio"].get(k)
            F = lambda q: q.as_fraction()   # noqa: E731
            if mn is not None and mx is not None and F(mn) > F(mx):
                errs.append(invalid(f"{ip}.min[{k}]", str(mn), f"min value {mn} is greater than max value {mx}"))
            if dr is not None and mn is not None and F(mn) > F(dr):
                errs.append(invalid(f"{ip}.defaultRequest[{k}]", str(dr), f"min value {mn} is greater than default request value {dr}"))
            if dr is not None and mx is not None and F(dr) > F(mx):
                errs.append(invalid(f"{ip}.defaultRequest[{k}]", str(dr), f"default request value {dr} is greater than max value {mx}"))
            if dr is not None and df is not None and F(dr) > F(df):
                errs.append(invalid(f"{ip}.defaultRequest[{k}]", str(dr), f"default request value {dr} is greater than default limit value {df}"))
            if df is not None and mn is not None and F(mn) > F(df):
                errs.append(invalid(f"{ip}.default[{k}]", str(mn), f"min value {mn} is greater than default value {df}"))
            if df is not None and mx is not None and F(df) > F(mx):
                errs.append(invalid(f"{ip}.default[{k}]", str(mx), f"default value {df} is greater than max value {mx}"))
            if ra is not None and F(ra) < 1:
                errs.append(invalid(f"{ip}.maxLimitRequestRatio[{k}]", str(ra), f"ratio {ra} is less than 1"))
            if ra is not None and mn is not None and mx is not None and F(mn) > 0:
                lim = float(F(mx) / F(mn))
                if float(F(ra)) > lim:
                    errs.append(invalid(f"{ip}.maxLimitRequestRatio[{k}]", str(ra), f"ratio {ra} is greater than max/min = {lim:f}"))
            if not overcommit_allowed(k) and df is not None and dr is not None and F(df) != F(dr):
                errs.append(invalid(f"{ip}.defaultRequest[{k}]", str(dr), f"default value {df} must equal to defaultRequest value {dr} in {k}"))
        for f in ("max", "min", "default", "defaultRequest", "maxLimitRequestRatio"):
            for k, q in (item.get(f) or {}).items():
                if _q(q) is None:
                    errs.append(invalid(f"{ip}.{f}[{k}]", q, "quantities must match the regular expression "
                                                              "'^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$'"))
    return errs


def validate_resource_quota_spec(spec, p) -> list[str]:
    errs = []
    hard = spec.get("hard") or {}
    for k, v in hard.items():
        errs += validate_quota_resource_name(k, f"{p}.hard[{k}]") + validate_quantity_value(k, v, f"{p}.hard[{k}]")
    scopes = spec.get("scopes") or []
    if scopes:
        sp = f"{p}.scopes"
        compute = {"cpu", "memory", "limits.cpu", "limits.memory", "requests.cpu", "requests.memory"}
        for sc in scopes:
            if sc not in QUOTA_SCOPES:
                errs.append(invalid(sp, _go(scopes), "unsupported scope"))
            for k in sorted(hard):
                if k in STANDARD_QUOTA or _quota_hugepages(k):
                    ok = (k == "pods" or k in compute) if sc in ("Terminating", "NotTerminating", "NotBestEffort") \
                        else (k == "pods") if sc == "BestEffort" else True
                    if not ok:
                        errs.append(invalid(sp, _go(scopes), "unsupported scope applied to resource"))
        for a, b in (("BestEffort", "NotBestEffort"), ("Terminating", "NotTerminating")):
            if a in scopes and b in scopes:
                errs.append(invalid(sp, _go(scopes), "conflicting scopes"))
    return errs


def validate_resource_quota(rq, old=None) -> list[str]:
    from .validation import validate_object_meta
    errs = validate_object_meta(rq, True) + validate_resource_quota_spec(rq.get("spec") or {}, "spec")
    st = rq.get("status") or {}
    for f in ("hard", "used"):
        for k, v in (st.get(f) or {}).items():
            errs += validate_quota_resource_name(k, f"status.{f}[{k}]") + validate_quantity_value(k, v, f"status.{f}[{k}]")
    if old is not None:
        if set((rq.get("spec") or {}).get("scopes") or []) != set((old.get("spec") or {}).get("scopes") or []):
            errs.append(invalid("spec.scopes", _go((rq.get("spec") or {}).get("scopes") or []), IMMUTABLE))
    return errs


# Deliberate deviation (docs/PARITY.md): amdkube's single-host local-up and hollow nodes run pods
# on the node's loopback address, so endpoints may point at 127.0.0.0/8; unspecified and
# link-local addresses are still refused.
ALLOW_LOOPBACK_ENDPOINTS = True


def validate_non_special_ip(ip, p) -> list[str]:
    a = parse_ip(ip)
    if a is None:
        return [invalid(p, ip, "must be a valid IP address")]
    errs = []
    if a.is_unspecified:
        errs.append(invalid(p, ip, "may not be unspecified (0.0.0.0)"))
    if a.is_loopback and not ALLOW_LOOPBACK_ENDPOINTS:
        errs.append(invalid(p, ip, "may not be in the loopback range (127.0.0.0/8)"))
    if a.is_link_local and not (a.version == 4 and a in ipaddress.ip_network("224.0.0.0/24")):
        errs.append(invalid(p, ip, "may not be in the link-local range (169.254.0.0/16)"))
    if (a.version == 4 and a in ipaddress.ip_network("224.0.0.0/24")) or \
            (a.version == 6 and a in ipaddress.ip_network("ff02::/16")):
        errs.append(invalid(p, ip, "may not be in the link-local multicast range (224.0.0.0/24)"))
    return errs


def validate_endpoints(ep, old=None) -> list[str]:
    from .validation import validate_object_meta
    errs = validate_object_meta(ep, True)
    old_nodes = {}
    for ss in ((old or {}).get("subsets") or []):
        for a in (ss.get("addresses") or []) + (ss.get("notReadyAddresses") or []):
            if a.get("nodeName"):
                old_nodes[a.get("ip")] = a["nodeName"]
    for i, ss in enumerate(ep.get("subsets") or []):
        ip = f"subsets[{i}]"
        if not ss.get("addresses") and not ss.get("notReadyAddresses"):
            errs.append(required(ip, "must specify `addresses` or `notReadyAddresses`"))
        for kind in ("addresses", "notReadyAddresses"):
            for j, a in enumerate(ss.get(kind) or []):
                ap = f"{ip}.{kind}[{j}]"
                ae = [invalid(f"{ap}.ip", a.get("ip") or "", m) for m in is_valid_ip(a.get("ip") or "")]
                if a.get("hostname"):
                    ae += dns_label(a["hostname"], f"{ap}.hostname")
                if a.get("nodeName") is not None:
                    ae += dns_subdomain(a["nodeName"], f"{ap}.nodeName")
                prev = old_nodes.get(a.get("ip"))
                if prev is not None and a.get("nodeName") != prev:
                    ae.append(forbidden(f"{ap}.nodeName", "Cannot change NodeName for " + str(a.get("ip")) + " to "
                                        + str(a.get("nodeName") or "")))
                if not ae:
                    ae = validate_non_special_ip(a.get("ip") or "", f"{ap}.ip")
                errs += ae
        ports = ss.get("ports") or []
        for j, port in enumerate(ports):
            pp = f"{ip}.ports[{j}]"
            if len(ports) > 1 and not port.get("name"):
                errs.append(required(f"{pp}.name"))
            elif port.get("name"):
                errs += dns_label(port["name"], f"{pp}.name")
            errs += [invalid(f"{pp}.port", port.get("port", 0), m) for m in is_valid_port_num(port.get("port", 0))]
            proto = port.get("protocol") or ""
            if not proto:
                errs.append(required(f"{pp}.protocol"))
            elif proto not in ("TCP", "UDP"):
                errs.append(not_supported(f"{pp}.protocol", proto, ["TCP", "UDP"]))
    return errs


def validate_service_account(sa, old=None) -> list[str]:
    from .validation import validate_object_meta
    return validate_object_meta(sa, True)


MAX_SECRET_SIZE = 1 * 1024 * 1024


def _b64len(v) -> int:
    import base64
    try:
        return len(base64.b64decode(v or "", validate=False))
    except Exception:
        return len(v or "")


def validate_secret(s, old=None) -> list[str]:
    import base64
    from .validation import is_config_map_key, validate_object_meta
    errs = validate_object_meta(s, True)
    data = dict(s.get("data") or {})
    for k, v in (s.get("stringData") or {}).items():
        data[k] = base64.b64encode(str(v).encode()).decode()
    total = 0
    for k, v in data.items():
        errs += [invalid(f"data[{k}]", k, m) for m in is_config_map_key(k)]
        total += _b64len(v)
    if total > MAX_SECRET_SIZE:
        errs.append(too_long("data", MAX_SECRET_SIZE))
    typ = s.get("type") or ""
    ann = (s.get("metadata") or {}).get("annotations") or {}

    def js(key):
        try:
            json.loads(base64.b64decode(data[key]).decode())
            return []
        except Exception as e:
            return [invalid(f"data[{key}]", "<secret contents redacted>", str(e))]
    if typ == "kubernetes.io/service-account-token":
        if not ann.get("kubernetes.io/service-account.name"):
            errs.append(required("metadata.annotations[kubernetes.io/service-account.name]"))
    elif typ == "kubernetes.io/dockercfg":
        errs += [required("data[.dockercfg]")] if ".dockercfg" not in data else js(".dockercfg")
    elif typ == "kubernetes.io/dockerconfigjson":
        errs += [required("data[.dockerconfigjson]")] if ".dockerconfigjson" not in data else js(".dockerconfigjson")
    elif typ == "kubernetes.io/basic-auth":
        if "username" not in data and "password" not in data:
            errs += [required("data[%s][username]"), required("data[%s][password]")]
    elif typ == "kubernetes.io/ssh-auth":
        if not _b64len(data.get("ssh-privatekey")):
            errs.append(required("data[%s][ssh-privatekey]"))
    elif typ == "kubernetes.io/tls":
        for k in ("tls.crt", "tls.key"):
            if k not in data:
                errs.append(required(f"data[{k}]"))
    if old is not None:
        ot = old.get("type") or ""
        if (s.get("type") or ot) != ot:
            errs.append(invalid("type", s.get("type"), IMMUTABLE))
    return errs


def validate_config_map(cm, old=None) -> list[str]:
    from .validation import is_config_map_key, validate_object_meta
    errs = validate_object_meta(cm, True)
    total = 0
    for field_ in ("data", "binaryData"):
        for k, v in (cm.get(field_) or {}).items():
            errs += [invalid(f"{field_}[{k}]", k, m) for m in is_config_map_key(k)]
            total += len(v or "")
    if total > MAX_SECRET_SIZE:
        errs.append(too_long("data", MAX_SECRET_SIZE))
    return errs


STANDARD_FINALIZERS = ("kubernetes", "orphan", "foregroundDeletion")


def validate_namespace(ns, old=None) -> list[str]:
    from .validation import validate_object_meta
    errs = validate_object_meta(ns, False, is_dns1123_label)
    for f in ((ns.get("spec") or {}).get("finalizers")) or []:
        ms = is_qualified_name(f)
        if ms:
            errs += [invalid("spec.finalizers", f, m) for m in ms]
        elif "/" not in f and f not in STANDARD_FINALIZERS:
            errs.append(invalid("spec.finalizers", f, "name is neither a standard finalizer name nor is it fully qualified"))
    return errs
