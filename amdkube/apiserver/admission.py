"""Admission chain: ordered mutating (`admit`) then validating (`validate`) plugins.

Reference: staging/src/k8s.io/apiserver/pkg/admission (chain, Attributes, Handler with
operation filter); plugin registry names in cmd/kube-apiserver/app/options/plugins.go:51,82.

Plugins implemented:
  * ResourceV2 — the fork's rewrite of legacy container limits into device-granular
    PodSpec.extendedResources (plugin/pkg/admission/resourcev2/admission.go:51-118).
    Deliberate change: the converted resource names are configurable
    and default to amd.com/gpu (the reference hard-codes nvidia.com/gpu at :64,79).
  * ExtendedResourceToleration — tolerate NoSchedule taints keyed by requested extended
    resources (plugin/pkg/admission/extendedresourcetoleration/admission.go:32-80); it
    also considers the fork's pod-level extendedResources.
  * NamespaceLifecycle, NamespaceAutoProvision/Exists, LimitRanger (Container/Pod/PVC
    defaults and min/max/maxLimitRequestRatio), ResourceQuota (evaluators of amdkube.quota,
    scopes, CAS-reserved status.used), ServiceAccount (default SA name),
    DefaultTolerationSeconds, Priority, PodNodeSelector, AlwaysAdmit, AlwaysDeny.
"""
from __future__ import annotations

import copy
import uuid

from ..api import meta as m
from ..api.helpers import (GPU_RESOURCE, pod_extended_resource_name, pod_requests, ExtendedResourceError,
                           is_extended_resource_name)
from ..api.quantity import Quantity

CREATE, UPDATE, DELETE, CONNECT = "CREATE", "UPDATE", "DELETE", "CONNECT"


class Attributes:
    __slots__ = ("operation", "resource", "subresource", "namespace", "name", "obj", "old", "user", "kind", "group",
                 "dry_run")

    def __init__(self, operation, resource, subresource, namespace, name, obj, old=None, user=None, kind="", group="",
                 dry_run=False):
        self.operation, self.resource, self.subresource = operation, resource, subresource
        self.namespace, self.name, self.obj, self.old, self.user, self.kind = namespace, name, obj, old, user, kind
        self.group = group
        self.dry_run = dry_run          # ?dryRun=All or a webhook preview: check, but change nothing


class Plugin:
    name = ""
    operations = (CREATE, UPDATE)

    def handles(self, op: str) -> bool:
        return op in self.operations

    def admit(self, a: Attributes, ctx) -> None:  # mutating
        pass

    def validate(self, a: Attributes, ctx) -> None:  # validating
        pass


def _resource_str(a) -> str:
    """schema.GroupResource.String(): `pods`, `deployments.extensions`."""
    return f"{a.resource}.{a.group}" if getattr(a, "group", "") else a.resource


def new_forbidden(a, err) -> m.StatusError:
    """admission.NewForbidden (apiserver/pkg/admission/errors.go): `<resource> "<name>" is
    forbidden: <err>`, the name from the request, else the object's name or generateName, else
    "Unknown"; a Forbidden error passes through unwrapped."""
    if isinstance(err, m.StatusError):
        if err.code == 403:
            return err
        err = err.message
    name = a.name
    if not name:
        md = ((a.obj or {}).get("metadata") or {}) if isinstance(a.obj, dict) else {}
        name = md.get("name") or md.get("generateName") or "Unknown"
    return m.forbidden(f'{_resource_str(a)} "{name}" is forbidden: {err}')


def forbidden_for(resource: str, name: str, err: str) -> m.StatusError:
    """errors.NewForbidden(qualifiedResource, name, err)."""
    return m.forbidden(f'{resource} "{name}" is forbidden: {err}')


def unknown_error(msg: str) -> m.StatusError:
    """A plain Go error returned by a plugin: the handler answers 500 with reason Unknown
    (responsewriters.ErrorToAPIStatus)."""
    return m.StatusError(500, "", msg)


def internal_error_message(msg: str) -> str:
    """errors.NewInternalError(err).Error()."""
    return f"Internal error occurred: {msg}"


def is_initialized(obj) -> bool:
    ini = ((obj or {}).get("metadata") or {}).get("initializers")
    return ini is None or not ini.get("pending")


def is_updating_initialized(a) -> bool:
    """kubeapiserver/admission/util IsUpdatingInitializedObject."""
    return a.operation == UPDATE and is_initialized(a.old)


def is_updating_uninitialized(a) -> bool:
    return a.operation == UPDATE and not is_initialized(a.old)


# ------------------------------------------------------- toleration helpers
def _tol(t, k):
    v = t.get(k)
    return "" if v is None and k != "tolerationSeconds" else v


def match_toleration(a: dict, b: dict) -> bool:
    """core Toleration.MatchToleration: key, effect, operator and value equal."""
    return all(_tol(a, k) == _tol(b, k) for k in ("key", "effect", "operator", "value"))


def tolerations_equal(a: dict, b: dict) -> bool:
    """pkg/util/tolerations AreEqual (tolerationSeconds included)."""
    return match_toleration(a, b) and a.get("tolerationSeconds") == b.get("tolerationSeconds")


def add_or_update_toleration(spec: dict, tol: dict) -> bool:
    """helper.AddOrUpdateTolerationInPod: a matching toleration is replaced (nothing happens when
    it is identical), otherwise the new one is appended."""
    out, updated = [], False
    for t in spec.get("tolerations") or []:
        if match_toleration(tol, t):
            if tolerations_equal(tol, t):
                return False
            out.append(dict(tol))
            updated = True
            continue
        out.append(t)
    if not updated:
        out.append(dict(tol))
    spec["tolerations"] = out
    return True


def _tol_map(ts) -> dict:
    """ConvertTolerationToAMap: keyed by (key, effect), the last one wins."""
    return {(_tol(t, "key"), _tol(t, "effect")): t for t in ts or []}


def tolerations_conflict(first, second) -> bool:
    """IsConflict: a (key, effect) present in both with another definition."""
    b = _tol_map(second)
    return any(k in b and not tolerations_equal(v, b[k]) for k, v in _tol_map(first).items())


def merge_tolerations(first, second) -> list:
    """MergeTolerations: `second`, then the tolerations of `first` whose (key, effect) it lacks."""
    b = _tol_map(second)
    return list(second or []) + [v for k, v in _tol_map(first).items() if k not in b]


def verify_against_whitelist(tolerations, whitelist) -> bool:
    if not whitelist:
        return True
    w = _tol_map(whitelist)
    return all(k in w and tolerations_equal(v, w[k]) for k, v in _tol_map(tolerations).items())


def convert_selector_to_labels_map(s: str) -> dict:
    """labels.ConvertSelectorToLabelsMap: `k=v, k2=v2` (spaces trimmed), keys and values
    validated as label keys and values."""
    from ..api.labels import is_qualified_name, is_valid_label_value
    out = {}
    if not s:
        return out
    for term in s.split(","):
        kv = term.strip().split("=")
        if len(kv) != 2:
            raise ValueError(f"invalid selector: {s}")
        k, v = kv[0].strip(), kv[1].strip()
        if is_qualified_name(k):
            raise ValueError(f"invalid label key {k!r}: {'; '.join(is_qualified_name(k))}")
        if is_valid_label_value(v):
            raise ValueError(f"invalid label value: {v!r}: {'; '.join(is_valid_label_value(v))}")
        out[k] = v
    return out


def labels_conflict(a: dict, b: dict) -> bool:
    return any(k in b and b[k] != v for k, v in a.items())


# MI355X partition resources advertised by the AMD plugin's "mixed" naming strategy
PARTITION_RESOURCES = tuple(f"amd.com/{cp}_{mp}" for cp in ("spx", "dpx", "qpx", "cpx") for mp in ("nps1", "nps2"))


class ResourceV2(Plugin):
    name = "ResourceV2"

    def __init__(self, resource_names=(GPU_RESOURCE,) + PARTITION_RESOURCES):
        self.resource_names = tuple(resource_names)

    def admit(self, a, ctx):
        if a.subresource or a.resource != "pods":
            return
        spec = a.obj.setdefault("spec", {})
        existing = {p.get("name"): p for p in spec.get("extendedResources") or []}
        for kind in ("initContainers", "containers"):
            for c in spec.get(kind) or []:
                res = c.get("resources") or {}
                lim = res.get("limits") or {}
                for rname in [r for r in lim if r in self.resource_names]:
                    val = lim[rname]
                    if Quantity(val).is_zero():
                        continue
                    # UPDATE of an already converted pod (e.g. `kubectl apply` of the original
                    # manifest): reuse the container's existing extended resource, do not mint a new one
                    reuse = [ref for ref in c.get("extendedResourceRequests") or []
                             if ((existing.get(ref) or {}).get("resources") or {}).get("limits", {}).get(rname) is not None
                             and Quantity(existing[ref]["resources"]["limits"][rname]) == Quantity(val)]
                    if a.operation == UPDATE and reuse:
                        lim.pop(rname, None)
                        (res.get("requests") or {}).pop(rname, None)
                        continue
                    name = str(uuid.uuid4())
                    spec.setdefault("extendedResources", []).append({
                        "name": name,
                        "resources": {"limits": {rname: val}, "requests": {rname: val}},
                    })
                    c["extendedResourceRequests"] = list(c.get("extendedResourceRequests") or []) + [name]
                    lim.pop(rname, None)
                    (res.get("requests") or {}).pop(rname, None)


class ExtendedResourceToleration(Plugin):
    """extendedresourcetoleration/admission.go Admit: every extended resource a container or
    init container asks for gets a `<name>:Exists:NoSchedule` toleration, in sorted order, through
    AddOrUpdateTolerationInPod. amdkube also reads limits (the request defaults to the limit) and
    the fork's pod-level extendedResources, which ResourceV2 writes before this plugin runs."""
    name = "ExtendedResourceToleration"

    def admit(self, a, ctx):
        if a.subresource or a.resource != "pods":
            return
        spec = a.obj.setdefault("spec", {})
        names = set()
        for kind in ("initContainers", "containers"):
            for c in spec.get(kind) or []:
                for rl in ((c.get("resources") or {}).get("requests") or {}, (c.get("resources") or {}).get("limits") or {}):
                    names.update(r for r in rl if is_extended_resource_name(r))
        for pres in spec.get("extendedResources") or []:
            try:
                names.add(pod_extended_resource_name(pres))
            except ExtendedResourceError:
                pass
        for n in sorted(names):
            add_or_update_toleration(spec, {"key": n, "operator": "Exists", "effect": "NoSchedule"})


class NamespaceLifecycle(Plugin):
    """apiserver/pkg/admission/plugin/namespace/lifecycle Admit: immortal namespaces cannot be
    deleted ("this namespace may not be deleted"); namespaced writes other than deletes (access
    reviews aside) need the namespace to exist (NotFound), and creations are refused while it is
    Terminating ("unable to create new content in namespace X because it is being
    terminated.")."""
    name = "NamespaceLifecycle"
    operations = (CREATE, UPDATE, DELETE)
    immortal = ("default", "kube-system", "kube-public")
    ACCESS_REVIEWS = ("localsubjectaccessreviews", "subjectaccessreviews")

    def validate(self, a, ctx):
        if a.resource == "namespaces" and not a.subresource:
            if a.operation == DELETE and a.name in self.immortal:
                raise forbidden_for("namespaces", a.name, "this namespace may not be deleted")
            return
        if not a.namespace or a.operation == DELETE:
            return
        if a.resource in self.ACCESS_REVIEWS and getattr(a, "group", "") in ("", "authorization.k8s.io"):
            return
        ns = ctx.get_namespace(a.namespace)
        if ns is None:
            raise m.not_found("namespaces", a.namespace)
        if a.operation == CREATE and (ns.get("status") or {}).get("phase") == "Terminating":
            raise new_forbidden(a, f"unable to create new content in namespace {a.namespace} because it is being "
                                   f"terminated.")


class NamespaceAutoProvision(Plugin):
    name = "NamespaceAutoProvision"
    operations = (CREATE,)

    def admit(self, a, ctx):
        if a.namespace and a.resource != "namespaces" and ctx.get_namespace(a.namespace) is None:
            ctx.create_namespace(a.namespace)


class NamespaceExists(Plugin):
    name = "NamespaceExists"
    operations = (CREATE, UPDATE, DELETE)

    def validate(self, a, ctx):
        if a.namespace and a.resource != "namespaces" and ctx.get_namespace(a.namespace) is None:
            raise m.not_found("namespaces", a.namespace)


MIRROR_POD_ANNOTATION = "kubernetes.io/config.mirror"
SA_TOKEN_MOUNT_PATH = "/var/run/secrets/kubernetes.io/serviceaccount"
ENFORCE_MOUNTABLE_SECRETS = "kubernetes.io/enforce-mountable-secrets"


def _forbid(pod: dict, msg: str) -> m.StatusError:
    """admission.NewForbidden: `pods "<name>" is forbidden: <why>`."""
    name = m.name_of(pod) or (pod.get("metadata") or {}).get("generateName", "")
    return m.forbidden(f'pods "{name}" is forbidden: {msg}')


def _parse_bool(v: str) -> bool:
    """strconv.ParseBool's true spellings (anything else, errors included, is false)."""
    return v in ("1", "t", "T", "TRUE", "true", "True")


class ServiceAccount(Plugin):
    """plugin/pkg/admission/serviceaccount/admission.go (create, and updates of uninitialized
    pods): default `serviceAccountName`; refuse a pod naming a ServiceAccount that does not
    exist; mount the first API token secret the account references (a token secret annotated
    with the account's name and, when set, uid) at /var/run/secrets/kubernetes.io/serviceaccount
    in every container without a mount there (unless the pod, else the account, sets
    automountServiceAccountToken: false); copy the account's imagePullSecrets into a pod without
    any; with the kubernetes.io/enforce-mountable-secrets annotation (or LimitSecretReferences)
    allow only secret volumes, env secretKeyRefs and imagePullSecrets the account references;
    keep mirror pods free of accounts and secrets.

    Deliberate difference: the reference also refuses a pod while the "default" account or its
    token does not exist yet (RequireAPIToken, "retry after the token is automatically
    created"); here a missing default account or token mounts nothing, so clusters run without
    the ServiceAccount/token controllers (the benches, the node e2e setups) still start pods.
    `require_api_token=True` restores the reference's refusal."""
    name = "ServiceAccount"
    operations = (CREATE, UPDATE)

    def __init__(self, require_api_token: bool = False, limit_secret_references: bool = False,
                 mount_service_account_token: bool = True):
        self.require_api_token = require_api_token
        self.limit_secret_references = limit_secret_references
        self.mount_token = mount_service_account_token

    @staticmethod
    def _ignore(a) -> bool:
        return a.resource != "pods" or getattr(a, "group", "") or not isinstance(a.obj, dict) or \
            (a.obj.get("kind") not in (None, "Pod")) or is_updating_initialized(a)

    def admit(self, a, ctx):
        if self._ignore(a):
            return
        pod = a.obj
        if MIRROR_POD_ANNOTATION in m.annotations_of(pod):
            return self.validate(a, ctx)
        spec = pod.setdefault("spec", {})
        if not spec.get("serviceAccountName"):
            spec["serviceAccountName"] = "default"
        sa_name = spec["serviceAccountName"]
        sa = ctx.get_object("serviceaccounts", a.namespace, sa_name)
        if sa is None:
            if sa_name != "default" or self.require_api_token:
                raise new_forbidden(a, f'error looking up service account {a.namespace}/{sa_name}: serviceaccount '
                                       f'"{sa_name}" not found')
            return
        automount = spec.get("automountServiceAccountToken")
        if automount is None:
            automount = sa.get("automountServiceAccountToken")
        if self.mount_token and automount is not False:
            self._mount_token(sa, pod, ctx)
        if not spec.get("imagePullSecrets") and sa.get("imagePullSecrets"):
            spec["imagePullSecrets"] = [dict(x) for x in sa["imagePullSecrets"]]
        self.validate(a, ctx)

    def validate(self, a, ctx):
        if self._ignore(a):
            return
        pod = a.obj
        spec = pod.get("spec") or {}
        if MIRROR_POD_ANNOTATION in m.annotations_of(pod):
            if spec.get("serviceAccountName"):
                raise new_forbidden(a, "a mirror pod may not reference service accounts")
            if pod_secret_names(pod):
                raise new_forbidden(a, "a mirror pod may not reference secrets")
            return
        sa_name = spec.get("serviceAccountName", "")
        sa = ctx.get_object("serviceaccounts", a.namespace, sa_name)
        if sa is None:
            if sa_name != "default" or self.require_api_token:
                raise new_forbidden(a, f'error looking up service account {a.namespace}/{sa_name}: serviceaccount '
                                       f'"{sa_name}" not found')
            return
        if self.limit_secret_references or _parse_bool(m.annotations_of(sa).get(ENFORCE_MOUNTABLE_SECRETS, "")):
            err = self._limit_secret_references(sa, pod)
            if err:
                raise new_forbidden(a, err)

    @staticmethod
    def _limit_secret_references(sa: dict, pod: dict) -> str:
        mountable = {r.get("name") for r in sa.get("secrets") or []}
        sa_name = m.name_of(sa)
        spec = pod.get("spec") or {}
        for v in spec.get("volumes") or []:
            if v.get("secret") is not None and v["secret"].get("secretName", "") not in mountable:
                return (f'volume with secret.secretName="{v["secret"].get("secretName", "")}" is not allowed because '
                        f"service account {sa_name} does not reference that secret")
        for kind, what in (("initContainers", "init container"), ("containers", "container")):
            for c in spec.get(kind) or []:
                for e in c.get("env") or []:
                    ref = (e.get("valueFrom") or {}).get("secretKeyRef")
                    if ref is not None and ref.get("name", "") not in mountable:
                        return (f'{what} {c.get("name", "")} with envVar {e.get("name", "")} referencing '
                                f'secret.secretName="{ref.get("name", "")}" is not allowed because service account '
                                f"{sa_name} does not reference that secret")
        pulls = {r.get("name") for r in sa.get("imagePullSecrets") or []}
        for i, ref in enumerate(spec.get("imagePullSecrets") or []):
            if ref.get("name") not in pulls:
                return (f'imagePullSecrets[{i}].name="{ref.get("name", "")}" is not allowed because service account '
                        f"{sa_name} does not reference that imagePullSecret")
        return ""

    @staticmethod
    def service_account_tokens(sa: dict, ctx) -> list[dict]:
        """getServiceAccountTokens: the namespace's token secrets that belong to the account
        (IsServiceAccountToken: the name annotation matches, the uid annotation when set)."""
        out = []
        for sec in ctx.list_objects("secrets", m.namespace_of(sa)):
            if sec.get("type") != "kubernetes.io/service-account-token":
                continue
            ann = m.annotations_of(sec)
            if ann.get("kubernetes.io/service-account.name") != m.name_of(sa):
                continue
            uid = ann.get("kubernetes.io/service-account.uid", "")
            if uid and uid != (sa.get("metadata") or {}).get("uid", ""):
                continue
            out.append(sec)
        return out

    def _token_secret(self, sa: dict, ctx) -> str:
        """getReferencedServiceAccountToken: the first of the account's secrets that is one of
        its tokens."""
        if not sa.get("secrets"):
            return ""
        tokens = {m.name_of(t) for t in self.service_account_tokens(sa, ctx)}
        return next((r.get("name") for r in sa["secrets"] if r.get("name") in tokens), "")

    def _mount_token(self, sa: dict, pod: dict, ctx):
        token = self._token_secret(sa, ctx)
        if not token:
            if self.require_api_token:
                raise m.StatusError(504, "ServerTimeout", f"No API token found for service account "
                                                          f"\"{m.name_of(sa)}\", retry after the token is "
                                                          f"automatically created and added to the service account")
            return
        spec = pod["spec"]
        volumes = spec.get("volumes") or []
        vol_name = next((v["name"] for v in volumes if (v.get("secret") or {}).get("secretName") == token), "")
        has_volume = bool(vol_name)
        if not vol_name:
            names = {v.get("name") for v in volumes}
            vol_name = token if token not in names else f"{token}-{uuid.uuid4().hex[:5]}"
        need = False
        for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
            if any(vm.get("mountPath") == SA_TOKEN_MOUNT_PATH for vm in c.get("volumeMounts") or []):
                continue
            c.setdefault("volumeMounts", []).append({"name": vol_name, "readOnly": True, "mountPath": SA_TOKEN_MOUNT_PATH})
            need = True
        if need and not has_volume:
            spec["volumes"] = list(volumes) + [{"name": vol_name, "secret": {"secretName": token}}]


NOT_READY_TAINT_KEY = "node.kubernetes.io/not-ready"
UNREACHABLE_TAINT_KEY = "node.kubernetes.io/unreachable"


class DefaultTolerationSeconds(Plugin):
    """defaulttolerationseconds/admission.go Admit (create and update): a pod that does not
    already tolerate node.kubernetes.io/not-ready:NoExecute (or unreachable) — a toleration with
    that key or no key, and NoExecute or no effect — gets `Exists:NoExecute` for
    --default-not-ready-toleration-seconds / --default-unreachable-toleration-seconds (300)."""
    name = "DefaultTolerationSeconds"

    def __init__(self, seconds=300, not_ready_seconds=None, unreachable_seconds=None):
        self.not_ready = seconds if not_ready_seconds is None else not_ready_seconds
        self.unreachable = seconds if unreachable_seconds is None else unreachable_seconds

    def admit(self, a, ctx):
        if a.resource != "pods" or a.subresource:
            return
        spec = a.obj.setdefault("spec", {})
        tols = spec.get("tolerations") or []

        def tolerates(key):
            return any(_tol(t, "key") in (key, "") and _tol(t, "effect") in ("NoExecute", "") for t in tols)
        nr, ur = tolerates(NOT_READY_TAINT_KEY), tolerates(UNREACHABLE_TAINT_KEY)
        if not nr:
            add_or_update_toleration(spec, {"key": NOT_READY_TAINT_KEY, "operator": "Exists", "effect": "NoExecute",
                                            "tolerationSeconds": self.not_ready})
        if not ur:
            add_or_update_toleration(spec, {"key": UNREACHABLE_TAINT_KEY, "operator": "Exists", "effect": "NoExecute",
                                            "tolerationSeconds": self.unreachable})


LIMIT_RANGER_ANNOTATION = "kubernetes.io/limit-ranger"


def _forbidden(a, msg: str) -> m.StatusError:
    """admission.NewForbidden: `<resource> "<name>" is forbidden: <reason>`."""
    return m.forbidden(f'{a.resource} "{a.name}" is forbidden: {msg}')


def _lr_values(req, lim, enforced) -> tuple[int, int, int]:
    """requestLimitEnforcedValues: milli-units unless a value would overflow them."""
    vals = [Quantity(x) if x is not None else Quantity(0) for x in (req, lim, enforced)]
    if all(v.value() <= _MAX_MILLI for v in vals):
        return tuple(v.milli_value() for v in vals)
    return tuple(v.value() for v in vals)


_MAX_MILLI = (1 << 63) // 1000


def _min_constraint(ltype, r, enforced, request, limit):
    req, lim = request.get(r), limit.get(r)
    rv, lv, ev = _lr_values(req, lim, enforced)
    if req is None:
        return f"minimum {r} usage per {ltype} is {Quantity(enforced)}.  No request is specified."
    if rv < ev:
        return f"minimum {r} usage per {ltype} is {Quantity(enforced)}, but request is {Quantity(req)}."
    if lim is not None and lv < ev:
        return f"minimum {r} usage per {ltype} is {Quantity(enforced)}, but limit is {Quantity(lim)}."
    return None


def _max_request_constraint(ltype, r, enforced, request):
    req = request.get(r)
    rv, _, ev = _lr_values(req, None, enforced)
    if req is None:
        return f"maximum {r} usage per {ltype} is {Quantity(enforced)}.  No request is specified."
    if rv > ev:
        return f"maximum {r} usage per {ltype} is {Quantity(enforced)}, but request is {Quantity(req)}."
    return None


def _max_constraint(ltype, r, enforced, request, limit):
    req, lim = request.get(r), limit.get(r)
    rv, lv, ev = _lr_values(req, lim, enforced)
    if lim is None:
        return f"maximum {r} usage per {ltype} is {Quantity(enforced)}.  No limit is specified."
    if lv > ev:
        return f"maximum {r} usage per {ltype} is {Quantity(enforced)}, but limit is {Quantity(lim)}."
    if req is not None and rv > ev:
        return f"maximum {r} usage per {ltype} is {Quantity(enforced)}, but request is {Quantity(req)}."
    return None


def _ratio_constraint(ltype, r, enforced, request, limit):
    req, lim = request.get(r), limit.get(r)
    rv, lv, _ = _lr_values(req, lim, enforced)
    e = Quantity(enforced)
    if req is None or rv == 0:
        return f"{r} max limit to request ratio per {ltype} is {e}, but no request is specified or request is 0."
    if lim is None or lv == 0:
        return f"{r} max limit to request ratio per {ltype} is {e}, but no limit is specified or limit is 0."
    observed = lv / rv
    shown = observed
    cap = float(e.value())
    if e.value() <= _MAX_MILLI:
        observed *= 1000
        cap = float(e.milli_value())
    if observed > cap:
        return f"{r} max limit to request ratio per {ltype} is {e}, but provided ratio is {shown:f}."
    return None


def _check_item(ltype, item, request, limit, errs):
    for r, v in (item.get("min") or {}).items():
        e = _min_constraint(ltype, r, v, request, limit)
        if e:
            errs.append(e)
    for r, v in (item.get("max") or {}).items():
        e = _max_constraint(ltype, r, v, request, limit)
        if e:
            errs.append(e)
    for r, v in (item.get("maxLimitRequestRatio") or {}).items():
        e = _ratio_constraint(ltype, r, v, request, limit)
        if e:
            errs.append(e)


def _sum_lists(lists: list[dict]) -> dict:
    """limitranger sum(): a resource is summed only when every container sets it."""
    keys = {k for rl in lists for k in rl}
    out = {}
    for k in keys:
        if all(k in rl for rl in lists):
            tot = sum(Quantity(rl[k]).milli_value() if k == "cpu" else Quantity(rl[k]).value() for rl in lists)
            out[k] = f"{tot}m" if k == "cpu" else str(tot)
    return out


def default_container_requirements(lr: dict) -> tuple[dict, dict]:
    """defaultContainerResourceRequirements: (default requests, default limits) of the Container
    items. A stored LimitRange is already defaulted (SetDefaults_LimitRangeItem, in
    amdkube.api.defaults: default <- max, defaultRequest <- default <- min)."""
    reqs, lims = {}, {}
    for item in (lr.get("spec") or {}).get("limits") or []:
        if item.get("type") != "Container":
            continue
        reqs.update(item.get("defaultRequest") or {})
        lims.update(item.get("default") or {})
    return reqs, lims


class LimitRanger(Plugin):
    """plugin/pkg/admission/limitranger/admission.go: mutate pods with the Container defaults
    (default / defaultRequest, recorded in the kubernetes.io/limit-ranger annotation), then
    enforce min / max / maxLimitRequestRatio per Container (containers and init containers), per
    Pod (the containers' sum, raised to the largest init container), and min / max storage
    request per PersistentVolumeClaim. Runs on CREATE and UPDATE, never on subresources."""
    name = "LimitRanger"
    operations = (CREATE, UPDATE)

    @staticmethod
    def _supports(a) -> bool:
        return not a.subresource and a.resource in ("pods", "persistentvolumeclaims") and a.obj is not None

    def admit(self, a, ctx):
        if not self._supports(a) or a.resource != "pods":
            return
        for lr in ctx.list_objects("limitranges", a.namespace):
            reqs, lims = default_container_requirements(lr)
            if not reqs and not lims:
                continue
            spec = a.obj.setdefault("spec", {})
            notes = []
            for kind, label in (("containers", "container"), ("initContainers", "init container")):
                for c in spec.get(kind) or []:
                    res = c.setdefault("resources", {})
                    cl, cr = res.setdefault("limits", {}), res.setdefault("requests", {})
                    set_l = sorted(k for k in lims if k not in cl)
                    set_r = sorted(k for k in reqs if k not in cr)
                    for k in set_l:
                        cl[k] = lims[k]
                    for k in set_r:
                        cr[k] = reqs[k]
                    if set_r:
                        notes.append(", ".join(set_r) + f" request for {label} {c.get('name', '')}")
                    if set_l:
                        notes.append(", ".join(set_l) + f" limit for {label} {c.get('name', '')}")
                    if not cl:
                        res.pop("limits")
                    if not cr:
                        res.pop("requests")
            if notes:
                a.obj.setdefault("metadata", {}).setdefault("annotations", {})[LIMIT_RANGER_ANNOTATION] = \
                    "LimitRanger plugin set: " + "; ".join(notes)

    def validate(self, a, ctx):
        if not self._supports(a):
            return
        for lr in ctx.list_objects("limitranges", a.namespace):
            errs: list[str] = []
            items = (lr.get("spec") or {}).get("limits") or []
            if a.resource == "persistentvolumeclaims":
                reqs = (((a.obj.get("spec") or {}).get("resources") or {}).get("requests") or {})
                for item in items:
                    if item.get("type") != "PersistentVolumeClaim":
                        continue
                    for r, v in (item.get("min") or {}).items():
                        e = _min_constraint("PersistentVolumeClaim", r, v, reqs, {})
                        if e:
                            errs.append(e)
                    for r, v in (item.get("max") or {}).items():
                        e = _max_request_constraint("PersistentVolumeClaim", r, v, reqs)
                        if e:
                            errs.append(e)
            else:
                spec = a.obj.get("spec") or {}
                for item in items:
                    t = item.get("type")
                    if t == "Container":
                        for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
                            res = c.get("resources") or {}
                            _check_item("Container", item, res.get("requests") or {}, res.get("limits") or {}, errs)
                    elif t == "Pod":
                        cs = spec.get("containers") or []
                        preq = _sum_lists([((c.get("resources") or {}).get("requests") or {}) for c in cs])
                        plim = _sum_lists([((c.get("resources") or {}).get("limits") or {}) for c in cs])
                        for c in spec.get("initContainers") or []:
                            res = c.get("resources") or {}
                            for dst, src in ((preq, res.get("requests") or {}), (plim, res.get("limits") or {})):
                                for k, v in src.items():
                                    if k not in dst or Quantity(dst[k]) < Quantity(v):
                                        dst[k] = v
                        _check_item("Pod", item, preq, plim, errs)
            if errs:
                raise _forbidden(a, errs[0] if len(errs) == 1 else "[" + ", ".join(errs) + "]")


class ResourceQuota(Plugin):
    """plugin/pkg/admission/resourcequota (controller.go checkRequest :372-517): for every quota
    in the namespace that the object's evaluator matches (a limited resource name, every scope),
    require the quota's status to be populated, check the container constraints, and charge the
    object's usage (its delta on UPDATE) against status.used; the charge is written back to the
    quota's status with a compare-and-swap on the quota object, re-checked against the current
    status on every CAS miss, so concurrent admissions (on one apiserver or several sharing an
    etcd) serialize on the quota and can never both take its last unit."""
    name = "ResourceQuota"
    operations = (CREATE, UPDATE)

    def validate(self, a, ctx):
        if a.subresource or not a.namespace or a.obj is None:
            return
        from .. import quota as Q
        ev = Q.evaluator_for(a.resource, a.group)
        if a.operation not in ev.operations:
            return
        quotas = [qq for qq in ctx.list_objects("resourcequotas", a.namespace) if ev.matches(qq, a.obj)]
        if not quotas:
            return
        for qq in quotas:
            hard_names = list(((qq.get("status") or {}).get("hard") or {}))
            err = ev.constraints(ev.matching_resources(hard_names), a.obj)
            if err:
                raise _forbidden(a, f"failed quota: {m.name_of(qq)}: {err}")
            if not Q.has_usage_stats(qq):
                raise _forbidden(a, f"status unknown for quota: {m.name_of(qq)}")
        delta = Q.pod_usage(a.obj) if ev is Q.POD_EVALUATOR else ev.usage(a.obj)
        neg = Q.negative(delta)
        if neg:
            raise _forbidden(a, f"quota usage is negative for resource(s): {', '.join(neg)}")
        if a.operation == UPDATE and a.old is not None:
            prev = Q.pod_usage(a.old) if ev is Q.POD_EVALUATOR else ev.usage(a.old)
            delta = Q.subtract_non_negative(delta, prev)
        if Q.is_zero(delta):
            return
        if a.dry_run:
            # a dry run (or the validating-webhook preview of a create) is checked against the
            # quotas as they stand, but takes nothing: the real request charges once
            for qq in quotas:
                self._charge(ctx, Q, qq, delta, a, check_only=True)
            return
        charged = []
        try:
            for qq in quotas:
                self._charge(ctx, Q, qq, delta, a)
                charged.append(qq)
        except m.StatusError:
            for qq in charged:             # give back what an earlier quota already took
                try:
                    self._charge(ctx, Q, qq, delta, a, refund=True)
                except m.StatusError:
                    pass                   # the quota controller recomputes usage anyway
            raise

    @staticmethod
    def _charge(ctx, Q, quota, delta, a, refund=False, check_only=False):
        name = m.name_of(quota)

        def apply(cur):
            if cur is None:
                raise _forbidden(a, f"status unknown for quota: {name}")
            st = cur.get("status") or {}
            hard = Q.parse_list(st.get("hard"))
            used = Q.parse_list(st.get("used"))
            requested = Q.mask(delta, hard)
            if not requested:
                return None
            if refund:
                new_used = Q.subtract_non_negative(used, requested)
            else:
                new_used = Q.add(used, requested)
                ok, exceeded = Q.less_than_or_equal(Q.mask(new_used, requested), hard)
                if not ok:
                    raise _forbidden(a, f"exceeded quota: {name}, requested: {Q.pretty(Q.mask(requested, exceeded))}, "
                                        f"used: {Q.pretty(Q.mask(used, exceeded))}, limited: {Q.pretty(Q.mask(hard, exceeded))}")
            out = m.deepcopy(cur)
            out.setdefault("status", {})["used"] = {**(st.get("used") or {}), **Q.format_list(Q.mask(new_used, requested))}
            return out
        if check_only:
            apply(quota)
            return
        ctx.guaranteed_update_object("resourcequotas", m.namespace_of(quota), name, apply)


SYSTEM_PRIORITY_CLASSES = {"system-cluster-critical": 2000000000, "system-node-critical": 2000001000}
HIGHEST_USER_DEFINABLE_PRIORITY = 1000000000


class Priority(Plugin):
    """priority/admission.go: a new pod may not carry spec.priority itself; it gets the value of
    its priorityClassName (the system classes are built in; an unknown name fails), else of the
    globalDefault class, else 0. PriorityClass writes are checked: value at most 1e9, the system
    names reserved, and only one globalDefault class."""
    name = "Priority"
    operations = (CREATE, UPDATE, DELETE)

    def admit(self, a, ctx):
        if a.subresource or a.resource != "pods" or a.operation != CREATE:
            return
        spec = a.obj.setdefault("spec", {})
        if spec.get("priority") is not None:
            raise new_forbidden(a, "the integer value of priority must not be provided in pod spec. Priority "
                                   "admission controller populates the value from the given PriorityClass name")
        pcn = spec.get("priorityClassName")
        if not pcn:
            dpc = self._default_class(ctx)
            spec["priority"] = int(dpc.get("value", 0)) if dpc else 0
            return
        if pcn in SYSTEM_PRIORITY_CLASSES:
            spec["priority"] = SYSTEM_PRIORITY_CLASSES[pcn]
            return
        pc = ctx.get_object("priorityclasses", "", pcn)
        if pc is None:
            raise unknown_error(f'failed to get default priority class {pcn}: priorityclass.scheduling.k8s.io "{pcn}" '
                                f'not found')
        spec["priority"] = int(pc.get("value", 0))

    @staticmethod
    def _default_class(ctx):
        return next((pc for pc in ctx.list_objects("priorityclasses", "", "scheduling.k8s.io") if pc.get("globalDefault")),
                    None)

    def validate(self, a, ctx):
        if a.subresource or a.resource != "priorityclasses" or a.operation == DELETE:
            return
        pc = a.obj or {}
        if int(pc.get("value") or 0) > HIGHEST_USER_DEFINABLE_PRIORITY:
            raise new_forbidden(a, f"maximum allowed value of a user defined priority is {HIGHEST_USER_DEFINABLE_PRIORITY}")
        if m.name_of(pc) in SYSTEM_PRIORITY_CLASSES:
            raise new_forbidden(a, f"the name of the priority class is a reserved name for system use only: {m.name_of(pc)}")
        if pc.get("globalDefault"):
            dpc = self._default_class(ctx)
            if dpc is not None and (a.operation == CREATE or m.name_of(dpc) != m.name_of(pc)):
                raise new_forbidden(a, f"PriorityClass {m.name_of(dpc)} is already marked as default. Only one default "
                                       f"can exist")


class PodNodeSelector(Plugin):
    """podnodeselector/admission.go: the namespace's scheduler.alpha.kubernetes.io/node-selector
    annotation (else the plugin's clusterDefaultNodeSelector; an empty annotation means none) is
    merged into the pod's nodeSelector — a label the pod sets differently is refused — and the
    result must stay within the namespace's whitelist from the plugin configuration. Updates of
    initialized pods are left alone (their node selector is immutable)."""
    name = "PodNodeSelector"
    ANNOTATION = "scheduler.alpha.kubernetes.io/node-selector"

    def __init__(self, cluster_node_selectors: dict | None = None, **config):
        # podNodeSelectorPluginConfig: {clusterDefaultNodeSelector: ..., <namespace>: <whitelist>}
        self.cluster = dict(cluster_node_selectors or config.get("podNodeSelectorPluginConfig") or {})

    @staticmethod
    def _ignore(a) -> bool:
        return a.resource != "pods" or bool(a.subresource) or not isinstance(a.obj, dict)

    def _namespace_selector(self, a, ctx) -> dict:
        ns = ctx.get_namespace(a.namespace)
        if ns is None:
            raise m.not_found("namespaces", a.namespace)
        ann = m.annotations_of(ns)
        try:
            if self.ANNOTATION in ann:
                return convert_selector_to_labels_map(ann[self.ANNOTATION])
            return convert_selector_to_labels_map(self.cluster.get("clusterDefaultNodeSelector", ""))
        except ValueError as e:
            raise unknown_error(str(e)) from None

    def admit(self, a, ctx):
        if self._ignore(a) or is_updating_initialized(a):
            return
        spec = a.obj.setdefault("spec", {})
        ns_sel = self._namespace_selector(a, ctx)
        pod_sel = spec.get("nodeSelector") or {}
        if labels_conflict(ns_sel, pod_sel):
            raise forbidden_for("pods", m.name_of(a.obj), "pod node label selector conflicts with its namespace node "
                                                           "label selector")
        merged = {**ns_sel, **pod_sel}
        if merged or spec.get("nodeSelector") is not None:
            spec["nodeSelector"] = merged
        self.validate(a, ctx)

    def validate(self, a, ctx):
        if self._ignore(a):
            return
        pod_sel = (a.obj.get("spec") or {}).get("nodeSelector") or {}
        ns_sel = self._namespace_selector(a, ctx)
        if labels_conflict(ns_sel, pod_sel):
            raise forbidden_for("pods", m.name_of(a.obj), "pod node label selector conflicts with its namespace node "
                                                           "label selector")
        try:
            whitelist = convert_selector_to_labels_map(self.cluster.get(a.namespace, ""))
        except ValueError as e:
            raise unknown_error(str(e)) from None
        # labels.AreLabelsInWhiteList: an empty whitelist allows everything
        if whitelist and any(k not in whitelist or whitelist[k] != v for k, v in pod_sel.items()):
            raise forbidden_for("pods", m.name_of(a.obj), "pod node label selector labels conflict with its namespace "
                                                           "whitelist")


DEFAULT_CLASS_ANNOTATIONS = ("storageclass.kubernetes.io/is-default-class",
                             "storageclass.beta.kubernetes.io/is-default-class")


class DefaultStorageClass(Plugin):
    """storageclass/setdefault/admission.go: a claim with neither spec.storageClassName nor the
    volume.beta.kubernetes.io/storage-class annotation gets the class annotated (GA or beta)
    is-default-class=true; more than one default is refused (a wrapped internal error)."""
    name = "DefaultStorageClass"
    operations = (CREATE,)

    def admit(self, a, ctx):
        if a.resource != "persistentvolumeclaims" or a.subresource or not isinstance(a.obj, dict):
            return
        spec = a.obj.setdefault("spec", {})
        if spec.get("storageClassName") is not None or "volume.beta.kubernetes.io/storage-class" in m.annotations_of(a.obj):
            return
        defaults = [sc for sc in ctx.list_objects("storageclasses", "", "storage.k8s.io")
                    if any(m.annotations_of(sc).get(k) == "true" for k in DEFAULT_CLASS_ANNOTATIONS)]
        if len(defaults) > 1:
            raise new_forbidden(a, internal_error_message(f"{len(defaults)} default StorageClasses were found"))
        if defaults:
            spec["storageClassName"] = m.name_of(defaults[0])


class StorageObjectInUseProtection(Plugin):
    """plugin/pkg/admission/storageobjectinuseprotection: new claims and volumes carry the
    kubernetes.io/pvc-protection / pv-protection finalizers."""
    name = "StorageObjectInUseProtection"
    operations = (CREATE,)

    def admit(self, a, ctx):
        fin = {"persistentvolumeclaims": "kubernetes.io/pvc-protection", "persistentvolumes": "kubernetes.io/pv-protection"}.get(
            a.resource)
        if fin and not a.subresource:
            md = a.obj.setdefault("metadata", {})
            if fin not in (md.get("finalizers") or []):
                md["finalizers"] = list(md.get("finalizers") or []) + [fin]


_SECRET_REF_SOURCES = ("cephfs", "flexVolume", "rbd", "scaleIO", "iscsi", "storageos")


def pod_secret_names(pod: dict) -> list[str]:
    """pkg/api/pod VisitPodSecretNames: imagePullSecrets, env/envFrom of every (init) container,
    and the secret-bearing volume sources."""
    spec = pod.get("spec") or {}
    out = [r.get("name", "") for r in spec.get("imagePullSecrets") or []]
    for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
        out += [ef["secretRef"].get("name", "") for ef in c.get("envFrom") or [] if ef.get("secretRef")]
        out += [e["valueFrom"]["secretKeyRef"].get("name", "") for e in c.get("env") or []
                if (e.get("valueFrom") or {}).get("secretKeyRef")]
    for v in spec.get("volumes") or []:
        if v.get("azureFile"):
            if v["azureFile"].get("secretName"):
                out.append(v["azureFile"]["secretName"])
        elif v.get("projected") is not None:
            out += [src["secret"].get("name", "") for src in v["projected"].get("sources") or [] if src.get("secret")]
        elif v.get("secret") is not None:
            out.append(v["secret"].get("secretName", ""))
        else:
            for k in _SECRET_REF_SOURCES:
                if v.get(k) is not None:
                    if (v[k].get("secretRef") or None) is not None:
                        out.append(v[k]["secretRef"].get("name", ""))
                    break
    return out


def pod_configmap_names(pod: dict) -> list[str]:
    """VisitPodConfigmapNames: env/envFrom of every (init) container, configMap and projected
    configMap volume sources."""
    spec = pod.get("spec") or {}
    out = []
    for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
        out += [ef["configMapRef"].get("name", "") for ef in c.get("envFrom") or [] if ef.get("configMapRef")]
        out += [e["valueFrom"]["configMapKeyRef"].get("name", "") for e in c.get("env") or []
                if (e.get("valueFrom") or {}).get("configMapKeyRef")]
    for v in spec.get("volumes") or []:
        if v.get("projected") is not None:
            out += [src["configMap"].get("name", "") for src in v["projected"].get("sources") or [] if src.get("configMap")]
        elif v.get("configMap") is not None:
            out.append(v["configMap"].get("name", ""))
    return out


def node_identity(user) -> tuple[str, bool]:
    """auth/nodeidentifier NodeIdentity: a `system:node:<name>` user in the system:nodes group."""
    name = (user or {}).get("name", "")
    if not name.startswith("system:node:") or "system:nodes" not in ((user or {}).get("groups") or []):
        return "", False
    return name[len("system:node:"):], True


class NodeRestriction(Plugin):
    """plugin/pkg/admission/noderestriction/admission.go: a kubelet (system:node:<name> in
    system:nodes) may create only mirror pods bound to itself that reference no service account,
    secret, configmap or claim; delete and evict only pods bound to itself; update the status of
    its own pods; touch only its own Node (no configSource on create, no new configSource on
    update); and change nothing of a claim but status.capacity and status.conditions (with
    ExpandPersistentVolumes)."""
    name = "NodeRestriction"
    operations = (CREATE, UPDATE, DELETE)

    def __init__(self, expand_persistent_volumes: bool | None = None):
        self.expand = expand_persistent_volumes

    def admit(self, a, ctx):
        node, is_node = node_identity(a.user)
        if not is_node:
            return
        if not node:
            raise new_forbidden(a, f'could not determine node from user "{(a.user or {}).get("name", "")}"')
        if a.resource == "pods" and not getattr(a, "group", ""):
            if a.subresource == "":
                return self._pod(node, a, ctx)
            if a.subresource == "status":
                return self._pod_status(node, a)
            if a.subresource == "eviction":
                return self._pod_eviction(node, a, ctx)
            raise new_forbidden(a, f'unexpected pod subresource "{a.subresource}"')
        if a.resource == "nodes" and not getattr(a, "group", ""):
            return self._node(node, a)
        if a.resource == "persistentvolumeclaims" and not getattr(a, "group", ""):
            if a.subresource == "status":
                return self._pvc_status(node, a)
            raise new_forbidden(a, "may only update PVC status")

    def _existing_pod(self, a, ctx, name):
        pod = ctx.get_object("pods", a.namespace, name)
        if pod is None:
            raise m.not_found("pods", name)
        return pod

    def _pod(self, node, a, ctx):
        if a.operation == CREATE:
            pod = a.obj or {}
            if MIRROR_POD_ANNOTATION not in m.annotations_of(pod):
                raise new_forbidden(a, f'pod does not have "{MIRROR_POD_ANNOTATION}" annotation, node "{node}" can only '
                                       f'create mirror pods')
            spec = pod.get("spec") or {}
            if spec.get("nodeName") != node:
                raise new_forbidden(a, f'node "{node}" can only create pods with spec.nodeName set to itself')
            if spec.get("serviceAccountName"):
                raise new_forbidden(a, f'node "{node}" can not create pods that reference a service account')
            if pod_secret_names(pod):
                raise new_forbidden(a, f'node "{node}" can not create pods that reference secrets')
            if pod_configmap_names(pod):
                raise new_forbidden(a, f'node "{node}" can not create pods that reference configmaps')
            if any(v.get("persistentVolumeClaim") is not None for v in spec.get("volumes") or []):
                raise new_forbidden(a, f'node "{node}" can not create pods that reference persistentvolumeclaims')
            return
        if a.operation == DELETE:
            existing = self._existing_pod(a, ctx, a.name)
            if (existing.get("spec") or {}).get("nodeName") != node:
                raise new_forbidden(a, f'node "{node}" can only delete pods with spec.nodeName set to itself')
            return
        raise new_forbidden(a, f'unexpected operation "{a.operation}"')

    def _pod_status(self, node, a):
        if a.operation != UPDATE:
            raise new_forbidden(a, f'unexpected operation "{a.operation}"')
        if ((a.old or {}).get("spec") or {}).get("nodeName") != node:
            raise new_forbidden(a, f'node "{node}" can only update pod status for pods with spec.nodeName set to itself')

    def _pod_eviction(self, node, a, ctx):
        if a.operation != CREATE:
            raise new_forbidden(a, f"unexpected operation {a.operation}")
        name = a.name or m.name_of(a.obj or {})
        if not name:
            raise new_forbidden(a, "could not determine pod from request data")
        existing = self._existing_pod(a, ctx, name)
        if (existing.get("spec") or {}).get("nodeName") != node:
            raise new_forbidden(a, f"node {node} can only evict pods with spec.nodeName set to itself")

    def _pvc_status(self, node, a):
        if a.operation != UPDATE:
            raise new_forbidden(a, f'unexpected operation "{a.operation}"')
        expand = self.expand
        if expand is None:
            from ..utils.features import DEFAULT
            expand = DEFAULT("ExpandPersistentVolumes")
        if not expand:
            raise new_forbidden(a, f'node "{node}" may not update persistentvolumeclaim metadata')

        def strip(o):
            o = copy.deepcopy(o or {})
            (o.get("metadata") or {}).pop("resourceVersion", None)
            st = o.get("status") or {}
            st.pop("capacity", None)
            st.pop("conditions", None)
            return o
        if strip(a.old) != strip(a.obj):
            raise new_forbidden(a, f'node "{node}" may not update fields other than status.capacity and '
                                   f'status.conditions')

    def _node(self, node, a):
        requested = a.name
        if a.operation == CREATE:
            if ((a.obj or {}).get("spec") or {}).get("configSource") is not None:
                raise new_forbidden(a, "cannot create with non-nil configSource")
            requested = requested or m.name_of(a.obj or {})
        if requested != node:
            raise new_forbidden(a, f'node "{node}" cannot modify node "{requested}"')
        if a.operation == UPDATE:
            new_cs = ((a.obj or {}).get("spec") or {}).get("configSource")
            if new_cs is not None and new_cs != ((a.old or {}).get("spec") or {}).get("configSource"):
                raise new_forbidden(a, "cannot update configSource to a new non-nil configSource")


class AlwaysAdmit(Plugin):
    name = "AlwaysAdmit"


class AlwaysDeny(Plugin):
    name = "AlwaysDeny"
    operations = (CREATE, UPDATE, DELETE, CONNECT)

    def validate(self, a, ctx):
        raise m.forbidden("admission control is denying all modifications")


REGISTRY = {p.name: p for p in (ResourceV2, ExtendedResourceToleration, NamespaceLifecycle, NamespaceAutoProvision,
                                 NamespaceExists, ServiceAccount, DefaultTolerationSeconds, LimitRanger, ResourceQuota,
                                 Priority, PodNodeSelector, DefaultStorageClass, StorageObjectInUseProtection, NodeRestriction,
                                 AlwaysAdmit, AlwaysDeny)}

# Matches the fork's recommended ordering (hack/local-up-cluster.sh:424 adds ResourceV2).
DEFAULT_CHAIN = ("NamespaceLifecycle", "LimitRanger", "ServiceAccount", "DefaultTolerationSeconds", "Priority",
                 "ResourceV2", "ExtendedResourceToleration", "DefaultStorageClass", "StorageObjectInUseProtection",
                 "ResourceQuota")


class Chain:
    def __init__(self, names=DEFAULT_CHAIN, config: dict | None = None):
        config = config or {}
        self.plugins: list[Plugin] = []
        for n in names:
            n = n.strip()
            if not n:
                continue
            if n not in REGISTRY:
                raise ValueError(f"unknown admission plugin {n!r}")
            self.plugins.append(REGISTRY[n](**config.get(n, {})))

    def has(self, name: str) -> bool:
        return any(p.name == name for p in self.plugins)

    async def admit_async(self, a: Attributes, ctx):
        """Plugins that call out (ImagePolicyWebhook): awaited by the apiserver before the
        synchronous chain runs on the same object."""
        for p in self.plugins:
            fn = getattr(p, "admit_async", None)
            if fn is not None and p.handles(a.operation):
                await fn(a, ctx)

    def admit(self, a: Attributes, ctx):
        for p in self.plugins:
            if p.handles(a.operation):
                p.admit(a, ctx)

    def validate(self, a: Attributes, ctx):
        for p in self.plugins:
            if p.handles(a.operation):
                p.validate(a, ctx)


from . import admission_ext as _ext  # noqa: E402  (the reference's remaining plugins)

REGISTRY.update({p.name: p for p in _ext.PLUGINS})
