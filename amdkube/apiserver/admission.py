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
        tols = spec.get("tolerations") or []
        for n in sorted(names):
            if not any(t.get("key") == n and t.get("operator") == "Exists" and t.get("effect") in ("NoSchedule", None, "") for t in tols):
                tols.append({"key": n, "operator": "Exists", "effect": "NoSchedule"})
        if tols:
            spec["tolerations"] = tols


class NamespaceLifecycle(Plugin):
    """Reject creation in missing/terminating namespaces; protect system namespaces."""
    name = "NamespaceLifecycle"
    operations = (CREATE, UPDATE, DELETE)
    immortal = ("default", "kube-system", "kube-public")

    def validate(self, a, ctx):
        if a.resource == "namespaces":
            if a.operation == DELETE and a.name in self.immortal:
                raise m.forbidden(f'namespace "{a.name}" is protected and cannot be deleted')
            return
        if not a.namespace or a.operation != CREATE:
            return
        if a.resource in ("events",) or a.subresource:
            return
        ns = ctx.get_namespace(a.namespace)
        if ns is None:
            raise m.not_found("namespaces", a.namespace)
        if (ns.get("status") or {}).get("phase") == "Terminating":
            raise m.forbidden(f'unable to create new content in namespace {a.namespace} because it is being terminated')


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


class ServiceAccount(Plugin):
    """plugin/pkg/admission/serviceaccount/admission.go: default `serviceAccountName`, refuse a
    pod naming a ServiceAccount that does not exist, mount the account's API token secret at
    /var/run/secrets/kubernetes.io/serviceaccount in every container (unless the pod or the
    account sets automountServiceAccountToken: false, or a container already mounts that path),
    copy the account's imagePullSecrets into a pod without any, enforce mountable secrets when
    the account asks for it, and keep mirror pods free of accounts and secrets.

    Deliberate difference: the reference also refuses a pod while the "default" account or its
    token does not exist yet (RequireAPIToken, "retry after the token is automatically
    created"); here a missing default account or token mounts nothing, so clusters run without
    the ServiceAccount/token controllers (the benches, the node e2e setups) still start pods.
    `require_api_token=True` restores the reference's refusal."""
    name = "ServiceAccount"
    operations = (CREATE,)

    def __init__(self, require_api_token: bool = False):
        self.require_api_token = require_api_token

    @staticmethod
    def _secret_names(pod: dict) -> set[str]:
        spec = pod.get("spec") or {}
        out = {v["secret"].get("secretName") for v in spec.get("volumes") or [] if (v.get("secret") or {}).get("secretName")}
        for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
            for e in c.get("env") or []:
                ref = ((e.get("valueFrom") or {}).get("secretKeyRef") or {}).get("name")
                if ref:
                    out.add(ref)
            for ef in c.get("envFrom") or []:
                ref = (ef.get("secretRef") or {}).get("name")
                if ref:
                    out.add(ref)
        return out

    def _token_secret(self, sa: dict, ctx) -> str:
        """The first API token secret the account references (getReferencedServiceAccountToken)."""
        ns, name = m.namespace_of(sa), m.name_of(sa)
        for ref in sa.get("secrets") or []:
            sec = ctx.get_object("secrets", ns, ref.get("name", ""))
            if sec and sec.get("type") == "kubernetes.io/service-account-token" and \
                    m.annotations_of(sec).get("kubernetes.io/service-account.name") == name:
                return m.name_of(sec)
        return ""

    def admit(self, a, ctx):
        if a.resource != "pods" or a.subresource:
            return
        pod = a.obj
        spec = pod.setdefault("spec", {})
        if MIRROR_POD_ANNOTATION in m.annotations_of(pod):
            if spec.get("serviceAccountName") or spec.get("serviceAccount"):
                raise _forbid(pod, "a mirror pod may not reference service accounts")
            if self._secret_names(pod):
                raise _forbid(pod, "a mirror pod may not reference secrets")
            return
        sa_name = spec.get("serviceAccountName") or spec.get("serviceAccount") or "default"
        spec["serviceAccountName"] = sa_name
        sa = ctx.get_object("serviceaccounts", a.namespace, sa_name)
        if sa is None:
            if sa_name != "default" or self.require_api_token:
                raise _forbid(pod, f"error looking up service account {a.namespace}/{sa_name}: "
                                                          f"serviceaccount \"{sa_name}\" not found")
            return
        automount = spec.get("automountServiceAccountToken")
        if automount is None:
            automount = sa.get("automountServiceAccountToken")
        if automount is not False:
            self._mount_token(sa, pod, ctx)
        if not spec.get("imagePullSecrets") and sa.get("imagePullSecrets"):
            spec["imagePullSecrets"] = [dict(x) for x in sa["imagePullSecrets"]]
        if m.annotations_of(sa).get(ENFORCE_MOUNTABLE_SECRETS) == "true":
            allowed = {r.get("name") for r in sa.get("secrets") or []}
            for sname in sorted(self._secret_names(pod)):
                if sname not in allowed:
                    raise _forbid(pod, f'volume with secret.secretName="{sname}" is not allowed '
                                                              f"because service account {sa_name} does not reference that secret")
            pulls = {r.get("name") for r in sa.get("imagePullSecrets") or []}
            for i, ref in enumerate(spec.get("imagePullSecrets") or []):
                if ref.get("name") not in pulls:
                    raise _forbid(pod, f'imagePullSecrets[{i}].name="{ref.get("name")}" is not '
                                                              f"allowed because service account {sa_name} does not "
                                                              f"reference that imagePullSecret")

    def _mount_token(self, sa: dict, pod: dict, ctx):
        token = self._token_secret(sa, ctx)
        if not token:
            if self.require_api_token:
                raise m.StatusError(504, "ServerTimeout", f"No API token found for service account "
                                                          f"\"{m.name_of(sa)}\", retry after the token is "
                                                          f"automatically created and added to the service account")
            return
        spec = pod["spec"]
        volumes = spec.setdefault("volumes", [])
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
            volumes.append({"name": vol_name, "secret": {"secretName": token}})


class DefaultTolerationSeconds(Plugin):
    name = "DefaultTolerationSeconds"
    operations = (CREATE,)

    def __init__(self, seconds=300):
        self.seconds = seconds

    def admit(self, a, ctx):
        if a.resource != "pods" or a.subresource:
            return
        tols = a.obj.setdefault("spec", {}).setdefault("tolerations", [])
        for key in ("node.kubernetes.io/not-ready", "node.kubernetes.io/unreachable"):
            if not any(t.get("key") == key and t.get("effect") in ("NoExecute", None, "") for t in tols):
                tols.append({"key": key, "operator": "Exists", "effect": "NoExecute", "tolerationSeconds": self.seconds})


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


class Priority(Plugin):
    name = "Priority"
    operations = (CREATE,)

    def admit(self, a, ctx):
        if a.resource != "pods" or a.subresource:
            return
        spec = a.obj.setdefault("spec", {})
        pcn = spec.get("priorityClassName")
        if pcn:
            pc = ctx.get_object("priorityclasses", "", pcn)
            if pc is None:
                if pcn in ("system-cluster-critical", "system-node-critical"):
                    spec["priority"] = 2000000000 if pcn == "system-cluster-critical" else 2000001000
                    return
                raise m.forbidden(f"no PriorityClass with name {pcn} was found")
            spec["priority"] = int(pc.get("value", 0))
        else:
            default = [pc for pc in ctx.list_objects("priorityclasses", "") if pc.get("globalDefault")]
            spec.setdefault("priority", int(default[0].get("value", 0)) if default else 0)


class PodNodeSelector(Plugin):
    """Merge the namespace annotation scheduler.alpha.kubernetes.io/node-selector."""
    name = "PodNodeSelector"
    operations = (CREATE,)
    ANNOTATION = "scheduler.alpha.kubernetes.io/node-selector"

    def admit(self, a, ctx):
        if a.resource != "pods" or a.subresource:
            return
        ns = ctx.get_namespace(a.namespace) or {}
        sel = m.annotations_of(ns).get(self.ANNOTATION)
        if not sel:
            return
        ns_sel = dict(kv.split("=", 1) for kv in sel.split(",") if "=" in kv)
        pod_sel = a.obj.setdefault("spec", {}).setdefault("nodeSelector", {})
        for k, v in ns_sel.items():
            if k in pod_sel and pod_sel[k] != v:
                raise m.forbidden("pod node label selector conflicts with its namespace node label selector")
            pod_sel[k] = v


class DefaultStorageClass(Plugin):
    """plugin/pkg/admission/storageclass/setdefault: a claim without a class gets the class
    annotated storageclass.kubernetes.io/is-default-class=true (more than one default: 403)."""
    name = "DefaultStorageClass"
    operations = (CREATE,)

    def admit(self, a, ctx):
        if a.resource != "persistentvolumeclaims" or a.subresource:
            return
        spec = a.obj.setdefault("spec", {})
        if "storageClassName" in spec or "volume.beta.kubernetes.io/storage-class" in (a.obj.get("metadata") or {}).get(
                "annotations", {}):
            return
        defaults = [sc for sc in ctx.list_objects("storageclasses", "", "storage.k8s.io")
                    if ((sc.get("metadata") or {}).get("annotations") or {}).get("storageclass.kubernetes.io/is-default-class") == "true"]
        if len(defaults) > 1:
            raise m.forbidden(f"{len(defaults)} default StorageClasses were found")
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


class NodeRestriction(Plugin):
    """plugin/pkg/admission/noderestriction: a kubelet (system:node:<name> in system:nodes) may
    create only mirror pods bound to itself, update the status of its own pods, and modify only
    its own Node object."""
    name = "NodeRestriction"
    operations = (CREATE, UPDATE, DELETE)

    def admit(self, a, ctx):
        u = a.user or {}
        if "system:nodes" not in (u.get("groups") or []) or not u.get("name", "").startswith("system:node:"):
            return
        node = u["name"][len("system:node:"):]
        if a.resource == "nodes":
            if a.name != node and m.name_of(a.obj or {}) != node:
                raise m.forbidden(f'node "{node}" cannot modify node "{a.name}"')
        elif a.resource == "pods":
            pod = a.obj if a.operation == CREATE else (a.old or {})
            if a.operation == CREATE and not a.subresource:
                ann = ((pod.get("metadata") or {}).get("annotations") or {})
                if "kubernetes.io/config.mirror" not in ann:
                    raise m.forbidden(f'pod does not have "kubernetes.io/config.mirror" annotation, node "{node}" can only create mirror pods')
                if (pod.get("spec") or {}).get("nodeName") != node:
                    raise m.forbidden(f'node "{node}" can only create pods with spec.nodeName set to itself')
            elif a.subresource in ("status", "") and (pod.get("spec") or {}).get("nodeName") != node:
                raise m.forbidden(f'node "{node}" can only update or delete pods bound to itself')


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
