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
  * NamespaceLifecycle, NamespaceAutoProvision/Exists, LimitRanger (default requests/
    limits), ResourceQuota (object-count + requests quota), ServiceAccount (default SA
    name), DefaultTolerationSeconds, Priority, PodNodeSelector, AlwaysAdmit, AlwaysDeny.
"""
from __future__ import annotations

import uuid

from ..api import meta as m
from ..api.helpers import (GPU_RESOURCE, pod_extended_resource_name, pod_requests, ExtendedResourceError,
                           is_extended_resource_name)
from ..api.quantity import Quantity

CREATE, UPDATE, DELETE, CONNECT = "CREATE", "UPDATE", "DELETE", "CONNECT"


class Attributes:
    __slots__ = ("operation", "resource", "subresource", "namespace", "name", "obj", "old", "user", "kind")

    def __init__(self, operation, resource, subresource, namespace, name, obj, old=None, user=None, kind=""):
        self.operation, self.resource, self.subresource = operation, resource, subresource
        self.namespace, self.name, self.obj, self.old, self.user, self.kind = namespace, name, obj, old, user, kind


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


class LimitRanger(Plugin):
    """Apply LimitRange container defaults (default / defaultRequest) and max checks."""
    name = "LimitRanger"
    operations = (CREATE,)

    def admit(self, a, ctx):
        if a.resource != "pods" or a.subresource:
            return
        for lr in ctx.list_objects("limitranges", a.namespace):
            for item in (lr.get("spec") or {}).get("limits") or []:
                if item.get("type") != "Container":
                    continue
                for c in a.obj.get("spec", {}).get("containers") or []:
                    res = c.setdefault("resources", {})
                    for k, v in (item.get("default") or {}).items():
                        res.setdefault("limits", {}).setdefault(k, v)
                    for k, v in (item.get("defaultRequest") or {}).items():
                        res.setdefault("requests", {}).setdefault(k, v)

    def validate(self, a, ctx):
        if a.resource != "pods" or a.subresource:
            return
        for lr in ctx.list_objects("limitranges", a.namespace):
            for item in (lr.get("spec") or {}).get("limits") or []:
                if item.get("type") != "Container":
                    continue
                for c in a.obj.get("spec", {}).get("containers") or []:
                    lim = (c.get("resources") or {}).get("limits") or {}
                    for k, mx in (item.get("max") or {}).items():
                        if k in lim and Quantity(lim[k]) > Quantity(mx):
                            raise m.forbidden(f"maximum {k} usage per Container is {mx}, but limit is {lim[k]}")


class ResourceQuota(Plugin):
    """Enforce `pods`, `count/<res>`, `requests.<r>` and extended-resource hard limits."""
    name = "ResourceQuota"
    operations = (CREATE,)

    def validate(self, a, ctx):
        if a.subresource or not a.namespace:
            return
        quotas = ctx.list_objects("resourcequotas", a.namespace)
        if not quotas:
            return
        pods = [p for p in ctx.list_objects("pods", a.namespace)
                if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")] if a.resource == "pods" else []
        for q in quotas:
            hard = (q.get("spec") or {}).get("hard") or {}
            for k, v in hard.items():
                lim = Quantity(v)
                if a.resource == "pods" and k == "pods" and len(pods) + 1 > lim.value():
                    raise m.forbidden(f'exceeded quota: {m.name_of(q)}, requested: pods=1, used: pods={len(pods)}, limited: pods={v}')
                if k == f"count/{a.resource}" and len(ctx.list_objects(a.resource, a.namespace)) + 1 > lim.value():
                    raise m.forbidden(f"exceeded quota: {m.name_of(q)}, requested: {k}=1, limited: {k}={v}")
                if a.resource == "pods" and (k.startswith("requests.") or is_extended_resource_name(k)):
                    r = k[len("requests."):] if k.startswith("requests.") else k
                    used = sum(_pod_usage(p, r) for p in pods)
                    want = _pod_usage(a.obj, r)
                    if want and used + want > (lim.milli_value() if r == "cpu" else lim.value()):
                        raise m.forbidden(f"exceeded quota: {m.name_of(q)}, requested: {k}={want}, used: {k}={used}, limited: {k}={v}")


def _pod_usage(pod, r):
    req = pod_requests(pod)
    if r in req:
        return req[r]
    n = 0
    for pres in (pod.get("spec") or {}).get("extendedResources") or []:
        lim = (pres.get("resources") or {}).get("limits") or {}
        if r in lim:
            n += Quantity(lim[r]).value()
    return n


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
