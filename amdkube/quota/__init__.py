"""Resource quota: usage evaluators shared by the ResourceQuota admission plugin and the
resource quota controller.

Reference: pkg/quota (resources.go: Add/Subtract/Max/Mask/LessThanOrEqual over ResourceLists;
generic/evaluator.go: Matches, object-count evaluators, ObjectCountQuotaResourceNameFor) and
pkg/quota/evaluator/core (pods.go :39-342, services.go :102-126, persistent_volume_claims.go
:94-186, registry.go legacy object-count aliases).

Resource lists are dict[str, Quantity]. The pod evaluator counts, as the reference does,
`pods`/`count/pods`, `cpu`/`memory`/`ephemeral-storage` (= requests), `requests.*` and `limits.*`
of the sum of the containers raised to the largest init container, only for pods that are not
terminal (and not past their deletion grace). Extension for the GPU fork: an extended resource
(`amd.com/gpu`) is charged under its bare name and `requests.<name>`/`limits.<name>`, counted
from the containers and from the device-granular spec.extendedResources that ResourceV2 writes.
"""
from __future__ import annotations

import time

from ..api import meta as m
from ..api.helpers import is_extended_resource_name
from ..api.quantity import Quantity

RL = dict  # str -> Quantity

SCOPES = ("Terminating", "NotTerminating", "BestEffort", "NotBestEffort")
STORAGE_CLASS_SUFFIX = ".storageclass.storage.k8s.io/"

POD_RESOURCES = ("count/pods", "cpu", "memory", "ephemeral-storage", "requests.cpu", "requests.memory",
                 "requests.ephemeral-storage", "limits.cpu", "limits.memory", "limits.ephemeral-storage", "pods")
POD_PREFIXES = ("hugepages-", "requests.hugepages-")
CONSTRAINED = ("cpu", "memory", "requests.cpu", "requests.memory", "limits.cpu", "limits.memory")
SERVICE_RESOURCES = ("count/services", "services", "services.loadbalancers", "services.nodeports")
PVC_RESOURCES = ("persistentvolumeclaims", "requests.storage")
# registry.go legacyObjectCountAliases
LEGACY_COUNTS = {"configmaps": "configmaps", "resourcequotas": "resourcequotas",
                 "replicationcontrollers": "replicationcontrollers", "secrets": "secrets"}


# ----------------------------------------------------------------- resource lists
def q(v) -> Quantity:
    return v if isinstance(v, Quantity) else Quantity(v)


def parse_list(d: dict | None) -> RL:
    return {k: q(v) for k, v in (d or {}).items()}


def format_list(rl: RL) -> dict:
    return {k: str(v) for k, v in rl.items()}


def add(a: RL, b: RL) -> RL:
    out = dict(a)
    for k, v in b.items():
        out[k] = out[k] + v if k in out else q(v)
    return out


def subtract_non_negative(a: RL, b: RL) -> RL:
    out = {}
    for k, v in a.items():
        d = v - b[k] if k in b else v
        out[k] = d if not d.as_fraction() < 0 else Quantity(0, d.format)
    return out


def max_list(a: RL, b: RL) -> RL:
    out = dict(a)
    for k, v in b.items():
        v = q(v)
        if k not in out or out[k] < v:
            out[k] = v
    return out


def mask(rl: RL, names) -> RL:
    names = set(names)
    return {k: v for k, v in rl.items() if k in names}


def less_than_or_equal(a: RL, b: RL) -> tuple[bool, list[str]]:
    bad = [k for k, v in b.items() if k in a and v < a[k]]
    return not bad, bad


def is_zero(rl: RL) -> bool:
    return all(v.is_zero() for v in rl.values())


def negative(rl: RL) -> list[str]:
    return sorted(k for k, v in rl.items() if v.as_fraction() < 0)


def pretty(rl: RL) -> str:
    return ",".join(f"{k}={rl[k]}" for k in sorted(rl))


def object_count_name(resource: str, group: str = "") -> str:
    return f"count/{resource}" + (f".{group}" if group else "")


# --------------------------------------------------------------------------- pods
def _requests_limits(c: dict) -> tuple[RL, RL]:
    res = c.get("resources") or {}
    return parse_list(res.get("requests")), parse_list(res.get("limits"))


def pod_compute_usage(requests: RL, limits: RL) -> RL:
    """pods.go podComputeUsageHelper (+ the extended-resource extension)."""
    out: RL = {"pods": Quantity(1)}
    for r in ("cpu", "memory", "ephemeral-storage"):
        if r in requests:
            out[r] = requests[r]
            out[f"requests.{r}"] = requests[r]
        if r in limits:
            out[f"limits.{r}"] = limits[r]
    for r, v in requests.items():
        if r.startswith("hugepages-") or is_extended_resource_name(r):
            out[r] = v
            out[f"requests.{r}"] = v
    for r, v in limits.items():
        if r.startswith("hugepages-") or is_extended_resource_name(r):
            out[f"limits.{r}"] = v
    return out


def is_terminating(pod: dict) -> bool:
    ads = (pod.get("spec") or {}).get("activeDeadlineSeconds")
    return ads is not None and int(ads) >= 0


def is_best_effort(pod: dict) -> bool:
    """qos.GetPodQOS == BestEffort: no container (or init container) requests or limits cpu/memory."""
    spec = pod.get("spec") or {}
    for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
        res = c.get("resources") or {}
        for kind in ("requests", "limits"):
            for r, v in (res.get(kind) or {}).items():
                if r in ("cpu", "memory") and not q(v).is_zero():
                    return False
    return True


def quota_pod(pod: dict, now: float | None = None) -> bool:
    """pods.go QuotaPod: terminal pods and pods past their deletion grace use nothing."""
    if (pod.get("status") or {}).get("phase") in ("Failed", "Succeeded"):
        return False
    md = pod.get("metadata") or {}
    if md.get("deletionTimestamp") and md.get("deletionGracePeriodSeconds") is not None:
        t = m.parse_time(md["deletionTimestamp"])
        if t is not None and (now if now is not None else time.time()) > t + int(md["deletionGracePeriodSeconds"]):
            return False
    return True


def pod_usage(pod: dict, now: float | None = None) -> RL:
    """pods.go PodUsageFunc."""
    out: RL = {"count/pods": Quantity(1)}
    if not quota_pod(pod, now):
        return out
    spec = pod.get("spec") or {}
    requests: RL = {}
    limits: RL = {}
    for c in spec.get("containers") or []:
        r, li = _requests_limits(c)
        requests, limits = add(requests, r), add(limits, li)
    for c in spec.get("initContainers") or []:
        r, li = _requests_limits(c)
        requests, limits = max_list(requests, r), max_list(limits, li)
    # device-granular extended resources (the fork's PodSpec.extendedResources)
    for pres in spec.get("extendedResources") or []:
        res = pres.get("resources") or {}
        lim = parse_list(res.get("limits"))
        req = parse_list(res.get("requests")) or lim
        requests, limits = add(requests, req), add(limits, lim)
    return add(out, pod_compute_usage(requests, limits))


def pod_matches_scope(scope: str, pod: dict) -> bool:
    if scope == "Terminating":
        return is_terminating(pod)
    if scope == "NotTerminating":
        return not is_terminating(pod)
    if scope == "BestEffort":
        return is_best_effort(pod)
    if scope == "NotBestEffort":
        return not is_best_effort(pod)
    return False


def pod_matching_resources(names) -> list[str]:
    return [n for n in names if n in POD_RESOURCES or n.startswith(POD_PREFIXES) or _extended_quota_name(n)]


def _extended_quota_name(n: str) -> bool:
    base = n.split(".", 1)[1] if n.startswith(("requests.", "limits.")) else n
    return is_extended_resource_name(base)


def pod_constraints(required, pod: dict) -> str | None:
    """pods.go Constraints: the containers' resource requirements are valid (a limit is never
    below its request: validation.ValidateResourceRequirements), and every container sets each
    compute resource the quota limits."""
    spec = pod.get("spec") or {}
    for kind in ("containers", "initContainers"):
        for i, c in enumerate(spec.get(kind) or []):
            r, li = _requests_limits(c)
            for k, v in r.items():
                if k in li and li[k] < v:
                    return (f"spec.{kind}[{i}].resources.requests: Invalid value: \"{v}\": "
                            f"must be less than or equal to {k} limit")
    req = set(required) & set(CONSTRAINED)
    if not req:
        return None
    missing = set()
    for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
        r, li = _requests_limits(c)
        have = set(pod_compute_usage(r, li))
        missing |= req - have
    return f"must specify {','.join(sorted(missing))}" if missing else None


# ----------------------------------------------------------------------- services
def service_usage(svc: dict) -> RL:
    spec = svc.get("spec") or {}
    ports = len(spec.get("ports") or [])
    out: RL = {"count/services": Quantity(1), "services": Quantity(1), "services.loadbalancers": Quantity(0),
               "services.nodeports": Quantity(0)}
    if spec.get("type") == "NodePort":
        out["services.nodeports"] = Quantity(ports)
    elif spec.get("type") == "LoadBalancer":
        out["services.nodeports"] = Quantity(ports)
        out["services.loadbalancers"] = Quantity(1)
    return out


# --------------------------------------------------------------------------- PVCs
def pvc_class(pvc: dict) -> str:
    ann = (pvc.get("metadata") or {}).get("annotations") or {}
    cls = ann.get("volume.beta.kubernetes.io/storage-class")
    if cls is not None:
        return cls
    return (pvc.get("spec") or {}).get("storageClassName") or ""


def pvc_usage(pvc: dict) -> RL:
    out: RL = {"persistentvolumeclaims": Quantity(1), "count/persistentvolumeclaims": Quantity(1)}
    cls = pvc_class(pvc)
    if cls:
        out[cls + STORAGE_CLASS_SUFFIX + "persistentvolumeclaims"] = Quantity(1)
    req = (((pvc.get("spec") or {}).get("resources") or {}).get("requests") or {}).get("storage")
    if req is not None:
        out["requests.storage"] = q(req)
        if cls:
            out[cls + STORAGE_CLASS_SUFFIX + "requests.storage"] = q(req)
    return out


def pvc_matching_resources(names) -> list[str]:
    out = []
    for n in names:
        if n == "count/persistentvolumeclaims" or n in PVC_RESOURCES or \
                any(n.endswith(STORAGE_CLASS_SUFFIX + r) for r in PVC_RESOURCES):
            out.append(n)
    return out


# --------------------------------------------------------------------- evaluators
class Evaluator:
    """quota.Evaluator for one group/resource."""

    def __init__(self, resource: str, group: str = "", usage=None, matching=None, scope=None, constraints=None,
                 operations=("CREATE",)):
        self.resource, self.group = resource, group
        count = object_count_name(resource, group)
        alias = LEGACY_COUNTS.get(resource) if not group else None
        self._usage = usage or (lambda obj: {count: Quantity(1), **({alias: Quantity(1)} if alias else {})})
        self._matching = matching or (lambda names: [n for n in names if n == count or (alias and n == alias)])
        self._scope = scope
        self._constraints = constraints
        self.operations = operations

    def matching_resources(self, names) -> list[str]:
        return self._matching(list(names))

    def usage(self, obj: dict) -> RL:
        return self._usage(obj)

    def matches_scope(self, scope: str, obj: dict) -> bool:
        return self._scope(scope, obj) if self._scope is not None else False

    def constraints(self, required, obj) -> str | None:
        return self._constraints(required, obj) if self._constraints is not None else None

    def matches(self, quota: dict, obj: dict) -> bool:
        """generic.Matches: the quota limits one of this resource's names and every scope holds."""
        hard = ((quota.get("status") or {}).get("hard") or (quota.get("spec") or {}).get("hard") or {})
        if not self.matching_resources(hard):
            return False
        return all(self.matches_scope(s, obj) for s in (quota.get("spec") or {}).get("scopes") or [])


POD_EVALUATOR = Evaluator("pods", usage=pod_usage, matching=pod_matching_resources, scope=pod_matches_scope,
                          constraints=pod_constraints)
SERVICE_EVALUATOR = Evaluator("services", usage=service_usage,
                              matching=lambda names: [n for n in names if n in SERVICE_RESOURCES],
                              operations=("CREATE", "UPDATE"))
PVC_EVALUATOR = Evaluator("persistentvolumeclaims", usage=pvc_usage, matching=pvc_matching_resources)
_FIXED = {("", "pods"): POD_EVALUATOR, ("", "services"): SERVICE_EVALUATOR,
          ("", "persistentvolumeclaims"): PVC_EVALUATOR}
_GENERIC: dict[tuple[str, str], Evaluator] = {}


def evaluator_for(resource: str, group: str = "") -> Evaluator:
    ev = _FIXED.get((group, resource))
    if ev is None:
        ev = _GENERIC.get((group, resource))
        if ev is None:
            ev = _GENERIC[(group, resource)] = Evaluator(resource, group)
    return ev


def resource_of_quota_name(name: str) -> tuple[str, str] | None:
    """The (group, resource) a quota key charges, for keys outside the fixed evaluators."""
    if name.startswith("count/"):
        rest = name[6:]
        res, _, group = rest.partition(".")
        return group, res
    if name in LEGACY_COUNTS:
        return "", LEGACY_COUNTS[name]
    return None


def has_usage_stats(quota: dict) -> bool:
    """controller.go hasUsageStats: status.hard is set and every hard resource has a used value."""
    st = quota.get("status") or {}
    hard = st.get("hard")
    if hard is None:
        return False
    used = st.get("used") or {}
    return all(k in used for k in hard)


def calculate_usage(quota: dict, objects_by_resource, now: float | None = None) -> RL:
    """The controller's status.used: for every evaluator whose names the quota limits, the summed
    usage of the namespace's objects that match the quota's scopes, masked to the hard names.
    `objects_by_resource(group, resource)` lists the namespace's objects."""
    hard = parse_list((quota.get("spec") or {}).get("hard"))
    scopes = (quota.get("spec") or {}).get("scopes") or []
    evs = [POD_EVALUATOR, SERVICE_EVALUATOR, PVC_EVALUATOR]
    seen = {(e.group, e.resource) for e in evs}
    for name in hard:
        gr = resource_of_quota_name(name)
        if gr is not None and gr not in seen:
            seen.add(gr)
            evs.append(evaluator_for(gr[1], gr[0]))
    used: RL = {}
    for ev in evs:
        names = ev.matching_resources(hard)
        if not names:
            continue
        for obj in objects_by_resource(ev.group, ev.resource):
            if not all(ev.matches_scope(s, obj) for s in scopes):
                continue
            u = pod_usage(obj, now) if ev is POD_EVALUATOR else ev.usage(obj)
            used = add(used, mask(u, names))
    # every hard resource reports a value, zero when nothing uses it
    return {k: used.get(k, Quantity(0, hard[k].format)) for k in hard}
