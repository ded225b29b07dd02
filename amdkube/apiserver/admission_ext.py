"""The reference release's remaining admission plugins (plugin/pkg/admission/* and
staging/src/k8s.io/apiserver/pkg/admission/plugin/initialization), registered by their
reference names (cmd/kube-apiserver/app/options/plugins.go):

  AlwaysPullImages, LimitPodHardAntiAffinityTopology, EventRateLimit, DenyEscalatingExec,
  DenyExecOnPrivileged, OwnerReferencesPermissionEnforcement, ImagePolicyWebhook,
  InitialResources, PersistentVolumeLabel, PersistentVolumeClaimResize, PodPreset,
  PodTolerationRestriction, PodSecurityPolicy, SecurityContextDeny, Initializers.

Plugins that call out over the network (ImagePolicyWebhook) implement `admit_async`, which the
apiserver awaits before the synchronous chain runs.
"""
from __future__ import annotations

import copy
import json
import logging
import time

from ..api import meta as m
from ..api.labels import selector_from_label_selector
from ..api.quantity import Quantity
from .admission import (CONNECT, CREATE, UPDATE, Plugin, forbidden_for, is_updating_uninitialized, merge_tolerations,
                        new_forbidden, tolerations_conflict, unknown_error, verify_against_whitelist)

log = logging.getLogger("amdkube.admission")


def _is_pod(a, sub=""):
    return a.resource == "pods" and a.subresource == sub


def _all_containers(pod):
    spec = pod.get("spec") or {}
    return list(spec.get("initContainers") or []) + list(spec.get("containers") or [])


# ------------------------------------------------------------------ AlwaysPullImages
class AlwaysPullImages(Plugin):
    """alwayspullimages/admission.go: every (init) container pulls; validation rejects a pod
    (create or update) that does not, naming the first offending field
    (`spec.initContainers[i].imagePullPolicy: Unsupported value: ...`)."""
    name = "AlwaysPullImages"

    def admit(self, a, ctx):
        if _is_pod(a) and a.obj is not None:
            for c in _all_containers(a.obj):
                c["imagePullPolicy"] = "Always"

    def validate(self, a, ctx):
        if not _is_pod(a) or a.obj is None:
            return
        from ..api.field import go_quote
        spec = a.obj.get("spec") or {}
        for kind in ("initContainers", "containers"):
            for i, c in enumerate(spec.get(kind) or []):
                if c.get("imagePullPolicy") != "Always":
                    raise new_forbidden(a, f"spec.{kind}[{i}].imagePullPolicy: Unsupported value: "
                                           f"{go_quote(c.get('imagePullPolicy') or '')}: supported values: \"Always\"")


# --------------------------------------------------- LimitPodHardAntiAffinityTopology
class LimitPodHardAntiAffinityTopology(Plugin):
    """antiaffinity/admission.go: required pod anti-affinity may only use the
    kubernetes.io/hostname topology key."""
    name = "LimitPodHardAntiAffinityTopology"

    def validate(self, a, ctx):
        if not _is_pod(a) or a.obj is None:
            return
        paa = (((a.obj.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity") or {})
        for t in paa.get("requiredDuringSchedulingIgnoredDuringExecution") or []:
            if t.get("topologyKey") != "kubernetes.io/hostname":
                raise forbidden_for("pods", m.name_of(a.obj),
                                    f"affinity.PodAntiAffinity.RequiredDuringScheduling has TopologyKey "
                                    f"{t.get('topologyKey') or ''} but only key kubernetes.io/hostname is allowed")


# ------------------------------------------------------------------- EventRateLimit
class _Bucket:
    """flowcontrol token bucket: starts full (burst tokens), refills at qps; TryAccept."""
    __slots__ = ("qps", "burst", "tokens", "t", "clock")

    def __init__(self, qps, burst, clock=time.monotonic):
        self.qps, self.burst, self.tokens, self.clock = float(qps), int(burst), float(burst), clock
        self.t = clock()

    def take(self) -> bool:
        now = self.clock()
        self.tokens = min(self.burst, self.tokens + (now - self.t) * self.qps)
        self.t = now
        if self.tokens >= 1.0:
            self.tokens -= 1.0
            return True
        return False


class EventRateLimit(Plugin):
    """eventratelimit/admission.go + limitenforcer.go: one token bucket per limit (Server), or per
    key in an LRU cache of cacheSize (default 4096) for Namespace, User and SourceAndObject (the
    source component and host and the involved object's kind, namespace, name, uid and
    apiVersion, concatenated); every limit takes its token for each Event create or update, and
    any exhausted one rejects it with 429 "limit reached on type T for key K"."""
    name = "EventRateLimit"
    operations = (CREATE, UPDATE)
    DEFAULT_CACHE_SIZE = 4096
    TYPES = ("Server", "Namespace", "User", "SourceAndObject")

    def __init__(self, limits=None, clock=time.monotonic):
        self.limits = limits or [{"type": "Server", "qps": 5000, "burst": 20000}]
        for lim in self.limits:
            if lim.get("type") not in self.TYPES:
                raise ValueError(f"unknown event rate limit type: {lim.get('type')}")
        self.clock = clock
        self.caches: list[tuple[dict, dict]] = [(lim, {}) for lim in self.limits]

    @staticmethod
    def _key(lim, a):
        t = lim.get("type")
        if t == "Server":
            return ""
        if t == "Namespace":
            return a.namespace
        if t == "User":
            return (a.user or {}).get("name", "")
        ev = a.obj if isinstance(a.obj, dict) else {}
        src, io = ev.get("source") or {}, ev.get("involvedObject") or {}
        return "".join(str(x or "") for x in (src.get("component"), src.get("host"), io.get("kind"), io.get("namespace"),
                                               io.get("name"), io.get("uid"), io.get("apiVersion")))

    def _bucket(self, lim, cache, key):
        if lim.get("type") == "Server":
            b = cache.get("")
            if b is None:
                b = cache[""] = _Bucket(lim.get("qps", 10), lim.get("burst", 100), self.clock)
            return b
        b = cache.pop(key, None) or _Bucket(lim.get("qps", 10), lim.get("burst", 100), self.clock)
        cache[key] = b                                   # most recently used last
        size = int(lim.get("cacheSize") or self.DEFAULT_CACHE_SIZE)
        while len(cache) > size:
            cache.pop(next(iter(cache)))
        return b

    def validate(self, a, ctx):
        kind = a.kind or ((a.obj or {}).get("kind") if isinstance(a.obj, dict) else "")
        if kind != "Event" or getattr(a, "group", ""):
            return
        rejection = None
        for lim, cache in self.caches:
            k = self._key(lim, a)
            if not self._bucket(lim, cache, k).take():
                rejection = m.too_many_requests(f"limit reached on type {lim.get('type')} for key {k}")
        if rejection is not None:
            raise rejection


# ---------------------------------------------------------------- exec restrictions
def _privileged(pod) -> bool:
    return any(((c.get("securityContext") or {}).get("privileged")) for c in _all_containers(pod))


class DenyEscalatingExec(Plugin):
    """exec/admission.go: no exec/attach into a privileged pod or one that shares the host's
    PID or IPC namespace; a pod that cannot be read is refused too."""
    name = "DenyEscalatingExec"
    operations = (CONNECT,)
    host_checks = True

    def validate(self, a, ctx):
        if a.resource != "pods" or a.subresource not in ("exec", "attach"):
            return
        pod = a.old or ctx.get_object("pods", a.namespace, a.name)
        if pod is None:
            raise new_forbidden(a, f'pods "{a.name}" not found')
        spec = pod.get("spec") or {}
        if self.host_checks and spec.get("hostPID"):
            raise new_forbidden(a, "cannot exec into or attach to a container using host pid")
        if self.host_checks and spec.get("hostIPC"):
            raise new_forbidden(a, "cannot exec into or attach to a container using host ipc")
        if _privileged(pod):
            raise new_forbidden(a, "cannot exec into or attach to a privileged container")


class DenyExecOnPrivileged(DenyEscalatingExec):
    name = "DenyExecOnPrivileged"
    host_checks = False


# ------------------------------------------------- OwnerReferencesPermissionEnforcement
class OwnerReferencesPermissionEnforcement(Plugin):
    """gc/gc_admission.go: changing metadata.ownerReferences (any difference, order included)
    needs `delete` on the object (subresource included; pods/status is whitelisted); each
    reference newly set to blockOwnerDeletion needs `update` on the owner's finalizers."""
    name = "OwnerReferencesPermissionEnforcement"
    WHITELIST = (("", "pods", "status"),)

    def validate(self, a, ctx):
        if (getattr(a, "group", ""), a.resource, a.subresource) in self.WHITELIST or not isinstance(a.obj, dict):
            return
        new = (a.obj.get("metadata") or {}).get("ownerReferences") or []
        if a.old is None:
            if not new:
                return
        elif new == (((a.old or {}).get("metadata") or {}).get("ownerReferences") or []):
            return
        if not ctx.authorize(a.user, "delete", getattr(a, "group", "") or _group_of(a.obj), a.resource, a.subresource,
                             a.namespace, a.name):
            raise new_forbidden(a, "cannot set an ownerRef on a resource you can't delete: , <nil>")
        olds = {r.get("uid"): r for r in ((a.old or {}).get("metadata") or {}).get("ownerReferences") or []}
        for r in new:
            if not r.get("blockOwnerDeletion"):
                continue
            prev = olds.get(r.get("uid"))
            if prev is not None and prev.get("blockOwnerDeletion"):
                continue
            av = r.get("apiVersion", "")
            plural = ctx.plural_for_kind(av, r.get("kind", ""))
            if plural is None:
                raise new_forbidden(a, f"cannot set blockOwnerDeletion in this case because cannot find RESTMapping for "
                                       f"APIVersion {av} Kind {r.get('kind', '')}: , no matches for kind")
            if not ctx.authorize(a.user, "update", av.rpartition("/")[0], plural, "finalizers", a.namespace, r.get("name", "")):
                raise new_forbidden(a, "cannot set blockOwnerDeletion if an ownerReference refers to a resource you can't "
                                       "set finalizers on: , <nil>")


def _group_of(obj):
    av = obj.get("apiVersion", "")
    return av.rpartition("/")[0] if "/" in av else ""


# -------------------------------------------------------------------- ImagePolicyWebhook
class ImagePolicyWebhook(Plugin):
    """imagepolicy/admission.go: every pod create asks a backend (ImageReview,
    imagepolicy.k8s.io/v1alpha1) whether its images may run; annotations matching
    `*.image-policy.k8s.io/*` are forwarded; answers are cached (allowTTL / denyTTL); an
    unreachable backend applies defaultAllow."""
    name = "ImagePolicyWebhook"
    operations = (CREATE, UPDATE)

    def __init__(self, url="", allow_ttl=300, deny_ttl=30, default_allow=False, timeout=5.0, ca_file=None,
                 insecure=False, client_cert=None, client_key=None):
        self.url, self.allow_ttl, self.deny_ttl, self.default_allow = url, allow_ttl, deny_ttl, default_allow
        self.timeout, self.ca_file, self.insecure = timeout, ca_file, insecure
        self.client_cert, self.client_key = client_cert, client_key
        self.cache: dict[str, tuple[float, bool, str]] = {}

    def review_for(self, pod, ns):
        ann = {k: v for k, v in m.annotations_of(pod).items() if ".image-policy.k8s.io/" in k}
        return {"apiVersion": "imagepolicy.k8s.io/v1alpha1", "kind": "ImageReview",
                "spec": {"containers": [{"image": c.get("image", "")} for c in _all_containers(pod)],
                         "annotations": ann, "namespace": ns}}

    async def admit_async(self, a, ctx):
        if not _is_pod(a) or a.obj is None:
            return
        if a.operation == UPDATE and [c.get("image") for c in _all_containers(a.obj)] == \
                [c.get("image") for c in _all_containers(a.old or {})]:
            return
        review = self.review_for(a.obj, a.namespace)
        key = json.dumps(review["spec"], sort_keys=True)
        hit = self.cache.get(key)
        if hit is not None and hit[0] > time.monotonic():
            allowed, reason = hit[1], hit[2]
        else:
            try:
                allowed, reason = await self._ask(review)
                self.cache[key] = (time.monotonic() + (self.allow_ttl if allowed else self.deny_ttl), allowed, reason)
            except Exception as e:
                log.warning("image policy webhook failed: %r (defaultAllow=%s)", e, self.default_allow)
                if not self.default_allow:
                    raise m.forbidden(f"image policy webhook backend denied one or more images: {e!r}")
                a.obj.setdefault("metadata", {}).setdefault("annotations", {})[
                    "alpha.image-policy.k8s.io/failed-open"] = "true"
                return
        if not allowed:
            raise m.forbidden(f"image policy webhook backend denied one or more images: {reason}")

    async def _ask(self, review):
        import ssl
        import aiohttp
        sslctx = None
        if self.url.startswith("https"):
            sslctx = ssl.create_default_context(cafile=self.ca_file) if self.ca_file else ssl.create_default_context()
            if self.insecure:
                sslctx.check_hostname, sslctx.verify_mode = False, ssl.CERT_NONE
            if self.client_cert:
                sslctx.load_cert_chain(self.client_cert, self.client_key)
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout)) as s:
            async with s.post(self.url, json=review, ssl=sslctx) as r:
                if r.status >= 400:
                    raise RuntimeError(f"HTTP {r.status}")
                st = (await r.json()).get("status") or {}
        return bool(st.get("allowed")), st.get("reason", "")


# -------------------------------------------------------------------- InitialResources
class InitialResources(Plugin):
    """initialresources/admission.go (deprecated upstream): containers without cpu/memory
    requests get the `percentile` of their image's historical usage (same image:tag, else
    any tag of the image) when at least 60 samples exist, and the pod is annotated with what was
    estimated. The data source is pluggable (`source.usage(resource, image, ns, exact) →
    samples`); the reference's InfluxDB/GCM/Hawkular sources need services this build has no
    access to, so a Prometheus source querying the kubelets' container metrics is provided."""
    name = "InitialResources"
    operations = (CREATE,)
    SAMPLES_THRESHOLD = 60

    def __init__(self, source=None, percentile=90, namespace_only=False):
        self.source, self.percentile, self.ns_only = source, percentile, namespace_only

    def admit(self, a, ctx):
        if not _is_pod(a) or a.obj is None or self.source is None:
            return
        notes = []
        for c in _all_containers(a.obj):
            req = (c.setdefault("resources", {})).setdefault("requests", {})
            lim = c["resources"].get("limits") or {}
            for res in ("cpu", "memory"):
                if res in req or res in lim:
                    continue
                v = self._estimate(res, c.get("image", ""), a.namespace if self.ns_only else "")
                if v is not None:
                    req[res] = f"{int(v)}m" if res == "cpu" else str(int(v))
                    notes.append(f"{res} request for container {c.get('name')}")
            if not req:
                c["resources"].pop("requests")
        if notes:
            a.obj.setdefault("metadata", {}).setdefault("annotations", {})["kubernetes.io/initial-resources"] = \
                "Initial Resources plugin set: " + "; ".join(notes)

    def _estimate(self, res, image, ns):
        for exact in (True, False):
            samples = sorted(self.source.usage(res, image, ns, exact) or [])
            if len(samples) >= self.SAMPLES_THRESHOLD:
                i = min(len(samples) - 1, int(len(samples) * self.percentile / 100))
                return samples[i]
        return None


class PrometheusUsageSource:
    """Usage samples for InitialResources from a Prometheus server scraping the kubelets'
    /metrics/cadvisor (container_cpu_usage_seconds_total rate in millicores, memory working set)."""

    def __init__(self, url: str, window: str = "30d"):
        self.url, self.window = url.rstrip("/"), window

    def usage(self, res, image, ns, exact):
        import urllib.parse
        import urllib.request
        sel = f'image="{image}"' if exact else f'image=~"{image.split(":")[0]}(:.*)?"'
        if ns:
            sel += f',namespace="{ns}"'
        q = (f"rate(container_cpu_usage_seconds_total{{{sel}}}[5m]) * 1000" if res == "cpu"
             else f"container_memory_working_set_bytes{{{sel}}}")
        url = f"{self.url}/api/v1/query_range?" + urllib.parse.urlencode(
            {"query": q, "start": time.time() - 86400 * 30, "end": time.time(), "step": "3600"})
        with urllib.request.urlopen(url, timeout=5) as r:
            data = json.loads(r.read())
        return [float(v) for s in data.get("data", {}).get("result", []) for _t, v in s.get("values", [])]


# -------------------------------------------------------------- PersistentVolumeLabel
class PersistentVolumeLabel(Plugin):
    """persistentvolume/label/admission.go: AWS EBS and GCE PD volumes get the zone/region
    labels of their disk from the cloud provider (`cloud.volume_labels(pv)`)."""
    name = "PersistentVolumeLabel"
    operations = (CREATE,)

    def __init__(self, cloud=None):
        self.cloud = cloud

    def admit(self, a, ctx):
        if a.resource != "persistentvolumes" or a.subresource or a.obj is None:
            return
        spec = a.obj.get("spec") or {}
        if "awsElasticBlockStore" not in spec and "gcePersistentDisk" not in spec:
            return
        cloud = self.cloud or getattr(ctx, "cloud", None)
        if cloud is None or not hasattr(cloud, "volume_labels"):
            raise m.forbidden("error querying volume labels: no cloud provider with volume support is configured")
        labels = cloud.volume_labels(a.obj) or {}
        if labels:
            a.obj.setdefault("metadata", {}).setdefault("labels", {}).update(labels)


# --------------------------------------------------------- PersistentVolumeClaimResize
RESIZABLE = ("glusterfs", "cinder", "rbd", "gcePersistentDisk", "awsElasticBlockStore")


def _claim_class(pvc) -> str:
    """helper.GetPersistentVolumeClaimClass: the beta annotation, else spec.storageClassName."""
    ann = m.annotations_of(pvc)
    if "volume.beta.kubernetes.io/storage-class" in ann:
        return ann["volume.beta.kubernetes.io/storage-class"]
    return (pvc.get("spec") or {}).get("storageClassName") or ""


class PersistentVolumeClaimResize(Plugin):
    """persistentvolume/resize/admission.go: growing a claim's storage request needs a bound
    claim whose (unchanged) StorageClass sets allowVolumeExpansion and whose volume is one the
    release can expand (GlusterFS, Cinder, RBD, GCE PD, AWS EBS)."""
    name = "PersistentVolumeClaimResize"
    operations = (UPDATE,)

    def validate(self, a, ctx):
        if a.resource != "persistentvolumeclaims" or a.subresource or not isinstance(a.obj, dict) or \
                not isinstance(a.old, dict):
            return

        def size(o):
            s = (((o.get("spec") or {}).get("resources") or {}).get("requests") or {}).get("storage")
            return Quantity(s) if s else Quantity(0)
        if not size(a.obj) > size(a.old):
            return
        if (a.old.get("status") or {}).get("phase") != "Bound":
            raise new_forbidden(a, "Only bound persistent volume claims can be expanded")
        new_sc, old_sc = _claim_class(a.obj), _claim_class(a.old)
        sc = ctx.get_object("storageclasses", "", new_sc) if new_sc and new_sc == old_sc else None
        if not sc or not sc.get("allowVolumeExpansion"):
            raise new_forbidden(a, "only dynamically provisioned pvc can be resized and the storageclass that provisions "
                                   "the pvc must support resize")
        pv = ctx.get_object("persistentvolumes", "", (a.obj.get("spec") or {}).get("volumeName", ""))
        if pv is None:
            raise new_forbidden(a, "Error updating persistent volume claim because fetching associated persistent volume "
                                   "failed")
        if not any((pv.get("spec") or {}).get(k) is not None for k in RESIZABLE):
            raise new_forbidden(a, "volume plugin does not support resize")


# ------------------------------------------------------------------------- PodPreset
PRESET_ANNOTATION_PREFIX = "podpreset.admission.kubernetes.io"


class PodPreset(Plugin):
    """podpreset/admission.go: on pod creation (mirror pods and pods annotated
    podpreset.admission.kubernetes.io/exclude=true aside) every preset of the namespace whose
    selector matches the pod's labels is merged in — volumes by name, each container's env by
    name, volumeMounts by name and by mount path, envFrom appended — unless any of them conflicts
    (same name or path, another definition), in which case the pod is left untouched; each
    applied preset is recorded as podpreset.admission.kubernetes.io/podpreset-<name>=<rv>."""
    name = "PodPreset"
    operations = (CREATE,)

    def admit(self, a, ctx):
        if not _is_pod(a) or a.obj is None or a.operation != CREATE:
            return
        pod = a.obj
        ann = m.annotations_of(pod)
        if "kubernetes.io/config.mirror" in ann or ann.get(f"{PRESET_ANNOTATION_PREFIX}/exclude") == "true":
            return
        labels = (pod.get("metadata") or {}).get("labels") or {}
        presets = [p for p in ctx.list_objects("podpresets", a.namespace, "settings.k8s.io")
                   if selector_from_label_selector((p.get("spec") or {}).get("selector") or {}).matches(labels)]
        if not presets:
            return
        errs = self.conflicts(pod, presets)
        if errs:
            log.warning("conflict occurred while applying podpresets: %s on pod: %s err: %s",
                        ",".join(m.name_of(p) for p in presets), (pod.get("metadata") or {}).get("generateName", ""), errs)
            return
        self.apply(pod, presets)

    @staticmethod
    def _merge_by(items, presets, field, keys, what):
        """mergeEnv / mergeVolumes / mergeVolumeMounts: the originals, then each preset item
        whose key is new; an existing key with another definition is an error."""
        merged = list(items or [])
        seen = [{it.get(k): it for it in merged} for k in keys]
        errs = []
        for p in presets:
            for it in (p.get("spec") or {}).get(field) or []:
                new = True
                for idx, k in enumerate(keys):
                    found = seen[idx].get(it.get(k))
                    if found is None:
                        seen[idx][it.get(k)] = it
                    else:
                        if idx == 0:
                            new = False
                        if found != it:
                            on = it.get(k) if k == "name" else f"mount path {it.get(k)}"
                            errs.append(f"merging {what} for {m.name_of(p)} has a conflict on {on}")
                if new:
                    merged.append(it)
        return merged, errs

    @classmethod
    def conflicts(cls, pod, presets) -> list[str]:
        """safeToApplyPodPresetsOnPod."""
        spec = pod.get("spec") or {}
        errs = cls._merge_by(spec.get("volumes"), presets, "volumes", ("name",), "volumes")[1]
        for c in spec.get("containers") or []:
            errs += cls._merge_by(c.get("env"), presets, "env", ("name",), "env")[1]
            errs += cls._merge_by(c.get("volumeMounts"), presets, "volumeMounts", ("name", "mountPath"), "volume mounts")[1]
        return errs

    @classmethod
    def apply(cls, pod, presets):
        """applyPodPresetsOnPod."""
        spec = pod.setdefault("spec", {})
        vols = cls._merge_by(spec.get("volumes"), presets, "volumes", ("name",), "volumes")[0]
        if vols:
            spec["volumes"] = vols
        else:
            spec.pop("volumes", None)
        for c in spec.get("containers") or []:
            for field, keys, what in (("env", ("name",), "env"), ("volumeMounts", ("name", "mountPath"), "volume mounts")):
                merged = cls._merge_by(c.get(field), presets, field, keys, what)[0]
                if merged:
                    c[field] = merged
            env_from = list(c.get("envFrom") or []) + [x for p in presets for x in (p.get("spec") or {}).get("envFrom") or []]
            if env_from:
                c["envFrom"] = env_from
        md = pod.setdefault("metadata", {})
        if md.get("annotations") is None:
            md["annotations"] = {}
        for p in presets:
            md["annotations"][f"{PRESET_ANNOTATION_PREFIX}/podpreset-{m.name_of(p)}"] = \
                (p.get("metadata") or {}).get("resourceVersion", "")


# ---------------------------------------------------------- PodTolerationRestriction
NS_DEFAULT_TOLERATIONS = "scheduler.alpha.kubernetes.io/defaultTolerations"
NS_WHITELIST_TOLERATIONS = "scheduler.alpha.kubernetes.io/tolerationsWhitelist"


MEMORY_PRESSURE_TOLERATION = {"key": "node.kubernetes.io/memory-pressure", "operator": "Exists", "effect": "NoSchedule"}


class PodTolerationRestriction(Plugin):
    """podtolerationrestriction/admission.go: a new pod (or an update of an uninitialized one)
    gets its namespace's default tolerations (the scheduler.alpha.kubernetes.io/defaultTolerations
    annotation, an empty value meaning none; without the annotation the plugin's cluster default)
    merged in (MergeTolerations; a (key, effect) defined differently is refused); non-BestEffort
    pods also tolerate node.kubernetes.io/memory-pressure:NoSchedule; every toleration must then
    be on the namespace's whitelist (annotation, else the cluster whitelist) when one is set."""
    name = "PodTolerationRestriction"

    def __init__(self, default=None, whitelist=None):
        self.default, self.whitelist = default or [], whitelist or []

    def _ns_list(self, ctx, ns, key):
        """extractNSTolerations: None without the annotation, [] for an empty value."""
        obj = ctx.get_namespace(ns)
        if obj is None:
            raise m.not_found("namespaces", ns)
        ann = m.annotations_of(obj)
        if key not in ann:
            return None
        if not ann[key]:
            return []
        try:
            v = json.loads(ann[key])
        except ValueError as e:
            raise unknown_error(str(e)) from None
        if v is not None and not isinstance(v, list):
            raise unknown_error(f"json: cannot unmarshal {type(v).__name__} into Go value of type []v1.Toleration")
        return v or []

    def admit(self, a, ctx):
        if not _is_pod(a) or not isinstance(a.obj, dict):
            return
        spec = a.obj.setdefault("spec", {})
        final = spec.get("tolerations") or []
        if a.operation == CREATE or is_updating_uninitialized(a):
            ts = self._ns_list(ctx, a.namespace, NS_DEFAULT_TOLERATIONS)
            if ts is None:
                ts = self.default
            if ts:
                if final:
                    if tolerations_conflict(ts, final):
                        raise unknown_error("namespace tolerations and pod tolerations conflict")
                    final = merge_tolerations(ts, final)
                else:
                    final = list(ts)
        from .registry import pod_qos
        if pod_qos(a.obj) != "BestEffort":
            final = merge_tolerations(final, [dict(MEMORY_PRESSURE_TOLERATION)])
        if final or spec.get("tolerations") is not None:
            spec["tolerations"] = final
        self.validate(a, ctx)

    def validate(self, a, ctx):
        if not _is_pod(a) or not isinstance(a.obj, dict):
            return
        tols = (a.obj.get("spec") or {}).get("tolerations") or []
        if not tols:
            return
        wl = self._ns_list(ctx, a.namespace, NS_WHITELIST_TOLERATIONS)
        if wl is None:
            wl = self.whitelist
        if wl and not verify_against_whitelist(tols, wl):
            raise unknown_error("pod tolerations (possibly merged with namespace default tolerations) conflict with its "
                                "namespace whitelist")


# ----------------------------------------------------------------- SecurityContextDeny
class SecurityContextDeny(Plugin):
    """securitycontext/scdeny/admission.go: pods may not set supplementalGroups, SELinux
    options, runAsUser or fsGroup, nor containers SELinux options or runAsUser."""
    name = "SecurityContextDeny"

    def validate(self, a, ctx):
        if not _is_pod(a) or not isinstance(a.obj, dict):
            return
        name = m.name_of(a.obj)
        psc = (a.obj.get("spec") or {}).get("securityContext")
        if psc is not None:
            for field, msg in (("supplementalGroups", "SecurityContext.SupplementalGroups is forbidden"),
                               ("seLinuxOptions", "pod.Spec.SecurityContext.SELinuxOptions is forbidden"),
                               ("runAsUser", "pod.Spec.SecurityContext.RunAsUser is forbidden"),
                               ("fsGroup", "SecurityContext.FSGroup is forbidden")):
                if psc.get(field) is not None:
                    raise forbidden_for("pods", name, msg)
        for c in _all_containers(a.obj):
            sc = c.get("securityContext")
            if sc is None:
                continue
            if sc.get("seLinuxOptions") is not None:
                raise forbidden_for("pods", name, "SecurityContext.SELinuxOptions is forbidden")
            if sc.get("runAsUser") is not None:
                raise forbidden_for("pods", name, "SecurityContext.RunAsUser is forbidden")


# ------------------------------------------------------------------- PodSecurityPolicy
PSP_ANNOTATION = "kubernetes.io/psp"


class PodSecurityPolicy(Plugin):
    """plugin/pkg/admission/security/podsecuritypolicy/admission.go over security/psp.py: every
    policy (name order) is tried on a copy of the pod; one that validates without changing the
    pod wins, else (create only) the first that validates with changes; the requesting user or
    the pod's service account must be authorized to `use` it; the winner is recorded as
    kubernetes.io/psp. On update the pod must be admitted unchanged. Forbidden otherwise,
    listing the errors of the policies the requester may use."""
    name = "PodSecurityPolicy"

    def __init__(self, fail_on_no_policies=True):
        self.fail_on_no_policies = fail_on_no_policies

    def _authorized(self, a, ctx, pod):
        sa = (pod.get("spec") or {}).get("serviceAccountName")
        sa_user = {"name": f"system:serviceaccount:{a.namespace}:{sa}",
                   "groups": ["system:serviceaccounts", f"system:serviceaccounts:{a.namespace}"]} if sa else None

        def ok(name):
            return (sa_user is not None and ctx.authorize(sa_user, "use", "extensions", "podsecuritypolicies", "",
                                                          a.namespace, name)) or \
                ctx.authorize(a.user or {}, "use", "extensions", "podsecuritypolicies", "", a.namespace, name)
        return ok

    def _compute(self, a, ctx, mutation_allowed):
        from ..security import psp
        policies = ctx.list_objects("podsecuritypolicies", "", "extensions")
        try:
            return psp.compute_security_context(policies, a.obj, self._authorized(a, ctx, a.obj), mutation_allowed,
                                                self.fail_on_no_policies)
        except PermissionError as e:
            raise m.forbidden(f"unable to validate against any pod security policy: {e}") from None

    @staticmethod
    def _ignore(a) -> bool:
        if not _is_pod(a) or a.obj is None:
            return True
        if a.operation == UPDATE and a.old is not None:
            strip = lambda o: {k: v for k, v in o.items() if k != "metadata"}   # noqa: E731
            if strip(a.obj) == strip(a.old):
                return True      # only metadata (GC fields, labels) changed: IsOnlyMutatingGCFields
        return False

    def admit(self, a, ctx):
        if self._ignore(a) or a.operation != CREATE:
            return
        allowed, name, errs = self._compute(a, ctx, True)
        if allowed is None:
            raise m.forbidden(f"unable to validate against any pod security policy: {[str(e) for e in errs]}")
        if allowed is not a.obj:
            a.obj.clear()
            a.obj.update(allowed)
        if name:
            md = a.obj.setdefault("metadata", {})
            if md.get("annotations") is None:
                md["annotations"] = {}
            md["annotations"][PSP_ANNOTATION] = name

    def validate(self, a, ctx):
        if self._ignore(a):
            return
        from ..security.psp import _semantic_equal
        allowed, _, errs = self._compute(a, ctx, False)
        if allowed is not None and _semantic_equal(allowed, a.obj):
            return
        raise m.forbidden(f"unable to validate against any pod security policy: {[str(e) for e in errs]}")


# ---------------------------------------------------------------------- Initializers
class Initializers(Plugin):
    """apiserver/pkg/admission/plugin/initialization: a new object whose resource matches an
    InitializerConfiguration rule gets metadata.initializers.pending (every matching
    initializer, in configuration order); it stays uninitialized — hidden from LIST/WATCH
    without includeUninitialized — until initializers remove themselves. Clients that are not
    allowed to `initialize` the resource may not set or change initializers."""
    name = "Initializers"
    operations = (CREATE, UPDATE)

    def admit(self, a, ctx):
        if a.obj is None or a.subresource or a.resource in ("initializerconfigurations",):
            return
        md = a.obj.setdefault("metadata", {})
        if a.operation == CREATE:
            if md.get("initializers") is not None:
                if not ctx.authorize(a.user or {}, "initialize", _group_of(a.obj), a.resource, "", a.namespace, a.name):
                    raise m.forbidden("must have the 'initialize' verb to set initializers on create")
                return
            names = []
            for ic in ctx.list_objects("initializerconfigurations", "", "admissionregistration.k8s.io"):
                for ini in ic.get("initializers") or []:
                    if any(_rule_matches(r, a) for r in ini.get("rules") or []) and ini["name"] not in names:
                        names.append(ini["name"])
            if names:
                md["initializers"] = {"pending": [{"name": n} for n in names]}
        else:
            old = ((a.old or {}).get("metadata") or {}).get("initializers")
            if md.get("initializers") != old:
                if old is None:
                    raise m.forbidden("field is immutable once initialization has completed")
                if not ctx.authorize(a.user or {}, "initialize", _group_of(a.obj), a.resource, "", a.namespace, a.name):
                    raise m.forbidden("must have the 'initialize' verb to modify initializers")
            if md.get("initializers") is not None and not (md["initializers"].get("pending")) \
                    and md["initializers"].get("result") is None:
                md.pop("initializers")


def _rule_matches(rule, a) -> bool:
    group = a.group if hasattr(a, "group") else ""
    def has(lst, v):
        return "*" in lst or v in lst
    groups = rule.get("apiGroups") or []
    gv = (a.obj or {}).get("apiVersion", "")
    g, _, v = gv.rpartition("/") if "/" in gv else ("", "", gv)
    return has(groups, g if not group else group) and has(rule.get("apiVersions") or [], v) and \
        has(rule.get("resources") or [], a.resource)


def is_uninitialized(obj) -> bool:
    ini = ((obj or {}).get("metadata") or {}).get("initializers")
    return bool(ini) and bool(ini.get("pending"))


PLUGINS = (AlwaysPullImages, LimitPodHardAntiAffinityTopology, EventRateLimit, DenyEscalatingExec, DenyExecOnPrivileged,
           OwnerReferencesPermissionEnforcement, ImagePolicyWebhook, InitialResources, PersistentVolumeLabel,
           PersistentVolumeClaimResize, PodPreset, PodTolerationRestriction, PodSecurityPolicy, SecurityContextDeny,
           Initializers)
