"""Kubelet eviction manager.

Reference: pkg/kubelet/eviction — api/types.go (signals, GetThresholdQuantity), helpers.go
(ParseThresholdConfig :101-287, makeSignalObservations :718-790, thresholdsMet :793-819, the
grace-period / transition-period bookkeeping :850-934, rankers :460-704, node-level reclaim
:1050-1092) and eviction_manager.go (Admit :121-145, synchronize :199-371, reclaimNodeLevelResources
:394-418, localStorageEviction :420-583).

One synchronize() pass: observe the signals from the stats summary (plus allocatable memory
from the capacity provider), find the thresholds met (a threshold met at the last pass stays
met until its minimum reclaim is satisfied), hold node conditions for the pressure transition
period, keep only thresholds whose grace period has elapsed and whose stats are newer than the
last pass, then reclaim the starved resource — node-level first (dead containers, unused
images), and failing that by killing the first pod of the resource's ranking (hard thresholds
kill with no grace, soft ones with MaxPodGracePeriodSeconds). Admit rejects BestEffort pods
under MemoryPressure and every pod under DiskPressure (critical pods excepted).

Times are seconds (the kubelet passes a monotonic clock); quantities are integers (bytes,
inodes). A Threshold is compared by identity as a map key, like the reference's struct with
pointer fields, and by value in mergeThresholds.
"""
from __future__ import annotations

import functools
import inspect
import time
from dataclasses import dataclass, field

import numpy as np

from ..api import meta as m
from ..api.quantity import Quantity

MEMORY, ALLOCATABLE_MEMORY = "memory.available", "allocatableMemory.available"
NODEFS, NODEFS_INODES = "nodefs.available", "nodefs.inodesFree"
IMAGEFS, IMAGEFS_INODES = "imagefs.available", "imagefs.inodesFree"
OP_LESS_THAN = "LessThan"
NODE_ALLOCATABLE_ENFORCEMENT_KEY = "pods"          # cm.NodeAllocatableEnforcementKey
REASON = "Evicted"
MESSAGE = "The node was low on resource: {}."

# internal resources of this module (helpers.go:44-55)
RESOURCE_DISK, RESOURCE_INODES = "disk", "inodes"
RESOURCE_IMAGEFS, RESOURCE_IMAGEFS_INODES = "imagefs", "imagefsInodes"
RESOURCE_NODEFS, RESOURCE_NODEFS_INODES = "nodefs", "nodefsInodes"

SIGNAL_TO_NODE_CONDITION = {MEMORY: "MemoryPressure", ALLOCATABLE_MEMORY: "MemoryPressure", IMAGEFS: "DiskPressure",
                            NODEFS: "DiskPressure", IMAGEFS_INODES: "DiskPressure", NODEFS_INODES: "DiskPressure"}
SIGNAL_TO_RESOURCE = {MEMORY: "memory", ALLOCATABLE_MEMORY: "memory", IMAGEFS: RESOURCE_IMAGEFS,
                      IMAGEFS_INODES: RESOURCE_IMAGEFS_INODES, NODEFS: RESOURCE_NODEFS, NODEFS_INODES: RESOURCE_NODEFS_INODES}
RESOURCE_CLAIM_TO_SIGNAL = {RESOURCE_NODEFS: [NODEFS], RESOURCE_IMAGEFS: [IMAGEFS], RESOURCE_NODEFS_INODES: [NODEFS_INODES],
                            RESOURCE_IMAGEFS_INODES: [IMAGEFS_INODES]}
SIGNALS = tuple(SIGNAL_TO_RESOURCE)
DEFAULT_HARD = "memory.available<100Mi,nodefs.available<10%,nodefs.inodesFree<5%"
FS_ROOT, FS_LOGS, FS_LOCAL_VOLUME = "root", "logs", "localVolumeSource"


# ---------------------------------------------------------------------------- thresholds
@dataclass(frozen=True, eq=False)
class ThresholdValue:
    quantity: int | None = None
    percentage: float = 0.0          # a float32 fraction, as the reference stores it

    def same(self, other: "ThresholdValue") -> bool:
        """compareThresholdValue (helpers.go:978-989)."""
        if self.quantity is not None:
            return other.quantity is not None and self.quantity == other.quantity
        return other.quantity is None and self.percentage == other.percentage


def threshold_quantity(v: ThresholdValue, capacity: int) -> int:
    """api.GetThresholdQuantity: the quantity, or int64(float64(capacity) * float64(percentage))."""
    if v.quantity is not None:
        return v.quantity
    return int(float(capacity) * float(v.percentage))


@dataclass(eq=False)
class Threshold:
    signal: str
    value: ThresholdValue
    grace: float = 0.0                          # seconds; 0 = a hard threshold
    min_reclaim: ThresholdValue | None = None
    operator: str = OP_LESS_THAN

    @property
    def hard(self) -> bool:
        return self.grace == 0

    def quantity(self, capacity: int) -> int:
        return threshold_quantity(self.value, capacity)

    # the node-allocatable reservation (cm.hard_eviction_reservation) reads these
    def value_of(self, capacity: int) -> int:
        return self.quantity(capacity)


def _float32_fraction(text: str) -> float:
    """parsePercentage: float32(ParseFloat(x, 32)) / 100 in float32 arithmetic."""
    return float(np.float32(np.float32(float(text)) / np.float32(100)))


def _parse_duration(s: str) -> float:
    """time.ParseDuration for the units the flags use (h, m, s, ms)."""
    s = s.strip()
    if not s:
        raise ValueError("time: invalid duration \"\"")
    total, i, sign = 0.0, 0, 1.0
    if s[0] in "+-":
        sign = -1.0 if s[0] == "-" else 1.0
        i = 1
    units = {"h": 3600.0, "m": 60.0, "s": 1.0, "ms": 1e-3, "us": 1e-6, "µs": 1e-6, "ns": 1e-9}
    if s[i:] == "0":
        return 0.0
    while i < len(s):
        j = i
        while j < len(s) and (s[j].isdigit() or s[j] == "."):
            j += 1
        if j == i:
            raise ValueError(f"time: invalid duration {s!r}")
        num = float(s[i:j])
        k = j
        while k < len(s) and not (s[k].isdigit() or s[k] == "."):
            k += 1
        unit = s[j:k]
        if unit not in units:
            raise ValueError(f"time: missing unit in duration {s!r}" if not unit else f"time: unknown unit {unit!r} in duration {s!r}")
        total += num * units[unit]
        i = k
    return sign * total


def _sign(q: Quantity) -> int:
    f = q.as_fraction()
    return (f > 0) - (f < 0)


_duration = _parse_duration        # the kubelet config file's durations


def parse_threshold_statement(signal: str, val: str) -> Threshold:
    if signal not in SIGNAL_TO_RESOURCE:
        raise ValueError(f"unsupported eviction signal {signal}")
    if val.endswith("%"):
        pct = _float32_fraction(val.rstrip("%"))
        if pct <= 0:
            raise ValueError(f"eviction percentage threshold {signal} must be positive: {val}")
        return Threshold(signal, ThresholdValue(percentage=pct))
    q = Quantity(val)
    if _sign(q) <= 0:
        raise ValueError(f"eviction threshold {signal} must be positive: {val}")
    return Threshold(signal, ThresholdValue(quantity=q.value()))


def get_allocatable_threshold(allocatable_config) -> list[Threshold]:
    if NODE_ALLOCATABLE_ENFORCEMENT_KEY in (allocatable_config or ()):
        return [Threshold(ALLOCATABLE_MEMORY, ThresholdValue(quantity=0), min_reclaim=ThresholdValue(quantity=0))]
    return []


def parse_threshold_config(allocatable_config=(), hard: dict | None = None, soft: dict | None = None,
                           soft_grace: dict | None = None, min_reclaim: dict | None = None) -> list[Threshold]:
    """ParseThresholdConfig (helpers.go:101-142)."""
    results = get_allocatable_threshold(allocatable_config)
    results += [parse_threshold_statement(s, v) for s, v in (hard or {}).items()]
    softs = [parse_threshold_statement(s, v) for s, v in (soft or {}).items()]
    graces = {}
    for s, v in (soft_grace or {}).items():
        if s not in SIGNAL_TO_RESOURCE:
            raise ValueError(f"unsupported eviction signal {s}")
        g = _parse_duration(v)
        if g < 0:
            raise ValueError(f"invalid eviction grace period specified: {v}, must be a positive value")
        graces[s] = g
    reclaims = {}
    for s, v in (min_reclaim or {}).items():
        if s not in SIGNAL_TO_RESOURCE:
            raise ValueError(f"unsupported eviction signal {s}")
        if v.endswith("%"):
            pct = _float32_fraction(v.rstrip("%"))
            if pct <= 0:
                raise ValueError(f"eviction percentage minimum reclaim {s} must be positive: {v}")
            reclaims[s] = ThresholdValue(percentage=pct)
            continue
        q = Quantity(v)
        if _sign(q) < 0:
            raise ValueError(f"negative eviction minimum reclaim specified for {s}")
        reclaims[s] = ThresholdValue(quantity=q.value())
    for t in softs:
        if t.signal not in graces:
            raise ValueError(f"grace period must be specified for the soft eviction threshold {t.signal}")
        t.grace = graces[t.signal]
    results += softs
    for t in results:
        if t.signal in reclaims:
            t.min_reclaim = reclaims[t.signal]
    return results


def split_flag(spec: str | None, sep: str) -> dict:
    """The `--eviction-*` flag syntax: `k<v,k<v` (thresholds) or `k=v,k=v`."""
    out = {}
    for part in filter(None, (x.strip() for x in (spec or "").split(","))):
        k, found, v = part.partition(sep)
        if not found:
            raise ValueError(f"malformed pair {part!r}, expecting \"k{sep}v\"")
        out[k.strip()] = v.strip()
    return out


def parse_thresholds(hard: str = "", soft: str = "", soft_grace: str = "", min_reclaim: str = "",
                     allocatable_config=()) -> list[Threshold]:
    """The kubelet's flags -> thresholds."""
    return parse_threshold_config(allocatable_config, split_flag(hard, "<"), split_flag(soft, "<"),
                                  split_flag(soft_grace, "="), split_flag(min_reclaim, "="))


# ---------------------------------------------------------------------------- observations
@dataclass
class Observation:
    available: int
    capacity: int
    time: object = None                # the stats' timestamp (None = unknown)


def _u(d, key):
    v = (d or {}).get(key)
    return None if v is None else int(v)


def pod_memory_usage(pod_stats: dict) -> int:
    return sum(int(((c.get("memory") or {}).get("workingSetBytes")) or 0) for c in pod_stats.get("containers") or [])


def stats_func_of(pods_stats: list[dict]):
    """cachedStatsFunc: pod -> its PodStats by UID (None when the summary has none)."""
    by_uid = {(p.get("podRef") or {}).get("uid"): p for p in pods_stats or []}
    return lambda pod: by_uid.get(m.uid_of(pod))


def make_signal_observations(summary: dict, capacity_provider, pods=()) -> tuple[dict, object]:
    """makeSignalObservations (helpers.go:718-790)."""
    node = summary.get("node") or {}
    res: dict[str, Observation] = {}
    mem = node.get("memory")
    if mem and mem.get("availableBytes") is not None and mem.get("workingSetBytes") is not None:
        res[MEMORY] = Observation(int(mem["availableBytes"]), int(mem["availableBytes"]) + int(mem["workingSetBytes"]),
                                  mem.get("time"))
    fs = node.get("fs")
    if fs:
        if fs.get("availableBytes") is not None and fs.get("capacityBytes") is not None:
            res[NODEFS] = Observation(int(fs["availableBytes"]), int(fs["capacityBytes"]), fs.get("time"))
        if fs.get("inodesFree") is not None and fs.get("inodes") is not None:
            res[NODEFS_INODES] = Observation(int(fs["inodesFree"]), int(fs["inodes"]), fs.get("time"))
    img = (node.get("runtime") or {}).get("imageFs")
    if img and img.get("availableBytes") is not None and img.get("capacityBytes") is not None:
        res[IMAGEFS] = Observation(int(img["availableBytes"]), int(img["capacityBytes"]), img.get("time"))
        if img.get("inodesFree") is not None and img.get("inodes") is not None:
            res[IMAGEFS_INODES] = Observation(int(img["inodesFree"]), int(img["inodes"]), img.get("time"))
    cap = (capacity_provider.capacity() or {}).get("memory") if capacity_provider is not None else None
    if cap is not None:
        avail = int(cap) - int((capacity_provider.reservation() or {}).get("memory", 0))
        for ps in summary.get("pods") or []:
            avail -= pod_memory_usage(ps)
        res[ALLOCATABLE_MEMORY] = Observation(avail, int(cap))
    return res, stats_func_of(summary.get("pods"))


def thresholds_met(thresholds, observations: dict, enforce_min_reclaim: bool) -> list[Threshold]:
    out = []
    for t in thresholds:
        obs = observations.get(t.signal)
        if obs is None:
            continue
        q = threshold_quantity(t.value, obs.capacity)
        if enforce_min_reclaim and t.min_reclaim is not None:
            q += threshold_quantity(t.min_reclaim, obs.capacity)
        if t.operator == OP_LESS_THAN and q > obs.available:
            out.append(t)
    return out


def _after(a, b) -> bool:
    return a is not None and (b is None or a > b)


def thresholds_updated_stats(thresholds, observations: dict, last: dict) -> list[Threshold]:
    """Only thresholds whose signal was observed anew since the last pass (helpers.go:850-865)."""
    out = []
    for t in thresholds:
        obs = observations.get(t.signal)
        if obs is None:
            continue
        prev = (last or {}).get(t.signal)
        if prev is None or obs.time is None or _after(obs.time, prev.time):
            out.append(t)
    return out


def thresholds_first_observed_at(thresholds, last_observed_at: dict, now) -> dict:
    return {t: last_observed_at.get(t, now) for t in thresholds}


def thresholds_met_grace_period(observed_at: dict, now) -> list[Threshold]:
    return [t for t, at in observed_at.items() if now - at >= t.grace]


def node_conditions(thresholds) -> list[str]:
    out = []
    for t in thresholds:
        c = SIGNAL_TO_NODE_CONDITION.get(t.signal)
        if c is not None and c not in out:
            out.append(c)
    return out


def node_conditions_last_observed_at(conditions, last: dict, now) -> dict:
    out = {c: now for c in conditions}
    for c, at in (last or {}).items():
        out.setdefault(c, at)
    return out


def node_conditions_observed_since(observed_at: dict, period: float, now) -> list[str]:
    return [c for c, at in observed_at.items() if now - at < period]


def has_threshold(items, t: Threshold) -> bool:
    return any(i.grace == t.grace and i.operator == t.operator and i.signal == t.signal and i.value.same(t.value)
               for i in items)


def merge_thresholds(a, b) -> list[Threshold]:
    out = list(a)
    for t in b:
        if not has_threshold(out, t):
            out.append(t)
    return out


def get_starved_resources(thresholds) -> list[str]:
    return [SIGNAL_TO_RESOURCE[t.signal] for t in thresholds if t.signal in SIGNAL_TO_RESOURCE]


def is_soft_eviction_thresholds(thresholds, starved: str) -> bool:
    return not any(SIGNAL_TO_RESOURCE.get(t.signal) == starved and t.hard for t in thresholds)


# ---------------------------------------------------------------------------- ranking
def _qty(v) -> int:
    return Quantity(v).value() if v not in (None, "") else 0


def pod_request(pod: dict, resource: str, local_storage: bool = True) -> int:
    """podRequest (helpers.go:594-625): max(sum of containers, largest init container)."""
    if resource == RESOURCE_DISK and not local_storage:
        return 0
    key = "memory" if resource == "memory" else "ephemeral-storage"
    spec = pod.get("spec") or {}
    total = sum(_qty(((c.get("resources") or {}).get("requests") or {}).get(key)) for c in spec.get("containers") or [])
    init = max([_qty(((c.get("resources") or {}).get("requests") or {}).get(key)) for c in spec.get("initContainers") or []]
               or [0])
    return max(total, init)


def local_volume_names(pod: dict) -> list[str]:
    return [v["name"] for v in (pod.get("spec") or {}).get("volumes") or []
            if "hostPath" in v or ("emptyDir" in v and (v["emptyDir"] or {}).get("medium") != "Memory")
            or "configMap" in v or "gitRepo" in v]


def local_ephemeral_volume_names(pod: dict) -> list[str]:
    return [v["name"] for v in (pod.get("spec") or {}).get("volumes") or []
            if "gitRepo" in v or ("emptyDir" in v and (v["emptyDir"] or {}).get("medium") != "Memory")
            or "configMap" in v or "downwardAPI" in v]


def _container_usage(pod_stats: dict, measure) -> tuple[int, int]:
    disk = inodes = 0
    for c in pod_stats.get("containers") or []:
        for kind, key in ((FS_ROOT, "rootfs"), (FS_LOGS, "logs")):
            if kind in measure:
                fs = c.get(key) or {}
                disk += int(fs.get("usedBytes") or 0)
                inodes += int(fs.get("inodesUsed") or 0)
    return disk, inodes


def _volume_usage(names, pod_stats: dict) -> tuple[int, int]:
    disk = inodes = 0
    vols = {v.get("name"): v for v in pod_stats.get("volume") or []}
    for n in names:
        v = vols.get(n)
        if v is not None:
            disk += int(v.get("usedBytes") or 0)
            inodes += int(v.get("inodesUsed") or 0)
    return disk, inodes


def pod_disk_usage(pod_stats: dict, pod: dict, measure) -> dict:
    disk, inodes = _container_usage(pod_stats, measure)
    if FS_LOCAL_VOLUME in measure:
        d, i = _volume_usage(local_volume_names(pod), pod_stats)
        disk, inodes = disk + d, inodes + i
    return {RESOURCE_DISK: disk, RESOURCE_INODES: inodes}


def pod_local_ephemeral_storage_usage(pod_stats: dict, pod: dict, measure) -> dict:
    disk, inodes = _container_usage(pod_stats, measure)
    if FS_LOCAL_VOLUME in measure:
        d, i = _volume_usage(local_ephemeral_volume_names(pod), pod_stats)
        disk, inodes = disk + d, inodes + i
    return {RESOURCE_DISK: disk, RESOURCE_INODES: inodes}


def _cmp_bool(a: bool, b: bool) -> int:
    """cmpBool: true sorts first."""
    return 0 if a == b else (-1 if a else 1)


def _cmp(a: int, b: int) -> int:
    return (a > b) - (a < b)


def priority(enabled: bool = True):
    """priority (helpers.go:519-533): lower priority first; all equal without the PodPriority gate."""
    def cmp(p1, p2):
        if not enabled:
            return 0
        return _cmp(int((p1.get("spec") or {}).get("priority") or 0), int((p2.get("spec") or {}).get("priority") or 0))
    return cmp


def _with_stats(stats, fn):
    """The rankers' common head: a pod without stats sorts first."""
    def cmp(p1, p2):
        s1, s2 = stats(p1), stats(p2)
        if s1 is None or s2 is None:
            return _cmp_bool(s1 is None, s2 is None)
        return fn(p1, s1, p2, s2)
    return cmp


def exceed_memory_requests(stats):
    return _with_stats(stats, lambda p1, s1, p2, s2: _cmp_bool(pod_memory_usage(s1) > pod_request(p1, "memory"),
                                                                pod_memory_usage(s2) > pod_request(p2, "memory")))


def memory(stats):
    """The larger working set above the memory request first."""
    return _with_stats(stats, lambda p1, s1, p2, s2: _cmp(pod_memory_usage(s2) - pod_request(p2, "memory"),
                                                          pod_memory_usage(s1) - pod_request(p1, "memory")))


def exceed_disk_requests(stats, measure, disk_resource: str, local_storage: bool = True):
    def used(p, s):
        return pod_disk_usage(s, p, measure)[disk_resource]
    return _with_stats(stats, lambda p1, s1, p2, s2: _cmp_bool(
        used(p1, s1) > pod_request(p1, disk_resource, local_storage),
        used(p2, s2) > pod_request(p2, disk_resource, local_storage)))


def disk(stats, measure, disk_resource: str, local_storage: bool = True):
    """The larger consumer above its request first; the request subtracted is the disk request
    even when ranking inodes (helpers.go:669-677)."""
    def used(p, s):
        return pod_disk_usage(s, p, measure)[disk_resource]
    return _with_stats(stats, lambda p1, s1, p2, s2: _cmp(
        used(p2, s2) - pod_request(p2, RESOURCE_DISK, local_storage),
        used(p1, s1) - pod_request(p1, RESOURCE_DISK, local_storage)))


def ordered_by(pods: list, *cmps):
    """orderedBy(...).Sort: the first comparator that separates two pods decides."""
    def cmp(a, b):
        for c in cmps:
            r = c(a, b)
            if r:
                return r
        return 0
    pods.sort(key=functools.cmp_to_key(cmp))


def rank_memory_pressure(pods: list, stats, priority_enabled: bool = True, local_storage: bool = True):
    """orderedBy(exceedMemoryRequests, priority, memory) (helpers.go:695-697)."""
    ordered_by(pods, exceed_memory_requests(stats), priority(priority_enabled), memory(stats))


def rank_disk_pressure_func(measure, disk_resource: str):
    def rank(pods: list, stats, priority_enabled: bool = True, local_storage: bool = True):
        ordered_by(pods, exceed_disk_requests(stats, measure, disk_resource, local_storage), priority(priority_enabled),
                   disk(stats, measure, disk_resource, local_storage))
    return rank


def build_resource_to_rank_func(with_image_fs: bool) -> dict:
    if with_image_fs:
        nodefs, imagefs = (FS_LOGS, FS_LOCAL_VOLUME), (FS_ROOT,)
    else:
        nodefs = imagefs = (FS_ROOT, FS_LOGS, FS_LOCAL_VOLUME)
    return {"memory": rank_memory_pressure,
            RESOURCE_NODEFS: rank_disk_pressure_func(nodefs, RESOURCE_DISK),
            RESOURCE_NODEFS_INODES: rank_disk_pressure_func(nodefs, RESOURCE_INODES),
            RESOURCE_IMAGEFS: rank_disk_pressure_func(imagefs, RESOURCE_DISK),
            RESOURCE_IMAGEFS_INODES: rank_disk_pressure_func(imagefs, RESOURCE_INODES)}


async def _maybe(v):
    return await v if inspect.isawaitable(v) else v


def _delete_containers(container_gc):
    async def reclaim():
        await _maybe(container_gc.delete_all_unused_containers())
        return 0                       # bytes freed is not known
    return reclaim


def _delete_images(image_gc, report_bytes: bool):
    async def reclaim():
        freed = await _maybe(image_gc.delete_unused_images())
        return int(freed or 0) if report_bytes else 0
    return reclaim


def build_resource_to_node_reclaim_funcs(image_gc, container_gc, with_image_fs: bool) -> dict:
    full = lambda report: [_delete_containers(container_gc), _delete_images(image_gc, report)]   # noqa: E731
    if with_image_fs:
        return {RESOURCE_NODEFS: [], RESOURCE_NODEFS_INODES: [], RESOURCE_IMAGEFS: full(True),
                RESOURCE_IMAGEFS_INODES: full(False)}
    return {RESOURCE_NODEFS: full(True), RESOURCE_NODEFS_INODES: full(False), RESOURCE_IMAGEFS: full(True),
            RESOURCE_IMAGEFS_INODES: full(False)}


# ---------------------------------------------------------------------------- the manager
def is_critical_pod(pod: dict) -> bool:
    from .qos import CRITICAL_ANNOTATION
    return m.namespace_of(pod) == "kube-system" and m.annotations_of(pod).get(CRITICAL_ANNOTATION) == ""


def is_static_pod(pod: dict) -> bool:
    return (m.annotations_of(pod).get("kubernetes.io/config.source") or "api") != "api"


def pod_is_evicted(status: dict) -> bool:
    return (status or {}).get("phase") == "Failed" and (status or {}).get("reason") == REASON


@dataclass
class Config:
    thresholds: list = field(default_factory=list)
    pressure_transition_period: float = 300.0
    max_pod_grace_period_seconds: int = 0


@dataclass
class CapacityProvider:
    """capacity (resource -> int) and the node-allocatable reservation (kube + system reserved)."""
    capacity_: dict = field(default_factory=dict)
    reservation_: dict = field(default_factory=dict)

    def capacity(self) -> dict:
        return self.capacity_

    def reservation(self) -> dict:
        return self.reservation_


class EvictionManager:
    """managerImpl: `kill_pod(pod, status, grace_override)`, `summary()` (the stats summary
    dict), `image_gc.delete_unused_images()` -> bytes, `container_gc.delete_all_unused_containers()`,
    `recorder.event(obj, type, reason, message)`; each may be sync or async."""

    def __init__(self, config: Config, kill_pod=None, summary=None, image_gc=None, container_gc=None, recorder=None,
                 node_ref=None, clock=time.monotonic, gates=None):
        self.config, self.kill_pod, self.summary = config, kill_pod, summary
        self.image_gc, self.container_gc, self.recorder, self.node_ref = image_gc, container_gc, recorder, node_ref
        self.clock = clock
        self.gates = gates or (lambda name: name == "PodPriority")
        self.node_conditions_: list[str] = []
        self.node_conditions_last_observed_at: dict = {}
        self.thresholds_first_observed_at: dict = {}
        self.thresholds_met_: list[Threshold] = []
        self.last_observations: dict = {}
        self.dedicated_image_fs: bool | None = None
        self.resource_to_rank_func: dict = {}
        self.resource_to_node_reclaim_funcs: dict = {}
        self.evictions = 0
        self.on_eviction = None            # callback(signal or resource) for metrics

    @property
    def thresholds(self) -> list[Threshold]:
        return self.config.thresholds

    # -------------------------------------------------------------- admission
    def admit(self, pod: dict) -> tuple[bool, str, str]:
        """Admit (eviction_manager.go:121-145) -> (admit, reason, message)."""
        from .qos import BEST_EFFORT, pod_qos
        conds = self.node_conditions_
        if not conds:
            return True, "", ""
        if self.gates("ExperimentalCriticalPodAnnotation") and is_critical_pod(pod):
            return True, "", ""
        if "MemoryPressure" in conds and pod_qos(pod) != BEST_EFFORT:
            return True, "", ""
        return False, REASON, MESSAGE.format("[" + " ".join(conds) + "]")

    def is_under_memory_pressure(self) -> bool:
        return "MemoryPressure" in self.node_conditions_

    def is_under_disk_pressure(self) -> bool:
        return "DiskPressure" in self.node_conditions_

    @property
    def conditions(self) -> set[str]:
        return set(self.node_conditions_)

    # -------------------------------------------------------------- synchronize
    async def _event(self, obj, typ, reason, msg):
        if self.recorder is not None:
            await _maybe(self.recorder.event(obj, typ, reason, msg))

    async def synchronize(self, has_dedicated_image_fs, active_pods, capacity_provider) -> list[dict] | None:
        """One pass (eviction_manager.go:199-371); returns the evicted pods, if any."""
        thresholds = self.config.thresholds
        if not thresholds:
            return None
        if self.dedicated_image_fs is None:
            try:
                with_image_fs = bool(await _maybe(has_dedicated_image_fs()))
            except Exception:
                return None
            self.dedicated_image_fs = with_image_fs
            self.resource_to_rank_func = build_resource_to_rank_func(with_image_fs)
            self.resource_to_node_reclaim_funcs = build_resource_to_node_reclaim_funcs(
                self.image_gc, self.container_gc, with_image_fs)
        pods = list(active_pods())
        summary = await _maybe(self.summary())
        observations, stats = make_signal_observations(summary, capacity_provider, pods)

        thresholds = thresholds_met(thresholds, observations, False)
        if self.thresholds_met_:
            thresholds = merge_thresholds(thresholds, thresholds_met(self.thresholds_met_, observations, True))
        now = self.clock()
        first = thresholds_first_observed_at(thresholds, self.thresholds_first_observed_at, now)
        conds = node_conditions(thresholds)
        last_at = node_conditions_last_observed_at(conds, self.node_conditions_last_observed_at, now)
        conds = node_conditions_observed_since(last_at, self.config.pressure_transition_period, now)
        thresholds = thresholds_met_grace_period(first, now)

        self.node_conditions_ = conds
        self.thresholds_first_observed_at = first
        self.node_conditions_last_observed_at = last_at
        self.thresholds_met_ = thresholds
        thresholds = thresholds_updated_stats(thresholds, observations, self.last_observations)
        self.last_observations = observations

        if self.gates("LocalStorageCapacityIsolation"):
            evicted = await self.local_storage_eviction(pods, summary)
            if evicted:
                return evicted

        starved = get_starved_resources(thresholds)
        if not starved:
            return None
        starved.sort(key=lambda r: r != "memory")          # byEvictionPriority: memory first
        resource = starved[0]
        soft = is_soft_eviction_thresholds(thresholds, resource)
        await self._event(self.node_ref, "Warning", "EvictionThresholdMet", f"Attempting to reclaim {resource}")
        if await self.reclaim_node_level_resources(resource, observations):
            return None
        rank = self.resource_to_rank_func.get(resource)
        if rank is None or not pods:
            return None
        rank(pods, stats, self.gates("PodPriority"), self.gates("LocalStorageCapacityIsolation"))
        for pod in pods:
            if self.gates("ExperimentalCriticalPodAnnotation") and is_critical_pod(pod) and is_static_pod(pod):
                continue
            msg = MESSAGE.format(resource)
            status = {"phase": "Failed", "message": msg, "reason": REASON}
            await self._event(pod, "Warning", REASON, msg)
            grace = self.config.max_pod_grace_period_seconds if soft else 0
            self.evictions += 1
            if self.on_eviction is not None:
                self.on_eviction(resource)
            try:
                await _maybe(self.kill_pod(pod, status, grace))
            except Exception:
                pass
            return [pod]
        return None

    async def reclaim_node_level_resources(self, resource: str, observations: dict) -> bool:
        """reclaimNodeLevelResources (eviction_manager.go:394-418): after each reclaim function,
        credit the freed bytes to the resource's signals and stop once no threshold met at this
        pass is still unresolved."""
        for fn in self.resource_to_node_reclaim_funcs.get(resource, []):
            try:
                freed = await fn()
            except Exception:
                freed = 0
            for sig in RESOURCE_CLAIM_TO_SIGNAL.get(resource, []):
                obs = observations.get(sig)
                if obs is not None:
                    obs.available += freed
            if not thresholds_met(self.thresholds_met_, observations, True):
                return True
        return False

    # -------------------------------------------------------------- local storage
    async def local_storage_eviction(self, pods, summary) -> list[dict]:
        stats = stats_func_of(summary.get("pods"))
        evicted = []
        for pod in pods:
            ps = stats(pod)
            if ps is None:
                continue
            if await self._empty_dir_limit_eviction(ps, pod) or await self._pod_ephemeral_limit_eviction(ps, pod) \
                    or await self._container_ephemeral_limit_eviction(ps, pod):
                evicted.append(pod)
        return evicted

    async def _empty_dir_limit_eviction(self, ps, pod) -> bool:
        used = {v.get("name"): int(v.get("usedBytes") or 0) for v in ps.get("volume") or []}
        for v in (pod.get("spec") or {}).get("volumes") or []:
            ed = v.get("emptyDir")
            if ed is None or not ed.get("sizeLimit"):
                continue
            size = Quantity(ed["sizeLimit"])
            u = used.get(v["name"])
            if u is not None and _sign(size) == 1 and u > size.value():
                return await self.evict_pod(pod, "EmptyDir", f'emptyDir usage exceeds the limit "{size}"')
        return False

    async def _pod_ephemeral_limit_eviction(self, ps, pod) -> bool:
        """PodRequestsAndLimits: the containers' ephemeral-storage limits summed (init containers
        max-merged), present when any container sets one."""
        spec = pod.get("spec") or {}
        lims = [((c.get("resources") or {}).get("limits") or {}).get("ephemeral-storage") for c in spec.get("containers") or []]
        ilims = [((c.get("resources") or {}).get("limits") or {}).get("ephemeral-storage") for c in spec.get("initContainers") or []]
        if not any(x for x in lims + ilims):
            return False
        limit = max([sum(_qty(x) for x in lims)] + [_qty(x) for x in ilims])
        measure = (FS_LOGS, FS_LOCAL_VOLUME) if self.dedicated_image_fs else (FS_ROOT, FS_LOGS, FS_LOCAL_VOLUME)
        usage = pod_local_ephemeral_storage_usage(ps, pod, measure)[RESOURCE_DISK]
        if usage > limit:
            return await self.evict_pod(pod, "ephemeral-storage",
                                        f"pod ephemeral local storage usage exceeds the total limit of containers {limit}")
        return False

    async def _container_ephemeral_limit_eviction(self, ps, pod) -> bool:
        limits = {}
        for c in (pod.get("spec") or {}).get("containers") or []:
            v = ((c.get("resources") or {}).get("limits") or {}).get("ephemeral-storage")
            if v and _qty(v) != 0:
                limits[c.get("name")] = v
        for cs in ps.get("containers") or []:
            used = int((cs.get("logs") or {}).get("usedBytes") or 0)
            if not self.dedicated_image_fs:
                used += int((cs.get("rootfs") or {}).get("usedBytes") or 0)
            lim = limits.get(cs.get("name"))
            if lim is not None and _qty(lim) < used:
                return await self.evict_pod(pod, "ephemeral-storage",
                                            f"container's ephemeral local storage usage exceeds the limit \"{lim}\"")
        return False

    async def evict_pod(self, pod, resource: str, evict_msg: str) -> bool:
        if self.gates("ExperimentalCriticalPodAnnotation") and is_critical_pod(pod) and is_static_pod(pod):
            return False
        status = {"phase": "Failed", "message": MESSAGE.format(resource), "reason": REASON}
        await self._event(pod, "Warning", REASON, evict_msg)
        self.evictions += 1
        if self.on_eviction is not None:
            self.on_eviction(resource)
        try:
            await _maybe(self.kill_pod(pod, status, 0))
        except Exception:
            pass
        return True


# ---------------------------------------------------------------------------- host observation
def observe(root_dir: str = "/", image_dir: str | None = None) -> dict:
    """A stats-summary-shaped node section from the host (psutil memory, statvfs filesystems)
    for callers without a kubelet stats provider."""
    import os
    import psutil
    vm = psutil.virtual_memory()
    node = {"memory": {"availableBytes": int(vm.available), "workingSetBytes": int(vm.total - vm.available)}}
    for key, path in (("fs", root_dir), ("imageFs", image_dir)):
        if path is None:
            continue
        try:
            st = os.statvfs(path)
        except OSError:
            continue
        fs = {"availableBytes": st.f_bavail * st.f_frsize, "capacityBytes": st.f_blocks * st.f_frsize,
              "inodesFree": st.f_favail, "inodes": st.f_files}
        if key == "fs":
            node["fs"] = fs
        else:
            node["runtime"] = {"imageFs": fs}
    return {"node": node, "pods": []}
