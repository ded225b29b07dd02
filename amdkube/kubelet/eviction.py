"""Kubelet eviction manager.

Reference: pkg/kubelet/eviction — api/types.go (signals memory.available, nodefs.available,
nodefs.inodesFree, imagefs.available, imagefs.inodesFree), helpers.go ParseThresholdConfig
(`--eviction-hard=memory.available<100Mi,nodefs.available<10%`, `--eviction-soft` with
`--eviction-soft-grace-period`, `--eviction-minimum-reclaim`), eviction_manager.go synchronize
(observe → thresholds met → soft thresholds only after their grace period → node conditions
MemoryPressure / DiskPressure held for --eviction-pressure-transition-period → rank → evict one
pod per pass), rank.go (memory: QoS class, then usage above requests; disk: QoS, then disk
usage), and Admit (MemoryPressure rejects BestEffort pods, DiskPressure rejects all).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

from ..api.quantity import Quantity

MEMORY, NODEFS, NODEFS_INODES, IMAGEFS, IMAGEFS_INODES = ("memory.available", "nodefs.available", "nodefs.inodesFree",
                                                         "imagefs.available", "imagefs.inodesFree")
SIGNALS = (MEMORY, NODEFS, NODEFS_INODES, IMAGEFS, IMAGEFS_INODES)
CONDITION = {MEMORY: "MemoryPressure", NODEFS: "DiskPressure", NODEFS_INODES: "DiskPressure",
             IMAGEFS: "DiskPressure", IMAGEFS_INODES: "DiskPressure"}
RESOURCE = {MEMORY: "memory", NODEFS: "ephemeral-storage", NODEFS_INODES: "inodes", IMAGEFS: "ephemeral-storage",
            IMAGEFS_INODES: "inodes"}
DEFAULT_HARD = "memory.available<100Mi,nodefs.available<10%,nodefs.inodesFree<5%"


@dataclass
class Threshold:
    signal: str
    quantity: int | None = None       # absolute (bytes / inodes)
    percentage: float | None = None   # of capacity
    grace: float = 0.0                # soft thresholds
    min_reclaim: int = 0              # absolute minimum reclaim
    min_reclaim_pct: float = 0.0      # minimum reclaim as a fraction of capacity
    hard: bool = True

    def value(self, capacity: int) -> int:
        return self.quantity if self.quantity is not None else int(capacity * (self.percentage or 0.0))

    def reclaim(self, capacity: int) -> int:
        return self.min_reclaim + int(capacity * self.min_reclaim_pct)

    @property
    def key(self):
        return (self.signal, self.hard)


def _duration(s: str) -> float:
    total, num = 0.0, ""
    units = {"h": 3600, "m": 60, "s": 1}
    for ch in s.strip():
        if ch.isdigit() or ch == ".":
            num += ch
        elif ch in units:
            total += float(num) * units[ch]
            num = ""
        else:
            raise ValueError(f"bad duration {s!r}")
    return total + (float(num) if num else 0.0)


def parse_thresholds(hard: str = "", soft: str = "", soft_grace: str = "", min_reclaim: str = "") -> list[Threshold]:
    def kv(spec, sep):
        out = {}
        for part in filter(None, (x.strip() for x in (spec or "").split(","))):
            k, _, v = part.partition(sep)
            if k not in SIGNALS:
                raise ValueError(f"unsupported eviction signal {k!r}")
            out[k] = v
        return out
    graces = {k: _duration(v) for k, v in kv(soft_grace, "=").items()}
    reclaims = {k: v for k, v in kv(min_reclaim, "=").items()}
    out = []
    for spec, is_hard in ((hard, True), (soft, False)):
        for sig, v in kv(spec, "<").items():
            t = Threshold(sig, hard=is_hard)
            if v.endswith("%"):
                t.percentage = float(v[:-1]) / 100.0
            else:
                t.quantity = Quantity(v).value()
            if not is_hard:
                if sig not in graces:
                    raise ValueError(f"soft eviction threshold {sig} needs a grace period")
                t.grace = graces[sig]
            if sig in reclaims:
                r = reclaims[sig]
                if r.endswith("%"):
                    t.min_reclaim_pct = float(r[:-1]) / 100.0
                else:
                    t.min_reclaim = int(Quantity(r).value())
            out.append(t)
    return out


def observe(root_dir: str = "/", image_dir: str | None = None) -> dict:
    """signal → (available, capacity) from the node (psutil memory; statvfs for the filesystems)."""
    import psutil
    vm = psutil.virtual_memory()
    obs = {MEMORY: (int(vm.available), int(vm.total))}
    for sig_b, sig_i, path in ((NODEFS, NODEFS_INODES, root_dir), (IMAGEFS, IMAGEFS_INODES, image_dir or root_dir)):
        try:
            st = os.statvfs(path)
            obs[sig_b] = (st.f_bavail * st.f_frsize, st.f_blocks * st.f_frsize)
            obs[sig_i] = (st.f_favail, st.f_files)
        except OSError:
            pass
    return obs


def _requests(p: dict, resource: str) -> int:
    tot = 0
    for c in (p.get("spec") or {}).get("containers") or []:
        res = c.get("resources") or {}
        r = (res.get("requests") or {}).get(resource) or (res.get("limits") or {}).get(resource)   # defaulting: requests := limits
        tot += Quantity(r).value() if r else 0
    return tot


def rank(pods: list[dict], signal: str, usage: dict[str, int], use_priority: bool = True) -> list[dict]:
    """helpers.go:695-703 orderedBy(exceedRequests, priority, usage): pods without stats first,
    then pods whose usage exceeds their request of the starved resource, then lower priority
    (only with the PodPriority gate, helpers.go:519-533), then the larger usage above request."""
    res = "memory" if RESOURCE[signal] == "memory" else "ephemeral-storage"

    def key(p):
        uid = (p.get("metadata") or {}).get("uid", "")
        if uid not in usage:
            return (0, 0, 0, 0)
        u, req = usage[uid], _requests(p, res)
        prio = int((p.get("spec") or {}).get("priority") or 0) if use_priority else 0
        return (1, 0 if u > req else 1, prio, -(u - req))
    return sorted(pods, key=key)


@dataclass
class EvictionManager:
    thresholds: list[Threshold]
    pressure_transition: float = 300.0
    max_pod_grace: int = 0
    observer: object = None
    clock: object = time.monotonic
    use_priority: bool = True
    first_seen: dict = field(default_factory=dict)     # signal → when the (soft) threshold was first met
    pressure_since: dict = field(default_factory=dict)  # condition → last time it was observed
    last_met: set = field(default_factory=set)          # keys of thresholds met at the last pass (m.thresholdsMet)
    evictions: int = 0

    def met(self, obs: dict) -> list[Threshold]:
        """eviction_manager.go:267-275: thresholds met now, merged with previously met ones that
        are not yet resolved, i.e. still below threshold + minimum reclaim."""
        out = []
        now = self.clock()
        for t in self.thresholds:
            if t.signal not in obs:
                continue
            avail, cap = obs[t.signal]
            bound = t.value(cap) + (t.reclaim(cap) if t.key in self.last_met else 0)
            if avail < bound:
                self.first_seen.setdefault(t.key, now)
                if t.hard or now - self.first_seen[t.key] >= t.grace:
                    out.append(t)
            else:
                self.first_seen.pop(t.key, None)
        self.last_met = {t.key for t in out}
        return out

    def conditions(self, obs: dict) -> set[str]:
        """Pressure conditions, held for the transition period after the last observation."""
        now = self.clock()
        for t in self.thresholds:
            if t.signal in obs and obs[t.signal][0] < t.value(obs[t.signal][1]):
                self.pressure_since[CONDITION[t.signal]] = now
        return {c for c, ts in self.pressure_since.items() if now - ts < self.pressure_transition or ts == now}

    def admit(self, pod: dict, conditions: set[str]) -> tuple[bool, str]:
        from .qos import pod_qos
        if "DiskPressure" in conditions:
            return False, "The node was low on resource: [DiskPressure]."
        if "MemoryPressure" in conditions and pod_qos(pod) == "BestEffort":
            return False, "The node was low on resource: [MemoryPressure]."
        return True, ""

    def choose(self, pods: list[dict], obs: dict, usage: dict[str, int]) -> tuple[dict | None, Threshold | None]:
        met = self.met(obs)
        if not met or not pods:
            return None, None
        t = sorted(met, key=lambda x: (x.signal != MEMORY, not x.hard))[0]   # memory first (reference order)
        return rank(pods, t.signal, usage, self.use_priority)[0], t

    def grace_for(self, pod: dict, t: Threshold) -> int:
        """eviction_manager.go:391-396: hard evictions kill immediately; soft ones get
        MaxPodGracePeriodSeconds (default 0), not the pod's own grace period."""
        return 0 if t.hard else int(self.max_pod_grace)
