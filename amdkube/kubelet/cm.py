"""Container-manager pieces of the kubelet: node allocatable and the pods cgroup limit.

Reference pkg/kubelet/cm/node_container_manager.go: GetNodeAllocatableReservation =
--kube-reserved + --system-reserved + the hard eviction thresholds (memory.available and
nodefs.available, hardEvictionReservation); kubelet_node_status.go setNodeStatusMachineInfo
sets allocatable = capacity − reservation (clamped at 0). --enforce-node-allocatable=pods
caps the top-level pods cgroup at allocatable (enforceNodeAllocatableCgroups); here the
kubepods cgroup (the QoS hierarchy rocshim creates under its cgroup root) gets memory.max and
cpu.max = allocatable when the cgroup v2 directory is writable.
"""
from __future__ import annotations

import logging
import os

from ..api.quantity import Quantity

log = logging.getLogger("amdkube.kubelet.cm")

RESERVABLE = ("cpu", "memory", "ephemeral-storage", "pods")


def parse_reserved(spec: str | dict | None) -> dict[str, int]:
    """`cpu=500m,memory=1Gi,ephemeral-storage=1Gi` → {resource: value} (cpu in millicores)."""
    if not spec:
        return {}
    items = spec.items() if isinstance(spec, dict) else (kv.split("=", 1) for kv in spec.split(",") if kv.strip())
    out = {}
    for k, v in items:
        k = k.strip()
        if k not in RESERVABLE:
            raise ValueError(f"cannot reserve {k!r} (only {', '.join(RESERVABLE)})")
        q = Quantity(str(v).strip())
        out[k] = q.milli_value() if k == "cpu" else q.value()
    return out


def hard_eviction_reservation(thresholds, capacity: dict[str, int]) -> dict[str, int]:
    """hardEvictionReservation: memory.available / nodefs.available hard thresholds reserve
    their absolute value (or percentage of capacity) of memory / ephemeral-storage."""
    out: dict[str, int] = {}
    for t in thresholds or ():
        if not t.hard:
            continue
        res = {"memory.available": "memory", "nodefs.available": "ephemeral-storage"}.get(t.signal)
        if res is None or res not in capacity:
            continue
        out[res] = out.get(res, 0) + t.quantity(capacity[res])
    return out


def _qty(res: str, v: int) -> str:
    if res == "cpu":
        return f"{v}m" if v % 1000 else str(v // 1000)
    if res == "memory" and v % 1024 == 0:
        return f"{v // 1024}Ki"
    return str(v)


def node_allocatable(capacity: dict[str, str], kube_reserved: dict[str, int], system_reserved: dict[str, int],
                     thresholds=()) -> dict[str, str]:
    """capacity (API strings) → allocatable (API strings); resources without a reservation
    (pods, extended resources) pass through unchanged."""
    cap = {k: (Quantity(v).milli_value() if k == "cpu" else Quantity(v).value()) for k, v in capacity.items()
           if k in RESERVABLE}
    ev = hard_eviction_reservation(thresholds, cap)
    out = dict(capacity)
    for k, v in cap.items():
        r = kube_reserved.get(k, 0) + system_reserved.get(k, 0) + ev.get(k, 0)
        if r:
            out[k] = _qty(k, max(0, v - r))
    return out


def enforce_pods_cgroup(cgroup_root: str, allocatable: dict[str, str], cpu_period_us: int = 100000,
                        manager=None) -> bool:
    """Write the pods cgroup's limits (cgroup v2) from allocatable, through the configured
    cgroup driver (`manager`, a cgroups.CgroupManager; cgroupfs under cgroup_root by default):
    /kubepods is the directory `kubepods` or, with systemd, the unit kubepods.slice. False when
    the cgroup tree is not there or not writable (e.g. an unprivileged node): allocatable is
    still reported and scheduled against, only the kernel cap is missing."""
    from .cgroups import CgroupManager
    manager = manager or CgroupManager("cgroupfs", cgroup_root)
    res = {}
    if "memory" in allocatable:
        res["memory"] = Quantity(allocatable["memory"]).value()
    if "cpu" in allocatable:
        res["cpu_quota"] = max(1000, Quantity(allocatable["cpu"]).milli_value() * cpu_period_us // 1000)
        res["cpu_period"] = cpu_period_us
    try:
        manager.create("/kubepods", res)
        return True
    except Exception as e:
        log.debug("pods cgroup limits not enforced under %s: %r", manager.path("/kubepods"), e)
        return False
