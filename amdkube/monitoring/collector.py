"""GPU metric collection (node + per-container) on top of the SMI backends.

Replaces cAdvisor's NVML accelerator collector (vendor/github.com/google/cadvisor/
accelerators/nvidia.go:140-252 — per-container AcceleratorStats{Make, Model, ID,
MemoryTotal, MemoryUsed, DutyCycle} found by parsing the devices cgroup for c 195:<minor>)
and its Prometheus export (vendor/github.com/google/cadvisor/metrics/prometheus.go:275-306).
The container↔GPU mapping comes from the kubelet's own allocation record (assigned device
IDs), not from cgroup-v1 parsing.

MemoryUsed is the container's own VRAM where the backend reports per-process usage (amd-smi
process list): the sum over the container's process tree (`container_pids`). A GPU shared by
several containers — compute partitions (CPX/DPX) over one memory pool, NPS modes, time
slicing — then reports each container's allocation instead of the whole device's. Without a
process list it falls back to the device's VRAM in use, as cAdvisor's NVML collector does.
"""
from __future__ import annotations

import os
import time

from ..smi import device_id


def container_pids(pid: int | None) -> set[int]:
    """The host PIDs of a container: its init process and every descendant."""
    if not pid:
        return set()
    try:
        import psutil
        root = psutil.Process(int(pid))
        return {root.pid} | {c.pid for c in root.children(recursive=True)}
    except Exception:
        return set()

# cAdvisor's DutyCycle is the NVML average over the last 10 s (accelerators/nvidia.go:216-252)
DUTY_CYCLE_WINDOW_S = 10.0


def duty_cycle(backend, index: int, sample: dict) -> int:
    """Percent busy over the last DUTY_CYCLE_WINDOW_S from the backend's activity sampler,
    else the instantaneous gfx activity of `sample`."""
    try:
        avg = backend.average_activity(index, DUTY_CYCLE_WINDOW_S)
    except Exception:
        avg = None
    if avg:
        return int(round(avg["gfx_activity"]))
    return int(sample.get("gfx_activity") or 0)


class AcceleratorCollector:
    def __init__(self, backend, node: str = ""):
        self.b = backend
        self.node = node
        self._gpus = None
        if backend:
            backend.start_sampling()

    def gpus(self):
        if self._gpus is None:
            self._gpus = self.b.gpus() if self.b else []
        return self._gpus

    def by_id(self):
        return {device_id(g): g for g in self.gpus()}

    def accelerator_stats(self, ids: list[str] | None, pids: set[int] | None = None) -> list[dict]:
        """stats/v1alpha1 AcceleratorStats for the given device IDs (None = all GPUs). With the
        container's `pids`, memoryUsed is what those processes hold on each device."""
        if not self.b:
            return []
        out = []
        bid = self.by_id()
        for did in (ids if ids is not None else list(bid)):
            g = bid.get(did)
            if g is None:
                continue
            try:
                s = self.b.sample(g["index"])
            except Exception:
                s = {}
            used = int(s.get("vram_used_bytes") or 0)
            if pids is not None and getattr(self.b, "per_process", False):
                try:
                    procs = self.b.processes(g["index"])
                except Exception:
                    procs = None
                # only when the SMI's PIDs are ours to compare (same PID namespace): otherwise keep
                # the device-level number rather than attribute nothing
                if procs is not None and (not procs or any(os.path.exists(f"/proc/{int(p.get('pid', -1))}") for p in procs)):
                    used = sum(int(p.get("vram_bytes") or 0) for p in procs if int(p.get("pid", -1)) in pids)
            out.append({"make": "amd", "model": g.get("market_name", ""), "id": did,
                        "memoryTotal": int(g.get("vram_total_bytes") or 0), "memoryUsed": used,
                        "dutyCycle": duty_cycle(self.b, g["index"], s)})
        return out

    def render_container_metrics(self, pod_devices: list[dict]) -> str:
        """container_accelerator_* exposition text (cadvisor metric names + labels)."""
        lines = ["# HELP container_accelerator_memory_total_bytes Total accelerator memory.",
                 "# TYPE container_accelerator_memory_total_bytes gauge",
                 "# HELP container_accelerator_memory_used_bytes Total accelerator memory allocated.",
                 "# TYPE container_accelerator_memory_used_bytes gauge",
                 "# HELP container_accelerator_duty_cycle Percent of time over the past sample period during which the accelerator was actively processing.",
                 "# TYPE container_accelerator_duty_cycle gauge"]
        for pd in pod_devices:
            for st in pd.get("stats") or self.accelerator_stats(pd["devices"], pd.get("pids")):
                lab = (f'container_name="{pd["container"]}",pod_name="{pd["pod"]}",namespace="{pd["namespace"]}",'
                       f'make="{st["make"]}",model="{st["model"]}",acc_id="{st["id"]}"')
                lines.append(f"container_accelerator_memory_total_bytes{{{lab}}} {st['memoryTotal']}")
                lines.append(f"container_accelerator_memory_used_bytes{{{lab}}} {st['memoryUsed']}")
                lines.append(f"container_accelerator_duty_cycle{{{lab}}} {st['dutyCycle']}")
        return "\n".join(lines) + "\n"


def now() -> float:
    return time.time()
