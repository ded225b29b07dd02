"""The AMD Instinct (MI355X) device plugin: advertises `amd.com/gpu` with device attributes,
tracks health from amd-smi RAS/ECC counters (plus an optional on-device HBM pattern probe),
and injects /dev/kfd + the GPU's DRM render node into containers.

Replaces the out-of-tree NVIDIA plugin the reference's DaemonSet deploys
(cluster/addons/device-plugins/nvidia-gpu/daemonset.yaml) and the legacy in-kubelet NVIDIA
path (pkg/kubelet/gpu/nvidia/nvidia_gpu_manager.go: /dev/nvidia* + nvidiactl + nvidia-uvm).

Published per-device Attributes (matchable by PodSpec extendedResources[].affinity.required,
SURVEY Appendix A.3; keys are single-slash qualified names, values label-safe — quirk #13):
  amd.com/gpu-type      MI355X            amd.com/gpu-memory  294896 (MiB, integer → Gt/Lt)
  amd.com/gfx           gfx950            amd.com/cu-count    256
  amd.com/numa-node     0                 amd.com/xgmi-hive   42a9…  (hex)
  amd.com/partition     SPX               amd.com/memory-partition NPS1
  amd.com/index         node-local index  amd.com/pci-bus     0000-23-00.0
  amd.com/partition-id  0..7 (partitioned GPUs only)   amd.com/parent-gpu  0000-23-00.0
Partitioned MI355X (compute partition DPX/QPX/CPX, memory NPS1/NPS2): every partition is a
device. Resource naming (`resource_groups`): "single" advertises everything as amd.com/gpu
(select partitions with the attributes above); "mixed" advertises whole GPUs as amd.com/gpu
and partitions as amd.com/<compute>_<memory> (e.g. amd.com/cpx_nps2), one plugin socket each.
Plugin labels (GetPluginInfoResponse.labels, field 2 of the fork's wire format) carry the
node's GPU link matrix as `amd.com/gpu-topology` JSON, which the kubelet copies into a node
annotation for the scheduler's xGMI/NUMA scorer.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import subprocess

from ..grpcdesc.deviceplugin import DEVICE_PLUGINS_PATH, HEALTHY, UNHEALTHY
from ..smi import Backend, device_id, visibility_token
from ..smi.backend import parent_key, partition_count
from .server import DevicePluginServer

from ..smi.health import HEALTH_REASON_ATTR  # noqa: E402

log = logging.getLogger("amdkube.deviceplugin.amd")

RESOURCE = "amd.com/gpu"
TOPOLOGY_LABEL = "amd.com/gpu-topology"
RUNTIME_ANNOTATION = "io.amdkube.runtime"
BIN_DIR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "_native", "bin")


def gpu_type(g: dict) -> str:
    name = (g.get("market_name") or g.get("product_name") or "").replace("AMD Instinct", "").strip()
    for known in ("MI355", "MI350", "MI325", "MI308", "MI300"):
        if known in name:
            return known + "X" if not name.startswith(known + "A") else known + "A"
    tok = name.split()[0] if name else (g.get("gfx_target") or "unknown")
    return "".join(ch for ch in tok if ch.isalnum() or ch in "-_.") or "unknown"


def attributes(g: dict) -> dict:
    a = {"amd.com/gpu-type": gpu_type(g), "amd.com/index": str(g.get("index", 0))}
    if g.get("vram_total_bytes"):
        a["amd.com/gpu-memory"] = str(int(g["vram_total_bytes"]) >> 20)
    if g.get("gfx_target"):
        a["amd.com/gfx"] = g["gfx_target"]
    if g.get("num_cu"):
        a["amd.com/cu-count"] = str(g["num_cu"])
    if g.get("numa_node") is not None:
        a["amd.com/numa-node"] = str(g["numa_node"])
    if g.get("xgmi_hive_id"):
        a["amd.com/xgmi-hive"] = f"{int(g['xgmi_hive_id']):x}"
    if g.get("compute_partition"):
        a["amd.com/partition"] = g["compute_partition"]
    if g.get("memory_partition"):
        a["amd.com/memory-partition"] = g["memory_partition"]
    if g.get("bdf"):
        a["amd.com/pci-bus"] = g["bdf"].replace(":", "-")
    if partition_count(g) > 1:
        a["amd.com/partition-id"] = str(int(g.get("partition_id") or 0))
        a["amd.com/parent-gpu"] = parent_key(g).replace(":", "-")
    return a


def resource_groups(gpus: list[dict], strategy: str = "single", base: str = RESOURCE) -> dict[str, list[dict]]:
    """Split a node's devices into advertised resources (see module doc)."""
    if strategy not in ("single", "mixed"):
        raise ValueError(f"unknown resource naming strategy {strategy!r} (single|mixed)")
    out: dict[str, list[dict]] = {}
    for g in gpus:
        if strategy == "single" or partition_count(g) <= 1 and str(g.get("memory_partition") or "NPS1").upper() == "NPS1":
            name = base
        else:
            cp = str(g.get("compute_partition") or "SPX").lower()
            mp = str(g.get("memory_partition") or "NPS1").lower()
            name = f"{base.split('/')[0]}/{cp}_{mp}"
        out.setdefault(name, []).append(g)
    return out


def topology_label(gpus: list[dict], topo: list[list[dict]]) -> str:
    """The `amd.com/gpu-topology` annotation the scheduler's allocator reads: device IDs, NUMA
    node, and a link cost per pair. The cost is the driver's link weight; where the driver
    reports the xGMI link bandwidth of every pair (amdsmi minmax bandwidth), the cost scales
    inversely with it (15 for the fastest pair), so a slower link costs more than a faster
    one rather than every xGMI hop costing the same."""
    ids = [device_id(g) for g in gpus]
    off = [e for i, row in enumerate(topo) for j, e in enumerate(row) if i != j]
    bws = [int(e.get("max_bw_mbps") or 0) for e in off]
    by_bw = bool(off) and all(b > 0 for b in bws)
    best = max(bws) if by_bw else 0
    link = []
    for i, row in enumerate(topo):
        r = []
        for j, e in enumerate(row):
            if i == j:
                r.append(0)
                continue
            if by_bw:
                w = max(1, round(15 * best / int(e["max_bw_mbps"])))
            else:
                w = e.get("weight")
                if not w:
                    w = {"xgmi": 15, "pcie": 40}.get(e.get("type"), 60) * max(1, int(e.get("hops") or 1))
            r.append(int(w))
        link.append(r)
    out = {"ids": ids, "numa": [int(g.get("numa_node") or 0) for g in gpus], "link": link,
           "type": [[(e.get("type") or "")[:4] for e in row] for row in topo]}
    if any(partition_count(g) > 1 for g in gpus):
        pk: dict[str, int] = {}
        out["parent"] = [pk.setdefault(parent_key(g), len(pk)) for g in gpus]
    return json.dumps(out, separators=(",", ":"))


def _attr_value(why: str) -> str:
    """An attribute value must be a valid label value (≤ 63 chars of [-A-Za-z0-9_.])."""
    import re
    v = re.sub(r"[^-A-Za-z0-9_.]+", "_", why).strip("-_.")
    return v[:63].rstrip("-_.") or "unhealthy"


class AMDGPUPlugin(DevicePluginServer):
    def __init__(self, backend: Backend, resource_name: str = RESOURCE, plugins_dir: str = DEVICE_PLUGINS_PATH,
                 health_interval: float = 10.0, health_probe: str = "none", dev_root: str = "/dev",
                 ecc_threshold: int = 0, expose_card: bool = True, init_timeout: int = 10,
                 devices: list[dict] | None = None, health_state: str | None = None):
        super().__init__(resource_name, plugins_dir, init_timeout)
        self.backend = backend
        self.health_interval = health_interval
        self.health_probe = health_probe
        self.dev_root = dev_root
        self.ecc_threshold = ecc_threshold
        self.expose_card = expose_card
        node_gpus = backend.gpus()
        # `devices`: the subset this socket advertises (resource_groups); topology stays node-wide
        self.gpus = node_gpus if devices is None else list(devices)
        self.by_id = {device_id(g): g for g in self.gpus}
        if len(self.by_id) != len(self.gpus):
            raise ValueError("device IDs are not unique on this node (partitions without distinct ids?)")
        self.reasons: dict[str, str] = {}
        from ..smi.health import HealthMonitor
        # health_state: checkpoint of RAS baselines + sticky faults, so a restart does not
        # re-advertise a faulted GPU Healthy (smi/health.py)
        by_index = {g["index"]: device_id(g) for g in node_gpus}
        self.monitor = HealthMonitor(backend, ecc_threshold, health_state, key_of=lambda i: by_index.get(i, str(i)))
        self._task: asyncio.Task | None = None
        try:
            self.labels[TOPOLOGY_LABEL] = topology_label(node_gpus, backend.topology())
        except Exception as e:  # topology is an optimisation, never a reason not to serve
            log.warning("gpu topology unavailable: %s", e)
        if node_gpus:  # node-wide facts: identical from every socket of a mixed-strategy plugin
            self.labels["amd.com/gpu.product"] = gpu_type(node_gpus[0])
            self.labels["amd.com/gpu.count"] = str(len({parent_key(g) for g in node_gpus}))
            modes = sorted({f"{g.get('compute_partition') or 'SPX'}_{g.get('memory_partition') or 'NPS1'}" for g in node_gpus})
            self.labels["amd.com/gpu.partition-modes"] = ",".join(modes)
        self.devices = [{"ID": device_id(g), "health": HEALTHY, "Attributes": attributes(g)} for g in self.gpus]

    async def start(self):
        for g in self.gpus:             # the RAS baseline new faults are judged against
            self.monitor.snapshot(g["index"])
        if self.health_probe != "none":
            await self._probe_all()
        self._check_health(push=False)
        await super().start()
        self._task = asyncio.create_task(self._health_loop(), name="amd-gpu-health")
        return self

    async def stop(self, grace: float = 0.5):
        from ..utils import cancel_and_wait
        await cancel_and_wait([self._task])
        await super().stop(grace)

    # ------------------------------------------------------------------ health
    def _check_health(self, push=True):
        devs = []
        for d in self.devices:
            g = self.by_id[d["ID"]]
            ok, why = self.monitor.check(g["index"])
            if d["ID"] in self.reasons and self.reasons[d["ID"]].startswith("probe:"):
                ok, why = False, self.reasons[d["ID"]]
            self.reasons[d["ID"]] = "" if ok else why
            h = HEALTHY if ok else UNHEALTHY
            if h != d.get("health"):
                log.warning("gpu %s is now %s %s", d["ID"], h, why)
            attrs = {k: v for k, v in d["Attributes"].items() if k != HEALTH_REASON_ATTR}
            if not ok:     # why it was taken out of service, for kubectl describe node / the scheduler
                attrs[HEALTH_REASON_ATTR] = _attr_value(why)
            devs.append(dict(d, health=h, Attributes=attrs))
        if devs != self.devices:
            if push:
                self.update(devs)
            else:
                self.devices = devs

    def _apply_resets(self):
        """`amdkube gpu-health reset`: clear the named devices' faults (fresh RAS baseline)."""
        ids = self.monitor.pending_resets()
        if not ids:
            return
        for did, g in self.by_id.items():
            if "all" in ids or did in ids:
                log.warning("gpu %s: health reset by the operator", did)
                self.monitor.reset(g["index"])
                if self.reasons.get(did, "").startswith("probe:"):
                    self.reasons[did] = ""

    def _apply_external_faults(self):
        """Kernel-log faults from the node-problem-detector's amdgpu rules: the named PCI address
        (a partitioned GPU's parent address covers all of its partitions) or device ID."""
        for ent in self.monitor.pending_faults():
            dev = str(ent["device"]).lower()
            why = f"{ent.get('source') or 'kernel log'}: {ent['reason']}"
            hit = False
            for did, g in self.by_id.items():
                if dev in (did.lower(), str(g.get("bdf") or "").lower(), str(g.get("parent_bdf") or "").lower()):
                    log.warning("gpu %s: %s", did, why)
                    self.monitor.fault(g["index"], why)
                    hit = True
            if not hit:
                log.info("kernel-log fault on %s names no GPU of this plugin", dev)

    async def _health_loop(self):
        while True:
            await asyncio.sleep(self.health_interval)
            try:
                self._apply_resets()
                self._apply_external_faults()
                self._check_health()
            except Exception as e:  # keep serving; the next tick retries
                log.error("health check failed: %s", e)

    async def _probe_all(self):
        """Run the HBM pattern probe on each GPU (subprocess → isolated HIP context)."""
        binp = os.path.join(BIN_DIR, "hbm-probe")
        for g in self.gpus:
            did = device_id(g)
            env = {k: v for k, v in os.environ.items() if k not in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
            env["ROCR_VISIBLE_DEVICES"] = visibility_token(g)
            try:
                r = await asyncio.to_thread(subprocess.run, [binp, "--mib", "512", "--iters", "2"], env=env,
                                            capture_output=True, text=True, timeout=60)
                if r.returncode != 0:
                    self.reasons[did] = f"probe: hbm-probe failed rc={r.returncode} {r.stdout.strip()[-200:]}"
            except Exception as e:
                self.reasons[did] = f"probe: {e}"

    # ------------------------------------------------------------ allocation
    def admit_pod(self, pod_name, containers, init_containers):
        for ids in list(containers.values()) + list(init_containers.values()):
            for did in ids:
                if did not in self.by_id:
                    raise ValueError(f"unknown device {did}")
        all_ids = sorted({d for ids in containers.values() for d in ids} | {d for ids in init_containers.values() for d in ids})
        return {"amd.com/gpu-devices": ",".join(all_ids)} if all_ids else {}

    def init_container(self, name, device_ids):
        gpus = [self.by_id[d] for d in device_ids if d in self.by_id]
        if len(gpus) != len(device_ids):
            raise ValueError(f"unknown device(s) in {device_ids}")
        devs = [{"container_path": f"{self.dev_root}/kfd", "host_path": f"{self.dev_root}/kfd", "permissions": "rw"}]
        for g in gpus:
            if g.get("render_minor") is not None:
                p = f"{self.dev_root}/dri/renderD{g['render_minor']}"
                devs.append({"container_path": p, "host_path": p, "permissions": "rw"})
            if self.expose_card and g.get("card_minor") is not None:
                p = f"{self.dev_root}/dri/card{g['card_minor']}"
                # the primary node is optional for compute: hand it out only where the node has it
                # (a container host may expose render nodes alone), never a path that is absent
                if self.backend.name != "fake" and not os.path.exists(p):
                    continue
                devs.append({"container_path": p, "host_path": p, "permissions": "rw"})
        envs = {"ROCR_VISIBLE_DEVICES": ",".join(visibility_token(g) for g in gpus),
                "AMD_GPU_DEVICE_IDS": ",".join(device_ids),
                "AMD_GPU_COUNT": str(len(gpus))}
        return {"envs": envs, "devices": devs, "mounts": [],
                "annotations": {"amd.com/gpus": ",".join(device_ids), RUNTIME_ANNOTATION: "rocm"}}


def make_plugins(backend: Backend, strategy: str = "single", resource_name: str = RESOURCE, **kw) -> list[AMDGPUPlugin]:
    """One AMDGPUPlugin (socket) per advertised resource of this node (see resource_groups)."""
    groups = resource_groups(backend.gpus(), strategy, resource_name)
    if not groups:
        return [AMDGPUPlugin(backend, resource_name, devices=[], **kw)]
    return [AMDGPUPlugin(backend, name, devices=devs, **kw) for name, devs in sorted(groups.items())]
