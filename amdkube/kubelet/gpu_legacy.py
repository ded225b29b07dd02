"""Legacy whole-GPU manager behind the `Accelerators` feature gate (alpha, off by default).

Reference: pkg/kubelet/gpu/nvidia/nvidia_gpu_manager.go, the pre-device-plugin
path for `alpha.kubernetes.io/nvidia-gpu`:
  * Start discovers the GPU device nodes and requires the shared control nodes
    (/dev/nvidiactl, /dev/nvidia-uvm);
  * Capacity reports the node-level count under the alpha resource name;
  * AllocateGPU(pod, container) hands out N whole devices from allGPUs − inUse, where
    inUse is rebuilt from the active pods' running containers (the reference inspects their
    Docker device lists), and returns the device paths plus the control nodes;
  * validation requires request == limit for the resource (validation.go:4448-4449).

The MI355X mapping: devices are the DRM render nodes /dev/dri/renderD<minor> (one per GPU
or partition from amd-smi), and the shared control node is /dev/kfd. The resource is
`alpha.kubernetes.io/amd-gpu`. Visibility is narrowed with ROCR_VISIBLE_DEVICES (GPU UUID
tokens), as the device plugin does. In-use state is rebuilt from the runtime's
container annotations (amdkube.io/legacy-gpus), so a kubelet restart never hands a busy GPU
to a second pod. The device-plugin path (F1-F20) supersedes this one and is what
`DevicePlugins` (beta, on) selects. Both can run, as in the reference.
"""
from __future__ import annotations

import os

from ..api import meta as m
from ..api.helpers import is_pod_terminal
from ..api.quantity import Quantity
from ..deviceplugin.amd import visibility_token

RESOURCE = "alpha.kubernetes.io/amd-gpu"
ANNOTATION = "amdkube.io/legacy-gpus"


class LegacyGPUError(RuntimeError):
    pass


def container_gpu_request(c: dict) -> int:
    v = ((c.get("resources") or {}).get("limits") or {}).get(RESOURCE)
    return Quantity(v).value() if v is not None else 0


class AMDGPUManager:
    def __init__(self, smi_backend=None, dev_root: str = "/dev"):
        self.smi, self.dev_root = smi_backend, dev_root
        self.gpus: dict[str, dict] = {}       # render node path -> gpu record
        self.allocated: dict[tuple[str, str], list[str]] = {}   # (pod uid, container) -> render paths

    def start(self):
        """Discover render nodes; like the reference, no shared control node → no GPUs."""
        gpus = list(self.smi.gpus()) if self.smi is not None else []
        if not gpus and os.path.isdir(os.path.join(self.dev_root, "dri")):
            gpus = [{"render_minor": int(f[len("renderD"):])} for f in sorted(os.listdir(os.path.join(self.dev_root, "dri")))
                    if f.startswith("renderD") and f[len("renderD"):].isdigit()]
        if self.smi is None and not os.path.exists(os.path.join(self.dev_root, "kfd")):
            gpus = []
        self.gpus = {f"{self.dev_root}/dri/renderD{g['render_minor']}": g for g in gpus if g.get("render_minor") is not None}
        return self

    def capacity(self) -> int:
        return len(self.gpus)

    def rebuild(self, running: list[tuple[str, str, dict]]):
        """running: (pod uid, container name, container annotations) of live containers."""
        self.allocated = {}
        for uid, cname, ann in running:
            paths = [p for p in (ann.get(ANNOTATION) or "").split(",") if p]
            if paths:
                self.allocated[(uid, cname)] = paths

    def in_use(self, active_uids: set[str]) -> set[str]:
        self.allocated = {k: v for k, v in self.allocated.items() if k[0] in active_uids}
        return {p for v in self.allocated.values() for p in v}

    def allocate(self, pod: dict, container: dict, active_pods: list[dict]) -> dict:
        """AllocateGPU: devices + env + annotation for one container (idempotent on restarts)."""
        n = container_gpu_request(container)
        if n == 0:
            return {"devices": [], "envs": {}, "annotations": {}}
        uid, cname = m.uid_of(pod), container["name"]
        have = self.allocated.get((uid, cname))
        if not have:
            active = {m.uid_of(p) for p in active_pods if not is_pod_terminal(p)} | {uid}
            free = [p for p in sorted(self.gpus) if p not in self.in_use(active)]
            if len(free) < n:
                raise LegacyGPUError(f"requested {n} {RESOURCE}, but only {len(free)} are available")
            have = free[:n]
            self.allocated[(uid, cname)] = have
        devs = [{"container_path": f"{self.dev_root}/kfd", "host_path": f"{self.dev_root}/kfd", "permissions": "rw"}]
        devs += [{"container_path": p, "host_path": p, "permissions": "rw"} for p in have]
        toks = [visibility_token(g) for g in map(self.gpus.get, have)
                if g.get("hip_uuid") or g.get("uuid") or "hip_id" in g]   # /dev/dri scans carry no identity
        envs = {"ROCR_VISIBLE_DEVICES": ",".join(toks)} if len(toks) == len(have) else {}
        return {"devices": devs, "envs": envs, "annotations": {ANNOTATION: ",".join(have)}}

    def release(self, uid: str):
        for k in [k for k in self.allocated if k[0] == uid]:
            del self.allocated[k]
