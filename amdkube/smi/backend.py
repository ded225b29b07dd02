"""GPU discovery / health / topology backends for MI355X.

Three interchangeable backends return the same dict shapes:

  * AmdSmiBackend — the C++ amd-smi shim (native/amdsmi_shim.cpp → amdkube._native._amdsmi),
    the MI355X replacement for the reference's NVML cgo binding
    (vendor/github.com/mindprince/gonvml/bindings.go:35-431);
  * SysfsBackend  — KFD topology fallback (/sys/class/kfd/kfd/topology/nodes/*/properties +
    io_links) for hosts where libamd_smi cannot initialise;
  * FakeBackend   — a JSON fixture (default: 8×MI355X, 288 GiB HBM3E, gfx950, full xGMI
    mesh, two NUMA nodes) so the whole stack is testable without a GPU.

`open_backend("auto")` tries amd-smi, then sysfs, and fails loudly when neither finds a GPU
on a machine that exposes /dev/kfd (no silent fake fallback on real hardware).
"""
from __future__ import annotations

import copy
import glob
import json
import logging
import os
import threading

log = logging.getLogger("amdkube.smi")
FIXTURE_DIR = os.path.join(os.path.dirname(__file__), "fixtures")
DEFAULT_FIXTURE = os.path.join(FIXTURE_DIR, "mi355x_8gpu.json")


class SMIError(RuntimeError):
    pass


def device_id(g: dict) -> str:
    """Stable device-plugin ID for a GPU (what the scheduler writes into `assigned`)."""
    u = g.get("uuid") or g.get("hip_uuid") or ""
    if u:
        return u if u.startswith("GPU-") else "GPU-" + u
    return "GPU-" + (g.get("bdf") or str(g.get("index"))).replace(":", "-")


def visibility_token(g: dict) -> str:
    """Value for ROCR_VISIBLE_DEVICES selecting exactly this GPU."""
    hu = g.get("hip_uuid") or ""
    if hu.startswith("GPU-") and len(hu) > 4:
        return hu
    return str(g.get("hip_id", g.get("index", 0)))


class Backend:
    name = "base"

    def gpus(self) -> list[dict]:
        raise NotImplementedError

    def sample(self, index: int) -> dict:
        return {}

    def topology(self) -> list[list[dict]]:
        n = len(self.gpus())
        return [[{"type": "self" if i == j else "unknown", "hops": 0 if i == j else 1, "weight": 0 if i == j else 40}
                 for j in range(n)] for i in range(n)]

    def processes(self, index: int) -> list[dict]:
        return []

    def link_metrics(self, index: int) -> list[dict]:
        return []

    def close(self):
        pass

    # derived ------------------------------------------------------------
    def health(self, index: int, ecc_uncorrectable_threshold: int = 0) -> tuple[bool, str]:
        try:
            s = self.sample(index)
        except Exception as e:  # a GPU we cannot even query is not schedulable
            return False, f"smi query failed: {e}"
        if s.get("ecc_uncorrectable", 0) > ecc_uncorrectable_threshold:
            return False, f"uncorrectable ECC errors: {s['ecc_uncorrectable']}"
        return True, ""


class AmdSmiBackend(Backend):
    name = "amdsmi"

    def __init__(self):
        from .._native import _amdsmi  # noqa: F401  (fails loudly if the shim was not built)
        self.lib = _amdsmi
        self.lib.init()
        self._lock = threading.Lock()
        self._gpus = None

    def gpus(self):
        with self._lock:
            if self._gpus is None:
                self._gpus = self.lib.list_gpus()
            return copy.deepcopy(self._gpus)

    def sample(self, index):
        with self._lock:
            return self.lib.sample(index)

    def topology(self):
        with self._lock:
            return self.lib.topology()

    def processes(self, index):
        with self._lock:
            return self.lib.processes(index)

    def link_metrics(self, index):
        with self._lock:
            return self.lib.link_metrics(index)

    def close(self):
        self.lib.shutdown()


def _props(path: str) -> dict:
    out = {}
    try:
        with open(path) as f:
            for line in f:
                parts = line.split()
                if len(parts) == 2:
                    try:
                        out[parts[0]] = int(parts[1])
                    except ValueError:
                        out[parts[0]] = parts[1]
    except OSError:
        pass
    return out


class SysfsBackend(Backend):
    """KFD topology reader (no library needed)."""
    name = "sysfs"

    def __init__(self, root: str = "/sys/class/kfd/kfd/topology/nodes"):
        self.root = root
        self._gpus = None

    def gpus(self):
        if self._gpus is not None:
            return copy.deepcopy(self._gpus)
        out = []
        nodes = sorted(glob.glob(os.path.join(self.root, "*")), key=lambda p: int(os.path.basename(p)))
        for nd in nodes:
            p = _props(os.path.join(nd, "properties"))
            if not p.get("simd_count") or not p.get("gfx_target_version"):
                continue  # CPU node
            v = int(p["gfx_target_version"])
            gfx = f"gfx{v // 10000}{(v // 100) % 100:x}{v % 100:x}"
            loc = int(p.get("location_id", 0))
            dom = int(p.get("domain", 0))
            bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
            mem = 0
            for b in glob.glob(os.path.join(nd, "mem_banks", "*", "properties")):
                mem += int(_props(b).get("size_in_bytes", 0))
            uid = p.get("unique_id", 0)
            idx = len(out)
            out.append({"index": idx, "uuid": f"GPU-{int(uid):016x}" if uid else "", "hip_uuid": f"GPU-{int(uid):016x}" if uid else "",
                        "bdf": bdf, "gfx_target": gfx, "num_cu": int(p.get("simd_count", 0)) // int(p.get("simd_per_cu", 4) or 4),
                        "vram_total_bytes": mem, "numa_node": max(0, int(p.get("numa_node", 0)) if isinstance(p.get("numa_node"), int) else 0),
                        "render_minor": int(p.get("drm_render_minor", 128 + idx)), "kfd_node_id": int(os.path.basename(nd)),
                        "market_name": "AMD Instinct" if gfx.startswith("gfx9") else gfx, "hip_id": idx,
                        "xgmi_hive_id": int(p.get("hive_id", 0))})
        self._gpus = out
        return copy.deepcopy(out)

    def topology(self):
        gpus = self.gpus()
        by_node = {g["kfd_node_id"]: g["index"] for g in gpus}
        n = len(gpus)
        mat = [[{"type": "self" if i == j else "pcie", "hops": 0 if i == j else 2, "weight": 0 if i == j else 40}
                for j in range(n)] for i in range(n)]
        for g in gpus:
            for lk in glob.glob(os.path.join(self.root, str(g["kfd_node_id"]), "io_links", "*", "properties")):
                p = _props(lk)
                dst = p.get("node_to")
                if dst in by_node:
                    t = {11: "xgmi", 2: "pcie"}.get(int(p.get("type", 0)), "unknown")
                    mat[g["index"]][by_node[dst]] = {"type": t, "hops": 1, "weight": int(p.get("weight", 15))}
        return mat


class FakeBackend(Backend):
    """Fixture-driven backend; mutable so tests can inject faults (ECC errors, lost GPUs)."""
    name = "fake"

    def __init__(self, fixture: str | dict | None = None, n: int | None = None):
        if isinstance(fixture, dict):
            data = fixture
        else:
            with open(fixture or DEFAULT_FIXTURE) as f:
                data = json.load(f)
        self.data = copy.deepcopy(data)
        if n is not None:
            self.data["gpus"] = self.data["gpus"][:n]
            self.data["topology"] = [row[:n] for row in self.data["topology"][:n]]
        self.samples = {g["index"]: dict(self.data.get("sample_defaults", {})) for g in self.data["gpus"]}
        self.procs: dict[int, list] = {}

    def gpus(self):
        return copy.deepcopy(self.data["gpus"])

    def sample(self, index):
        if index not in self.samples:
            raise SMIError(f"gpu {index} not found")
        return dict(self.samples[index])

    def topology(self):
        return copy.deepcopy(self.data["topology"])

    def processes(self, index):
        return list(self.procs.get(index, []))

    def link_metrics(self, index):
        n = len(self.data["gpus"])
        return [{"peer_bdf": self.data["gpus"][j]["bdf"], "type": "xgmi", "bit_rate_gbps": 32, "max_bandwidth_gbps": 1224,
                 "read_kb": 0, "write_kb": 0} for j in range(n) if j != index]

    # fault injection
    def inject_ecc(self, index, uncorrectable=1):
        self.samples[index]["ecc_uncorrectable"] = self.samples[index].get("ecc_uncorrectable", 0) + uncorrectable

    def set_sample(self, index, **kw):
        self.samples[index].update(kw)


def has_kfd() -> bool:
    return os.path.exists("/dev/kfd")


def open_backend(kind: str = "auto", fixture: str | None = None, n: int | None = None) -> Backend:
    kind = kind or "auto"
    if kind == "fake":
        return FakeBackend(fixture, n)
    errs = []
    if kind in ("auto", "amdsmi"):
        try:
            b = AmdSmiBackend()
            if b.gpus():
                return _Limited(b, n) if n else b
            errs.append("amd-smi found no GPUs")
        except Exception as e:
            errs.append(f"amd-smi: {e}")
            if kind == "amdsmi":
                raise SMIError("; ".join(errs))
    if kind in ("auto", "sysfs"):
        b = SysfsBackend()
        if b.gpus():
            return _Limited(b, n) if n else b
        errs.append("KFD sysfs topology lists no GPUs")
    if kind == "auto" and not has_kfd():
        log.warning("no AMD GPU on this host (%s); using the fake 8xMI355X fixture", "; ".join(errs))
        return FakeBackend(fixture, n)
    raise SMIError("no AMD GPU backend available: " + "; ".join(errs))


class _Limited(Backend):
    """Expose only the first n GPUs (allocatable-GPU scaling runs: 1/2/4/8)."""

    def __init__(self, inner: Backend, n: int):
        self.inner, self.n = inner, n
        self.name = inner.name

    def gpus(self):
        return self.inner.gpus()[: self.n]

    def sample(self, index):
        return self.inner.sample(index)

    def topology(self):
        return [row[: self.n] for row in self.inner.topology()[: self.n]]

    def processes(self, index):
        return self.inner.processes(index)

    def link_metrics(self, index):
        return self.inner.link_metrics(index)

    def close(self):
        self.inner.close()
