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

import atexit
import collections
import copy
import glob
import json
import logging
import os
import threading
import time

log = logging.getLogger("amdkube.smi")
FIXTURE_DIR = os.path.join(os.path.dirname(__file__), "fixtures")
DEFAULT_FIXTURE = os.path.join(FIXTURE_DIR, "mi355x_8gpu.json")


class SMIError(RuntimeError):
    pass


def device_id(g: dict) -> str:
    """Stable device-plugin ID for a GPU (what the scheduler writes into `assigned`).

    A compute partition (CPX/QPX/DPX) of a physical GPU may report its parent's UUID, so
    partitions get a `-p<partition>` suffix whenever they are not the whole device.
    """
    u = g.get("uuid") or g.get("hip_uuid") or ""
    if u:
        base = u if u.startswith("GPU-") else "GPU-" + u
    else:
        base = "GPU-" + (g.get("bdf") or str(g.get("index"))).replace(":", "-")
    if partition_count(g) > 1 and not g.get("uuid_is_unique"):
        return f"{base}-p{int(g.get('partition_id') or 0)}"
    return base


def visibility_token(g: dict) -> str:
    """Value for ROCR_VISIBLE_DEVICES selecting exactly this GPU (or GPU partition).

    The HIP UUID is position-independent and preferred; partitions that share their parent's
    UUID are selected by their ROCr agent ordinal instead.
    """
    hu = g.get("hip_uuid") or ""
    if hu.startswith("GPU-") and len(hu) > 4 and (partition_count(g) <= 1 or g.get("uuid_is_unique")):
        return hu
    return str(g.get("hip_id", g.get("index", 0)))


COMPUTE_PARTITIONS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}   # MI355X: 8 XCDs split 1/2/4/8 ways
MEMORY_PARTITIONS = {"NPS1": 1, "NPS2": 2}                      # MI355X: HBM interleaved 1 or 2 ways


def partition_count(g: dict) -> int:
    return COMPUTE_PARTITIONS.get(str(g.get("compute_partition") or "SPX").upper(), 1)


def parent_key(g: dict) -> str:
    """Identity of the physical GPU a (possibly partitioned) device belongs to."""
    return str(g.get("parent_bdf") or g.get("bdf") or g.get("uuid") or g.get("index"))


def partition_fixture(data: dict, compute: str = "SPX", memory: str = "NPS1") -> dict:
    """Expand a whole-GPU fixture into the devices a node in `compute`/`memory` mode exposes.

    Each physical MI355X (8 XCDs × 32 CUs, 288 GiB HBM3E) becomes `parts` KFD nodes / render
    nodes / HIP devices with 256/parts CUs. Under NPS1 every partition addresses all of HBM;
    under NPSn each partition sees its 1/n memory domain. Partitions of one GPU link to
    each other on-package (type "xcp", cheaper than an xGMI hop); cross-GPU links inherit the
    parents' xGMI entries.
    """
    compute, memory = compute.upper(), memory.upper()
    if compute not in COMPUTE_PARTITIONS or memory not in MEMORY_PARTITIONS:
        raise ValueError(f"unknown partition mode {compute}/{memory}")
    parts, nps = COMPUTE_PARTITIONS[compute], MEMORY_PARTITIONS[memory]
    if parts % nps:
        raise ValueError(f"{compute} cannot be combined with {memory} (partitions must divide evenly over memory domains)")
    out = copy.deepcopy(data)
    if parts == 1 and nps == 1:
        return out
    gpus, topo = out["gpus"], out["topology"]
    new_gpus, owner = [], []
    for g in gpus:
        for pid in range(parts):
            d = dict(g)
            i = len(new_gpus)
            d.update(index=i, hip_id=i, hsa_id=i + 1,
                     compute_partition=compute, memory_partition=memory, partition_id=pid,
                     parent_index=g["index"], parent_bdf=g.get("bdf"), num_cu=int(g.get("num_cu", 256)) // parts,
                     vram_total_bytes=int(g.get("vram_total_bytes", 0)) // nps,
                     render_minor=128 + i, card_minor=None if pid else g.get("card_minor"),
                     kfd_node_id=int(g.get("kfd_node_id", 0)) * parts + pid)
            new_gpus.append(d)
            owner.append(g["index"])
    pos = {g["index"]: k for k, g in enumerate(gpus)}
    new_topo = []
    for i, pi in enumerate(owner):
        row = []
        for j, pj in enumerate(owner):
            if i == j:
                row.append({"type": "self", "hops": 0, "weight": 0, "p2p": True})
            elif pi == pj:
                row.append({"type": "xcp", "hops": 0, "weight": 5, "p2p": True})
            else:
                row.append(dict(topo[pos[pi]][pos[pj]]))
        new_topo.append(row)
    out["gpus"], out["topology"] = new_gpus, new_topo
    out["description"] = f"{out.get('description', '')} [{compute}/{memory}: {len(gpus)} GPUs x {parts} partitions]"
    return out


class Backend:
    name = "base"
    per_process = False     # processes() reports per-PID VRAM (container attribution)

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

    def ras(self, index: int) -> dict:
        """RAS state beyond the ECC totals: xgmi_error (0 none, 1 error, 2 multiple),
        bad_pages{,_retired,_pending,_unreservable}, bad_page_threshold; absent = unknown."""
        return {}

    def start_sampling(self, period_ms: float = 100.0) -> bool:
        """Begin background activity sampling for average_activity(); False = not supported
        (callers then fall back to the instantaneous sample)."""
        return False

    def average_activity(self, index: int, window_s: float = 10.0) -> dict | None:
        """Mean {gfx_activity, umc_activity, samples, span_s} over the last window_s seconds
        (gonvml AverageGPUUtilization, vendor/github.com/mindprince/gonvml/bindings.go:218-260),
        or None when nothing was sampled in the window."""
        return None

    def close(self):
        pass

    # derived ------------------------------------------------------------
    def health(self, index: int, ecc_uncorrectable_threshold: int = 0) -> tuple[bool, str]:
        """Stateless check against lifetime totals (kept for tools); the device plugin uses
        smi.health.HealthMonitor, which judges NEW faults since it started."""
        try:
            s = self.sample(index)
        except Exception as e:  # a GPU we cannot even query is not schedulable
            return False, f"smi query failed: {e}"
        if s.get("ecc_uncorrectable", 0) > ecc_uncorrectable_threshold:
            return False, f"uncorrectable ECC errors: {s['ecc_uncorrectable']}"
        return True, ""


class AmdSmiBackend(Backend):
    per_process = True

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

    def ras(self, index):
        with self._lock:
            return self.lib.ras(index)

    def link_metrics(self, index):
        with self._lock:
            return self.lib.link_metrics(index)

    def start_sampling(self, period_ms: float = 100.0) -> bool:
        """Native sampler thread (native/sampler_core.h); its ring holds >= 60 s of samples."""
        with self._lock:
            if not self.lib.sampler_state()["running"]:
                self.lib.start_sampler(period_ms, max(64, int(60_000 / period_ms)))
                atexit.register(self.lib.stop_sampler)  # joined before the library goes away
        return True

    def average_activity(self, index, window_s=10.0):
        return self.lib.average_activity(index, window_s)

    def close(self):
        self.lib.shutdown()  # stops the sampler first


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
    per_process = True

    """Fixture-driven backend; mutable so tests can inject faults (ECC errors, lost GPUs)."""
    name = "fake"

    def __init__(self, fixture: str | dict | None = None, n: int | None = None, compute_partition: str = "SPX",
                 memory_partition: str = "NPS1"):
        if isinstance(fixture, dict):
            data = fixture
        else:
            with open(fixture or DEFAULT_FIXTURE) as f:
                data = json.load(f)
        self.data = copy.deepcopy(data)
        if n is not None:  # n physical GPUs (before partitioning)
            self.data["gpus"] = self.data["gpus"][:n]
            self.data["topology"] = [row[:n] for row in self.data["topology"][:n]]
        self.data = partition_fixture(self.data, compute_partition, memory_partition)
        self.samples = {g["index"]: dict(self.data.get("sample_defaults", {})) for g in self.data["gpus"]}
        self.ras_state: dict[int, dict] = {}
        self.procs: dict[int, list] = {}
        self.sampling = False
        self.history: dict[int, collections.deque] = {i: collections.deque(maxlen=1024) for i in self.samples}

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
        gpus = self.data["gpus"]
        me = parent_key(gpus[index])
        peers = []
        for g in gpus:  # one xGMI link per peer physical GPU, whatever the partition mode
            k = parent_key(g)
            if k != me and k not in peers:
                peers.append(k)
        return [{"peer_bdf": k, "type": "xgmi", "bit_rate_gbps": 32, "max_bandwidth_gbps": 1224,
                 "read_kb": 0, "write_kb": 0} for k in peers]

    def ras(self, index):
        if index not in self.samples:
            raise SMIError(f"gpu {index} not found")
        r = self.ras_state.setdefault(index, {"xgmi_error": 0, "bad_pages": 0, "bad_pages_retired": 0,
                                              "bad_pages_pending": 0, "bad_pages_unreservable": 0,
                                              "bad_page_threshold": 512})
        return dict(r)

    # fault injection
    def inject_ecc(self, index, uncorrectable=1):
        self.samples[index]["ecc_uncorrectable"] = self.samples[index].get("ecc_uncorrectable", 0) + uncorrectable

    def inject_xgmi_error(self, index, status=1):
        self.ras(index)
        self.ras_state[index]["xgmi_error"] = status

    def inject_bad_page(self, index, pending=1, retired=0):
        r = self.ras(index)
        r = self.ras_state[index]
        r["bad_pages_pending"] += pending
        r["bad_pages_retired"] += retired
        r["bad_pages"] += pending + retired

    def set_sample(self, index, **kw):
        self.samples[index].update(kw)
        if self.sampling and ("gfx_activity" in kw or "umc_activity" in kw):
            self._record(index)

    # activity sampling: every set_sample() while sampling is one sample
    def _record(self, index, t: float | None = None):
        s = self.samples[index]
        self.history[index].append((time.monotonic() if t is None else t, float(s.get("gfx_activity") or 0),
                                    s.get("umc_activity")))

    def start_sampling(self, period_ms: float = 100.0) -> bool:
        if not self.sampling:
            self.sampling = True
            for i in self.samples:
                self._record(i)
        return True

    def average_activity(self, index, window_s=10.0):
        if index not in self.history:
            raise SMIError(f"gpu {index} not found")
        since = time.monotonic() - window_s
        pts = [p for p in self.history[index] if p[0] >= since]
        if not pts:
            return None
        out = {"gfx_activity": sum(p[1] for p in pts) / len(pts), "samples": len(pts), "span_s": pts[-1][0] - pts[0][0]}
        umc = [float(p[2]) for p in pts if p[2] is not None]
        if umc:
            out["umc_activity"] = sum(umc) / len(umc)
        return out


def has_kfd() -> bool:
    return os.path.exists("/dev/kfd")


def open_backend(kind: str = "auto", fixture: str | None = None, n: int | None = None, partition: str | None = None) -> Backend:
    """`partition` ("CPX/NPS2" style) applies to the fake backend; real GPUs report their own mode."""
    kind = kind or "auto"
    if kind == "fake":
        cp, _, mp = (partition or "SPX/NPS1").partition("/")
        return FakeBackend(fixture, n, cp or "SPX", mp or "NPS1")
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
    @property
    def per_process(self):
        return self.inner.per_process

    """Expose only the first n physical GPUs (allocatable-GPU scaling runs: 1/2/4/8); on a
    partitioned node every partition of those GPUs stays visible."""

    def __init__(self, inner: Backend, n: int):
        self.inner, self.n = inner, n
        self.name = inner.name
        parents: list[str] = []
        self.keep: list[int] = []
        for pos, g in enumerate(inner.gpus()):
            k = parent_key(g)
            if k not in parents:
                if len(parents) >= n:
                    continue
                parents.append(k)
            self.keep.append(pos)

    def gpus(self):
        all_ = self.inner.gpus()
        return [all_[i] for i in self.keep]

    def sample(self, index):
        return self.inner.sample(index)

    def topology(self):
        t = self.inner.topology()
        return [[t[i][j] for j in self.keep] for i in self.keep]

    def processes(self, index):
        return self.inner.processes(index)

    def link_metrics(self, index):
        return self.inner.link_metrics(index)

    def start_sampling(self, period_ms: float = 100.0) -> bool:
        return self.inner.start_sampling(period_ms)

    def average_activity(self, index, window_s=10.0):
        return self.inner.average_activity(index, window_s)

    def close(self):
        self.inner.close()
