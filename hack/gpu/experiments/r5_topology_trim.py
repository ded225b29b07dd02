"""Does trimming foreign GPUs' KFD topology (devview: caches_count 0) shorten hsa_init on MI355X?

Runs kernels/hsa_vector_add (AMDKUBE_VADD_TRACE=1) in three modes, each after a 1 s idle gap
(no predecessor KFD release window: pure init cost) and back to back (the pod cadence):
  plain  — no preload (ROCr sees every GPU of the host);
  view   — the devview preload hiding the GPUs the container was not given (what pods get today);
  trim   — the same preload with the foreign GPUs' topology trimmed (the new default).
Also times a Python walk of the topology's properties files, with and without caches.
Writes one JSON document to argv[1].
"""
import glob
import json
import os
import re
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.path.join(ROOT, "amdkube", "_native", "bin", "hsa-vector-add")
LIB = os.path.join(ROOT, "amdkube", "_native", "lib", "libamdkube-devview.so")
TOPO = "/sys/devices/virtual/kfd/kfd/topology/nodes"


def own_render_node():
    for p in sorted(glob.glob("/dev/dri/renderD*")):
        try:
            os.close(os.open(p, os.O_RDWR))
            return p
        except OSError:
            continue
    return None


def run_once(env):
    t0 = time.perf_counter()
    r = subprocess.run([BIN, "-n", "50000"], env=env, capture_output=True, text=True, timeout=60)
    wall = (time.perf_counter() - t0) * 1000
    phases = {m.group(1): float(m.group(2)) for m in re.finditer(r"\[trace\] (\S+)\s+([\d.]+) ms", r.stderr)}
    return {"rc": r.returncode, "wall_ms": round(wall, 2), "phases": phases,
            "err": r.stderr[-300:] if r.returncode else ""}


REFUSED = {}


def _read(path):
    try:
        with open(path) as f:
            f.read()
    except OSError as e:
        REFUSED[path.split("/nodes/")[1].split("/")[0]] = e.strerror


def topo_walk(with_caches: bool) -> float:
    t0 = time.perf_counter()
    for node in glob.glob(TOPO + "/*"):
        _read(node + "/properties")
        if with_caches:
            for c in glob.glob(node + "/caches/*/properties"):
                _read(c)
    return (time.perf_counter() - t0) * 1000


def main(out):
    node = own_render_node()
    base = dict(os.environ, AMDKUBE_VADD_TRACE="1")
    view = dict(base, LD_PRELOAD=LIB, AMDKUBE_DEVVIEW_ROOT="/dev", AMDKUBE_DEVVIEW_ALLOW=f"/dev/kfd,{node}",
                AMDKUBE_DEVVIEW_TOPOLOGY="full")
    trim = dict(view)
    trim.pop("AMDKUBE_DEVVIEW_TOPOLOGY")
    caches = sum(len(glob.glob(n + "/caches/*")) for n in glob.glob(TOPO + "/*"))
    res = {"render_node": node, "topology_nodes": len(glob.glob(TOPO + "/*")), "cache_entries": caches,
           "walk_ms": {"with_caches": [round(topo_walk(True), 2) for _ in range(5)],
                       "nodes_only": [round(topo_walk(False), 2) for _ in range(5)]}, "modes": {}}
    res["refused_nodes"] = dict(REFUSED)
    print(json.dumps({k: res[k] for k in ("render_node", "topology_nodes", "cache_entries", "walk_ms", "refused_nodes")}),
          flush=True)
    for cadence in ("idle", "back_to_back"):
        for rnd in range(8):                       # interleave the modes so box drift hits all alike
            for mode, env in (("plain", base), ("view", view), ("trim", trim)):
                if cadence == "idle":
                    time.sleep(1.0)
                r = run_once(env)
                res["modes"].setdefault(f"{mode}/{cadence}", []).append(r)
                print(mode, cadence, rnd, r["rc"], r["wall_ms"], r["phases"].get("hsa_init"), flush=True)
    summary = {}
    for key, runs in res["modes"].items():
        ok = [r for r in runs if r["rc"] == 0]
        summary[key] = {"ok": len(ok), "of": len(runs),
                        "wall_ms_median": round(statistics.median(r["wall_ms"] for r in ok), 2) if ok else None,
                        "hsa_init_ms_median": round(statistics.median(r["phases"].get("hsa_init", 0) for r in ok), 2) if ok else None}
    res["summary"] = summary
    print(json.dumps(summary, indent=1), flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
