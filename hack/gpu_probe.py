"""One-shot MI355X environment probe: amd-smi view, HIP kernels, pod-binary start latency.

Writes gpurun_out/gpu_probe.json. Used to calibrate the device plugin's visibility token and
to measure what a GPU pod's process start costs (the floor of GPU-pod startup latency).
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BIN = os.path.join(ROOT, "amdkube", "_native", "bin")
OUT = os.path.join(ROOT, "gpurun_out")
os.makedirs(OUT, exist_ok=True)
res = {}


def timed_run(cmd, env=None, timeout=120):
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout)
    return {"rc": r.returncode, "s": round(time.perf_counter() - t0, 4), "out": r.stdout[-1500:], "err": r.stderr[-800:]}


from amdkube._native import _amdsmi  # noqa: E402

_amdsmi.init()
res["amdsmi_gpus"] = _amdsmi.list_gpus()
res["amdsmi_topology_row0"] = _amdsmi.topology()[0] if _amdsmi.count() else []
res["amdsmi_links0"] = _amdsmi.link_metrics(0) if _amdsmi.count() else []
res["amdsmi_procs0"] = _amdsmi.processes(0) if _amdsmi.count() else []
_amdsmi.shutdown()
print("amdsmi ok", len(res["amdsmi_gpus"]), flush=True)

env = dict(os.environ)
res["env_visible"] = {k: v for k, v in env.items() if "VISIBLE" in k or k.startswith("HSA") or k.startswith("HIP")}
res["vadd_plain"] = [timed_run([os.path.join(BIN, "rocm-vector-add"), "--json"]) for _ in range(3)]
g0 = res["amdsmi_gpus"][0] if res["amdsmi_gpus"] else {}
for label, tok in (("hip_uuid", g0.get("hip_uuid")), ("index", "0"), ("uuid", g0.get("uuid"))):
    if tok:
        e = dict(env, ROCR_VISIBLE_DEVICES=str(tok))
        res[f"vadd_rocr_{label}"] = timed_run([os.path.join(BIN, "rocm-vector-add"), "--json"], env=e)
print("vadd done", flush=True)
res["pause"] = timed_run([os.path.join(BIN, "pause"), "--version"])
res["hbm_probe"] = timed_run([os.path.join(BIN, "hbm-probe"), "--mib", "2048", "--iters", "10"])
res["gpu_burn"] = timed_run([os.path.join(BIN, "gpu-burn"), "--ms", "500"])
res["xgmi_probe"] = timed_run([os.path.join(BIN, "xgmi-probe"), "--max-mib", "64", "--iters", "5"])
print("binaries done", flush=True)
from amdkube._native import _hipops  # noqa: E402

res["hipops"] = {"info": _hipops.device_info(0), "vadd": _hipops.vector_add(1 << 24, 0),
                 "hbm": _hipops.hbm_probe(2048, 10, 0), "burn": _hipops.mfma_burn(300.0, 0)}
json.dump(res, open(os.path.join(OUT, "gpu_probe.json"), "w"), indent=1, default=str)
print(json.dumps({k: (v if k.startswith("vadd") or k in ("hbm_probe", "gpu_burn", "hipops") else "...") for k, v in res.items()}, indent=1, default=str)[:6000])
