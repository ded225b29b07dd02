"""Where do a GPU pod's ~200 ms of ROCr init go, and is it stable? (run on the gpurun box)

A/B-interleaves plain vs HSAKMT_DEBUG_LEVEL=7 hsa_init, times the thunk phases (KFD open,
topology snapshot), idle-gap sensitivity, and sysfs topology size."""
import glob, json, os, statistics as st, subprocess, time
D = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
os.makedirs(OUT, exist_ok=True)
def one(cmd, env=None):
    t = time.perf_counter(); r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=60)
    w = (time.perf_counter() - t) * 1000
    last = (r.stdout.strip().splitlines() or [""])[-1]
    try: j = json.loads(last)
    except Exception: j = {"raw": last[-200:], "rc": r.returncode}
    j["wall"] = round(w, 1); return j
res = {"kmt": [], "hsa": [], "hsa_dbg": [], "gap": {}, "vadd": []}
base = dict(os.environ)
for i in range(8):
    res["kmt"].append(one([D + "/kmt_phases"]))
    res["hsa"].append(one([D + "/hsa_init"]))
    res["hsa_dbg"].append(one([D + "/hsa_init"], dict(base, HSAKMT_DEBUG_LEVEL="7")))
for gap in (0.0, 0.5, 2.0, 5.0):
    xs = []
    for _ in range(3):
        time.sleep(gap); xs.append(one([D + "/hsa_init"]))
    res["gap"][str(gap)] = xs
V = os.path.join(D, "..", "..", "amdkube", "_native", "bin", "rocm-vector-add")
for _ in range(5):
    res["vadd"].append(one([V, "--json"]))
t = time.perf_counter(); n = 0
for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/**/properties", recursive=True):
    try: open(p).read(); n += 1
    except Exception: pass
res["sysfs"] = {"property_files": n, "read_all_ms": round((time.perf_counter() - t) * 1000, 1),
                "nodes": len(glob.glob("/sys/class/kfd/kfd/topology/nodes/*")),
                "caches": len(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/caches/*"))}
pw = {}
for p in glob.glob("/sys/class/drm/card*/device/power/runtime_status") + glob.glob("/sys/module/amdgpu/parameters/runpm"):
    try: pw[p] = open(p).read().strip()
    except Exception as e: pw[p] = repr(e)
res["power"] = pw
def med(xs, k):
    v = [x[k] for x in xs if k in x]; return round(st.median(v), 2) if v else None
res["summary"] = {"kmt_open": med(res["kmt"], "open"), "kmt_topology": med(res["kmt"], "topology"), "kmt_wall": med(res["kmt"], "wall"),
                  "hsa_init": med(res["hsa"], "init"), "hsa_wall": med(res["hsa"], "wall"),
                  "hsa_dbg_init": med(res["hsa_dbg"], "init"), "hsa_dbg_wall": med(res["hsa_dbg"], "wall"),
                  "gap": {g: med(x, "init") for g, x in res["gap"].items()}, "vadd_wall": med(res["vadd"], "wall")}
print(json.dumps(res["summary"]))
json.dump(res, open(os.path.join(OUT, "init_var.json"), "w"), indent=1)
