import json, os, subprocess, time, statistics as st
B = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hip_init_phases")
V = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "amdkube", "_native", "bin", "rocm-vector-add")
def runs(cmd, env, n=5):
    out = []
    for _ in range(n):
        t = time.perf_counter(); r = subprocess.run(cmd, env=env, capture_output=True, text=True); w = (time.perf_counter() - t) * 1000
        out.append((w, r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-200:]))
    return {"wall_ms_median": round(st.median(w for w, _ in out), 1), "last": out[-1][1]}
base = dict(os.environ)
res = {}
res["true"] = runs(["/bin/true"], base)
for mode in (1, 2, 3, 4):
    res[f"phases_mode{mode}"] = runs([B, str(mode)], base)
variants = {"default": {}, "queues1": {"GPU_MAX_HW_QUEUES": "1"}, "no_interrupt": {"HSA_ENABLE_INTERRUPT": "0"},
            "sdma0": {"HSA_ENABLE_SDMA": "0"}, "lazy": {"HIP_ENABLE_DEFERRED_LOADING": "1"}, "eager": {"HIP_ENABLE_DEFERRED_LOADING": "0"},
            "no_scratch_reclaim": {"HSA_NO_SCRATCH_RECLAIM": "1"}, "hip_vis_unset": {"HIP_VISIBLE_DEVICES": None, "ROCR_VISIBLE_DEVICES": None}}
for name, ch in variants.items():
    e = dict(base)
    for k, v in ch.items():
        if v is None: e.pop(k, None)
        else: e[k] = v
    res["vadd_" + name] = runs([V, "--json"], e)
    res["phases_" + name] = runs([B, "4"], e)
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "init_exp.json"), "w"), indent=1)
