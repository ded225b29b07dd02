import json, os, subprocess, time, statistics as st
D = os.path.dirname(os.path.abspath(__file__))
def runs(cmd, env, n=8):
    ws, last = [], ""
    for _ in range(n):
        t = time.perf_counter(); r = subprocess.run(cmd, env=env, capture_output=True, text=True); ws.append((time.perf_counter() - t) * 1000)
        last = (r.stdout.strip().splitlines() or [r.stderr[-200:]])[-1]
    return {"wall_ms": round(st.median(ws), 1), "last": last}
base = dict(os.environ)
res = {"hsa": runs([D + "/hsa_init"], base),
       "hsa_nointr": runs([D + "/hsa_init"], dict(base, HSA_ENABLE_INTERRUPT="0")),
       "hsa_no_sdma": runs([D + "/hsa_init"], dict(base, HSA_ENABLE_SDMA="0")),
       "hip_count": runs([D + "/hip_init_phases", "1"], base),
       "hip_count_direct_dispatch0": runs([D + "/hip_init_phases", "1"], dict(base, AMD_DIRECT_DISPATCH="0")),
       "env": {k: v for k, v in base.items() if k.startswith(("HSA", "HIP", "ROC", "GPU_", "AMD", "LD_"))}}
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "hsa_exp.json"), "w"), indent=1)
