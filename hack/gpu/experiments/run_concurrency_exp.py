"""Does ROCr/KFD init serialise across processes? k concurrent GPU processes, wall per batch."""
import json, os, subprocess, time, statistics as st
D = os.path.dirname(os.path.abspath(__file__))
V = os.path.join(D, "..", "..", "amdkube", "_native", "bin", "rocm-vector-add")
H = os.path.join(D, "hsa_init")
res = {}
for name, cmd in (("hsa_init", [H]), ("vector_add", [V, "--json"])):
    for k in (1, 2, 4, 8):
        walls = []
        for _ in range(4):
            t = time.perf_counter()
            ps = [subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL) for _ in range(k)]
            rc = [p.wait(60) for p in ps]
            walls.append((time.perf_counter() - t) * 1000)
            assert not any(rc), rc
        res[f"{name}_x{k}"] = round(st.median(walls), 1)
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "concurrency_exp.json"), "w"), indent=1)
