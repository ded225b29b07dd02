import json, os, subprocess, time, statistics as st
D = os.path.dirname(os.path.abspath(__file__))
V = os.path.join(D, "..", "..", "amdkube", "_native", "bin", "rocm-vector-add")
def runs(cmd, env, n=10):
    ws = []
    for _ in range(n):
        t = time.perf_counter(); subprocess.run(cmd, env=env, capture_output=True); ws.append((time.perf_counter() - t) * 1000)
    return round(st.median(ws), 1)
base = dict(os.environ)
q1 = dict(base, GPU_MAX_HW_QUEUES="1")
res = {"true": runs(["/bin/true"], base), "load_only": runs([D + "/hip_init_phases", "0"], base),
       "init_only": runs([D + "/hip_init_phases", "1"], base),
       "normal_exit": runs([D + "/exit_variants", "0"], base), "quick_exit": runs([D + "/exit_variants", "1"], base),
       "free_quick_exit": runs([D + "/exit_variants", "2"], base),
       "normal_exit_q1": runs([D + "/exit_variants", "0"], q1), "quick_exit_q1": runs([D + "/exit_variants", "1"], q1),
       "quick_exit_q1_nointr": runs([D + "/exit_variants", "1"], dict(q1, HSA_ENABLE_INTERRUPT="0")),
       "vadd": runs([V, "--json"], base), "vadd_q1": runs([V, "--json"], q1)}
r = subprocess.run([D + "/exit_variants", "1"], env=dict(base, LD_DEBUG="statistics"), capture_output=True, text=True)
res["ld_debug"] = [l.strip() for l in r.stderr.splitlines() if "total startup time" in l or "relocation processing" in l or "number of relocations" in l][:6]
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "exit_exp.json"), "w"), indent=1)
