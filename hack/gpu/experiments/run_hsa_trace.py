"""Timeline of hsa_init: timestamp each libhsakmt / ROCr debug line as it is written."""
import json, os, subprocess, time
D = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
for name, env in (("kmt", {"HSAKMT_DEBUG_LEVEL": "7"}), ("hip", {"AMD_LOG_LEVEL": "4"})):
    cmd = [os.path.join(D, "hsa_init")] if name == "kmt" else [os.path.join(D, "hip_init_phases"), "1"]
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, env=dict(os.environ, **env), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1)
    lines = [f"{(time.perf_counter() - t0) * 1000:8.2f} {l.rstrip()}" for l in p.stdout]
    p.wait(60)
    open(os.path.join(OUT, f"hsa_trace_{name}.txt"), "w").write("\n".join(lines) + "\n")
    print(name, len(lines), lines[-1] if lines else "")
