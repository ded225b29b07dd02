"""Scale proxy, procs=1 only, N from argv; optional daemon cProfiles (AMDKUBE_CPROFILE) at the
largest N, summarised to gpurun_out/scale_prof_<comp>.txt."""
import glob, json, os, pstats, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ns = [int(x) for x in (sys.argv[1:] or ["1", "8"])]
out = {}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for i, n in enumerate(ns):
    env = dict(os.environ)
    prof = i == len(ns) - 1
    if prof:
        pdir = os.path.join(ROOT, "gpurun_out", "prof")
        os.makedirs(pdir, exist_ok=True)
        env["AMDKUBE_CPROFILE"] = os.path.join(pdir, "p")
    cmds = "".join(json.dumps(c) + "\n" for c in ({"cmd": "run", "steps": 2}, {"cmd": "run", "steps": 10}, {"cmd": "quit"}))
    r = subprocess.run([sys.executable, "-m", "amdkube.benchmark.podbench", "--gpus", str(n), "--backend", "fake",
                        "--procs", "1", "--image", "busybox", "--", "-c", "sleep 0.3"], input=cmds, cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=env)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    d = json.loads(lines[-1]) if len(lines) >= 3 else {"error": r.stderr[-500:]}
    out[f"n{n}"] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items()
                    if k in ("pods_per_s", "gpu_pods_per_s", "elapsed_s", "p50_startup_all_pods_ms", "p99_startup_all_pods_ms",
                             "p50_schedule_ms", "p50_node_startup_ms", "error")}
    print(f"n={n}", out[f"n{n}"], flush=True)
    if prof:
        for f in glob.glob(os.path.join(pdir, "p.*")):
            s = pstats.Stats(f)
            with open(f + ".txt", "w") as fh:
                s.stream = fh
                fh.write(f"total {s.total_tt:.2f}s\n")
                s.sort_stats("tottime").print_stats(25)
                s.sort_stats("cumtime").print_stats(40)
            os.unlink(f)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "scale_proxy2.json"), "w"), indent=1)
