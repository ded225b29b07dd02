"""Round 4: control-plane scaling rehearsal with fake devices (0.3 s pods) at N = 1, 2, 4, 8 —
the density step bench.py runs, without GPU processes, so the node path's own cost per step
shows. Writes gpurun_out/scale_rehearsal_r4.json."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = {}
for n in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8"])]:
    cmds = "".join(json.dumps(c) + "\n" for c in ({"cmd": "run", "steps": 3}, {"cmd": "run", "steps": 15}, {"cmd": "quit"}))
    r = subprocess.run([sys.executable, "-m", "amdkube.benchmark.podbench", "--gpus", str(n), "--backend", "fake", "--procs", "1",
                        "--image", "busybox", "--", "-c", "sleep 0.3"], input=cmds, cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    d = json.loads(lines[-1]) if len(lines) >= 3 else {"error": r.stderr[-800:]}
    keep = ("pods_per_s", "gpu_pods_per_s", "elapsed_s", "p50_startup_ms", "p50_node_startup_ms", "p50_schedule_ms",
            "p99_startup_all_pods_ms", "node_cpu_s", "error")
    out[f"n{n}"] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items() if k in keep}
    out[f"n{n}"]["ms_per_step"] = round(d.get("elapsed_s", 0) / 15 * 1000, 1)
    print(f"n={n}", json.dumps(out[f"n{n}"]), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "scale_rehearsal_r4.json"), "w"), indent=1)
