"""Control-plane proxy for the driver's 8-GPU SCALE run, on a 1-GPU box: the density step
at N = 1/2/4/8 *simulated* GPUs (fake amd-smi backend) with a 300 ms CPU workload standing in
for vector-add, node daemons in-process (procs=0) vs separate processes (procs=1)."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = {}
for procs in (1, 0):
    for n in (1, 2, 4, 8):
        cmds = json.dumps({"cmd": "run", "steps": 2}) + "\n" + json.dumps({"cmd": "run", "steps": 10}) + "\n" + json.dumps({"cmd": "quit"}) + "\n"
        r = subprocess.run([sys.executable, "-m", "amdkube.benchmark.podbench", "--gpus", str(n), "--backend", "fake",
                            "--procs", str(procs), "--image", "busybox", "--", "-c", "sleep 0.3"], input=cmds, cwd=ROOT,
                           capture_output=True, text=True, timeout=300)
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        d = json.loads(lines[-1]) if len(lines) >= 3 else {"error": r.stderr[-500:]}
        out[f"procs{procs}_n{n}"] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items()
                                     if k in ("pods_per_s", "gpu_pods_per_s", "elapsed_s", "p50_startup_all_pods_ms",
                                              "p99_startup_all_pods_ms", "p50_schedule_ms", "p50_node_startup_ms", "error")}
        print(f"procs={procs} n={n}", out[f"procs{procs}_n{n}"], flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "scale_proxy.json"), "w"), indent=1)
