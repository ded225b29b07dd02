import json, subprocess, sys, time, os
n=int(sys.argv[1]); procs=(sys.argv[2:] or ["1"])[0]
cmds = json.dumps({"cmd": "run", "steps": 2}) + "\n" + json.dumps({"cmd": "run", "steps": 10}) + "\n" + json.dumps({"cmd": "quit"}) + "\n"
t=time.time()
r = subprocess.run([sys.executable, "-m", "amdkube.benchmark.podbench", "--gpus", str(n), "--backend", "fake",
                    "--procs", procs, "--image", "busybox", "--", "-c", "sleep 0.3"], input=cmds, cwd=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                   capture_output=True, text=True, timeout=300)
lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
d=json.loads(lines[-1]) if lines else {"err": r.stderr[-2000:]}
print({k: d.get(k) for k in ("pods_per_s","gpu_pods_per_s","elapsed_s","p50_startup_all_pods_ms","p99_startup_all_pods_ms","p50_schedule_ms","p50_node_startup_ms","ms_per_step","err")})
