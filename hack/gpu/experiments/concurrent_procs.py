"""How do N concurrent rocm-vector-add processes on one GPU overlap (ROCr init / KFD teardown)?
Prints one JSON line per (N, rep): wall time of the whole batch and per-process lifetimes."""
import json, subprocess, sys, time
BIN = "./amdkube/_native/bin/rocm-vector-add"
for n in (1, 2, 4, 8):
    for rep in range(3):
        t0 = time.perf_counter()
        procs = [subprocess.Popen(["timeout", "-k", "5", "60", BIN], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                 for _ in range(n)]
        ends = []
        for p in procs:
            rc = p.wait()
            ends.append((time.perf_counter() - t0) * 1e3)
            if rc != 0:
                print(json.dumps({"n": n, "rep": rep, "rc": rc}), flush=True)
                sys.exit(1)
        print(json.dumps({"n": n, "rep": rep, "wall_ms": round(max(ends), 1), "first_exit_ms": round(min(ends), 1)}), flush=True)
