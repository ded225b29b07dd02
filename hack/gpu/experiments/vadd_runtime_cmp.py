"""HIP vs bare-HSA vector-add pod workload: per-process wall time, run back to back as consecutive
GPU pods run. A process's hsa_init waits out its predecessor's KFD release, so each variant runs
in its own block of REPS+1 consecutive runs (its own kind as predecessor; the first run of a block
is dropped). One JSON line per run, then a summary line."""
import json, statistics, subprocess, sys, time
BINS = {"hip": ["./amdkube/_native/bin/rocm-vector-add"], "hsa": ["./amdkube/_native/bin/hsa-vector-add"],
        "hsa-shutdown": ["./amdkube/_native/bin/hsa-vector-add", "--shutdown"]}
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 12
walls = {k: [] for k in BINS}
for k, b in BINS.items():
    for rep in range(REPS + 1):
        t0 = time.perf_counter()
        p = subprocess.run(["timeout", "-k", "5", "30", *b, "--json"], capture_output=True, text=True)
        ms = (time.perf_counter() - t0) * 1e3
        ok = p.returncode == 0 and "Test PASSED" in p.stdout
        print(json.dumps({"rep": rep, "runtime": k, "wall_ms": round(ms, 1), "ok": ok, "rc": p.returncode,
                          "out": p.stdout.strip().splitlines()[-2:] if p.stdout else [], "err": p.stderr[-300:]}), flush=True)
        if not ok:
            sys.exit(1)
        if rep:
            walls[k].append(ms)
print(json.dumps({"summary": {k: {"median_ms": round(statistics.median(v), 1), "min_ms": round(min(v), 1),
                                  "max_ms": round(max(v), 1)} for k, v in walls.items()}}), flush=True)
