"""Where does a new process block when it opens /dev/kfd right after another KFD process
exited? Samples /proc/<pid>/wchan of the opener every ~100 µs (readable for our own
processes) and prints a histogram of kernel wait channels plus the open time, for
predecessors: none, open/close only, and the rocm-vector-add workload."""
import collections
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
OPEN = os.path.join(HERE, "kfd_open")
VADD = os.path.join(HERE, "..", "..", "amdkube", "_native", "bin", "rocm-vector-add")


def sample(pred):
    if pred == "kfd_open":
        subprocess.run([OPEN], capture_output=True, timeout=30)
    elif pred == "vector_add":
        subprocess.run([VADD], capture_output=True, timeout=60)
    elif pred == "idle":
        time.sleep(0.5)
    t_exit = time.monotonic() * 1e3
    p = subprocess.Popen([OPEN], stdout=subprocess.PIPE, text=True)
    hist = collections.Counter()
    path = f"/proc/{p.pid}/wchan"
    while p.poll() is None:
        try:
            with open(path) as f:
                w = f.read().strip() or "(running)"
        except OSError:
            break
        hist[w] += 1
        time.sleep(0.0001)
    out = json.loads(p.stdout.read().strip().splitlines()[-1])
    out["gap_ms"] = round(out["t_open_end"] - out["open_ms"] - t_exit, 3)
    out["wchan"] = dict(hist.most_common(6))
    return out


res = {}
for pred in ("idle", "kfd_open", "vector_add"):
    runs = [sample(pred) for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6)]
    tot = collections.Counter()
    for r in runs:
        tot.update(r["wchan"])
    res[pred] = {"open_ms": sorted(r["open_ms"] for r in runs), "gap_ms_first": runs[0]["gap_ms"],
                 "wchan_samples": dict(tot.most_common(8))}
    print(pred, json.dumps(res[pred]), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/kfd_wchan.json", "w"), indent=1)
