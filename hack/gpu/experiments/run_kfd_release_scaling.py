"""Is the KFD process-release path host-serialised? K processes open+close /dev/kfd and exit
together; then (a) one opener, (b) K openers at once measure their open() wait. With a
serialised release the single opener's wait grows ~K× (the N-GPU density step's bound)."""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
OPEN = os.path.join(HERE, "kfd_open")
VADD = os.path.join(HERE, "..", "..", "amdkube", "_native", "bin", "rocm-vector-add")


def burst(k, prog):
    ps = [subprocess.Popen([prog], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL) for _ in range(k)]
    for p in ps:
        p.wait(60)


def openers(k):
    ps = [subprocess.Popen([OPEN], stdout=subprocess.PIPE, text=True) for _ in range(k)]
    return sorted(json.loads(p.communicate(timeout=60)[0].strip().splitlines()[-1])["open_ms"] for p in ps)


res = {}
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for prog_name, prog in (("kfd_open", OPEN), ("vector_add", VADD)):
    for k in (1, 2, 4, 8):
        one, many = [], []
        for _ in range(reps):
            time.sleep(0.4)
            burst(k, prog)
            one += openers(1)
            time.sleep(0.4)
            burst(k, prog)
            many.append(openers(k))
        res[f"{prog_name}_k{k}"] = {"single_opener_ms": sorted(round(x, 1) for x in one),
                                    "k_openers_max_ms": sorted(round(max(x), 1) for x in many),
                                    "k_openers_median_ms": sorted(round(x[len(x) // 2], 1) for x in many)}
        print(prog_name, k, json.dumps(res[f"{prog_name}_k{k}"]), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/kfd_release_scaling.json", "w"), indent=1)
