"""Why is a GPU process slow to start right after another one exits? (run on the gpurun box)

E1: predecessor A (kfd open only / topology / hsa_init / vector-add) then B = kmt_phases: B's open ms.
E2: B's open after a gap of g seconds following a vector-add exit.
E3: the same back-to-back chain with a resident keeper (thunk-only or HIP context) alive."""
import json, os, statistics as st, subprocess, time
D = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
os.makedirs(OUT, exist_ok=True)
V = os.path.join(D, "..", "..", "amdkube", "_native", "bin", "rocm-vector-add")
K = os.path.join(D, "kmt_phases")


def run(cmd):
    t = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
    w = (time.perf_counter() - t) * 1000
    last = (r.stdout.strip().splitlines() or [""])[-1]
    try:
        j = json.loads(last)
    except Exception:
        j = {"raw": last[-100:], "rc": r.returncode}
    j["wall"] = round(w, 1)
    return j


A = {"none": None, "kfd_open": [K, "open"], "kfd_topo": [K, "topo"], "hsa_init": [D + "/hsa_init"], "vadd": [V, "--json"]}
res = {"E1": {}, "E2": {}, "E3": {}}


def chain(reps=5, pre=None):
    xs = []
    for _ in range(reps):
        if pre:
            run(pre)
        else:
            time.sleep(1.0)
        xs.append(run([K]))
    return xs


for name, cmd in A.items():
    res["E1"][name] = chain(5, cmd)
for gap in (0.02, 0.05, 0.1, 0.15, 0.2, 0.3):
    xs = []
    for _ in range(4):
        run([V, "--json"])
        time.sleep(gap)
        xs.append(run([K]))
    res["E2"][str(gap)] = xs
for kname, kcmd in (("thunk_keeper", [K, "hold"]), ("hip_keeper", [D + "/gpu_keeper"])):
    p = subprocess.Popen(kcmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    first = p.stdout.readline()
    time.sleep(1.0)
    xs = {"kmt_after_vadd": chain(5, [V, "--json"]), "vadd_chain": [run([V, "--json"]) for _ in range(6)]}
    p.stdin.close()
    p.wait(30)
    res["E3"][kname] = dict(xs, started=first.strip())


def med(xs, k="open"):
    v = [x[k] for x in xs if k in x]
    return round(st.median(v), 1) if v else None


summ = {"E1_open_after": {k: med(v) for k, v in res["E1"].items()},
        "E2_open_after_gap": {k: med(v) for k, v in res["E2"].items()},
        "E3": {k: {"open_after_vadd": med(v["kmt_after_vadd"]), "vadd_wall": med(v["vadd_chain"], "wall")}
               for k, v in res["E3"].items()}}
res["summary"] = summ
print(json.dumps(summ))
json.dump(res, open(os.path.join(OUT, "teardown_exp.json"), "w"), indent=1)
