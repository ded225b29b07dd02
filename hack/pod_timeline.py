"""Join AMDKUBE_POD_TRACE files (one per process) into per-stage startup latencies.

usage: python hack/pod_timeline.py <trace path prefix> [--json out.json]
Every stage is reported as milliseconds after the pod's `bench_create` stamp (p50/p90/max
over pods that reached it), in order of median, so the stage where latency accumulates stands out.
"""
import glob
import json
import statistics
import sys


def load(prefix):
    pods = {}
    for f in glob.glob(prefix + ".*"):
        for line in open(f):
            try:
                r = json.loads(line)
            except ValueError:
                continue
            pods.setdefault(r["uid"], {}).setdefault(r["stage"], r["t"])
    return pods


def summarize(pods):
    rel = {}
    for st in pods.values():
        t0 = st.get("bench_create")
        if t0 is None:
            continue
        for k, t in st.items():
            rel.setdefault(k, []).append((t - t0) * 1000)
    out = []
    for k, v in rel.items():
        v.sort()
        out.append({"stage": k, "n": len(v), "p50_ms": round(statistics.median(v), 2),
                    "p90_ms": round(v[int(0.9 * (len(v) - 1))], 2), "max_ms": round(v[-1], 2)})
    return sorted(out, key=lambda r: r["p50_ms"])


if __name__ == "__main__":
    rows = summarize(load(sys.argv[1]))
    for r in rows:
        print(f"{r['stage']:24s} n={r['n']:4d}  p50 {r['p50_ms']:8.2f}  p90 {r['p90_ms']:8.2f}  max {r['max_ms']:8.2f}")
    if "--json" in sys.argv:
        json.dump(rows, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
