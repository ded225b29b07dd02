"""Summarise rocprofv3 rocpd databases (--kernel-trace) as a markdown table per kernel:
calls, total/avg/min/max duration, launch shape and register/LDS use.

  python hack/rocpd_summary.py gpurun_out/<tag>/prof_x/x_results.db [...] > profiles/<file>.md
"""
import sqlite3
import sys


def summary(path: str) -> str:
    db = sqlite3.connect(path)
    rows = db.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(grid_x), max(workgroup_x), max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    out = [f"### `{path.rsplit('/', 1)[-1]}`", "",
           "| kernel | calls | total µs | avg µs | min µs | max µs | grid | wg | VGPR | AGPR | SGPR | LDS B |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for n, c, tot, avg, mn, mx, gx, wx, v, a, s, lds in rows:
        out.append(f"| `{n}` | {c} | {tot / 1e3:.1f} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | {gx} | {wx} | "
                   f"{v} | {a} | {s} | {lds} |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print("\n".join(summary(p) for p in sys.argv[1:]))
