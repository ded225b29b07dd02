"""Extract the Job controller tables from the reference into a JSON fixture.

Source: pkg/controller/job/job_controller_test.go — TestControllerSyncJob and
TestSyncJobPastDeadline: `testCases := map[string]struct{<fields>}{"name": {<positional>}, …}`.
Field names are read from the struct type, the values by hack/goexpr.py.

  python hack/extract_job_cases.py [REFERENCE_ROOT]  ->  tests/fixtures/job_cases.json
"""
from __future__ import annotations

import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goexpr import Evaluator, block_after, line_of  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = "pkg/controller/job/job_controller_test.go"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures", "job_cases.json")


def table(src: str, test: str, ev: Evaluator) -> list[dict]:
    at = src.index(f"func {test}(")
    type_body, end = block_after(src, "testCases := map[string]struct", at)
    fields = [ln.split()[0] for ln in (re.sub(r"//[^\n]*", "", type_body[1:-1])).splitlines() if ln.strip()]
    lit, _ = block_after(src, "{", end)
    rows = ev.eval(lit)
    out = []
    for name, vals in rows.items():
        if len(vals) != len(fields):
            raise ValueError(f"{test} {name!r}: {len(vals)} values for {len(fields)} fields")
        out.append({"name": name, "line": line_of(src, src.index(f'"{name}"', at)), **dict(zip(fields, vals))})
    return out


def main():
    src = open(os.path.join(REF, SRC)).read()
    ev = Evaluator({"fmt.Errorf": lambda msg, *a: {"error": msg}},
                   {"jobConditionComplete": "Complete", "jobConditionFailed": "Failed"})
    out = {"source": SRC, "TestControllerSyncJob": table(src, "TestControllerSyncJob", ev),
           "TestSyncJobPastDeadline": table(src, "TestSyncJobPastDeadline", ev)}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT}: {len(out['TestControllerSyncJob'])} + {len(out['TestSyncJobPastDeadline'])} cases")


if __name__ == "__main__":
    main()
