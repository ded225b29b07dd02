"""Extract pkg/controller/cronjob/cronjob_controller_test.go's tables (TestSyncOne_RunOrNot,
TestCleanupFinishedJobs_DeleteOrNot, TestSyncOne_Status) into tests/fixtures/cronjob_cases.json
(replayed by tests/test_cronjob_parity.py).

    python hack/extract_cronjob_cases.py [REFERENCE_ROOT]
"""
from __future__ import annotations

import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goexpr import Evaluator, eval_locals, func_body, table  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = "pkg/controller/cronjob/cronjob_controller_test.go"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures", "cronjob_cases.json")


def main():
    src = open(os.path.join(REF, SRC)).read()
    # the time helpers return fixed RFC 3339 instants; read them from their bodies
    funcs = {name: (lambda v: (lambda: v))(val)
             for name, val in re.findall(r'func (\w+)\(\) time\.Time \{\s*T1, err := time\.Parse\(time\.RFC3339, "([^"]+)"\)', src)}
    funcs["int32"] = lambda x: x
    names = {"batchV1beta1.AllowConcurrent": "Allow", "batchV1beta1.ForbidConcurrent": "Forbid",
             "batchV1beta1.ReplaceConcurrent": "Replace", "NoDeadline": None}
    # package-level `var ( name type = value )` constants: the deadlines, policies and booleans
    ev = Evaluator(funcs, names)
    for name, expr in re.findall(r"^\t(\w+)\s+[\w.]+\s+=\s+(.+)$", src, re.M):
        expr = expr.strip()
        if re.fullmatch(r"[\d\s*]+", expr):          # integer products: 2 * 60 * 60
            v = 1
            for x in expr.split("*"):
                v *= int(x)
            ev.names[name] = v
            continue
        try:
            ev.names[name] = ev.eval(expr)
        except (SyntaxError, NameError):
            pass
    for name, expr in re.findall(r"^\t(\w+)\s+string\s+=\s+(\".*\")$", src, re.M):
        ev.names[name] = ev.eval(expr)
    out = {"source": SRC, "times": {k: f() for k, f in funcs.items() if k != "int32"}}
    for fn in ("TestSyncOne_RunOrNot", "TestCleanupFinishedJobs_DeleteOrNot", "TestSyncOne_Status"):
        start, end = func_body(src, fn)
        eval_locals(src, ev, start, end)
        cases, line = table(src, ev, "testCases", start)
        out[fn] = {"line": line, "cases": cases}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}: " + ", ".join(f"{k} {len(v['cases'])}" for k, v in out.items() if isinstance(v, dict) and "cases" in v))


if __name__ == "__main__":
    main()
