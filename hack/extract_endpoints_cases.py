"""Extract pkg/api/v1/endpoints/util_test.go's TestPackSubsets table into
tests/fixtures/endpoints_cases.json (replayed by tests/test_endpoints_parity.py).

    python hack/extract_endpoints_cases.py [REFERENCE_ROOT]
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from goexpr import Evaluator, eval_locals, func_body, k8s_hook, table  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = "pkg/api/v1/endpoints/util_test.go"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures", "endpoints_cases.json")


def pod_ref(uid: str) -> dict:
    """podRef(uid): an ObjectReference carrying only the UID (an empty one serializes as {})."""
    return {"uid": uid} if uid else {}


def main():
    src = open(os.path.join(REF, SRC)).read()
    ev = Evaluator({"podRef": pod_ref}, hook=k8s_hook)
    start, end = func_body(src, "TestPackSubsets")
    eval_locals(src, ev, start, end)
    cases, line = table(src, ev, "testCases", start)
    with open(OUT, "w") as f:
        json.dump({"source": SRC, "PackSubsets": {"line": line, "cases": cases}}, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}: {len(cases)} cases")


if __name__ == "__main__":
    main()
