"""Extract the reference's strategic-merge-patch table tests into a JSON fixture
(tests/fixtures/strategicpatch_cases.json), so tests/test_strategicpatch.py can run them against
amdkube/api/strategicpatch.py without the reference tree.

Source: staging/src/k8s.io/apimachinery/pkg/util/strategicpatch/patch_test.go —
customStrategicMergePatchTestCaseData / customStrategicMergePatchRawTestCases (patch
application only, TestCustomStrategicMergePatch) and createStrategicMergePatchTestCaseData /
strategicMergePatchRawTestCases (two-way + three-way creation and application,
TestStrategicMergePatch). The YAML documents are kept as parsed JSON values; "sorted" marks the
struct-form cases, whose inputs and expectations the reference sorts by merge key first.

  python hack/extract_smp_cases.py /root/reference
"""
import json
import os
import re
import sys

import yaml

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                   "strategicpatch_cases.json")
SRC = "staging/src/k8s.io/apimachinery/pkg/util/strategicpatch/patch_test.go"
FIELDS = {"Original": "original", "Modified": "modified", "Current": "current", "TwoWay": "twoWay",
          "ThreeWay": "threeWay", "Result": "result", "TwoWayResult": "twoWayResult"}


def yaml_var(text: str, name: str) -> list[dict]:
    m = re.search(rf"var {name} = \[\]byte\(`(.*?)`\)", text, re.S)
    return yaml.safe_load(m.group(1))["testCases"]


def raw_var(text: str, name: str) -> list[dict]:
    start = text.index(f"var {name} = ")
    end = text.index("\n}\n", start)
    block = text[start:end]
    out = []
    for chunk in re.split(r"\n\t\{\n\t\tDescription: ", block)[1:]:
        desc = json.loads(chunk[:chunk.index("\n")].rstrip(","))
        case = {"description": desc}
        for fname, body in re.findall(r"(\w+):\s*\[\]byte\(`(.*?)`\)", chunk, re.S):
            if fname in FIELDS:
                case[FIELDS[fname]] = yaml.safe_load(body)
        e = re.search(r'ExpectedError:\s*"([^"]*)"', chunk)
        if e:
            case["expectedError"] = e.group(1)
        out.append(case)
    return out


def main(ref: str):
    text = open(os.path.join(ref, SRC)).read()
    data = {"source": SRC,
            "apply": [dict(c, sorted=True) for c in yaml_var(text, "customStrategicMergePatchTestCaseData")]
            + raw_var(text, "customStrategicMergePatchRawTestCases"),
            "create": [dict(c, sorted=True) for c in yaml_var(text, "createStrategicMergePatchTestCaseData")]
            + raw_var(text, "strategicMergePatchRawTestCases")}
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(f"{len(data['apply'])} apply + {len(data['create'])} create cases -> {OUT}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
