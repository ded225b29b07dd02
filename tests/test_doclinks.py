"""cmd/linkcheck for this repository's documents: every relative markdown link and every
backticked repository path (amdkube/…, native/…, kernels/…, tests/…, hack/…, deploy/…,
profiles/…, docs/…) in README.md and docs/*.md names a file or directory that exists."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOPS = ("amdkube/", "native/", "kernels/", "tests/", "hack/", "deploy/", "profiles/", "docs/")
LINK = re.compile(r"\]\(([^)#\s]+)\)")
TICK = re.compile(r"`([^`\s]+)`")


def _exists(path: str) -> bool:
    path = path.split("::")[0].rstrip(".,;:")
    if any(ch in path for ch in "*<>{}$"):
        return glob.glob(os.path.join(ROOT, re.sub(r"<[^>]*>|\{[^}]*\}", "*", path))) != []
    return os.path.exists(os.path.join(ROOT, path))


def test_document_paths_exist():
    bad = []
    for doc in ["README.md", *sorted(glob.glob(os.path.join(ROOT, "docs", "*.md")))]:
        text = open(os.path.join(ROOT, doc)).read()
        rel = os.path.relpath(os.path.join(ROOT, doc), ROOT)
        for target in LINK.findall(text):
            if "://" in target:
                continue
            p = os.path.normpath(os.path.join(os.path.dirname(rel), target))
            if not os.path.exists(os.path.join(ROOT, p)):
                bad.append(f"{rel}: link {target}")
        for target in TICK.findall(text):
            if target.startswith(TOPS) and "/" in target[:-1] and not _exists(target):
                bad.append(f"{rel}: path {target}")
    assert not bad, "\n".join(bad)
