"""cmd/clicheck (pkg/kubectl/cmd/util/sanity/cmd_sanity.go) on this build's CLIs, plus the
documentation generators (cmd/gendocs, genkubedocs, genman, genyaml)."""
import argparse
import contextlib
import io
import re

import yaml

from amdkube.cmd import gendocs
from amdkube.cmd.components import COMPONENTS
from amdkube.kubectl import help as kh
from amdkube.kubectl.main import main as kubectl, parser

FLAG_RE = re.compile(r"^[a-z0-9]+(-[a-z0-9]+)*$")   # cmd_sanity.go CheckFlags


def _subparsers():
    root = parser()
    return root, next(a for a in root._actions if isinstance(a, argparse._SubParsersAction)).choices


def test_every_kubectl_command_has_normalized_help():
    _, subs = _subparsers()
    errors = []
    for name in subs:
        short, long_, _ = kh.HELP.get(name, ("", "", ""))
        if not short:
            errors.append(f"{name}: no short description")
        if short.endswith("."):
            errors.append(f"{name}: short description ends with a period")
        if kh.long_desc(name) != kh.long_desc(name).strip(" \t\n") or not long_:
            errors.append(f"{name}: long description missing or not normalized")     # CheckLongDesc
        for line in kh.examples(name).splitlines():                                     # CheckExamples
            if not line.startswith(kh.INDENT):
                errors.append(f"{name}: example line not indented: {line!r}")
            if line.strip().startswith("//"):
                errors.append(f"{name}: examples use // comments")
        if "kubectl " + name not in kh.examples(name):
            errors.append(f"{name}: no example invocation")
    assert not errors, errors
    assert set(kh.HELP) == set(subs), set(kh.HELP) ^ set(subs)


def test_flag_names_follow_the_convention():
    root, subs = _subparsers()
    bad = []
    parsers = [("kubectl", root)] + [(f"kubectl {n}", p) for n, p in subs.items()]
    for name in sorted(set(COMPONENTS) - set(gendocs.GENERATORS)):
        p = gendocs.capture_parser(COMPONENTS[name])
        assert p is not None, name
        parsers.append((name, p))
    for where, p in parsers:
        for act in p._actions:
            for opt in act.option_strings:
                if opt.startswith("--") and not FLAG_RE.match(opt[2:]):
                    bad.append(f"{where}: {opt}")
    assert not bad, bad


def test_kubectl_help_and_overview():
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        assert kubectl([]) == 0
        assert kubectl(["help", "get"]) == 0
        assert kubectl(["help"]) == 0
    text = out.getvalue()
    assert "Basic Commands (Beginner):" in text and "Troubleshooting and Debugging Commands:" in text
    assert "kubectl get pods" in text and "Examples:" in text
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        try:
            kubectl(["top", "--help"])
        except SystemExit as e:
            assert e.code == 0
    assert "GPU usage per device" in out.getvalue()


def test_doc_generators_cover_every_command(tmp_path):
    _, subs = _subparsers()
    for fmt, fn in (("md", gendocs.gendocs), ("man", gendocs.genman), ("yaml", gendocs.genyaml)):
        d = tmp_path / fmt
        assert fn(["--out", str(d)]) == 0
        names = {p.name for p in d.iterdir()}
        ext = {"md": ".md", "man": ".1", "yaml": ".yaml"}[fmt]
        sep = "-" if fmt == "man" else "_"
        for c in subs:
            assert f"kubectl{sep}{c}{ext}" in names, (fmt, c)
        for comp in ("kubelet", "kube-scheduler", "kube-apiserver", "amd-device-plugin", "kubeadm"):
            assert f"{comp}{ext}" in names, (fmt, comp)
    doc = yaml.safe_load((tmp_path / "yaml" / "kubectl_get.yaml").read_text())
    assert doc["name"] == "kubectl get" and doc["synopsis"] == kh.short("get")
    assert any(o["name"] == "output" and o.get("shorthand") == "o" for o in doc["options"])
    assert any(o["name"] == "server" for o in doc["inherited_options"])
    kubelet_md = (tmp_path / "md" / "kubelet.md").read_text()
    assert "--container-runtime-endpoint" in kubelet_md and "### Options" in kubelet_md
    man = (tmp_path / "man" / "kubectl-get.1").read_text()
    assert man.startswith('.TH "KUBECTL-GET" "1"') and ".SH EXAMPLE" in man
