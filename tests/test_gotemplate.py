"""`kubectl -o go-template`: the text/template subset kubectl templates use, with Go's output
(pkg/printers/template.go over text/template; the cases mirror template_test.go-style usage and
the kubectl docs' examples). Parity unpinned beyond these: the reference has no table of its own
for text/template, whose tests live in Go's standard library."""
import pytest

from amdkube.kubectl.gotemplate import TemplateError, render

POD_LIST = {"kind": "List", "items": [
    {"metadata": {"name": "a", "labels": {"app": "web", "tier": "fe"}}, "status": {"phase": "Running"},
     "spec": {"containers": [{"name": "c1", "image": "nginx"}, {"name": "c2", "image": "redis"}],
              "extendedResources": [{"name": "gpus", "assigned": ["GPU-0", "GPU-1"]}]}},
    {"metadata": {"name": "b", "labels": {"app": "db"}}, "status": {"phase": "Pending"}, "spec": {"containers": []}},
]}

CASES = [
    ("{{range .items}}{{.metadata.name}}{{\"\\n\"}}{{end}}", "a\nb\n"),
    ("{{range .items}}{{index .metadata.labels \"app\"}} {{end}}", "web db "),
    ("{{range .items}}{{if eq .status.phase \"Running\"}}{{.metadata.name}}{{end}}{{end}}", "a"),
    ("{{range .items}}{{.metadata.name}}:{{len .spec.containers}};{{end}}", "a:2;b:0;"),
    ("{{range $i, $p := .items}}{{$i}}={{$p.metadata.name}} {{end}}", "0=a 1=b "),
    ("{{range $k, $v := (index .items 0).metadata.labels}}{{$k}}={{$v}},{{end}}", "app=web,tier=fe,"),
    ("{{with index .items 0}}{{.metadata.name}}{{end}}", "a"),
    ("{{(index .items 1).metadata.name}}", "b"),
    ("{{range .items}}{{.missing}}|{{end}}", "<no value>|<no value>|"),
    ("{{printf \"%s has %d\" (index .items 0).metadata.name 2}}", "a has 2"),
    ("{{range .items}}{{if .spec.extendedResources}}{{range .spec.extendedResources}}{{.assigned}}{{end}}{{else}}none{{end}} {{end}}",
     "[GPU-0 GPU-1] none "),
    ("{{range .items}}{{if eq .status.phase \"Pending\"}}P{{else if eq .status.phase \"Running\"}}R{{else}}?{{end}}{{end}}", "RP"),
    ("{{- range .items }}\n  {{ .metadata.name -}}\n{{ end }}", "\n  a\n  b"),
    ("{{- range .items -}}\n  {{ .metadata.name -}}\n{{ end }}", "ab"),
    ("{{/* a comment */}}x{{$n := len .items}}{{$n}}", "x2"),
    ("{{range .items}}{{if exists . \"spec\" \"extendedResources\"}}{{.metadata.name}}{{end}}{{end}}", "a"),
    ("{{(index .items 0).metadata.labels}}", "map[app:web tier:fe]"),
    ("{{.kind | printf \"%q\"}}", "\"List\""),
    ("{{range .nothing}}x{{else}}empty{{end}}", "empty"),
    ("{{if and .kind (not .missing)}}ok{{end}}", "ok"),
    ("{{define \"n\"}}[{{.metadata.name}}]{{end}}{{range .items}}{{template \"n\" .}}{{end}}", "[a][b]"),
]


@pytest.mark.parametrize("tpl,expected", CASES)
def test_templates(tpl, expected):
    assert render(tpl, POD_LIST) == expected


def test_missing_key_is_an_error_when_not_allowed():
    with pytest.raises(TemplateError):
        render("{{.missing}}", POD_LIST, allow_missing_keys=False)


@pytest.mark.parametrize("tpl", ["{{if .kind}}x", "{{end}}", "{{nosuchfunc .kind}}", "{{.kind .kind}}"])
def test_bad_templates_fail(tpl):
    with pytest.raises(TemplateError):
        render(tpl, POD_LIST)
