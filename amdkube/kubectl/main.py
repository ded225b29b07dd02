"""kubectl for amdkube.

Reference command set: pkg/kubectl/cmd/cmd.go:216 (create/apply/get/describe/delete/logs/
exec/label/annotate/cordon/uncordon/drain/scale/patch/run/top/version/api-resources/
cluster-info), create.go:64,146; rollout/expose/autoscale/taint/set/replace/edit/config/
auth/certificate/port-forward/proxy/cp/explain and the create generators live in extra.py. Output: tables (GPU columns added, SURVEY §7.6
#17), -o json|yaml|name|wide|jsonpath={...}. Server from --server, $AMDKUBE_SERVER or
~/.amdkube/config ({"server": ..., "token": ...}).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import re
import sys
import time

from ..api import meta as m
from ..runtime import spdy
from ..api.scheme import SCHEME, dump_yaml, load_manifests
from ..client import Client
from . import printers

CONFIG = os.path.expanduser("~/.amdkube/config")


def _client(a) -> Client:
    kc = getattr(a, "kubeconfig", None) or os.environ.get("KUBECONFIG")
    if kc and not a.server:
        return Client.from_kubeconfig(kc, getattr(a, "context", None), user_agent="kubectl/amdkube")
    server, token = a.server, a.token
    if not server:
        server = os.environ.get("AMDKUBE_SERVER")
    if (not server or not token) and os.path.exists(CONFIG):
        cfg = json.load(open(CONFIG))
        server = server or cfg.get("server")
        token = token or cfg.get("token")
    return Client(server or "http://127.0.0.1:8080", token=token, user_agent="kubectl/amdkube")


def _jsonpath(obj, expr: str, allow_missing: bool = True):
    from .jsonpath import JSONPath
    return JSONPath("jsonpath", allow_missing).parse(expr).execute(obj)


def _read_template(a, value: str, kind: str) -> str:
    """-o <kind>=<template> or <kind>-file=<path>, or --template."""
    if value:
        return value
    tpl = getattr(a, "template", None)
    if tpl:
        return tpl
    raise SystemExit(f"error: template format specified but no template given")


def _emit(objs, a, kind=None, single=False, out=None, with_headers=True):
    """The printer -o selects (pkg/kubectl/cmd/util/printing.go PrinterForOptions): json, yaml,
    name, wide, jsonpath[-file], go-template[-file], custom-columns[-file], or the table;
    --sort-by orders a list first (SortingPrinter)."""
    from . import gotemplate
    from .jsonpath import JSONPathError
    out = out or sys.stdout
    o = a.output or ""
    allow_missing = getattr(a, "allow_missing_template_keys", True)
    sort_by = getattr(a, "sort_by", None)
    if sort_by and not single and len(objs) > 1:
        try:
            objs = printers.sort_objects(objs, sort_by)
        except (ValueError, JSONPathError) as e:
            raise SystemExit(f"error: {e}")
    data = objs[0] if single and len(objs) == 1 else {"apiVersion": "v1", "kind": "List", "items": objs,
                                                      "metadata": {"resourceVersion": "", "selfLink": ""}}
    if o == "json":
        print(json.dumps(data, indent=4), file=out)
    elif o == "yaml":
        print(dump_yaml(data), file=out, end="")
    elif o == "name":
        for x in objs:
            print(f"{(x.get('kind') or kind or '').lower()}/{m.name_of(x)}", file=out)
    elif o.startswith(("jsonpath=", "jsonpath-file=")) or o == "jsonpath":
        expr = o.split("=", 1)[1] if "=" in o else ""
        if o.startswith("jsonpath-file="):
            expr = open(expr).read()
        expr = _read_template(a, expr, "jsonpath")
        try:
            print(_jsonpath(data, expr, allow_missing), file=out, end="")
        except JSONPathError as e:
            raise SystemExit(f"error: error executing jsonpath {expr!r}: {e}")
    elif o.startswith(("go-template=", "go-template-file=", "template=", "templatefile=")) or o in ("go-template", "template"):
        tpl = o.split("=", 1)[1] if "=" in o else ""
        if o.startswith(("go-template-file=", "templatefile=")):
            tpl = open(tpl).read()
        tpl = _read_template(a, tpl, "go-template")
        try:
            print(gotemplate.render(tpl, data, allow_missing), file=out, end="")
        except gotemplate.TemplateError as e:
            raise SystemExit(f"error: error executing template {tpl!r}: {e}")
    elif o.startswith(("custom-columns=", "custom-columns-file=")):
        spec = o.split("=", 1)[1]
        try:
            if o.startswith("custom-columns-file="):
                ccp = printers.CustomColumnsPrinter.from_template(open(spec).read())
            else:
                ccp = printers.CustomColumnsPrinter.from_spec(spec, getattr(a, "no_headers", False))
        except (ValueError, JSONPathError) as e:
            raise SystemExit(f"error: {e}")
        print(ccp.print(objs), file=out, end="")
    elif o in ("", "wide"):
        k = kind or (objs[0].get("kind") if objs else "")
        if k == "Pod" and not single and not getattr(a, "show_all", True):
            objs = [p for p in objs if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")]
        if not objs:
            print("No resources found.", file=sys.stderr)
            return
        label_cols = []
        for spec in getattr(a, "label_columns", None) or []:
            label_cols += [x.strip() for x in spec.split(",") if x.strip()]
        txt = printers.print_table(objs, k, wide=o == "wide", with_namespace=getattr(a, "all_namespaces", False),
                                   show_labels=getattr(a, "show_labels", False), label_columns=label_cols,
                                   no_headers=getattr(a, "no_headers", False) or not with_headers,
                                   with_kind=getattr(a, "show_kind", False))
        print(txt, file=out)
    else:
        raise SystemExit(f"error: unable to match a printer suitable for the output format \"{o}\", allowed formats "
                         f"are: custom-columns,custom-columns-file,go-template,go-template-file,json,jsonpath,"
                         f"jsonpath-file,name,template,templatefile,wide,yaml")


MANIFEST_EXTS = (".yaml", ".yml", ".json")


def manifest_paths(p: str, recursive: bool = False) -> list[str]:
    """A directory's manifests (resource.FileVisitorForSTDIN / ExpandPathsToFileVisitors: only
    .json/.yaml/.yml, sub-directories with --recursive), or the file itself."""
    if not os.path.isdir(p):
        return [p]
    out = []
    for f in sorted(os.listdir(p)):
        fp = os.path.join(p, f)
        if os.path.isdir(fp):
            if recursive:
                out += manifest_paths(fp, True)
        elif f.endswith(MANIFEST_EXTS):
            out.append(fp)
    return out


def _read_files(paths, recursive: bool = False) -> list[dict]:
    docs = []
    for p in paths:
        if p == "-":
            docs += load_manifests(sys.stdin.read())
            continue
        for fp in manifest_paths(p, recursive):
            with open(fp) as f:
                docs += load_manifests(f.read())
    return docs


def standard_error_message(e: m.StatusError) -> str:
    """cmdutil checkErr (helpers.go:124-170) for API errors: an Invalid error lists its causes
    ("The Pod "x" is invalid: ..." — one per line after "* " when there are several), any other
    is `Error from server (<Reason>): <message>`."""
    d = e.details or {}
    if e.code == 422 and e.reason == "Invalid" and d.get("kind"):
        head = f'The {d.get("kind")} "{d.get("name", "")}" is invalid'
        causes = [(c.get("field") + ": " if c.get("field") else "") + c.get("message", "") for c in d.get("causes") or []]
        if not causes:
            return head
        if len(causes) == 1:
            return f"{head}: {causes[0]}"
        return f"{head}: \n" + "\n".join(f"* {c}" for c in causes)
    return f"Error from server ({e.reason}): {e.message}"


def parse_duration_flag(s: str) -> float:
    """A Go duration flag (`5m`, `30s`, `1h30m`) in seconds; a bare number is seconds."""
    try:
        return float(s)
    except ValueError:
        from ..api.protobuf import parse_duration
        return parse_duration(s) / 1e9


def timeout_of(a, default: float = 30.0) -> float:
    """--timeout when given, else the command's own default."""
    t = getattr(a, "timeout", None)
    return default if t is None else float(t)


def _ns(a, ri=None):
    if ri is not None and not ri.namespaced:
        return ""
    return "" if getattr(a, "all_namespaces", False) else (a.namespace or "default")


def _split_targets(args):
    """['pods', 'a', 'b'] | ['pod/a', 'node/b'] -> [(resource, name|None)]"""
    out = []
    if not args:
        return out
    if all("/" in x for x in args):
        for x in args:
            r, n = x.split("/", 1)
            out.append((r, n))
        return out
    res = args[0].split(",")
    names = args[1:]
    for r in res:
        if names:
            out += [(r, n) for n in names]
        else:
            out.append((r, None))
    return out


async def cmd_get(c, a):
    from .get import cmd_get as get
    return await get(c, a)


async def cmd_describe(c, a):
    from .describe import describe, gather_extra
    for r, name in _split_targets(a.args):
        ri = SCHEME.resolve(r)
        if ri is None:
            raise SystemExit(f'error: the server doesn\'t have a resource type "{r}"')
        ns = _ns(a, ri)
        res = ri.plural if not ri.group else f"{ri.plural}.{ri.group}"
        objs = [await c.get(res, name, ns)] if name else (await c.list(res, ns, a.selector))[0]
        for o in objs:
            o.setdefault("kind", ri.kind)
            o.setdefault("apiVersion", ri.api_version)
            fs = f"involvedObject.name={m.name_of(o)},involvedObject.kind={ri.kind}"
            try:
                evs, _ = await c.list("events", m.namespace_of(o) or ("default" if ri.namespaced else ""), field_selector=fs)
            except m.StatusError:
                evs = []
            evs = [e for e in evs if (e.get("involvedObject") or {}).get("uid") in (None, "", m.uid_of(o))]
            print(describe(o, evs, **(await gather_extra(c, o))))
            print()


async def _create_or_apply(c, a, apply=False):
    for doc in _read_files(a.filename):
        ri = SCHEME.for_object(doc)
        if ri is None:
            raise SystemExit(f"error: unknown kind {doc.get('apiVersion')}/{doc.get('kind')}")
        ns = (m.namespace_of(doc) or a.namespace or "default") if ri.namespaced else ""
        if ri.namespaced:
            doc.setdefault("metadata", {})["namespace"] = ns
        name = m.name_of(doc)
        res = ri.plural if not ri.group else f"{ri.plural}.{ri.group}"
        if apply and name:
            cur = await c.get_or_none(res, name, ns)
            if cur is not None:
                patch = {k: v for k, v in doc.items() if k not in ("status",)}
                patch.setdefault("metadata", {}).setdefault("annotations", {})[
                    "kubectl.kubernetes.io/last-applied-configuration"] = json.dumps(doc, sort_keys=True)
                from ..api import strategicpatch as smp
                ptype = "application/strategic-merge-patch+json" if smp.schema_for(doc.get("apiVersion"), doc.get("kind")) \
                    else "application/merge-patch+json"        # custom resources have no strategic schema
                await c.patch(res, name, patch, ns, patch_type=ptype)
                print(f"{ri.kind.lower()}/{name} configured")
                continue
            doc.setdefault("metadata", {}).setdefault("annotations", {})[
                "kubectl.kubernetes.io/last-applied-configuration"] = json.dumps(doc, sort_keys=True)
        obj = await c.create(doc, ns)
        print(f"{ri.kind.lower()}/{m.name_of(obj)} created")


async def cmd_create(c, a):
    if not a.filename:
        from .extra import cmd_create_generator
        if await cmd_create_generator(c, a):
            return
        raise SystemExit("error: must specify -f or a generator (namespace, configmap, secret generic, serviceaccount, "
                         "deployment, job, priorityclass, quota, role, clusterrole, rolebinding, clusterrolebinding)")
    await _create_or_apply(c, a)


async def cmd_apply(c, a):
    await _create_or_apply(c, a, apply=True)


async def cmd_delete(c, a):
    from .delete import cmd_delete as delete
    return await delete(c, a)


async def cmd_logs(c, a):
    from .logs import cmd_logs as logs
    return await logs(c, a)


async def kubelet_exec(c, ns: str, name: str, container: str | None, cmd: list[str]) -> tuple[bytes, int]:
    """Run a command in a container through its node's kubelet (/run), returning (output, exit code)."""
    pod = await c.get("pods", name, ns)
    node = await c.get("nodes", pod["spec"]["nodeName"])
    st = node.get("status") or {}
    port = st["daemonEndpoints"]["kubeletEndpoint"]["Port"]
    addr = next((x["address"] for x in st.get("addresses") or [] if x.get("type") == "InternalIP"), "127.0.0.1")
    container = container or pod["spec"]["containers"][0]["name"]
    import aiohttp
    async with aiohttp.ClientSession() as s:
        async with s.post(f"http://{addr}:{port}/run/{ns}/{name}/{container}", params=[("cmd", x) for x in cmd]) as r:
            return await r.read(), int(r.headers.get("X-Exit-Code", "0"))


async def _stdin_chunks():
    loop = asyncio.get_running_loop()
    while True:
        data = await loop.run_in_executor(None, sys.stdin.buffer.read1, 65536)
        if not data:
            return
        yield data


def stream_transport() -> str:
    """exec / attach / port-forward / cp speak SPDY/3.1 like a v1.9 kubectl;
    AMDKUBE_STREAM_TRANSPORT=websocket selects the WebSocket channel protocol."""
    return os.environ.get("AMDKUBE_STREAM_TRANSPORT", "spdy")


def _term_size():
    try:
        sz = os.get_terminal_size(sys.stdout.fileno())
        return sz.columns, sz.lines
    except OSError:
        return None


async def cmd_exec(c, a):
    """exec through the apiserver (pods/exec, SPDY or WebSocket), -i forwards stdin, -t asks for a tty."""
    from ..client.stream import exec_stream
    out = lambda b: (sys.stdout.buffer.write(b), sys.stdout.buffer.flush())   # noqa: E731
    err = lambda b: (sys.stderr.buffer.write(b), sys.stderr.buffer.flush())   # noqa: E731
    return await exec_stream(c, a.namespace or "default", a.args[0].split("/", 1)[-1], a.command, a.container,
                             stdin=_stdin_chunks() if a.stdin else None, tty=a.tty, on_stdout=out, on_stderr=err,
                             transport=stream_transport(), resize=_term_size() if a.tty else None)


async def cmd_attach(c, a):
    from ..client.stream import exec_stream
    out = lambda b: (sys.stdout.buffer.write(b), sys.stdout.buffer.flush())   # noqa: E731
    return await exec_stream(c, a.namespace or "default", a.args[0].split("/", 1)[-1], [], a.container, attach=True,
                             on_stdout=out, on_stderr=out, transport=stream_transport())


async def cmd_label(c, a):
    from .metacmds import cmd_label as label
    return await label(c, a)


async def cmd_annotate(c, a):
    from .metacmds import cmd_annotate as annotate
    return await annotate(c, a)


async def cmd_cordon(c, a):
    from .drain import cmd_cordon as cordon
    return await cordon(c, a)


async def cmd_uncordon(c, a):
    from .drain import cmd_uncordon as uncordon
    return await uncordon(c, a)


async def cmd_drain(c, a):
    from .drain import cmd_drain as drain
    return await drain(c, a)


async def cmd_scale(c, a):
    from .scale import cmd_scale as scale
    return await scale(c, a)


async def cmd_run(c, a):
    from .run import cmd_run as run_
    return await run_(c, a)


async def cmd_top(c, a):
    from .top import cmd_top as top
    await top(c, a)


async def cmd_version(c, a):
    from .. import GIT_VERSION
    print(f"Client Version: {GIT_VERSION}")
    try:
        v = await c.request("GET", "/version")
        print(f"Server Version: {v['gitVersion']}")
    except Exception as e:
        print(f"Server Version: unavailable ({e})")


async def cmd_api_resources(c, a):
    rows = [["NAME", "SHORTNAMES", "APIGROUP", "NAMESPACED", "KIND"]]
    for ri in sorted(SCHEME.storage_versions(), key=lambda r: (r.group, r.plural)):
        rows.append([ri.plural, ",".join(ri.short_names), ri.group, str(ri.namespaced).lower(), ri.kind])
    print(printers.table(rows))


async def cmd_cluster_info(c, a):
    if a.args and a.args[0] == "dump":
        from .more import cmd_cluster_info_dump
        return await cmd_cluster_info_dump(c, a)
    print(f"Kubernetes master is running at {c.server}")


async def cmd_wait(c, a):
    r, name = _split_targets(a.args)[0]
    ri = SCHEME.resolve(r)
    cond = a.for_.split("=", 1)[1] if "=" in a.for_ else a.for_
    end = time.time() + timeout_of(a)
    while time.time() < end:
        o = await c.get_or_none(ri.plural, name, _ns(a, ri))
        if a.for_ == "delete" and o is None:
            print(f"{ri.kind.lower()}/{name} deleted")
            return
        if o is not None:
            st = o.get("status") or {}
            if st.get("phase") == cond or any(x.get("type") == cond and x.get("status") == "True" for x in st.get("conditions") or []):
                print(f"{ri.kind.lower()}/{name} condition met")
                return
        await asyncio.sleep(0.2)
    raise SystemExit(f"error: timed out waiting for the condition on {r}/{name}")


COMMANDS = {"get": cmd_get, "describe": cmd_describe, "create": cmd_create, "apply": cmd_apply, "delete": cmd_delete,
            "logs": cmd_logs, "exec": cmd_exec, "label": cmd_label, "annotate": cmd_annotate, "cordon": cmd_cordon,
            "uncordon": cmd_uncordon, "drain": cmd_drain, "scale": cmd_scale, "run": cmd_run,
            "top": cmd_top, "version": cmd_version, "api-resources": cmd_api_resources, "cluster-info": cmd_cluster_info,
            "wait": cmd_wait, "attach": cmd_attach}
from .extra import COMMANDS as _EXTRA, add_arguments as _extra_args  # noqa: E402
from . import more as _more  # noqa: E402
from . import logs as _logs  # noqa: E402
from . import drain as _drain  # noqa: E402
from . import metacmds as _metacmds  # noqa: E402
from . import scale as _scale  # noqa: E402
from . import run as _run  # noqa: E402
from . import delete as _delete  # noqa: E402
from . import expose as _expose  # noqa: E402
from . import taint as _taint  # noqa: E402
from . import autoscale as _autoscale  # noqa: E402
from . import patch as _patch  # noqa: E402
from . import replace as _replace  # noqa: E402
COMMANDS.update(_EXTRA)
COMMANDS.update(_more.COMMANDS)
COMMANDS["apply"] = _more.cmd_apply       # three-way merge, --prune, *-last-applied
COMMANDS["set"] = _more.cmd_set           # env/image/resources/selector/serviceaccount/subject
from .diff import cmd_alpha  # noqa: E402
COMMANDS["alpha"] = cmd_alpha             # alpha diff LOCAL|LIVE|LAST|MERGED
COMMANDS["expose"] = _expose.cmd_expose   # service/v2 generator
COMMANDS["taint"] = _taint.cmd_taint      # ParseTaints / ReorganizeTaints
COMMANDS["autoscale"] = _autoscale.cmd_autoscale   # horizontalpodautoscaler/v1 generator
COMMANDS["patch"] = _patch.cmd_patch      # patched / not patched, --local, -f
COMMANDS["replace"] = _replace.cmd_replace   # unconditional PUT, --force delete-and-create


_RESOURCE_CMDS = {"get", "describe", "delete", "label", "annotate", "scale", "patch", "wait", "edit", "explain", "expose",
                  "autoscale"}


def parser():
    p = argparse.ArgumentParser(prog="kubectl", description="amdkube kubectl")
    p.add_argument("--server", "-s", default=None)
    p.add_argument("--token", default=None)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--context", default=None)
    p.add_argument("-n", "--namespace", default=None)
    sub = p.add_subparsers(dest="cmd", required=True, metavar="command")
    from . import help as _help
    for name in list(COMMANDS) + ["config", "help"]:
        sp = sub.add_parser(name, help=_help.short(name), description=_help.long_desc(name),
                            epilog="Examples:\n" + _help.examples(name),
                            formatter_class=argparse.RawDescriptionHelpFormatter)
        _extra_args(sp)
        _more.add_arguments(sp)
        _logs.add_arguments(sp)
        _drain.add_arguments(sp)
        _metacmds.add_arguments(sp)
        _scale.add_arguments(sp)
        _run.add_arguments(sp)
        _delete.add_arguments(sp)
        _expose.add_arguments(sp)
        sp.add_argument("args", nargs="*")
        sp.add_argument("-n", "--namespace", default=argparse.SUPPRESS)
        sp.add_argument("-o", "--output", default=None)
        sp.add_argument("-l", "--selector", default=None)
        sp.add_argument("--field-selector", default=None)
        sp.add_argument("-A", "--all-namespaces", action="store_true")
        sp.add_argument("-w", "--watch", action="store_true")
        sp.add_argument("-f", "--filename", action="append", default=[])
        sp.add_argument("-c", "--container", default=None)
        sp.add_argument("-i", "--stdin", action="store_true")
        sp.add_argument("-t", "--tty", action="store_true")
        sp.add_argument("--tail", type=int, default=-1)
        sp.add_argument("--all", action="store_true")
        sp.add_argument("--grace-period", type=int, default=-1)
        sp.add_argument("--save-config", action="store_true")
        sp.add_argument("--cascade", type=lambda s: s != "false", default=True)
        sp.add_argument("--ignore-not-found", action="store_const", const=True, default=None)
        sp.add_argument("--ignore-daemonsets", action="store_true")
        sp.add_argument("--replicas", "-r", type=int, default=None)
        sp.add_argument("-p", "--patch", default=None)
        sp.add_argument("--type", default=None)
        sp.add_argument("--image", default=None)
        sp.add_argument("--gpus", type=int, default=0)
        sp.add_argument("--restart", default="Always")
        sp.add_argument("--for", dest="for_", default="condition=Ready")
        sp.add_argument("--timeout", type=parse_duration_flag, default=None)
        sp.add_argument("--command", nargs=argparse.REMAINDER, default=None)
        sp.add_argument("--validate", nargs="?", const=True, default=True,
                        type=lambda s: s.lower() not in ("false", "0", "no"))
        sp.add_argument("--recursive", action="store_true")
        sp.add_argument("--api-version", dest="explain_api_version", default=None)
        # printing flags (pkg/kubectl/cmd/util/printing.go AddPrinterFlags / AddOutputFlags)
        sp.add_argument("--show-labels", action="store_true")
        sp.add_argument("-L", "--label-columns", action="append", default=[])
        sp.add_argument("--sort-by", default=None)
        sp.add_argument("--no-headers", action="store_true")
        sp.add_argument("--template", default=None)
        sp.add_argument("--allow-missing-template-keys", type=lambda s: s != "false", default=True)
        sp.add_argument("-a", "--show-all", action="store_true")
        sp.add_argument("--show-kind", action="store_true")
    return p


async def openapi_definitions(c) -> dict:
    """The server's /openapi/v2 definitions (kubectl's cached OpenAPI getter); this build's own
    document when the server does not serve one."""
    from ..api.openapi import definitions
    try:
        doc = await c.request("GET", "/openapi/v2")
        if isinstance(doc, dict) and doc.get("definitions"):
            return doc["definitions"]
    except Exception:
        pass
    return definitions()


async def validate_files(c, paths) -> list[str]:
    """--validate (cmd/util/openapi/validation): one message per invalid file."""
    from ..api.openapi import validate
    defs = await openapi_definitions(c)
    out = []
    for p in paths:
        files = [os.path.join(p, f) for f in sorted(os.listdir(p)) if f.endswith((".yaml", ".yml", ".json"))] \
            if p != "-" and os.path.isdir(p) else [p]
        for f in files:
            if f == "-":
                continue        # stdin is read once, by the command itself
            errs = []
            for doc in load_manifests(open(f).read()):
                errs += validate(doc, defs)
            if errs:
                out.append(f'error validating "{f}": error validating data: [{", ".join(errs)}]; '
                           "if you choose to ignore these errors, turn validation off with --validate=false")
    return out


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        from .help import overview
        print(overview())
        return 0
    cmd_tail = []
    if "--" in argv:
        i = argv.index("--")
        argv, cmd_tail = argv[:i], argv[i + 1:]
    argv = _logs.rewrite_short_flags(argv)
    argv = _expose.rewrite_flags(argv)
    command_flag = "--command" in argv
    p = parser()
    a, extra = p.parse_known_args(argv)
    a.command_flag = command_flag
    if any(x.startswith("-") for x in extra):
        p.error(f"unrecognized arguments: {' '.join(extra)}")
    a.args = list(a.args) + extra      # positionals after flags (kubectl alpha diff -f x LAST LOCAL)
    if cmd_tail:
        a.command = cmd_tail
    elif a.command is None:
        a.command = []

    if a.cmd == "help":
        from .help import command_help, overview
        print(command_help(a.args[0]) if a.args else overview())
        return 0
    if a.cmd == "config":   # kubeconfig edits need no server
        from .extra import cmd_config_sync
        return cmd_config_sync(a)

    async def go():
        c = _client(a)
        try:
            if a.cmd in _RESOURCE_CMDS and a.args:
                first = a.args[0].split("/")[0].split(",")[0]
                if a.cmd == "explain":
                    first = first.split(".")[0]
                if SCHEME.resolve(first) is None:
                    await c.discover()          # a custom resource: learn it from the server
            elif a.filename and any(SCHEME.for_object(d) is None for d in _read_files(a.filename)):
                await c.discover()
            if a.cmd in ("create", "apply", "replace") and a.filename and a.validate:
                bad = await validate_files(c, a.filename)
                if bad:
                    for msg in bad:
                        print(f"error: {msg}", file=sys.stderr)
                    return 1
            rc = await COMMANDS[a.cmd](c, a)
            if a.cmd == "exec" and isinstance(rc, int) and rc > 0:
                # remotecommand v4: a non-zero exit is an ExitError, printed by checkErr
                print(f"command terminated with exit code {rc}", file=sys.stderr)
            return rc
        except m.StatusError as e:
            print(standard_error_message(e), file=sys.stderr)
            return 1
        except spdy.UpgradeRefused as e:
            se = e.status_error()
            print(standard_error_message(se) if se is not None else f"error: {e}", file=sys.stderr)
            return 1
        finally:
            await c.close()
    rc = asyncio.run(go())
    return rc if isinstance(rc, int) else 0


if __name__ == "__main__":
    sys.exit(main())
