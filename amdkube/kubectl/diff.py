"""kubectl alpha diff (pkg/kubectl/cmd/diff.go): compare two versions of the objects in -f files.

Versions: LOCAL (the file), LIVE (the server's object), LAST (its last-applied-configuration
annotation) and MERGED (what `kubectl apply` would produce: the three-way patch of LAST → LOCAL
applied to LIVE). LOCAL and LIVE by default; one keyword diffs it against LIVE. Each version is
written as one YAML file per object into a directory named after the version and the two
directories are compared with `diff -u -N`, or with $KUBERNETES_EXTERNAL_DIFF.
"""
from __future__ import annotations

import copy
import json
import os
import shlex
import subprocess
import sys
import tempfile

import yaml

from ..api import meta as m
from ..api.scheme import SCHEME
from .extra import _res
from .more import _SAME, LAST_APPLIED, three_way

VERSIONS = ("LOCAL", "LIVE", "LAST", "MERGED")


def _file_name(obj: dict) -> str:
    av = obj.get("apiVersion", "").replace("/", ".")
    ns = m.namespace_of(obj)
    return ".".join(x for x in (av, obj.get("kind", ""), ns, m.name_of(obj)) if x)


def merged(local: dict, live: dict | None) -> dict:
    """The object apply would leave on the server."""
    from ..api import strategicpatch as smp
    if live is None:
        out = copy.deepcopy(local)
        out.setdefault("metadata", {}).setdefault("annotations", {})[LAST_APPLIED] = json.dumps(local, sort_keys=True)
        return out
    original = json.loads(m.annotations_of(live).get(LAST_APPLIED) or "{}")
    modified = copy.deepcopy(local)
    modified.setdefault("metadata", {}).setdefault("annotations", {})[LAST_APPLIED] = json.dumps(local, sort_keys=True)
    patch = three_way(original, modified, live)
    if patch is _SAME:
        return copy.deepcopy(live)
    node = smp.schema_for(live.get("apiVersion"), live.get("kind"))
    if node is None and SCHEME.for_object(live) is None:
        from ..apiserver.registry import _json_merge_patch
        return _json_merge_patch(copy.deepcopy(live), patch)
    return smp.apply(live, patch, node)


async def version_of(c, which: str, local: dict, ns_default: str) -> dict | None:
    ri = SCHEME.for_object(local)
    if ri is None:
        raise SystemExit(f"error: unknown kind {local.get('apiVersion')}/{local.get('kind')}")
    ns = (m.namespace_of(local) or ns_default) if ri.namespaced else ""
    if ri.namespaced:
        local.setdefault("metadata", {})["namespace"] = ns
    if which == "LOCAL":
        return local
    live = await c.get_or_none(_res(ri), m.name_of(local), ns)
    if which == "LIVE":
        return live
    if which == "LAST":
        la = m.annotations_of(live or {}).get(LAST_APPLIED)
        return json.loads(la) if la else None
    return merged(local, live)


async def cmd_alpha(c, a):
    if not a.args or a.args[0] != "diff":
        raise SystemExit("error: unknown alpha command (available: diff)")
    from .main import _read_files
    kw = [x.upper() for x in a.args[1:]]
    for x in kw:
        if x not in VERSIONS:
            raise SystemExit(f'error: Invalid parameter "{x}", must be either "LOCAL", "LIVE", "LAST" or "MERGED"')
    if len(kw) > 2:
        raise SystemExit("error: Invalid number of arguments: expected at most 2.")
    frm, to = (kw + ["LOCAL", "LIVE"])[:2] if len(kw) != 1 else (kw[0], "LIVE")
    if not a.filename:
        raise SystemExit("error: Missing filename (-f)")
    docs = _read_files(a.filename)
    with tempfile.TemporaryDirectory(prefix="kubectl-diff-") as tmp:
        dirs = {}
        for label in dict.fromkeys((frm, to)):
            dirs[label] = os.path.join(tmp, label)
            os.makedirs(dirs[label])
        for doc in docs:
            ri = SCHEME.for_object(doc)
            if ri is not None and ri.namespaced:
                doc.setdefault("metadata", {}).setdefault("namespace", a.namespace or "default")
            for label in dirs:
                obj = await version_of(c, label, copy.deepcopy(doc), a.namespace or "default")
                if obj is None:
                    continue
                with open(os.path.join(dirs[label], _file_name(doc)), "w") as f:
                    yaml.safe_dump(obj, f, sort_keys=True)
        tool = shlex.split(os.environ.get("KUBERNETES_EXTERNAL_DIFF", "")) or ["diff", "-u", "-N"]
        r = subprocess.run([*tool, dirs[frm], dirs[to]], capture_output=True, text=True)
        sys.stdout.write(r.stdout.replace(tmp + "/", ""))
        sys.stderr.write(r.stderr)
        return 0 if r.returncode in (0, 1) else r.returncode
