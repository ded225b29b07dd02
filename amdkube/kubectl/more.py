"""kubectl: the rest of the reference release's command set (pkg/kubectl/cmd).

  * apply with a real three-way merge (apply.go: patch = last-applied → manifest → live,
    deletions for fields the manifest dropped, `$patch: delete` for list items, all driven by
    the kind's patch strategies and merge keys — api/strategicpatch.py), a JSON-merge three-way
    patch for custom resources, 409 retries and --force re-creation,
    `--prune -l` (apply.go pruner: objects with a last-applied annotation matching the selector
    that the manifests no longer contain), `apply view-last-applied|set-last-applied|
    edit-last-applied`;
  * set env|resources|selector|serviceaccount|subject (cmd/set/*.go);
  * create secret docker-registry|tls, create service clusterip|nodeport|loadbalancer|
    externalname, create poddisruptionbudget (cmd/create_*.go);
  * rolling-update for ReplicationControllers (rolling_updater.go: new RC with a deployment
    hash, scale up one / down one until the old one is gone, rename);
  * convert (to another served version), api-versions, completion (bash), options, plugin
    (plugins from ~/.kube/plugins/<name>/plugin.yaml, KUBECTL_PLUGINS_* environment),
    cluster-info dump.
"""
from __future__ import annotations

import base64
import copy
import hashlib
import json
import os
import subprocess
import sys

import yaml

from ..api import meta as m
from ..api import strategicpatch as smp
from ..api.scheme import SCHEME
from .extra import _ns, _res, _target

LAST_APPLIED = "kubectl.kubernetes.io/last-applied-configuration"
# ---------------------------------------------------------------- three-way merge
def apply_patch_for(original: dict | None, modified: dict, current: dict) -> tuple[dict | None, str]:
    """(patch, content type) that turns `current` into `modified`, deleting what `original`
    (the last applied manifest) had and `modified` drops (apply.go patcher.patchSimple):
    a strategic three-way patch over the kind's schema (strategicpatch.CreateThreeWayMergePatch)
    for built-in kinds, a JSON merge three-way patch for kinds without one (custom resources).
    None when nothing changes."""
    node = smp.schema_for(modified.get("apiVersion"), modified.get("kind"))
    if node is None:
        patch, ctype = smp.create_three_way_json_merge(original, modified, current), "application/merge-patch+json"
    else:
        patch, ctype = smp.create_three_way(original, modified, current, node), "application/strategic-merge-patch+json"
    return (patch or None), ctype


def three_way(original, modified, current):
    """The apply patch alone (kubectl diff's MERGED view and tests); _SAME when empty."""
    patch, _ = apply_patch_for(original, modified, current)
    return _SAME if patch is None else patch


class _Same:
    def __repr__(self):
        return "<same>"


_SAME = _Same()


async def apply_docs(c, a, docs, out=print, allow_empty: bool = False):
    """`out`: where the per-object result lines go. With -l only the manifests whose labels
    match are applied (the builder's LabelSelectorParam filters local files too), and
    `allow_empty` lets a prune run when none match (apply.go returns "no objects passed to
    apply" first, so removing an addon's last manifest never prunes it; the addon manager
    passes True)."""
    from ..api.labels import parse_selector
    sel = parse_selector(a.selector) if getattr(a, "selector", None) else None
    applied = set()
    count = 0
    for doc in docs:
        if sel is not None and not sel.matches(m.labels_of(doc)):
            continue
        count += 1
        ri = SCHEME.for_object(doc)
        if ri is None:
            raise SystemExit(f"error: unknown kind {doc.get('apiVersion')}/{doc.get('kind')}")
        ns = (m.namespace_of(doc) or a.namespace or "default") if ri.namespaced else ""
        if ri.namespaced:
            doc.setdefault("metadata", {})["namespace"] = ns
        name = m.name_of(doc)
        res = _res(ri)
        applied.add((ri.group, ri.plural, ns, name))
        manifest = json.dumps(doc, sort_keys=True)
        cur = await c.get_or_none(res, name, ns) if name else None
        if cur is None:
            doc.setdefault("metadata", {}).setdefault("annotations", {})[LAST_APPLIED] = manifest
            obj = await c.create(doc, ns)
            applied.add(m.uid_of(obj))
            out(f"{ri.kind.lower()}/{m.name_of(obj)} created")
            continue
        applied.add(m.uid_of(cur))
        original = json.loads(m.annotations_of(cur).get(LAST_APPLIED) or "{}")
        modified = copy.deepcopy(doc)
        modified.setdefault("metadata", {}).setdefault("annotations", {})[LAST_APPLIED] = manifest
        for attempt in range(5):            # apply.go maxPatchRetry: a 409 re-reads the live object
            try:
                patch, ctype = apply_patch_for(original, modified, cur)
            except smp.PatchError as e:
                raise SystemExit(f"error: {ri.kind.lower()}/{name}: {e}")
            if patch is None:
                out(f"{ri.kind.lower()}/{name} unchanged")
                break
            try:
                await c.patch(res, name, patch, ns, patch_type=ctype)
            except m.StatusError as e:
                if e.code == 409 and attempt < 4:
                    cur = await c.get(res, name, ns)
                    continue
                if getattr(a, "force", False) and e.code in (409, 422):
                    await c.delete(res, name, ns)             # --force: delete and re-create
                    await _wait_gone(c, res, name, ns)
                    doc.setdefault("metadata", {}).setdefault("annotations", {})[LAST_APPLIED] = manifest
                    applied.add(m.uid_of(await c.create(doc, ns)))
                    out(f"{ri.kind.lower()}/{name} replaced")
                    break
                raise
            out(f"{ri.kind.lower()}/{name} configured")
            break
    if count == 0 and not allow_empty:
        raise SystemExit("error: no objects passed to apply")
    if getattr(a, "prune", False):
        await _prune(c, a, applied, out)
    return applied


async def _wait_gone(c, res, name, ns, timeout: float = 30.0):
    import asyncio
    import time
    end = time.monotonic() + timeout
    while await c.get_or_none(res, name, ns) is not None:
        if time.monotonic() > end:
            raise SystemExit(f"error: timed out waiting for {res}/{name} to be deleted")
        await asyncio.sleep(0.2)


PRUNE_WHITELIST = ("configmaps", "endpoints", "namespaces", "persistentvolumeclaims", "persistentvolumes", "pods",
                   "replicationcontrollers", "secrets", "services", "jobs.batch", "cronjobs.batch", "daemonsets.apps",
                   "deployments.apps", "replicasets.apps", "statefulsets.apps", "ingresses.extensions")


def prune_resources(whitelist) -> list[str]:
    """--prune-whitelist <group>/<version>/<Kind> entries (core/v1/ConfigMap) → resources."""
    if not whitelist:
        return list(PRUNE_WHITELIST)
    out = []
    for gvk in whitelist:
        parts = gvk.split("/")
        if len(parts) != 3:
            raise SystemExit(f"error: invalid GroupVersionKind format: {gvk}, please follow <group/version/kind>")
        group = "" if parts[0] == "core" else parts[0]
        ri = SCHEME.for_object({"apiVersion": f"{group}/{parts[1]}" if group else parts[1], "kind": parts[2]})
        if ri is None:
            raise SystemExit(f"error: unknown prune resource {gvk}")
        out.append(ri.plural if not ri.group else f"{ri.plural}.{ri.group}")
    return out


async def _prune(c, a, applied, out=print):
    if not a.selector and not a.all:
        raise SystemExit("error: all resources selected for prune without explicitly passing --all or -l")
    # `applied`: (group, plural, namespace, name) of every manifest plus the UIDs it created or
    # patched; the pruner skips visited UIDs (apply.go visitedUids), so a kind served by two
    # groups (extensions and apps DaemonSets) is never pruned through its other name
    namespaces = {t[2] for t in applied if isinstance(t, tuple) and t[2]} or {a.namespace or "default"}
    for res in prune_resources(getattr(a, "prune_whitelist", None)):
        ri = SCHEME.resolve(res)
        for ns in (namespaces if ri.namespaced else {""}):
            items, _ = await c.list(res, ns, a.selector)
            for o in items:
                if LAST_APPLIED not in m.annotations_of(o):
                    continue
                if m.uid_of(o) in applied or \
                        (ri.group, ri.plural, m.namespace_of(o) if ri.namespaced else "", m.name_of(o)) in applied:
                    continue
                await c.delete(res, m.name_of(o), m.namespace_of(o) if ri.namespaced else "")
                out(f"{ri.kind.lower()}/{m.name_of(o)} pruned")


async def cmd_apply(c, a):
    from .main import _emit, _read_files
    if a.args and a.args[0] in ("view-last-applied", "set-last-applied", "edit-last-applied"):
        sub = a.args[0]
        if sub == "set-last-applied":
            for doc in _read_files(a.filename):
                ri = SCHEME.for_object(doc)
                ns = (m.namespace_of(doc) or a.namespace or "default") if ri.namespaced else ""
                cur = await c.get_or_none(_res(ri), m.name_of(doc), ns)
                if cur is None:
                    if not a.create_annotation:
                        raise SystemExit(f"error: no last-applied-configuration annotation found on resource: {m.name_of(doc)}")
                    continue
                await c.patch(_res(ri), m.name_of(doc), {"metadata": {"annotations": {
                    LAST_APPLIED: json.dumps(doc, sort_keys=True)}}}, ns)
                print(f"{ri.kind.lower()}/{m.name_of(doc)} configured")
            return
        ri, name, _ = _target(a, 1)
        ns = _ns(a, ri)
        cur = await c.get(_res(ri), name, ns)
        la = m.annotations_of(cur).get(LAST_APPLIED)
        if la is None:
            raise SystemExit(f"error: no last-applied-configuration annotation found on resource: {name}")
        if sub == "view-last-applied":
            obj = json.loads(la)
            print(json.dumps(obj, indent=2) if a.output == "json" else yaml.safe_dump(obj, sort_keys=False), end="")
            return
        # edit-last-applied: $EDITOR on the annotation, then store it
        import tempfile
        with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
            yaml.safe_dump(json.loads(la), f, sort_keys=False)
        subprocess.run([os.environ.get("KUBE_EDITOR") or os.environ.get("EDITOR") or "vi", f.name], check=False)
        new = yaml.safe_load(open(f.name))
        os.unlink(f.name)
        await c.patch(_res(ri), name, {"metadata": {"annotations": {LAST_APPLIED: json.dumps(new, sort_keys=True)}}}, ns)
        print(f"{ri.kind.lower()}/{name} edited")
        return
    docs = _read_files(a.filename, getattr(a, "recursive", False))
    if a.output and a.dry_run:
        _emit(docs, a, docs[0]["kind"] if docs else "List")
        return
    await apply_docs(c, a, docs)


# ----------------------------------------------------------------------------- set
def _podspec(obj):
    return obj.get("spec") if obj.get("kind") == "Pod" else ((obj.get("spec") or {}).get("template") or {}).get("spec")


async def cmd_set(c, a):
    from .extra import cmd_set as set_image
    if not a.args:
        raise SystemExit("error: set env|image|resources|selector|serviceaccount|subject ...")
    sub = a.args[0]
    if sub == "image":
        return await set_image(c, a)
    ri, name, rest = _target(a, 1)
    ns = _ns(a, ri)
    obj = await c.get(_res(ri), name, ns)
    if sub == "env":
        ps = _podspec(obj)
        sets = [kv.split("=", 1) for kv in rest + list(a.env) if "=" in kv and not kv.endswith("-")]
        unsets = [kv[:-1] for kv in rest + list(a.env) if kv.endswith("-")]
        for ct in ps.get("containers") or []:
            if a.container and ct["name"] != a.container:
                continue
            env = [e for e in ct.get("env") or [] if e["name"] not in unsets and e["name"] not in dict(sets)]
            env += [{"name": k, "value": v} for k, v in sets]
            ct["env"] = env
        await c.update(obj)
        print(f"{ri.kind.lower()}/{name} env updated")
    elif sub == "resources":
        ps = _podspec(obj)
        def parse(s):
            return dict(kv.split("=", 1) for kv in (s or "").split(",") if kv)
        lim, req = parse(a.limits), parse(a.requests)
        for ct in ps.get("containers") or []:
            if a.container and ct["name"] != a.container:
                continue
            res = ct.setdefault("resources", {})
            if lim:
                res.setdefault("limits", {}).update(lim)
            if req:
                res.setdefault("requests", {}).update(req)
        await c.update(obj)
        print(f"{ri.kind.lower()}/{name} resource requirements updated")
    elif sub == "selector":
        sel = dict(kv.split("=", 1) for kv in rest[0].split(",")) if rest else {}
        if ri.kind == "Service":
            obj.setdefault("spec", {})["selector"] = sel
        else:
            obj.setdefault("spec", {})["selector"] = {"matchLabels": sel}
        await c.update(obj)
        print(f"{ri.kind.lower()}/{name} selector updated")
    elif sub == "serviceaccount":
        ps = _podspec(obj)
        ps["serviceAccountName"] = rest[0]
        await c.update(obj)
        print(f"{ri.kind.lower()}/{name} serviceaccount updated")
    elif sub == "subject":
        subs = list(obj.get("subjects") or [])
        for u in a.user:
            subs.append({"kind": "User", "name": u, "apiGroup": "rbac.authorization.k8s.io"})
        for g in a.group:
            subs.append({"kind": "Group", "name": g, "apiGroup": "rbac.authorization.k8s.io"})
        for sa in a.serviceaccount:
            sns, _, sname = sa.partition(":")
            subs.append({"kind": "ServiceAccount", "namespace": sns, "name": sname})
        dedup = []
        for s in subs:
            if s not in dedup:
                dedup.append(s)
        obj["subjects"] = dedup
        await c.update(obj)
        print(f"{ri.kind.lower()}/{name} subjects updated")
    else:
        raise SystemExit(f"error: unknown set subcommand {sub!r}")


# --------------------------------------------------------------------- generators
async def create_more(c, a, kind, rest) -> dict | None:
    if kind == "secret" and rest and rest[0] == "docker-registry":
        # secret_for_docker_registry.go: the four fields checked, .dockerconfigjson compact with
        # the credentialprovider entry's omitempty fields (username, password, email, auth)
        from .generators import secret_hash
        name = rest[1] if len(rest) > 1 else ""
        server = a.docker_server or "https://index.docker.io/v1/"
        for val, what in ((name, "name"), (a.docker_username, "username"), (a.docker_password, "password"), (server, "server")):
            if not val:
                raise SystemExit(f"error: {what} must be specified")
        entry = {"username": a.docker_username, "password": a.docker_password}
        if a.docker_email:
            entry["email"] = a.docker_email
        entry["auth"] = base64.b64encode(f"{a.docker_username}:{a.docker_password}".encode()).decode()
        cfg = json.dumps({"auths": {server: entry}}, separators=(",", ":"))
        sec = {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": name}, "type": "kubernetes.io/dockerconfigjson",
               "data": {".dockerconfigjson": base64.b64encode(cfg.encode()).decode()}}
        if getattr(a, "append_hash", False):
            sec["metadata"]["name"] = f"{name}-{secret_hash(sec)}"
        return sec
    if kind == "secret" and rest and rest[0] == "tls":
        # secret_for_tls.go: key and certificate required and loadable as a pair
        import ssl
        from .generators import secret_hash
        name = rest[1] if len(rest) > 1 else ""
        if not a.key:
            raise SystemExit("error: key must be specified")
        if not a.cert:
            raise SystemExit("error: certificate must be specified")
        try:
            ssl.create_default_context(ssl.Purpose.CLIENT_AUTH).load_cert_chain(a.cert, a.key)
        except (OSError, ssl.SSLError) as e:
            raise SystemExit(f"error: failed to load key pair {e}") from None
        with open(a.cert, "rb") as fc, open(a.key, "rb") as fk:
            sec = {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": name}, "type": "kubernetes.io/tls",
                   "data": {"tls.crt": base64.b64encode(fc.read()).decode(), "tls.key": base64.b64encode(fk.read()).decode()}}
        if getattr(a, "append_hash", False):
            sec["metadata"]["name"] = f"{name}-{secret_hash(sec)}"
        return sec
    if kind in ("service", "svc") and rest:
        from .generators import SERVICE_TYPES, GenerateError, generate_service
        stype = SERVICE_TYPES.get(rest[0])
        if stype is None:
            raise SystemExit("error: create service clusterip|nodeport|loadbalancer|externalname NAME")
        try:
            return generate_service(rest[1] if len(rest) > 1 else "", stype, a.tcp, a.clusterip or "",
                                    a.external_name or "", int(a.node_port or 0) if stype == "NodePort" else 0)
        except GenerateError as e:
            raise SystemExit(f"error: {e}") from None
    if kind in ("poddisruptionbudget", "pdb") and rest:
        from .generators import GenerateError, generate_pdb
        try:
            return generate_pdb(rest[0], a.selector or "", a.min_available or "", a.max_unavailable or "")
        except GenerateError as e:
            raise SystemExit(f"error: {e}") from None
    return None


# ------------------------------------------------------------------ rolling-update
async def cmd_rolling_update(c, a):
    """rolling_updater.go for ReplicationControllers: the new RC (image change or -f) gets a
    deployment label; pods are added one at a time, waiting until ready, and the old RC is
    scaled down one at a time; finally the old RC is deleted and the new one takes its name."""
    import asyncio
    old_name = a.args[0]
    ns = a.namespace or "default"
    old = await c.get("replicationcontrollers", old_name, ns)
    replicas = (old.get("spec") or {}).get("replicas", 1)
    if a.filename:
        from .main import _read_files
        new = _read_files(a.filename)[0]
    else:
        new = copy.deepcopy(old)
        for k in ("resourceVersion", "uid", "creationTimestamp", "generation", "selfLink"):
            new["metadata"].pop(k, None)
        new.pop("status", None)
        ct = new["spec"]["template"]["spec"]["containers"][0]
        ct["image"] = a.image
    h = hashlib.md5(json.dumps(new["spec"]["template"], sort_keys=True).encode()).hexdigest()[:8]
    keep_name = not a.filename or m.name_of(new) == old_name
    new_name = f"{old_name}-{h}" if keep_name else m.name_of(new)
    new["metadata"]["name"] = new_name
    for obj in (new,):
        obj["spec"].setdefault("selector", dict(obj["spec"]["template"]["metadata"].get("labels") or {}))
        obj["spec"]["selector"]["deployment"] = h
        obj["spec"]["template"]["metadata"].setdefault("labels", {})["deployment"] = h
    new["spec"]["replicas"] = 0
    if await c.get_or_none("replicationcontrollers", new_name, ns) is None:
        await c.create(new, ns)
    print(f"Created {new_name}")

    async def ready(name, want):
        for _ in range(int(_timeout_of(a) * 10)):
            rc = await c.get("replicationcontrollers", name, ns)
            if (rc.get("status") or {}).get("readyReplicas", 0) >= want:
                return
            await asyncio.sleep(0.1)
        raise SystemExit(f"error: timed out waiting for {name} to have {want} ready replicas")
    up, down = 0, replicas
    while up < replicas or down > 0:
        if up < replicas:
            up += 1
            await c.patch("replicationcontrollers", new_name, {"spec": {"replicas": up}}, ns)
            await ready(new_name, up)
            print(f"Scaling {new_name} up to {up}")
        if down > 0:
            down -= 1
            await c.patch("replicationcontrollers", old_name, {"spec": {"replicas": down}}, ns)
            print(f"Scaling {old_name} down to {down}")
    await c.delete("replicationcontrollers", old_name, ns)
    if keep_name:
        final = await c.get("replicationcontrollers", new_name, ns)
        for k in ("resourceVersion", "uid", "creationTimestamp", "generation"):
            final["metadata"].pop(k, None)
        final.pop("status", None)
        final["metadata"]["name"] = old_name
        await c.create(final, ns)
        await c.delete("replicationcontrollers", new_name, ns, propagation="Orphan")
        new_name = old_name
    print(f'Update succeeded. Deleting old controller: {old_name}\nRenaming {new_name} to {old_name}'
          if keep_name else f"Update succeeded. Deleting {old_name}")
    print(f'replicationcontroller "{old_name}" rolling updated' + ("" if keep_name else f' to "{new_name}"'))


# ------------------------------------------------------------------- small commands
async def cmd_convert(c, a):
    """convert: manifests to --output-version (any version the scheme serves for the kind)."""
    from .main import _read_files
    out = []
    for doc in _read_files(a.filename):
        ri = SCHEME.for_object(doc)
        if ri is None:
            raise SystemExit(f"error: unknown kind {doc.get('apiVersion')}/{doc.get('kind')}")
        target = a.output_version or SCHEME.storage_of(ri).api_version
        g, _, v = target.rpartition("/") if "/" in target else ("", "", target)
        served = SCHEME.served(g, v, ri.plural)
        if served is None or SCHEME.storage_of(served) is not SCHEME.storage_of(ri):
            raise SystemExit(f"error: {ri.kind} is not served as {target}")
        doc = SCHEME.to_storage(copy.deepcopy(doc))
        doc["apiVersion"] = served.api_version
        out.append(doc)
    obj = out[0] if len(out) == 1 else {"apiVersion": "v1", "kind": "List", "items": out}
    print(json.dumps(obj, indent=2) if a.output == "json" else yaml.safe_dump(obj, sort_keys=False), end="")


async def cmd_api_versions(c, a):
    d = await c.request("GET", "/apis")
    vs = ["v1"] + sorted(v["groupVersion"] for g in d.get("groups") or [] for v in g.get("versions") or [])
    print("\n".join(vs))


async def cmd_options(c, a):
    print("The following options can be passed to any command:\n\n"
          "  --kubeconfig='': Path to the kubeconfig file to use for CLI requests.\n"
          "  --context='': The name of the kubeconfig context to use\n"
          "  -n, --namespace='': If present, the namespace scope for this CLI request\n"
          "  -s, --server='': The address and port of the Kubernetes API server\n"
          "  --token='': Bearer token for authentication to the API server")


def completion_script(commands) -> str:
    cmds = " ".join(sorted(commands))
    return ("# kubectl bash completion (amdkube)\n"
            "_amdkube_kubectl() {\n"
            "    local cur=${COMP_WORDS[COMP_CWORD]}\n"
            "    if [ $COMP_CWORD -eq 1 ]; then\n"
            f"        COMPREPLY=( $(compgen -W \"{cmds}\" -- \"$cur\") )\n"
            "    else\n"
            "        COMPREPLY=( $(compgen -W \"$(kubectl api-resources 2>/dev/null | awk 'NR>1{print $1}')\" -- \"$cur\") )\n"
            "    fi\n"
            "}\n"
            "complete -F _amdkube_kubectl kubectl\n")


async def cmd_completion(c, a):
    from .main import COMMANDS
    if a.args and a.args[0] not in ("bash", "zsh"):
        raise SystemExit(f"error: Unsupported shell type {a.args[0]!r}")
    print(completion_script(list(COMMANDS)), end="")


def plugin_dirs():
    env = os.environ.get("KUBECTL_PLUGINS_PATH")
    if env:
        return env.split(os.pathsep)
    return [os.path.expanduser("~/.kube/plugins"),
            os.path.join(os.environ.get("XDG_DATA_DIRS", "/usr/local/share").split(os.pathsep)[0], "kubectl", "plugins")]


def find_plugins() -> dict[str, tuple[str, dict]]:
    """plugins/loader.go: <dir>/<name>/plugin.yaml with name, shortDesc, command."""
    out = {}
    for d in plugin_dirs():
        if not os.path.isdir(d):
            continue
        for n in sorted(os.listdir(d)):
            p = os.path.join(d, n, "plugin.yaml")
            if os.path.isfile(p):
                try:
                    desc = yaml.safe_load(open(p)) or {}
                except yaml.YAMLError:
                    continue
                out.setdefault(desc.get("name", n), (os.path.join(d, n), desc))
    return out


async def cmd_plugin(c, a):
    plugins = find_plugins()
    if not a.args:
        for n, (_d, desc) in sorted(plugins.items()):
            print(f"  {n:<20} {desc.get('shortDesc', '')}")
        return
    name = a.args[0]
    if name not in plugins:
        raise SystemExit(f"error: unknown plugin {name!r}")
    d, desc = plugins[name]
    env = dict(os.environ, KUBECTL_PLUGINS_CALLER=sys.argv[0], KUBECTL_PLUGINS_CURRENT_NAMESPACE=a.namespace or "default",
               KUBECTL_PLUGINS_DESCRIPTOR_NAME=name, KUBECTL_PLUGINS_DESCRIPTOR_COMMAND=desc.get("command", ""),
               KUBECTL_PLUGINS_DESCRIPTOR_SHORT_DESC=desc.get("shortDesc", ""), KUBECTL_PLUGINS_GLOBAL_FLAG_SERVER=c.server)
    r = subprocess.run(["sh", "-c", desc.get("command", "") + ' "$@"', name, *a.args[1:]], cwd=d, env=env)
    return r.returncode


async def cmd_cluster_info_dump(c, a):
    """cluster-info dump: nodes, then events/rcs/services/daemonsets/deployments/replicasets/
    pods (and pod logs) of kube-system and default, as JSON."""
    out_dir = a.output_directory
    sections = [("nodes", "")]
    for ns in ([a.namespace] if a.namespace else ["kube-system", "default"]):
        sections += [(r, ns) for r in ("events", "replicationcontrollers", "services", "daemonsets.apps", "deployments.apps",
                                       "replicasets.apps", "pods")]
    for res, ns in sections:
        ri = SCHEME.resolve(res)
        items, _ = await c.list(res, ns)
        doc = json.dumps({"kind": ri.list_kind, "apiVersion": ri.api_version, "items": items}, indent=2)
        if out_dir:
            p = os.path.join(out_dir, ns or "", f"{ri.plural}.json")
            os.makedirs(os.path.dirname(p), exist_ok=True)
            open(p, "w").write(doc)
        else:
            print(doc)
        if ri.plural == "pods":
            for p in items:
                for ct in (p.get("spec") or {}).get("containers") or []:
                    try:
                        logs = await c.logs(ns, m.name_of(p), ct["name"])
                    except m.StatusError:
                        continue
                    if out_dir:
                        lp = os.path.join(out_dir, ns, m.name_of(p), "logs.txt")
                        os.makedirs(os.path.dirname(lp), exist_ok=True)
                        open(lp, "a").write(logs)
                    else:
                        print(f"==== START logs for container {ct['name']} of pod {ns}/{m.name_of(p)} ====\n{logs}"
                              f"==== END logs for container {ct['name']} of pod {ns}/{m.name_of(p)} ====")
    if out_dir:
        print(f"Cluster info dumped to {out_dir}")


def add_arguments(sp):
    sp.add_argument("--prune", action="store_true")
    sp.add_argument("--prune-whitelist", action="append", default=[])
    sp.add_argument("--dry-run", action="store_true")
    sp.add_argument("--create-annotation", action="store_true")
    sp.add_argument("--env", "-e", action="append", default=[])
    sp.add_argument("--limits", default=None)
    sp.add_argument("--requests", default=None)
    sp.add_argument("--docker-server", default="https://index.docker.io/v1/")
    sp.add_argument("--docker-username", default="")
    sp.add_argument("--docker-password", default="")
    sp.add_argument("--docker-email", default="")
    sp.add_argument("--cert", default=None)
    sp.add_argument("--key", default=None)
    sp.add_argument("--tcp", action="append", default=[])
    sp.add_argument("--node-port", type=int, default=0)
    sp.add_argument("--external-name", default="")
    sp.add_argument("--clusterip", default="")
    sp.add_argument("--min-available", default=None)
    sp.add_argument("--max-unavailable", default=None)
    sp.add_argument("--output-version", default=None)
    sp.add_argument("--output-directory", default=None)
    sp.add_argument("--containers", action="store_true")
    # kubectl config set-cluster / set-credentials / set-context / view --minify
    sp.add_argument("--certificate-authority", default=None)
    sp.add_argument("--insecure-skip-tls-verify", default=None, choices=("true", "false"))
    sp.add_argument("--embed-certs", action="store_true")
    sp.add_argument("--client-certificate", default=None)
    sp.add_argument("--client-key", default=None)
    sp.add_argument("--username", default=None)
    sp.add_argument("--password", default=None)
    sp.add_argument("--cluster", dest="cfg_cluster", default=None)
    sp.add_argument("--current", action="store_true")
    sp.add_argument("--minify", action="store_true")
    sp.add_argument("--token", dest="cfg_token", default=None, help="set-credentials bearer token")
    import argparse as _ap
    sp.add_argument("--server", default=_ap.SUPPRESS, help="set-cluster: the API server URL (also the global flag)")


COMMANDS = {"rolling-update": cmd_rolling_update, "convert": cmd_convert, "api-versions": cmd_api_versions,
            "options": cmd_options, "completion": cmd_completion, "plugin": cmd_plugin}


def _timeout_of(a, default: float = 30.0) -> float:
    t = getattr(a, "timeout", None)
    return default if t is None else float(t)
