"""kubectl commands beyond the core CRUD set.

Reference: pkg/kubectl/cmd/cmd.go:216-330 command groups — rollout (rollout/rollout.go:
status, history, undo, pause, resume), expose.go, autoscale.go, taint.go, set/set_image.go,
replace.go, edit.go, config/ (view, current-context, use-context, get-contexts),
auth/cani.go, certificates.go (approve/deny), portforward.go, proxy.go, cp.go, explain.go,
create_*.go generators (namespace, configmap, secret generic, serviceaccount, deployment,
job, priorityclass, quota, role/clusterrole/rolebinding/clusterrolebinding).

exec/attach/port-forward/cp go through the apiserver's WebSocket subresources (the reference
also speaks SPDY; amdkube serves the WebSocket channel protocols only).
"""
from __future__ import annotations

import asyncio
import base64
import json
import os
import subprocess
import sys
import tempfile
import time

from ..api import meta as m
from ..api.scheme import SCHEME, dump_yaml, load_manifests
from . import printers

REVISION = "deployment.kubernetes.io/revision"
CHANGE_CAUSE = "kubernetes.io/change-cause"


def _res(ri) -> str:
    return ri.plural if not ri.group else f"{ri.plural}.{ri.group}"


def _target(a, idx=0):
    args = a.args[idx:]
    if not args:
        raise SystemExit("error: a resource is required")
    if "/" in args[0]:
        r, n = args[0].split("/", 1)
        rest = args[1:]
    else:
        r, n, rest = args[0], (args[1] if len(args) > 1 else None), args[2:]
    ri = SCHEME.resolve(r)
    if ri is None:
        raise SystemExit(f'error: the server doesn\'t have a resource type "{r}"')
    return ri, n, rest


def _ns(a, ri=None):
    if ri is not None and not ri.namespaced:
        return ""
    return a.namespace or "default"


# ------------------------------------------------------------------ rollout
async def _owned_rs(c, d):
    items, _ = await c.list("replicasets.apps", m.namespace_of(d))
    uid = m.uid_of(d)
    return [r for r in items if (m.controller_ref(r) or {}).get("uid") == uid]


def _rev(o) -> int:
    try:
        return int(((o.get("metadata") or {}).get("annotations") or {}).get(REVISION, "0"))
    except ValueError:
        return 0


async def _owned_revisions(c, obj) -> list[dict]:
    """The ControllerRevisions a DaemonSet or StatefulSet recorded, oldest first."""
    items, _ = await c.list("controllerrevisions.apps", m.namespace_of(obj))
    uid = m.uid_of(obj)
    return sorted((r for r in items if (m.controller_ref(r) or {}).get("uid") == uid), key=lambda r: int(r.get("revision", 0)))


def _revision_template(r) -> dict:
    """The template a revision restores (its data is a `$patch: replace` of spec.template)."""
    tpl = json.loads(json.dumps(((r.get("data") or {}).get("spec") or {}).get("template") or {}))
    tpl.pop("$patch", None)
    return tpl


async def _rollout_history_based(c, a, sub, ri, name, ns, res):
    """rollout history/undo/status of DaemonSets and StatefulSets (pkg/kubectl/history.go
    DaemonSetHistoryViewer/StatefulSetHistoryViewer, rollback.go, rollout_status.go)."""
    kind = ri.kind
    if sub == "history":
        obj = await c.get(res, name, ns)
        revs = await _owned_revisions(c, obj)
        if a.revision:
            r = next((x for x in revs if int(x.get("revision", 0)) == a.revision), None)
            if r is None:
                raise SystemExit(f"error: unable to find the specified revision {a.revision}")
            print(f'{kind.lower()}s "{name}" with revision #{a.revision}')
            print(dump_yaml({"Pod Template": _revision_template(r)}), end="")
            return 0
        rows = [["REVISION", "CHANGE-CAUSE"]]
        for r in revs:
            rows.append([str(r.get("revision", 0)), ((r.get("metadata") or {}).get("annotations") or {}).get(CHANGE_CAUSE, "<none>")])
        print(f'{kind.lower()}s "{name}"')
        print(printers.table(rows))
        return 0
    if sub == "undo":
        obj = await c.get(res, name, ns)
        revs = await _owned_revisions(c, obj)
        if a.to_revision:
            target = next((r for r in revs if int(r.get("revision", 0)) == a.to_revision), None)
            if target is None:
                raise SystemExit(f"error: unable to find specified revision {a.to_revision} in history")
        else:
            if len(revs) < 2:
                raise SystemExit("error: no last revision to roll back to")
            target = revs[-2]
        tpl = _revision_template(target)
        if tpl == ((obj.get("spec") or {}).get("template") or {}):
            print(f"{kind.lower()}.apps/{name} skipped rollback (current template already matches revision "
                  f"{target.get('revision')})")
            return 0
        obj["spec"]["template"] = tpl
        await c.update(dict(obj, apiVersion=obj.get("apiVersion") or "apps/v1", kind=kind))
        print(f"{kind.lower()}.apps/{name} rolled back")
        return 0
    return await _rollout_status(c, a, kind, res, name, ns)


async def _rollout_status(c, a, kind, res, name, ns):
    """rollout.go RunStatus over the StatusViewers of kubectl/rollout.py: print each new
    message; without --watch stop after the first."""
    from . import rollout as R
    end = time.time() + _timeout_of(a)
    last = None
    while True:
        obj = await c.get(res, name, ns)
        try:
            if kind == "Deployment":
                msg, done = R.deployment_status(obj, name, int(getattr(a, "revision", 0) or 0))
            else:
                msg, done = R.VIEWERS[kind](obj, name)
        except R.StatusError as e:
            print(f"error: {e}", file=sys.stderr)
            return 1
        if msg != last:
            print(msg, end="")
            last = msg
        if done:
            return 0
        if not a.watch_status or time.time() > end:
            return 1
        await asyncio.sleep(0.2)


async def cmd_rollout(c, a):
    if not a.args:
        raise SystemExit("error: rollout needs a subcommand: status|history|undo|pause|resume")
    sub = a.args[0]
    ri, name, _ = _target(a, 1)
    ns = _ns(a, ri)
    res = _res(ri)
    if ri.kind in ("DaemonSet", "StatefulSet"):
        if sub in ("pause", "resume"):
            raise SystemExit(f"error: {ri.plural} \"{name}\" is not supported ({sub} works on deployments)")
        if sub in ("history", "undo", "status"):
            return await _rollout_history_based(c, a, sub, ri, name, ns, res)
    if sub == "pause" or sub == "resume":
        await c.patch(res, name, {"spec": {"paused": sub == "pause" or None}}, ns)
        print(f"{ri.kind.lower()}/{name} {'paused' if sub == 'pause' else 'resumed'}")
        return 0
    if sub == "history":
        d = await c.get(res, name, ns)
        rows = [["REVISION", "CHANGE-CAUSE"]]
        for r in sorted(await _owned_rs(c, d), key=_rev):
            rows.append([str(_rev(r)), ((r.get("metadata") or {}).get("annotations") or {}).get(CHANGE_CAUSE, "<none>")])
        print(f"{ri.kind.lower()}s \"{name}\"")
        print(printers.table(rows))
        return 0
    if sub == "undo":
        d = await c.get(res, name, ns)
        rss = sorted(await _owned_rs(c, d), key=_rev)
        want = a.to_revision
        if want == 0:
            if len(rss) < 2:
                raise SystemExit("error: no rollout history found")
            target = rss[-2]
        else:
            target = next((r for r in rss if _rev(r) == want), None)
            if target is None:
                raise SystemExit(f"error: unable to find specified revision {want} in history")
        tpl = json.loads(json.dumps((target.get("spec") or {}).get("template") or {}))
        ((tpl.get("metadata") or {}).get("labels") or {}).pop("pod-template-hash", None)
        await c.patch(res, name, {"spec": {"template": tpl}}, ns)
        print(f"{ri.kind.lower()}/{name} rolled back")
        return 0
    if sub == "status":
        return await _rollout_status(c, a, "Deployment", res, name, ns)
    raise SystemExit(f"error: unknown rollout subcommand {sub!r}")


# ------------------------------------------------------------------ generators
async def cmd_expose(c, a):
    ri, name, _ = _target(a)
    ns = _ns(a, ri)
    obj = await c.get(_res(ri), name, ns)
    spec = obj.get("spec") or {}
    if ri.kind == "Pod":
        sel = m.labels_of(obj)
    elif ri.kind == "Service":
        sel = spec.get("selector") or {}
    else:
        s = spec.get("selector") or {}
        sel = s.get("matchLabels", s) if isinstance(s, dict) else {}
        if isinstance(s, dict) and s.get("matchExpressions"):
            raise SystemExit("error: cannot expose an object whose selector uses matchExpressions")
    if not sel:
        raise SystemExit("error: couldn't find a selector to expose")
    port = a.port
    if port is None:
        ports = [p for ct in ((spec.get("template") or {}).get("spec") or spec).get("containers") or []
                 for p in ct.get("ports") or []]
        if not ports:
            raise SystemExit("error: couldn't find port via --port flag or introspection")
        port = ports[0]["containerPort"]
    svc_type = a.type if a.type not in (None, "strategic", "merge", "json") else "ClusterIP"   # --type is shared with patch
    svc = {"apiVersion": "v1", "kind": "Service",
           "metadata": {"name": a.name or name, "labels": dict(sel)},
           "spec": {"selector": dict(sel), "type": svc_type,
                    "ports": [{"port": int(port), "protocol": a.protocol,
                               "targetPort": int(a.target_port) if str(a.target_port or "").isdigit() else (a.target_port or int(port))}]}}
    out = await c.create(svc, ns)
    print(f"service/{m.name_of(out)} exposed")


async def cmd_set(c, a):
    if not a.args or a.args[0] != "image":
        raise SystemExit("error: supported: set image RESOURCE/NAME CONTAINER=IMAGE ...")
    ri, name, rest = _target(a, 1)
    ns = _ns(a, ri)
    obj = await c.get(_res(ri), name, ns)
    pairs = dict(x.split("=", 1) for x in rest)
    podspec = ((obj.get("spec") or {}).get("template") or {}).get("spec") if ri.kind != "Pod" else obj.get("spec")
    cs = []
    for key in ("initContainers", "containers"):
        for ct in (podspec or {}).get(key) or []:
            if ct["name"] in pairs or "*" in pairs:
                ct["image"] = pairs.get(ct["name"], pairs.get("*"))
                cs.append(ct["name"])
    missing = set(pairs) - set(cs) - {"*"}
    if missing:
        raise SystemExit(f"error: unable to find container named {sorted(missing)[0]!r}")
    patch = {"spec": {"template": {"spec": podspec}}} if ri.kind != "Pod" else {"spec": podspec}
    if a.record:
        patch["metadata"] = {"annotations": {CHANGE_CAUSE: "kubectl set image " + " ".join(a.args[1:])}}
    await c.patch(_res(ri), name, patch, ns)
    print(f"{ri.kind.lower()}/{name} image updated")


async def cmd_edit(c, a):
    ri, name, _ = _target(a)
    ns = _ns(a, ri)
    obj = await c.get(_res(ri), name, ns)
    editor = os.environ.get("KUBE_EDITOR") or os.environ.get("EDITOR") or "vi"
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
        f.write(dump_yaml(obj))
        path = f.name
    try:
        rc = subprocess.call(editor.split() + [path])
        if rc != 0:
            raise SystemExit(f"error: editor exited with {rc}")
        new = load_manifests(open(path).read())
    finally:
        os.unlink(path)
    if not new or new[0] == obj:
        print("Edit cancelled, no changes made.")
        return 0
    await c.update(new[0])
    print(f"{ri.kind.lower()}/{name} edited")


# ------------------------------------------------------------------ config / auth / certs
def _kubeconfig_path(a):
    return getattr(a, "kubeconfig", None) or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")


def _named(cfg, section, name, create=False, inner=None):
    lst = cfg.setdefault(section, []) if create else (cfg.get(section) or [])
    ent = next((x for x in lst if x.get("name") == name), None)
    if ent is None and create:
        ent = {"name": name, inner: {}}
        lst.append(ent)
    return ent


def _file_data(path):
    import base64
    with open(path, "rb") as f:
        return base64.b64encode(f.read()).decode()


def _set_path(cfg, path: str, value):
    """`kubectl config set PROPERTY_NAME VALUE`: dotted path where a list of named entries is
    addressed by name (clusters.<name>.server, users.<name>.token, contexts.<name>.namespace)."""
    parts = path.split(".")
    cur = cfg
    i = 0
    while i < len(parts) - 1:
        k = parts[i]
        if k in ("clusters", "users", "contexts") and i + 1 < len(parts):
            inner = {"clusters": "cluster", "users": "user", "contexts": "context"}[k]
            ent = _named(cfg if cur is cfg else cur, k, parts[i + 1], create=value is not None, inner=inner)
            if ent is None:
                raise SystemExit(f"error: {path}: no {inner} named {parts[i + 1]!r}")
            cur = ent.setdefault(inner, {})
            i += 2
            continue
        cur = cur.setdefault(k, {}) if value is not None else cur.get(k, {})
        i += 1
    if value is None:
        cur.pop(parts[-1], None)
    else:
        cur[parts[-1]] = value


def cmd_config_sync(a):
    """kubectl config (pkg/kubectl/cmd/config): view, current-context, get-contexts,
    get-clusters, use-context, set-context, set-cluster, set-credentials, set, unset,
    delete-context, delete-cluster, rename-context. Edits are written back to the kubeconfig."""
    import yaml
    path = _kubeconfig_path(a)
    sub = a.args[0] if a.args else "view"
    cfg = yaml.safe_load(open(path)) if os.path.exists(path) else {}
    cfg = cfg or {}
    cfg.setdefault("apiVersion", "v1")
    cfg.setdefault("kind", "Config")

    def save(msg):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            yaml.safe_dump(cfg, f, sort_keys=False)
        os.replace(tmp, path)
        print(msg)

    def arg(i):
        if len(a.args) <= i:
            raise SystemExit(f"error: config {sub}: missing argument")
        return a.args[i]

    if sub == "view":
        view = json.loads(json.dumps(cfg))
        if getattr(a, "minify", False) and view.get("current-context"):
            ctx = _named(view, "contexts", view["current-context"]) or {}
            cc = ctx.get("context") or {}
            view["contexts"] = [ctx] if ctx else []
            view["clusters"] = [x for x in view.get("clusters") or [] if x.get("name") == cc.get("cluster")]
            view["users"] = [x for x in view.get("users") or [] if x.get("name") == cc.get("user")]
        if not a.raw:
            for u in view.get("users") or []:
                for k in ("client-key-data", "token", "client-certificate-data", "password"):
                    if k in (u.get("user") or {}):
                        u["user"][k] = "REDACTED"
            for cl in view.get("clusters") or []:
                if "certificate-authority-data" in (cl.get("cluster") or {}):
                    cl["cluster"]["certificate-authority-data"] = "DATA+OMITTED"
        print(yaml.safe_dump(view, sort_keys=False), end="")
    elif sub == "current-context":
        cur = cfg.get("current-context")
        if not cur:
            raise SystemExit("error: current-context is not set")
        print(cur)
    elif sub == "get-contexts":
        rows = [["CURRENT", "NAME", "CLUSTER", "AUTHINFO", "NAMESPACE"]]
        for ctx in cfg.get("contexts") or []:
            if len(a.args) > 1 and ctx.get("name") not in a.args[1:]:
                continue
            cc = ctx.get("context") or {}
            rows.append(["*" if ctx.get("name") == cfg.get("current-context") else "", ctx.get("name", ""),
                         cc.get("cluster", ""), cc.get("user", ""), cc.get("namespace", "")])
        print(printers.table(rows))
    elif sub == "get-clusters":
        print("\n".join(["NAME"] + [x.get("name", "") for x in cfg.get("clusters") or []]))
    elif sub == "use-context":
        name = arg(1)
        if _named(cfg, "contexts", name) is None:
            raise SystemExit(f"error: no context exists with the name: {name!r}")
        cfg["current-context"] = name
        save(f'Switched to context "{name}".')
    elif sub == "set-context":
        name = cfg.get("current-context") if getattr(a, "current", False) else arg(1)
        if not name:
            raise SystemExit("error: no current context is set")
        new = _named(cfg, "contexts", name) is None
        ctx = _named(cfg, "contexts", name, create=True, inner="context")
        for kv in a.args[2:]:
            k, _, v = kv.lstrip("-").partition("=")
            ctx["context"][k] = v
        if getattr(a, "cfg_cluster", None):
            ctx["context"]["cluster"] = a.cfg_cluster
        if getattr(a, "user", None):      # --user is shared with the rolebinding generators (a list)
            ctx["context"]["user"] = a.user[-1]
        if a.namespace:
            ctx["context"]["namespace"] = a.namespace
        save(f'Context "{name}" {"created" if new else "modified"}.')
    elif sub == "set-cluster":
        name = arg(1)
        new = _named(cfg, "clusters", name) is None
        cl = _named(cfg, "clusters", name, create=True, inner="cluster")["cluster"]
        if a.server:
            cl["server"] = a.server
        if a.certificate_authority:
            if a.embed_certs:
                cl["certificate-authority-data"] = _file_data(a.certificate_authority)
                cl.pop("certificate-authority", None)
            else:
                cl["certificate-authority"] = os.path.abspath(a.certificate_authority)
        if a.insecure_skip_tls_verify is not None:
            cl["insecure-skip-tls-verify"] = a.insecure_skip_tls_verify == "true"
        save(f'Cluster "{name}" {"set" if new else "modified"}.')
    elif sub == "set-credentials":
        name = arg(1)
        new = _named(cfg, "users", name) is None
        u = _named(cfg, "users", name, create=True, inner="user")["user"]
        if getattr(a, "cfg_token", None):
            u["token"] = a.cfg_token
        if a.username:
            u["username"] = a.username
        if a.password:
            u["password"] = a.password
        for src, key in ((a.client_certificate, "client-certificate"), (a.client_key, "client-key")):
            if src:
                if a.embed_certs:
                    u[key + "-data"] = _file_data(src)
                    u.pop(key, None)
                else:
                    u[key] = os.path.abspath(src)
        save(f'User "{name}" {"set" if new else "modified"}.')
    elif sub == "set":
        _set_path(cfg, arg(1), arg(2))
        save(f'Property "{a.args[1]}" set.')
    elif sub == "unset":
        _set_path(cfg, arg(1), None)
        save(f'Property "{a.args[1]}" unset.')
    elif sub in ("delete-context", "delete-cluster"):
        section = "contexts" if sub == "delete-context" else "clusters"
        name = arg(1)
        lst = cfg.get(section) or []
        if not any(x.get("name") == name for x in lst):
            raise SystemExit(f"error: cannot delete {section[:-1]} {name}, not in {path}")
        cfg[section] = [x for x in lst if x.get("name") != name]
        if section == "contexts" and cfg.get("current-context") == name:
            print(f"warning: this removed your active context, use \"kubectl config use-context\" to select a different one")
        save(f"deleted {section[:-1]} {name} from {path}")
    elif sub == "rename-context":
        old, new_name = arg(1), arg(2)
        ctx = _named(cfg, "contexts", old)
        if ctx is None:
            raise SystemExit(f"error: cannot rename the context {old!r}, it's not in {path}")
        if _named(cfg, "contexts", new_name) is not None:
            raise SystemExit(f"error: cannot rename the context {old!r}, the context {new_name!r} already exists in {path}")
        ctx["name"] = new_name
        if cfg.get("current-context") == old:
            cfg["current-context"] = new_name
        save(f'Context "{old}" renamed to "{new_name}".')
    else:
        raise SystemExit(f"error: unknown config subcommand {sub!r}")
    return 0


async def auth_reconcile(c, a):
    """`kubectl auth reconcile -f FILE` (pkg/kubectl/cmd/auth/reconcile.go:153 RunReconcile):
    Roles / ClusterRoles gain missing rules (coverage-checked, api/rbac.py), bindings gain
    missing subjects and are re-created when their roleRef changed; objects annotated
    rbac.authorization.kubernetes.io/autoupdate=false are left alone. Nothing is removed."""
    from ..api import rbac
    from .main import _read_files
    if not a.filename:
        raise SystemExit('error: required flag(s) "filename" not set')
    kinds = {"Role": ("roles", rbac.reconcile_role), "ClusterRole": ("clusterroles", rbac.reconcile_role),
             "RoleBinding": ("rolebindings", rbac.reconcile_binding),
             "ClusterRoleBinding": ("clusterrolebindings", rbac.reconcile_binding)}
    for doc in _read_files(a.filename):
        kind = doc.get("kind")
        if kind not in kinds or not str(doc.get("apiVersion", "")).startswith("rbac.authorization.k8s.io/"):
            continue                                         # reconcile visits RBAC objects only
        res, fn = kinds[kind]
        res = res + ".rbac.authorization.k8s.io"
        name = m.name_of(doc)
        ns = (m.namespace_of(doc) or a.namespace or "default") if kind in ("Role", "RoleBinding") else ""
        if ns:
            doc.setdefault("metadata", {})["namespace"] = ns
            if await c.get_or_none("namespaces", ns) is None:   # RoleModifier creates the namespace
                await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
        for attempt in range(4):
            cur = await c.get_or_none(res, name, ns)
            r = fn(cur, doc)
            if r["protected"]:
                break
            try:
                if r["operation"] == rbac.RECREATE:
                    await c.delete(res, name, ns, uid=m.uid_of(cur))
                if r["operation"] in (rbac.CREATE, rbac.RECREATE):
                    obj = dict(r["object"])
                    obj.setdefault("metadata", {}).pop("resourceVersion", None)
                    obj["metadata"].pop("uid", None)
                    await c.create(obj, ns)
                elif r["operation"] == rbac.UPDATE:
                    await c.update(r["object"])
                break
            except m.StatusError as e:
                if e.code in (404, 409) and attempt < 3:        # changed under us: re-run
                    continue
                raise
        print(f"{kind.lower()}.rbac.authorization.k8s.io/{name} reconciled")
    return 0


async def cmd_auth(c, a):
    if a.args and a.args[0] == "reconcile":
        return await auth_reconcile(c, a)
    if len(a.args) < 3 or a.args[0] != "can-i":
        raise SystemExit("error: auth can-i VERB RESOURCE[/NAME] | auth reconcile -f FILE")
    verb, target = a.args[1], a.args[2]
    r, _, name = target.partition("/")
    ri = SCHEME.resolve(r)
    ra = {"verb": verb, "resource": ri.plural if ri else r, "group": ri.group if ri else "",
          "namespace": "" if (ri and not ri.namespaced) else (a.namespace or "default")}
    if name:
        ra["name"] = name
    if a.as_user:
        body = {"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
                "spec": {"resourceAttributes": ra, "user": a.as_user, "groups": a.as_group or []}}
        out = await c.request("POST", "/apis/authorization.k8s.io/v1/subjectaccessreviews", body=body)
    else:
        body = {"apiVersion": "authorization.k8s.io/v1", "kind": "SelfSubjectAccessReview", "spec": {"resourceAttributes": ra}}
        out = await c.request("POST", "/apis/authorization.k8s.io/v1/selfsubjectaccessreviews", body=body)
    ok = bool((out.get("status") or {}).get("allowed"))
    print("yes" if ok else "no")
    return 0 if ok else 1


async def cmd_certificate(c, a):
    if len(a.args) < 2 or a.args[0] not in ("approve", "deny"):
        raise SystemExit("error: certificate approve|deny NAME...")
    approve = a.args[0] == "approve"
    for name in a.args[1:]:
        csr = await c.get("certificatesigningrequests.certificates.k8s.io", name)
        conds = [x for x in (csr.get("status") or {}).get("conditions") or [] if x.get("type") not in ("Approved", "Denied")]
        conds.append({"type": "Approved" if approve else "Denied", "reason": "KubectlApprove" if approve else "KubectlDeny",
                      "message": f"This CSR was {'approved' if approve else 'denied'} by kubectl certificate {a.args[0]}.",
                      "lastUpdateTime": m.now_rfc3339()})
        csr.setdefault("status", {})["conditions"] = conds
        await c.request("PUT", f"/apis/certificates.k8s.io/v1beta1/certificatesigningrequests/{name}/approval", body=csr)
        print(f"certificatesigningrequest.certificates.k8s.io/{name} {'approved' if approve else 'denied'}")


# ------------------------------------------------------------------ data plane helpers
async def _pod_ip(c, ns, name) -> str:
    p = await c.get("pods", name, ns)
    ip = (p.get("status") or {}).get("podIP")
    if not ip:
        raise SystemExit(f"error: pod {name} has no IP yet")
    return ip


async def _pipe(r, w):
    try:
        while True:
            data = await r.read(65536)
            if not data:
                break
            w.write(data)
            await w.drain()
    except (ConnectionError, asyncio.CancelledError):
        pass
    finally:
        try:
            w.close()
        except Exception:
            pass


async def port_forward(c, ns, name, mappings, ready=None, stop=None):
    """Listen on 127.0.0.1:LOCAL for each LOCAL:REMOTE and splice to podIP:REMOTE."""
    ip = await _pod_ip(c, ns, name)
    servers = []
    for mp in mappings:
        local, _, remote = mp.partition(":")
        remote = int(remote or local)

        async def handle(r, w, remote=remote):
            try:
                pr, pw = await asyncio.open_connection(ip, remote)
            except OSError:
                w.close()
                return
            await asyncio.gather(_pipe(r, pw), _pipe(pr, w))

        srv = await asyncio.start_server(handle, "127.0.0.1", int(local or 0))
        servers.append(srv)
        print(f"Forwarding from 127.0.0.1:{srv.sockets[0].getsockname()[1]} -> {remote}", flush=True)
    if ready is not None:
        ready.set_result([s.sockets[0].getsockname()[1] for s in servers])
    try:
        await (stop.wait() if stop is not None else asyncio.Event().wait())
    finally:
        for s in servers:
            s.close()


async def cmd_port_forward(c, a):
    """Through the apiserver (pods/portforward WebSocket → kubelet → runtime), like the reference."""
    from ..client.stream import port_forward as api_port_forward
    ri, name, rest = _target(a) if "/" in a.args[0] else (SCHEME.resolve("pods"), a.args[0], a.args[1:])
    if ri.kind != "Pod":
        obj = await c.get(_res(ri), name, _ns(a, ri))
        sel = ((obj.get("spec") or {}).get("selector") or {})
        sel = sel.get("matchLabels", sel)
        pods, _ = await c.list("pods", _ns(a, ri), ",".join(f"{k}={v}" for k, v in sel.items()))
        running = [p for p in pods if (p.get("status") or {}).get("phase") == "Running"]
        if not running:
            raise SystemExit("error: no running pod found")
        name = m.name_of(running[0])
    from .main import stream_transport
    await api_port_forward(c, a.namespace or "default", name, rest, transport=stream_transport())


async def cmd_proxy(c, a):
    """Local HTTP proxy to the apiserver that adds the client's credentials (proxy.go)."""
    from aiohttp import web

    async def handle(req):
        body = await req.read()
        try:
            r = await c.request(req.method, req.rel_url.path, params=dict(req.query), body=body or None, raw=True,
                                content_type=req.headers.get("Content-Type", "application/json"))
        except m.StatusError as e:
            return web.json_response(e.status(), status=e.code)
        return web.Response(body=r, content_type="application/json")

    app = web.Application()
    app.router.add_route("*", "/{tail:.*}", handle)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", a.port or 8001)
    await site.start()
    print(f"Starting to serve on 127.0.0.1:{a.port or 8001}", flush=True)
    await asyncio.Event().wait()


async def cmd_cp(c, a):
    """Files move through exec streams (cat / sh -c 'cat > f'), as kubectl cp uses tar over exec."""
    from ..client.stream import exec_stream
    from .main import stream_transport
    if len(a.args) != 2:
        raise SystemExit("error: cp SRC DST (one side as [NAMESPACE/]POD:PATH)")
    src, dst = a.args
    errb = bytearray()
    if ":" in src:
        pod, _, path = src.partition(":")
        ns, _, pod = pod.rpartition("/")
        outb = bytearray()
        rc = await exec_stream(c, ns or a.namespace or "default", pod, ["cat", path], a.container,
                               on_stdout=outb.extend, on_stderr=errb.extend, transport=stream_transport())
        if rc != 0:
            raise SystemExit(f"error: {errb.decode(errors='replace').strip()}")
        with open(dst, "wb") as f:
            f.write(outb)
    else:
        pod, _, path = dst.partition(":")
        ns, _, pod = pod.rpartition("/")
        data = open(src, "rb").read()
        rc = await exec_stream(c, ns or a.namespace or "default", pod, ["sh", "-c", 'cat > "$0"', path], a.container,
                               stdin=data, on_stderr=errb.extend, transport=stream_transport())
        if rc != 0:
            raise SystemExit(f"error: {errb.decode(errors='replace').strip()}")


async def cmd_explain(c, a):
    """kubectl explain RESOURCE[.FIELD...] [--recursive] [--api-version] from the server's OpenAPI
    document (pkg/kubectl/explain: field lookup, model printer, recursive field printer)."""
    from ..api.openapi import explain
    from .main import openapi_definitions
    if not a.args:
        raise SystemExit("error: You must specify the type of resource to explain. Use \"kubectl api-resources\" for a complete list of supported resources.")
    parts = a.args[0].split(".")
    ri, fields = None, []
    for n in range(len(parts), 0, -1):      # the longest resource[.group] prefix (deployments.apps.spec…)
        ri = SCHEME.resolve(".".join(parts[:n]))
        if ri is not None:
            fields = parts[n:]
            break
    if ri is None:
        raise SystemExit(f'error: the server doesn\'t have a resource type "{parts[0]}"')
    api_version = a.explain_api_version or ri.api_version
    try:
        print(explain(await openapi_definitions(c), api_version, ri.kind, fields, recursive=a.recursive), end="")
    except KeyError as e:
        raise SystemExit(f"error: {e.args[0]}")


# ------------------------------------------------------------------ create <generator>
async def cmd_create_generator(c, a) -> bool:
    """`kubectl create <kind> NAME ...` generators; False when args are not a generator."""
    if not a.args:
        return False
    kind, rest = a.args[0], a.args[1:]
    ns = a.namespace or "default"

    if kind in ("namespace", "ns", "serviceaccount", "sa") and not rest:
        raise SystemExit("error: name must be specified")      # namespace.go / serviceaccount.go validate()
    if kind in ("namespace", "ns"):
        obj = {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": rest[0]}}
    elif kind in ("configmap", "cm"):
        from .generators import GenerateError, generate_config_map
        try:
            obj = generate_config_map(rest[0] if rest else "", a.from_file, a.from_literal, a.from_env_file, a.append_hash)
        except GenerateError as e:
            raise SystemExit(f"error: {e}") from None
    elif (kind == "secret" and rest and rest[0] in ("docker-registry", "tls")) or kind in ("service", "svc", "poddisruptionbudget", "pdb"):
        from .more import create_more
        obj = await create_more(c, a, kind, rest)
    elif kind == "secret":
        if not rest or rest[0] != "generic":
            raise SystemExit("error: create secret generic|docker-registry|tls NAME")
        from .generators import GenerateError, generate_secret
        try:
            obj = generate_secret(rest[1] if len(rest) > 1 else "", a.type or "", a.from_file, a.from_literal,
                                  a.from_env_file, a.append_hash)
        except GenerateError as e:
            raise SystemExit(f"error: {e}") from None
    elif kind in ("serviceaccount", "sa"):
        obj = {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": rest[0]}}
    elif kind in ("deployment", "deploy"):
        # deployment.go BaseDeploymentGenerator: a name and an image are required; the container is
        # named after the image's last path element without tag or digest
        if not rest:
            raise SystemExit("error: name must be specified")
        if not a.image:
            raise SystemExit("error: at least one image must be specified")
        cname = a.image.split("/")[-1]
        cname = cname.split(":")[0] if ":" in cname else cname.split("@")[0]
        ct = {"name": cname, "image": a.image}
        if a.gpus:
            ct["resources"] = {"limits": {"amd.com/gpu": str(a.gpus)}}
        obj = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": rest[0], "labels": {"app": rest[0]}},
               "spec": {"replicas": a.replicas if a.replicas is not None else 1, "selector": {"matchLabels": {"app": rest[0]}},
                        "template": {"metadata": {"labels": {"app": rest[0]}}, "spec": {"containers": [ct]}}}}
    elif kind == "job":
        ct = {"name": rest[0], "image": a.image or "busybox"}
        if a.command:
            ct["command"] = a.command
        obj = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": rest[0]},
               "spec": {"template": {"spec": {"restartPolicy": "Never", "containers": [ct]}}}}
    elif kind in ("priorityclass", "pc"):
        obj = {"apiVersion": "scheduling.k8s.io/v1alpha1", "kind": "PriorityClass", "metadata": {"name": rest[0]},
               "value": a.value, "globalDefault": a.global_default, "description": a.description}
    elif kind in ("quota", "resourcequota"):
        from .generators import GenerateError, generate_quota
        try:
            obj = generate_quota(rest[0] if rest else "", a.hard or "", getattr(a, "scopes", "") or "")
        except GenerateError as e:
            raise SystemExit(f"error: {e}") from None
    elif kind in ("role", "clusterrole"):
        from .generators import GenerateError, generate_role
        try:
            obj = generate_role("Role" if kind == "role" else "ClusterRole", rest[0] if rest else "",
                                [v for x in a.verb for v in x.split(",")], [r for x in a.resource for r in x.split(",")],
                                [n for x in a.resource_name for n in x.split(",")],
                                [u for x in a.non_resource_url for u in x.split(",")] if kind == "clusterrole" else [])
        except GenerateError as e:
            raise SystemExit(f"error: {e}") from None
    elif kind in ("rolebinding", "clusterrolebinding"):
        from .generators import GenerateError, generate_role_binding
        try:
            obj = generate_role_binding("RoleBinding" if kind == "rolebinding" else "ClusterRoleBinding",
                                        rest[0] if rest else "", a.role or "", a.clusterrole or "", a.user, a.group,
                                        a.serviceaccount)
        except GenerateError as e:
            raise SystemExit(f"error: {e}") from None
    else:
        return False
    ri = SCHEME.for_object(obj)
    if a.output:
        from .main import _emit
        _emit([obj], a, obj["kind"], single=True)
        return True
    out = await c.create(obj, ns if ri.namespaced else "")
    print(f"{obj['kind'].lower()}/{m.name_of(out)} created")
    return True


COMMANDS = {"rollout": cmd_rollout, "expose": cmd_expose, "set": cmd_set,
            "edit": cmd_edit, "auth": cmd_auth, "certificate": cmd_certificate,
            "port-forward": cmd_port_forward, "proxy": cmd_proxy, "cp": cmd_cp, "explain": cmd_explain}


def add_arguments(sp):
    sp.add_argument("--to-revision", type=int, default=0)
    sp.add_argument("--revision", type=int, default=0, help="rollout history: show this revision's template")
    sp.add_argument("--watch-status", type=lambda s: s != "false", default=True)
    sp.add_argument("--port", default=None)
    sp.add_argument("--target-port", default=None)
    sp.add_argument("--name", default=None)
    sp.add_argument("--protocol", default=None)
    sp.add_argument("--min", type=int, default=None)
    sp.add_argument("--max", type=int, default=None)
    sp.add_argument("--cpu-percent", type=int, default=None)
    sp.add_argument("--overwrite", action="store_true")
    sp.add_argument("--record", action="store_true")
    sp.add_argument("--force", action="store_true")
    sp.add_argument("--raw", action="store_true")
    sp.add_argument("--as", dest="as_user", default=None)
    sp.add_argument("--as-group", action="append", default=[])
    sp.add_argument("--from-literal", action="append", default=[])
    sp.add_argument("--from-file", action="append", default=[])
    sp.add_argument("--from-env-file", default="")
    sp.add_argument("--append-hash", action="store_true")
    sp.add_argument("--value", type=int, default=0)
    sp.add_argument("--global-default", action="store_true")
    sp.add_argument("--description", default="")
    sp.add_argument("--hard", default=None)
    sp.add_argument("--scopes", default=None)
    sp.add_argument("--verb", action="append", default=[])
    sp.add_argument("--resource", action="append", default=[])
    sp.add_argument("--resource-name", action="append", default=[])
    sp.add_argument("--non-resource-url", action="append", default=[])
    sp.add_argument("--user", action="append", default=[])
    sp.add_argument("--group", action="append", default=[])
    sp.add_argument("--serviceaccount", action="append", default=[])
    sp.add_argument("--clusterrole", default=None)
    sp.add_argument("--role", default=None)


__all__ = ["COMMANDS", "add_arguments", "cmd_config_sync", "cmd_create_generator", "port_forward", "sys"]


def _timeout_of(a, default: float = 30.0) -> float:
    t = getattr(a, "timeout", None)
    return default if t is None else float(t)
