"""kubectl get.

Reference: pkg/kubectl/cmd/resource/get.go RunGet (:230-418) —
  * arguments: `TYPE[,TYPE...] [NAME...]`, `TYPE/NAME...`, -f files, and the `all` category
    (categories.go legacyUserResources: pods, replicationcontrollers, services, statefulsets,
    horizontalpodautoscalers, jobs, cronjobs, daemonsets, deployments, replicasets);
  * errors of single objects (NotFound) do not stop the others (ContinueOnError) and are
    reported after the output; --ignore-not-found drops NotFound;
  * generic printers (json, yaml, name, jsonpath, go-template, custom-columns) get one List of
    everything, or the object itself when exactly one was named;
  * the table printer prints one table per resource type, a blank line (on stderr) between
    them; names carry the resource's short form (`po/x`, `svc/y`: kubectl.go
    ResourceShortFormFor) when several types were asked for, or with --show-kind;
  * lists hide finished pods unless --show-all (DefaultResourceFilterFunc), and
    PrintFilterCount says "No resources found." (or "..., use --show-all to see completed
    objects.") when nothing is shown.
"""
from __future__ import annotations

import sys

from ..api import meta as m
from ..api.scheme import SCHEME

ALL = ("pods", "replicationcontrollers", "services", "statefulsets", "horizontalpodautoscalers", "jobs", "cronjobs",
       "daemonsets", "deployments", "replicasets")
SHORT_FORMS = {"configmaps": "cm", "componentstatuses": "cs", "endpoints": "ep", "events": "ev", "limitranges": "limits",
               "nodes": "no", "namespaces": "ns", "pods": "po", "persistentvolumeclaims": "pvc", "persistentvolumes": "pv",
               "resourcequotas": "quota", "replicationcontrollers": "rc", "replicasets": "rs", "serviceaccounts": "sa",
               "services": "svc", "horizontalpodautoscalers": "hpa", "certificatesigningrequests": "csr",
               "poddisruptionbudgets": "pdb", "deployments": "deploy", "daemonsets": "ds", "ingresses": "ing",
               "networkpolicies": "netpol", "podsecuritypolicies": "psp"}
GENERIC = ("json", "yaml", "name")


def _is_generic(o: str) -> bool:
    return o in GENERIC or o.startswith(("jsonpath", "go-template", "template", "custom-columns"))


def expand(args: list[str]) -> tuple[list[tuple], bool, bool]:
    """[(ri, [names] | None)], whether several types were requested (MultipleTypesRequested),
    and whether the arguments named single items."""
    if not args:
        raise SystemExit("error: You must specify the type of resource to get. Valid resource types include:\n\n"
                         "    * all\n    * pods (aka 'po')\n    * services (aka 'svc')\n    * deployments (aka 'deploy')\n"
                         "    * nodes (aka 'no')\n    ...")
    groups: list[tuple] = []

    def resolve(t):
        if t == "all":
            return [SCHEME.resolve(r) for r in ALL]
        ri = SCHEME.resolve(t)
        if ri is None:
            raise SystemExit(f'error: the server doesn\'t have a resource type "{t}"')
        return [ri]
    if all("/" in a for a in args):
        seen = {}
        for a in args:
            t, n = a.split("/", 1)
            for ri in resolve(t):
                if ri.plural not in seen:
                    seen[ri.plural] = (ri, [])
                    groups.append(seen[ri.plural])
                seen[ri.plural][1].append(n)
        return groups, len(groups) > 1, True
    types = args[0].split(",")
    names = args[1:] or None
    if names and any("/" in n for n in names):
        raise SystemExit("error: there is no need to specify a resource type as a separate argument when passing "
                         "arguments in resource/name form (e.g. 'kubectl get resource/<resource_name>' instead of "
                         "'kubectl get resource resource/<resource_name>'")
    for t in types:
        for ri in resolve(t):
            groups.append((ri, list(names) if names else None))
    return groups, len(types) > 1 or "all" in types, bool(names)


async def cmd_get(c, a):
    from . import printers
    from .main import _emit, _ns
    try:
        await c.discover()
    except Exception:
        pass
    if a.filename and not a.args:
        from .main import _read_files
        groups, index = [], {}
        for d in _read_files(a.filename):
            ri = SCHEME.for_object(d)
            if ri.plural not in index:
                index[ri.plural] = (ri, [])
                groups.append(index[ri.plural])
            index[ri.plural][1].append(m.name_of(d))
        multiple, singles = len(groups) > 1, True
    else:
        groups, multiple, singles = expand(list(a.args))
    errors: list[str] = []
    fetched: list[tuple] = []          # (ri, [objs], list resourceVersion, resource, namespace)
    for ri, names in groups:
        ns = _ns(a, ri)
        res = ri.plural if not ri.group else f"{ri.plural}.{ri.group}"
        objs, rv = [], ""
        if names:
            for n in names:
                try:
                    objs.append(await c.get(res, n, ns))
                except m.StatusError as e:
                    if not (a.ignore_not_found and m.is_not_found(e)):
                        errors.append(f"Error from server ({e.reason}): {e.message}")
        else:
            objs, rv = await c.list(res, ns, a.selector, a.field_selector)
        for o in objs:
            o.setdefault("kind", ri.kind)
            o.setdefault("apiVersion", ri.api_version)
        fetched.append((ri, objs, rv, res, ns))
    o = a.output or ""
    all_objs = [x for _, objs, *_ in fetched for x in objs]
    if _is_generic(o):
        single = singles and len(all_objs) == 1 and len(groups) == 1 and len(groups[0][1] or []) == 1
        if all_objs or not errors:
            _emit(all_objs, a, groups[0][0].kind if len(groups) == 1 else None, single=single)
    else:
        shown = hidden = 0
        first = True
        show_kind = multiple or getattr(a, "show_kind", False)
        for ri, objs, *_ in fetched:
            vis = objs
            if ri.kind == "Pod" and not singles and not getattr(a, "show_all", False):
                vis = [p for p in objs if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")]
            hidden += len(objs) - len(vis)
            if not vis:
                continue
            if not first and not getattr(a, "no_headers", False):
                print("", file=sys.stderr)
            first = False
            shown += len(vis)
            label_cols = []
            for spec in getattr(a, "label_columns", None) or []:
                label_cols += [x.strip() for x in spec.split(",") if x.strip()]
            print(printers.print_table(vis, ri.kind, wide=o == "wide",
                                       with_namespace=getattr(a, "all_namespaces", False) and ri.namespaced,
                                       show_labels=getattr(a, "show_labels", False), label_columns=label_cols,
                                       no_headers=getattr(a, "no_headers", False),
                                       with_kind=SHORT_FORMS.get(ri.plural, ri.plural) if show_kind else False))
        found = len(all_objs)
        if not errors and not a.ignore_not_found and found <= hidden:
            print("No resources found." if found == 0 else "No resources found, use --show-all to see completed objects.",
                  file=sys.stderr)
    for e in errors:
        print(e, file=sys.stderr)
    if a.watch and fetched:
        ri, _, rv, res, ns = fetched[0]
        async for _typ, obj in c.watch(res, ns, rv, a.selector, a.field_selector):
            obj.setdefault("kind", ri.kind)
            _emit([obj], a, ri.kind, with_headers=False)
    return 1 if errors else 0
