"""Human-readable printers for `kubectl get` / `describe`.

Reference printers live in pkg/printers/internalversion (7,649 LoC) and have no support for
the fork's ExtendedResources (zero references). amdkube adds GPU columns:
pods show `GPUS` (count and assigned device IDs with -o wide), nodes show `GPU` capacity /
allocatable / healthy and the GPU model.
"""
from __future__ import annotations

import time

from ..api import meta as m
from ..api.helpers import get_condition, is_gpu_resource, pod_gpu_request


def age(ts: str | None) -> str:
    t = m.parse_time(ts)
    if t is None:
        return "<unknown>"
    s = max(0, int(time.time() - t))
    if s < 120:
        return f"{s}s"
    if s < 7200:
        return f"{s // 60}m"
    if s < 172800:
        return f"{s // 3600}h"
    return f"{s // 86400}d"


def table(rows: list[list[str]]) -> str:
    if not rows:
        return ""
    widths = [max(len(str(r[i])) for r in rows) for i in range(len(rows[0]))]
    return "\n".join("   ".join(str(c).ljust(widths[i]) for i, c in enumerate(r)).rstrip() for r in rows)


def pod_gpu_ids(pod) -> list[str]:
    out = []
    for pres in (pod.get("spec") or {}).get("extendedResources") or []:
        out.extend(pres.get("assigned") or [])
    return out


def pod_status_reason(pod) -> str:
    st = pod.get("status") or {}
    if (pod.get("metadata") or {}).get("deletionTimestamp"):
        return "Terminating"
    reason = st.get("reason") or st.get("phase") or "Pending"
    for cs in st.get("initContainerStatuses") or []:
        s = cs.get("state") or {}
        if "terminated" in s and s["terminated"].get("exitCode") == 0:
            continue
        if "waiting" in s:
            return f"Init:{s['waiting'].get('reason', 'Waiting')}"
        if "running" in s:
            return "Init:Running"
    for cs in st.get("containerStatuses") or []:
        s = cs.get("state") or {}
        if "waiting" in s and s["waiting"].get("reason"):
            reason = s["waiting"]["reason"]
        elif "terminated" in s and s["terminated"].get("reason"):
            reason = s["terminated"]["reason"]
    return reason


def pods_table(items, wide=False, all_ns=False) -> str:
    head = (["NAMESPACE"] if all_ns else []) + ["NAME", "READY", "STATUS", "RESTARTS", "GPUS", "AGE"]
    if wide:
        head += ["IP", "NODE", "GPU IDS"]
    rows = [head]
    for p in items:
        st = p.get("status") or {}
        cs = st.get("containerStatuses") or []
        ready = sum(1 for c in cs if c.get("ready"))
        total = len((p.get("spec") or {}).get("containers") or [])
        restarts = sum(int(c.get("restartCount", 0)) for c in cs)
        n = pod_gpu_request(p)
        row = ([m.namespace_of(p)] if all_ns else []) + [m.name_of(p), f"{ready}/{total}", pod_status_reason(p), str(restarts),
                                                         str(n) if n else "-", age((p.get("metadata") or {}).get("creationTimestamp"))]
        if wide:
            ids = pod_gpu_ids(p)
            row += [st.get("podIP") or "<none>", (p.get("spec") or {}).get("nodeName") or "<none>", ",".join(ids) if ids else "<none>"]
        rows.append(row)
    return table(rows)


def node_gpu_summary(node) -> tuple[str, str, str, str]:
    """Totals over amd.com/gpu and the partition resources; model shows the partition mode
    when the node's GPUs are partitioned (e.g. MI355X/CPX)."""
    st = node.get("status") or {}
    cap = sum(int(v) for r, v in (st.get("capacity") or {}).items() if is_gpu_resource(r))
    alloc = sum(int(v) for r, v in (st.get("allocatable") or {}).items() if is_gpu_resource(r))
    devs = {}
    for r, dom in ((st.get("extendedResources") or {}).items()):
        if is_gpu_resource(r):
            devs.update((dom or {}).get("resources") or {})
    healthy = sum(1 for d in devs.values() if d.get("health") == "Healthy")
    attrs = next((d.get("attributes") or {} for d in devs.values()), {})
    model = attrs.get("amd.com/gpu-type") or "-"
    if attrs.get("amd.com/partition-id") is not None and attrs.get("amd.com/partition"):
        model += "/" + attrs["amd.com/partition"]
    return str(cap), str(alloc), str(healthy), model


def nodes_table(items, wide=False) -> str:
    head = ["NAME", "STATUS", "ROLES", "AGE", "VERSION", "GPU", "GPU-ALLOC", "GPU-HEALTHY", "GPU-MODEL"]
    if wide:
        head += ["INTERNAL-IP", "CONTAINER-RUNTIME"]
    rows = [head]
    for n in items:
        ready = get_condition(n, "Ready")
        status = "Ready" if ready and ready.get("status") == "True" else ("NotReady" if ready else "Unknown")
        if (n.get("spec") or {}).get("unschedulable"):
            status += ",SchedulingDisabled"
        roles = ",".join(k.split("/", 1)[1] for k in m.labels_of(n) if k.startswith("node-role.kubernetes.io/")) or "<none>"
        cap, alloc, healthy, model = node_gpu_summary(n)
        st = n.get("status") or {}
        row = [m.name_of(n), status, roles, age((n.get("metadata") or {}).get("creationTimestamp")),
               (st.get("nodeInfo") or {}).get("kubeletVersion", ""), cap, alloc, healthy, model]
        if wide:
            ip = next((a["address"] for a in st.get("addresses") or [] if a.get("type") == "InternalIP"), "<none>")
            row += [ip, (st.get("nodeInfo") or {}).get("containerRuntimeVersion", "")]
        rows.append(row)
    return table(rows)


def generic_table(items, kind, all_ns=False) -> str:
    head = (["NAMESPACE"] if all_ns else []) + ["NAME"]
    extra = []
    if kind in ("Deployment", "ReplicaSet", "DaemonSet", "Job"):
        extra = {"Deployment": ["READY", "UP-TO-DATE", "AVAILABLE"], "ReplicaSet": ["DESIRED", "CURRENT", "READY"],
                 "DaemonSet": ["DESIRED", "CURRENT", "READY"], "Job": ["COMPLETIONS"]}[kind]
    elif kind == "Namespace":
        extra = ["STATUS"]
    elif kind == "Event":
        extra = ["TYPE", "REASON", "OBJECT", "MESSAGE"]
    rows = [head + extra + ["AGE"]]
    for o in items:
        st, sp = o.get("status") or {}, o.get("spec") or {}
        ex = []
        if kind == "Deployment":
            ex = [f"{st.get('readyReplicas', 0)}/{sp.get('replicas', 0)}", str(st.get("updatedReplicas", 0)), str(st.get("availableReplicas", 0))]
        elif kind == "ReplicaSet":
            ex = [str(sp.get("replicas", 0)), str(st.get("replicas", 0)), str(st.get("readyReplicas", 0))]
        elif kind == "DaemonSet":
            ex = [str(st.get("desiredNumberScheduled", 0)), str(st.get("currentNumberScheduled", 0)), str(st.get("numberReady", 0))]
        elif kind == "Job":
            ex = [f"{st.get('succeeded', 0)}/{sp.get('completions', 1)}"]
        elif kind == "Namespace":
            ex = [st.get("phase", "")]
        elif kind == "Event":
            io = o.get("involvedObject") or {}
            ex = [o.get("type", ""), o.get("reason", ""), f"{io.get('kind', '').lower()}/{io.get('name', '')}", (o.get("message") or "")[:80]]
        ts = (o.get("metadata") or {}).get("creationTimestamp")
        rows.append(([m.namespace_of(o)] if all_ns else []) + [m.name_of(o)] + ex + [age(ts)])
    return table(rows)


def describe(obj, events=()) -> str:
    """kubectl describe: key fields + the fork's device details + events."""
    md, sp, st = obj.get("metadata") or {}, obj.get("spec") or {}, obj.get("status") or {}
    out = [f"Name:         {md.get('name')}"]
    if md.get("namespace"):
        out.append(f"Namespace:    {md['namespace']}")
    out.append(f"Labels:       {', '.join(f'{k}={v}' for k, v in (md.get('labels') or {}).items()) or '<none>'}")
    out.append(f"Annotations:  {', '.join(f'{k}={v[:60]}' for k, v in (md.get('annotations') or {}).items()) or '<none>'}")
    kind = obj.get("kind")
    if kind == "Pod":
        out.append(f"Node:         {sp.get('nodeName') or '<none>'}")
        out.append(f"Status:       {pod_status_reason(obj)}")
        if st.get("message"):
            out.append(f"Message:      {st['message']}")
        out.append("Extended Resources:")
        for pres in sp.get("extendedResources") or []:
            lim = (pres.get("resources") or {}).get("limits") or {}
            sel = ", ".join(f"{r.get('key')} {r.get('operator')} {r.get('values') or ''}" for r in (pres.get("affinity") or {}).get("required") or [])
            out.append(f"  {pres.get('name')}: {', '.join(f'{k}={v}' for k, v in lim.items())}")
            out.append(f"    Affinity:  {sel or '<none>'}")
            out.append(f"    Assigned:  {', '.join(pres.get('assigned') or []) or '<not yet scheduled>'}")
        out.append("Containers:")
        for c in sp.get("containers") or []:
            out.append(f"  {c['name']}:")
            out.append(f"    Image:     {c.get('image')}")
            if c.get("extendedResourceRequests"):
                out.append(f"    Extended Resource Requests: {', '.join(c['extendedResourceRequests'])}")
            lim = (c.get("resources") or {}).get("limits")
            if lim:
                out.append(f"    Limits:    {', '.join(f'{k}={v}' for k, v in lim.items())}")
        out.append("Conditions:")
        for c in st.get("conditions") or []:
            out.append(f"  {c.get('type'):<16}{c.get('status')}")
    elif kind == "Node":
        out.append("Capacity:")
        for k, v in (st.get("capacity") or {}).items():
            out.append(f"  {k}: {v}")
        out.append("Allocatable:")
        for k, v in (st.get("allocatable") or {}).items():
            out.append(f"  {k}: {v}")
        out.append("Extended Resources:")
        for r, dom in (st.get("extendedResources") or {}).items():
            out.append(f"  {r}:")
            for did, d in sorted((dom.get("resources") or {}).items()):
                a = d.get("attributes") or {}
                out.append(f"    {did}  {d.get('health')}  type={a.get('amd.com/gpu-type', '-')} mem={a.get('amd.com/gpu-memory', '-')}MiB "
                           f"numa={a.get('amd.com/numa-node', '-')} partition={a.get('amd.com/partition', '-')}")
        out.append("Conditions:")
        for c in st.get("conditions") or []:
            out.append(f"  {c.get('type'):<16}{c.get('status'):<8}{c.get('reason', '')}")
        if sp.get("taints"):
            taints = ", ".join("%s=%s:%s" % (t.get("key"), t.get("value", ""), t.get("effect")) for t in sp["taints"])
            out.append(f"Taints:       {taints}")
    else:
        if sp:
            out.append(f"Spec:         {str(sp)[:400]}")
        if st:
            out.append(f"Status:       {str(st)[:400]}")
    out.append("Events:")
    if not events:
        out.append("  <none>")
    for e in events:
        out.append(f"  {e.get('type', ''):<8}{e.get('reason', ''):<20}{age(e.get('lastTimestamp'))} ago  {e.get('source', {}).get('component', '')}  {e.get('message', '')}")
    return "\n".join(out)
