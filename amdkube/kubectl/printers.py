"""Human-readable output for `kubectl get`: tables, custom columns, sorting.

Reference:
  * pkg/printers/internalversion/printers.go — the column definitions of every kind
    (AddHandlers :74-430) and their row functions (printPod, printNode, printService with
    getServiceExternalIP / makePortString, printIngress with formatHosts, printEndpoints with
    formatEndpoints, printHorizontalPodAutoscaler with formatHPAMetrics, printPersistentVolume,
    …); translateTimestamp / ShortHumanDuration (printers/common.go);
  * pkg/printers/humanreadable.go — headers upper-cased, wide-only columns (priority 1), the
    NAMESPACE prefix, `-L` label columns (headers from the key's last path segment) and the
    trailing LABELS column for --show-labels; a text/tabwriter(minwidth 10, tabwidth 4,
    padding 3) aligned table;
  * pkg/printers/customcolumn.go — `-o custom-columns=` / `custom-columns-file=`;
  * pkg/kubectl/sorting_printer.go — `--sort-by`: a JSONPath field, natural string order,
    numbers, timestamps; objects without the field first.

amdkube adds GPU columns the reference has no notion of: pods show `GPUS`
(count, device IDs with -o wide), nodes the GPU capacity / allocatable / healthy count and model.
"""
from __future__ import annotations

import functools
import json
import time

from ..api import meta as m
from ..api.helpers import get_condition, is_gpu_resource, pod_gpu_request
from . import jsonpath as jp

# ---------------------------------------------------------------------------- time
def short_human_duration(seconds: float) -> str:
    """printers.ShortHumanDuration."""
    s = int(seconds)
    if s < -1:
        return "<invalid>"
    if s < 0:
        return "0s"
    if s < 60:
        return f"{s}s"
    if s // 60 < 60:
        return f"{s // 60}m"
    h = s // 3600
    if h < 24:
        return f"{h}h"
    if h < 24 * 365:
        return f"{h // 24}d"
    return f"{h // 24 // 365}y"


def age(ts: str | None) -> str:
    """translateTimestamp: <unknown> for a zero time."""
    t = m.parse_time(ts)
    if t is None:
        return "<unknown>"
    return short_human_duration(time.time() - t)


# ---------------------------------------------------------------------------- tabwriter
def tabwrite(text: str, minwidth: int = 10, padding: int = 3) -> str:
    """Go text/tabwriter with the printer's settings (minwidth 10, padding 3, padchar ' ',
    no flags): tab-terminated cells aligned per column block; a line's last cell is not part
    of its column's width."""
    lines = [ln.split("\t") for ln in text.split("\n")]
    out: list[str] = []
    widths: list[int] = []

    def write_lines(l0, l1):
        for i in range(l0, l1):
            cells = lines[i]
            parts = []
            for j, c in enumerate(cells):
                parts.append(c)
                if j < len(widths) and j < len(cells) - 1:
                    parts.append(" " * (widths[j] - len(c)))
            out.append("".join(parts))

    def fmt(l0, l1):
        column = len(widths)
        this = l0
        while this < l1:
            if column >= len(lines[this]) - 1:
                this += 1
                continue
            write_lines(l0, this)
            l0 = this
            width = minwidth
            while this < l1 and column < len(lines[this]) - 1:
                width = max(width, len(lines[this][column]) + padding)
                this += 1
            widths.append(width)
            fmt(l0, this)
            widths.pop()
            l0 = this
        write_lines(l0, l1)
    fmt(0, len(lines))
    return "\n".join(out)


def table(rows: list[list]) -> str:
    """Rows of cells → the aligned table (no trailing newline)."""
    if not rows:
        return ""
    return tabwrite("\n".join("\t".join(str(c) for c in r) for r in rows))


# ---------------------------------------------------------------------------- helpers
def format_labels(labels: dict | None) -> str:
    """labels.FormatLabels: sorted k=v pairs, <none> when empty."""
    if not labels:
        return "<none>"
    return ",".join(f"{k}={labels[k]}" for k in sorted(labels))


def format_label_selector(sel: dict | None) -> str:
    """metav1.FormatLabelSelector."""
    from ..api.labels import SelectorError, selector_from_label_selector
    if sel is None:
        return "<none>"
    try:
        s = str(selector_from_label_selector(sel))
    except SelectorError:
        return "<error>"
    return s or "<none>"


def _cell(v) -> str:
    if v is None:
        return "<nil>"
    return v if isinstance(v, str) else jp.go_fmt(v)


def layout_containers(containers) -> tuple[str, str]:
    containers = containers or []
    return ",".join(c.get("name", "") for c in containers), ",".join(c.get("image", "") for c in containers)


def pod_gpu_ids(pod) -> list[str]:
    out = []
    for pres in (pod.get("spec") or {}).get("extendedResources") or []:
        out.extend(pres.get("assigned") or [])
    return out


def _term(s) -> dict:
    return (s or {}).get("terminated") or {}


def pod_status_reason(pod) -> tuple[str, int, int]:
    """printPod: (status reason, ready containers, restarts)."""
    st, sp = pod.get("status") or {}, pod.get("spec") or {}
    reason = st.get("reason") or st.get("phase") or ""
    restarts = ready = 0
    initializing = False
    inits = st.get("initContainerStatuses") or []
    for i, c in enumerate(inits):
        restarts += int(c.get("restartCount") or 0)
        s = c.get("state") or {}
        t = s.get("terminated")
        if t is not None and int(t.get("exitCode") or 0) == 0:
            continue
        if t is not None:
            if not t.get("reason"):
                reason = f"Init:Signal:{t['signal']}" if t.get("signal") else f"Init:ExitCode:{int(t.get('exitCode') or 0)}"
            else:
                reason = "Init:" + t["reason"]
        elif (s.get("waiting") or {}).get("reason") and s["waiting"]["reason"] != "PodInitializing":
            reason = "Init:" + s["waiting"]["reason"]
        else:
            reason = f"Init:{i}/{len(sp.get('initContainers') or [])}"
        initializing = True
        break
    if not initializing:
        restarts = 0
        for c in reversed(st.get("containerStatuses") or []):
            restarts += int(c.get("restartCount") or 0)
            s = c.get("state") or {}
            w, t = s.get("waiting"), s.get("terminated")
            if w is not None and w.get("reason"):
                reason = w["reason"]
            elif t is not None and t.get("reason"):
                reason = t["reason"]
            elif t is not None:
                reason = f"Signal:{t['signal']}" if t.get("signal") else f"ExitCode:{int(t.get('exitCode') or 0)}"
            elif c.get("ready") and s.get("running") is not None:
                ready += 1
    md = pod.get("metadata") or {}
    if md.get("deletionTimestamp") and st.get("reason") == "NodeLost":
        reason = "Unknown"
    elif md.get("deletionTimestamp"):
        reason = "Terminating"
    return reason, ready, restarts


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


def node_roles(node) -> list[str]:
    roles = set()
    for k, v in m.labels_of(node).items():
        if k.startswith("node-role.kubernetes.io/") and k[len("node-role.kubernetes.io/"):]:
            roles.add(k[len("node-role.kubernetes.io/"):])
        elif k == "kubernetes.io/role" and v:
            roles.add(v)
    return sorted(roles)


def node_status(node) -> str:
    ready = get_condition(node, "Ready")
    status = [] if ready is None else (["Ready"] if ready.get("status") == "True" else ["NotReady"])
    if not status:
        status = ["Unknown"]
    if (node.get("spec") or {}).get("unschedulable"):
        status.append("SchedulingDisabled")
    return ",".join(status)


LOAD_BALANCER_WIDTH = 16


def load_balancer_status(lb: dict | None, wide: bool) -> str:
    ips = sorted({i.get("ip") or i.get("hostname") for i in (lb or {}).get("ingress") or []
                  if i.get("ip") or i.get("hostname")})
    r = ",".join(ips)
    if not wide and len(r) > LOAD_BALANCER_WIDTH:
        r = r[:LOAD_BALANCER_WIDTH - 3] + "..."
    return r


def service_external_ip(svc, wide) -> str:
    sp = svc.get("spec") or {}
    t = sp.get("type") or "ClusterIP"
    ext = sp.get("externalIPs") or []
    if t in ("ClusterIP", "NodePort"):
        return ",".join(ext) if ext else "<none>"
    if t == "LoadBalancer":
        lb = load_balancer_status((svc.get("status") or {}).get("loadBalancer"), wide)
        if ext:
            return ",".join(([*lb.split(",")] if lb else []) + ext)
        return lb or "<pending>"
    if t == "ExternalName":
        return sp.get("externalName", "")
    return "<unknown>"


def port_string(ports) -> str:
    out = []
    for p in ports or []:
        proto = p.get("protocol") or "TCP"
        out.append(f"{p.get('port')}:{p['nodePort']}/{proto}" if p.get("nodePort") else f"{p.get('port')}/{proto}")
    return ",".join(out)


def _join_host_port(ip, port) -> str:
    return f"[{ip}]:{port}" if ":" in (ip or "") else f"{ip}:{port}"


def format_endpoints(ep, ports=None) -> str:
    subsets = ep.get("subsets") or []
    if not subsets:
        return "<none>"
    lst, more, count, mx = [], False, 0, 3
    for ss in subsets:
        for port in ss.get("ports") or []:
            if ports is None or port.get("name", "") in ports:
                for addr in ss.get("addresses") or []:
                    if len(lst) == mx:
                        more = True
                    if not more:
                        lst.append(_join_host_port(addr.get("ip"), port.get("port")))
                    count += 1
    ret = ",".join(lst)
    return f"{ret} + {count - mx} more..." if more else ret


def format_hosts(rules) -> str:
    lst, more, mx = [], False, 3
    for r in rules or []:
        if len(lst) == mx:
            more = True
        if not more and r.get("host"):
            lst.append(r["host"])
    if not lst:
        return "*"
    ret = ",".join(lst)
    return f"{ret} + {len(rules) - mx} more..." if more else ret


def format_hpa_metrics(hpa) -> str:
    """formatHPAMetrics over the autoscaling/v1 object: the v1 CPU target plus the metrics the
    v2 fields carry in the autoscaling.alpha.kubernetes.io annotations."""
    sp, st = hpa.get("spec") or {}, hpa.get("status") or {}
    ann = m.annotations_of(hpa)
    specs, statuses = [], []
    try:
        specs = json.loads(ann.get("autoscaling.alpha.kubernetes.io/metrics") or "[]")
        statuses = json.loads(ann.get("autoscaling.alpha.kubernetes.io/current-metrics") or "[]")
    except ValueError:
        pass
    if sp.get("targetCPUUtilizationPercentage") is not None or not specs:
        specs = [{"type": "Resource", "resource": {"name": "cpu",
                                                   "targetAverageUtilization": sp.get("targetCPUUtilizationPercentage")}}] + specs
        statuses = [{"type": "Resource", "resource": {"currentAverageUtilization": st.get("currentCPUUtilizationPercentage")}}
                    if st.get("currentCPUUtilizationPercentage") is not None else {}] + statuses
        if sp.get("targetCPUUtilizationPercentage") is None and len(specs) == 1:
            specs, statuses = [], []
    if not specs:
        return "<none>"
    lst = []
    for i, s in enumerate(specs):
        cur = statuses[i] if i < len(statuses) else {}
        t = s.get("type")
        if t == "Pods":
            c = ((cur.get("pods") or {}).get("currentAverageValue")) or "<unknown>"
            lst.append(f"{c} / {(s.get('pods') or {}).get('targetAverageValue')}")
        elif t == "Object":
            c = ((cur.get("object") or {}).get("currentValue")) or "<unknown>"
            lst.append(f"{c} / {(s.get('object') or {}).get('targetValue')}")
        elif t == "Resource":
            r = s.get("resource") or {}
            if r.get("targetAverageValue") is not None:
                c = ((cur.get("resource") or {}).get("currentAverageValue")) or "<unknown>"
                lst.append(f"{c} / {r['targetAverageValue']}")
            else:
                cu = (cur.get("resource") or {}).get("currentAverageUtilization")
                c = f"{cu}%" if cu is not None else "<unknown>"
                tgt = f"{r['targetAverageUtilization']}%" if r.get("targetAverageUtilization") is not None else "<auto>"
                lst.append(f"{c} / {tgt}")
        else:
            lst.append("<unknown type>")
    if len(lst) > 2:
        return ", ".join(lst[:2]) + f" + {len(lst) - 2} more..."
    return ", ".join(lst)


ACCESS_MODES = (("ReadWriteOnce", "RWO"), ("ReadOnlyMany", "ROX"), ("ReadWriteMany", "RWX"))


def access_modes_string(modes) -> str:
    """helper.GetAccessModesAsString."""
    modes = modes or []
    return ",".join(short for full, short in ACCESS_MODES if full in modes)


def pv_class(pv) -> str:
    ann = m.annotations_of(pv).get("volume.beta.kubernetes.io/storage-class")
    return ann if ann is not None else ((pv.get("spec") or {}).get("storageClassName") or "")


def subjects_strings(subjects):
    users, groups, sas = [], [], []
    for s in subjects or []:
        k = s.get("kind")
        if k == "User":
            users.append(s.get("name", ""))
        elif k == "Group":
            groups.append(s.get("name", ""))
        elif k == "ServiceAccount":
            sas.append(f"{s.get('namespace', '')}/{s.get('name', '')}")
    return users, groups, sas


def csr_status(csr) -> str:
    approved = denied = False
    for c in (csr.get("status") or {}).get("conditions") or []:
        if c.get("type") == "Approved":
            approved = True
        elif c.get("type") == "Denied":
            denied = True
    s = "Denied" if denied else ("Approved" if approved else "Pending")
    if (csr.get("status") or {}).get("certificate"):
        s += ",Issued"
    return s


# ---------------------------------------------------------------------------- per-kind rows
def _ts(o):
    return age((o.get("metadata") or {}).get("creationTimestamp"))


def _pod_row(p, wide):
    reason, ready, restarts = pod_status_reason(p)
    total = len((p.get("spec") or {}).get("containers") or [])
    n = pod_gpu_request(p)
    row = [m.name_of(p), f"{ready}/{total}", reason, restarts, str(n) if n else "-", _ts(p)]
    if wide:
        ids = pod_gpu_ids(p)
        row += [(p.get("status") or {}).get("podIP") or "<none>", (p.get("spec") or {}).get("nodeName") or "<none>",
                ",".join(ids) if ids else "<none>"]
    return row


def _node_row(n, wide):
    st = n.get("status") or {}
    info = st.get("nodeInfo") or {}
    cap, alloc, healthy, model = node_gpu_summary(n)
    row = [m.name_of(n), node_status(n), ",".join(node_roles(n)) or "<none>", _ts(n), info.get("kubeletVersion", ""),
           cap, alloc, healthy, model]
    if wide:
        ext = next((a.get("address") for a in st.get("addresses") or [] if a.get("type") == "ExternalIP"), "<none>")
        row += [ext, info.get("osImage") or "<unknown>", info.get("kernelVersion") or "<unknown>",
                info.get("containerRuntimeVersion") or "<unknown>"]
    return row


def _tpl_containers(o, *path):
    spec = o
    for k in path:
        spec = (spec or {}).get(k) or {}
    return layout_containers((spec or {}).get("containers"))


def _workload(extra_fn, tpl_path=("spec", "template", "spec"), selector=lambda o: format_label_selector(
        (o.get("spec") or {}).get("selector")), containers=True):
    def row(o, wide):
        r = [m.name_of(o)] + extra_fn(o) + [_ts(o)]
        if wide and containers:
            names, images = _tpl_containers(o, *tpl_path)
            r += [names, images] + ([selector(o)] if selector else [])
        return r
    return row


def _sp(o):
    return o.get("spec") or {}


def _st(o):
    return o.get("status") or {}


def _svc_row(s, wide):
    sp = _sp(s)
    row = [m.name_of(s), sp.get("type") or "ClusterIP", sp.get("clusterIP") or "<none>", service_external_ip(s, wide),
           port_string(sp.get("ports")) or "<none>", _ts(s)]
    if wide:
        row.append(format_labels(sp.get("selector")))
    return row


def _binding_row(b, wide):
    row = [m.name_of(b), _ts(b)]
    if wide:
        ref = b.get("roleRef") or {}
        users, groups, sas = subjects_strings(b.get("subjects"))
        row += [f"{ref.get('kind', '')}/{ref.get('name', '')}", ", ".join(users), ", ".join(groups), ", ".join(sas)]
    return row


def _pdb_row(p, wide):
    sp = _sp(p)
    mn = sp.get("minAvailable")
    mx = sp.get("maxUnavailable")
    return [m.name_of(p), "N/A" if mn is None else str(mn), "N/A" if mx is None else str(mx),
            _st(p).get("disruptionsAllowed", _st(p).get("podDisruptionsAllowed", 0)), _ts(p)]


def _pv_row(pv, wide):
    sp, st = _sp(pv), _st(pv)
    cr = sp.get("claimRef")
    claim = f"{cr.get('namespace', '')}/{cr.get('name', '')}" if cr else ""
    return [m.name_of(pv), (sp.get("capacity") or {}).get("storage", "0"), access_modes_string(sp.get("accessModes")),
            sp.get("persistentVolumeReclaimPolicy", ""), st.get("phase", ""), claim, pv_class(pv), st.get("reason", ""),
            _ts(pv)]


def _pvc_row(c, wide):
    sp, st = _sp(c), _st(c)
    phase = "Terminating" if (c.get("metadata") or {}).get("deletionTimestamp") else st.get("phase", "")
    cap = modes = ""
    if sp.get("volumeName"):
        modes = access_modes_string(st.get("accessModes"))
        cap = (st.get("capacity") or {}).get("storage", "0")
    ann = m.annotations_of(c).get("volume.beta.kubernetes.io/storage-class")
    cls = ann if ann is not None else (sp.get("storageClassName") or "")
    return [m.name_of(c), phase, sp.get("volumeName", ""), cap, modes, cls, _ts(c)]


def _cron_row(cj, wide):
    sp, st = _sp(cj), _st(cj)
    last = age(st["lastScheduleTime"]) if st.get("lastScheduleTime") else "<none>"
    susp = sp.get("suspend")
    row = [m.name_of(cj), sp.get("schedule", ""), "<unset>" if susp is None else jp.go_fmt(bool(susp)),
           len(st.get("active") or []), last, _ts(cj)]
    if wide:
        jt = ((sp.get("jobTemplate") or {}).get("spec") or {})
        names, images = layout_containers(((jt.get("template") or {}).get("spec") or {}).get("containers"))
        row += [names, images, format_label_selector(jt.get("selector"))]
    return row


def _event_row(e, wide):
    io, src = e.get("involvedObject") or {}, e.get("source") or {}
    source = src.get("component", "") + (f", {src['host']}" if src.get("host") else "")
    return [age(e.get("lastTimestamp")), age(e.get("firstTimestamp")), e.get("count", 0), m.name_of(e),
            io.get("kind", ""), io.get("fieldPath", ""), e.get("type", ""), e.get("reason", ""), source,
            e.get("message", "")]


def _sc_row(sc, wide):
    name = m.name_of(sc)
    ann = m.annotations_of(sc)
    if ann.get("storageclass.kubernetes.io/is-default-class") == "true" or \
            ann.get("storageclass.beta.kubernetes.io/is-default-class") == "true":
        name += " (default)"
    return [name, sc.get("provisioner", ""), _ts(sc)]


def _cr_row(r, wide):
    ref = next((o for o in (r.get("metadata") or {}).get("ownerReferences") or [] if o.get("controller")), None)
    return [m.name_of(r), f"{ref.get('kind')}/{ref.get('name')}" if ref else "<none>", r.get("revision", 0), _ts(r)]


def _cs_row(c, wide):
    status, msg, err = "Unknown", "", ""
    for cond in c.get("conditions") or []:
        if cond.get("type") == "Healthy":
            status = "Healthy" if cond.get("status") == "True" else "Unhealthy"
            msg, err = cond.get("message", ""), cond.get("error", "")
            break
    return [m.name_of(c), status, msg, err]


def _psp_row(p, wide):
    sp = _sp(p)
    return [m.name_of(p), jp.go_fmt(bool(sp.get("privileged"))), jp.go_fmt(sp.get("allowedCapabilities") or []),
            (sp.get("seLinux") or {}).get("rule", ""), (sp.get("runAsUser") or {}).get("rule", ""),
            (sp.get("fsGroup") or {}).get("rule", ""), (sp.get("supplementalGroups") or {}).get("rule", ""),
            jp.go_fmt(bool(sp.get("readOnlyRootFilesystem"))), jp.go_fmt(sp.get("volumes") or [])]


def _meta_row(o, wide):
    return [m.name_of(o), _ts(o)]


W = 1   # a wide-only column (TableColumnDefinition Priority 1)
CONTAINER_COLS = [("Containers", W), ("Images", W), ("Selector", W)]
PRINTERS: dict[str, tuple[list, object]] = {
    "Pod": ([("Name", 0), ("Ready", 0), ("Status", 0), ("Restarts", 0), ("GPUs", 0), ("Age", 0), ("IP", W), ("Node", W),
             ("GPU IDs", W)], _pod_row),
    "PodTemplate": ([("Name", 0), ("Containers", 0), ("Images", 0), ("Pod Labels", 0)],
                    lambda o, w: [m.name_of(o), *_tpl_containers(o, "template", "spec"),
                                  format_labels(((o.get("template") or {}).get("metadata") or {}).get("labels"))]),
    "PodDisruptionBudget": ([("Name", 0), ("Min Available", 0), ("Max Unavailable", 0), ("Allowed Disruptions", 0),
                             ("Age", 0)], _pdb_row),
    "ReplicationController": ([("Name", 0), ("Desired", 0), ("Current", 0), ("Ready", 0), ("Age", 0)] + CONTAINER_COLS,
                              _workload(lambda o: [_sp(o).get("replicas", 0), _st(o).get("replicas", 0),
                                                   _st(o).get("readyReplicas", 0)],
                                        selector=lambda o: format_labels(_sp(o).get("selector")))),
    "ReplicaSet": ([("Name", 0), ("Desired", 0), ("Current", 0), ("Ready", 0), ("Age", 0)] + CONTAINER_COLS,
                   _workload(lambda o: [_sp(o).get("replicas", 0), _st(o).get("replicas", 0), _st(o).get("readyReplicas", 0)])),
    "DaemonSet": ([("Name", 0), ("Desired", 0), ("Current", 0), ("Ready", 0), ("Up-to-date", 0), ("Available", 0),
                   ("Node Selector", 0), ("Age", 0)] + CONTAINER_COLS,
                  _workload(lambda o: [_st(o).get("desiredNumberScheduled", 0), _st(o).get("currentNumberScheduled", 0),
                                       _st(o).get("numberReady", 0), _st(o).get("updatedNumberScheduled", 0),
                                       _st(o).get("numberAvailable", 0),
                                       format_labels((((_sp(o).get("template") or {}).get("spec")) or {}).get("nodeSelector"))])),
    "Job": ([("Name", 0), ("Desired", 0), ("Successful", 0), ("Age", 0)] + CONTAINER_COLS,
            _workload(lambda o: [str(_sp(o)["completions"]) if _sp(o).get("completions") is not None else "<none>",
                                 _st(o).get("succeeded", 0)])),
    "CronJob": ([("Name", 0), ("Schedule", 0), ("Suspend", 0), ("Active", 0), ("Last Schedule", 0), ("Age", 0)]
                + CONTAINER_COLS, _cron_row),
    "Service": ([("Name", 0), ("Type", 0), ("Cluster-IP", 0), ("External-IP", 0), ("Port(s)", 0), ("Age", 0),
                 ("Selector", W)], _svc_row),
    "Ingress": ([("Name", 0), ("Hosts", 0), ("Address", 0), ("Ports", 0), ("Age", 0)],
                lambda o, w: [m.name_of(o), format_hosts(_sp(o).get("rules")),
                              load_balancer_status(_st(o).get("loadBalancer"), w),
                              "80, 443" if _sp(o).get("tls") else "80", _ts(o)]),
    "StatefulSet": ([("Name", 0), ("Desired", 0), ("Current", 0), ("Age", 0), ("Containers", W), ("Images", W)],
                    _workload(lambda o: [_sp(o).get("replicas", 0), _st(o).get("replicas", 0)], selector=None)),
    "Endpoints": ([("Name", 0), ("Endpoints", 0), ("Age", 0)], lambda o, w: [m.name_of(o), format_endpoints(o), _ts(o)]),
    "Node": ([("Name", 0), ("Status", 0), ("Roles", 0), ("Age", 0), ("Version", 0), ("GPU", 0), ("GPU-Alloc", 0),
              ("GPU-Healthy", 0), ("GPU-Model", 0), ("External-IP", W), ("OS-Image", W), ("Kernel-Version", W),
              ("Container-Runtime", W)], _node_row),
    "Event": ([("Last Seen", 0), ("First Seen", 0), ("Count", 0), ("Name", 0), ("Kind", 0), ("Subobject", 0),
               ("Type", 0), ("Reason", 0), ("Source", 0), ("Message", 0)], _event_row),
    "Namespace": ([("Name", 0), ("Status", 0), ("Age", 0)], lambda o, w: [m.name_of(o), _st(o).get("phase", ""), _ts(o)]),
    "Secret": ([("Name", 0), ("Type", 0), ("Data", 0), ("Age", 0)],
               lambda o, w: [m.name_of(o), o.get("type", ""), len(o.get("data") or {}), _ts(o)]),
    "ServiceAccount": ([("Name", 0), ("Secrets", 0), ("Age", 0)],
                       lambda o, w: [m.name_of(o), len(o.get("secrets") or []), _ts(o)]),
    "PersistentVolume": ([("Name", 0), ("Capacity", 0), ("Access Modes", 0), ("Reclaim Policy", 0), ("Status", 0),
                          ("Claim", 0), ("StorageClass", 0), ("Reason", 0), ("Age", 0)], _pv_row),
    "PersistentVolumeClaim": ([("Name", 0), ("Status", 0), ("Volume", 0), ("Capacity", 0), ("Access Modes", 0),
                               ("StorageClass", 0), ("Age", 0)], _pvc_row),
    "ComponentStatus": ([("Name", 0), ("Status", 0), ("Message", 0), ("Error", 0)], _cs_row),
    "Deployment": ([("Name", 0), ("Desired", 0), ("Current", 0), ("Up-to-date", 0), ("Available", 0), ("Age", 0)]
                   + CONTAINER_COLS,
                   _workload(lambda o: [_sp(o).get("replicas", 0), _st(o).get("replicas", 0), _st(o).get("updatedReplicas", 0),
                                        _st(o).get("availableReplicas", 0)])),
    "HorizontalPodAutoscaler": ([("Name", 0), ("Reference", 0), ("Targets", 0), ("MinPods", 0), ("MaxPods", 0),
                                 ("Replicas", 0), ("Age", 0)],
                                lambda o, w: [m.name_of(o), f"{(_sp(o).get('scaleTargetRef') or {}).get('kind', '')}/"
                                                            f"{(_sp(o).get('scaleTargetRef') or {}).get('name', '')}",
                                              format_hpa_metrics(o),
                                              str(_sp(o)["minReplicas"]) if _sp(o).get("minReplicas") is not None else "<unset>",
                                              _sp(o).get("maxReplicas", 0), _st(o).get("currentReplicas", 0), _ts(o)]),
    "ConfigMap": ([("Name", 0), ("Data", 0), ("Age", 0)],
                  lambda o, w: [m.name_of(o), len(o.get("data") or {}) + len(o.get("binaryData") or {}), _ts(o)]),
    "PodSecurityPolicy": ([("Name", 0), ("Data", 0), ("Caps", 0), ("SELinux", 0), ("RunAsUser", 0), ("FsGroup", 0),
                           ("SupGroup", 0), ("ReadOnlyRootFs", 0), ("Volumes", 0)], _psp_row),
    "NetworkPolicy": ([("Name", 0), ("Pod-Selector", 0), ("Age", 0)],
                      lambda o, w: [m.name_of(o), format_label_selector(_sp(o).get("podSelector") or {}), _ts(o)]),
    "RoleBinding": ([("Name", 0), ("Age", 0), ("Role", W), ("Users", W), ("Groups", W), ("ServiceAccounts", W)],
                    _binding_row),
    "ClusterRoleBinding": ([("Name", 0), ("Age", 0), ("Role", W), ("Users", W), ("Groups", W), ("ServiceAccounts", W)],
                           _binding_row),
    "CertificateSigningRequest": ([("Name", 0), ("Age", 0), ("Requestor", 0), ("Condition", 0)],
                                  lambda o, w: [m.name_of(o), _ts(o), _sp(o).get("username", ""), csr_status(o)]),
    "StorageClass": ([("Name", 0), ("Provisioner", 0), ("Age", 0)], _sc_row),
    "ControllerRevision": ([("Name", 0), ("Controller", 0), ("Revision", 0), ("Age", 0)], _cr_row),
}
META_COLUMNS = [("Name", 0), ("Age", 0)]


def columns_for(kind: str, wide: bool) -> list[str]:
    cols, _ = PRINTERS.get(kind, (META_COLUMNS, None))
    return [n.upper() for n, prio in cols if wide or not prio]


def rows_for(obj, kind: str, wide: bool) -> list:
    cols, fn = PRINTERS.get(kind, (META_COLUMNS, _meta_row))
    return [_cell(c) for c in fn(obj, wide)]


def label_headers(label_columns) -> list[str]:
    return [c.split("/")[-1].upper() for c in label_columns or []]


def print_table(objs, kind: str, wide: bool = False, with_namespace: bool = False, show_labels: bool = False,
                label_columns=(), no_headers: bool = False, with_kind: bool | str = False) -> str:
    """printRowsForHandlerEntry + printRows: the aligned table of one kind; `with_kind` prefixes
    each name with that resource name (True: the kind, lower-cased)."""
    rows = []
    if not no_headers:
        head = columns_for(kind, wide) + label_headers(label_columns) + (["LABELS"] if show_labels else [])
        rows.append((["NAMESPACE"] if with_namespace else []) + head)
    for o in objs:
        cells = rows_for(o, kind, wide)
        if with_kind:
            cells[0] = f"{with_kind if isinstance(with_kind, str) else kind.lower()}/{cells[0]}"
        labels = m.labels_of(o)
        cells += [labels.get(c, "") for c in label_columns or []]
        if show_labels:
            cells.append(format_labels(labels))
        rows.append(([m.namespace_of(o)] if with_namespace else []) + cells)
    return table(rows)


# kept for the GPU-aware callers (and older tests)
def pods_table(items, wide=False, all_ns=False) -> str:
    return print_table(items, "Pod", wide, all_ns)


def nodes_table(items, wide=False) -> str:
    return print_table(items, "Node", wide)


def generic_table(items, kind, all_ns=False) -> str:
    return print_table(items, kind, False, all_ns)


def describe(obj, events=()) -> str:
    from .describe import describe as _describe
    return _describe(obj, events)


# ---------------------------------------------------------------------------- custom columns
class CustomColumnsPrinter:
    """customcolumn.go: (header, JSONPath) columns; an empty result prints <none>, several
    results are comma-joined."""

    def __init__(self, columns: list[tuple[str, str]], no_headers: bool = False):
        self.columns, self.no_headers = columns, no_headers

    @classmethod
    def from_spec(cls, spec: str, no_headers: bool = False) -> "CustomColumnsPrinter":
        if not spec:
            raise ValueError("custom-columns format specified but no custom columns given")
        cols = []
        for part in spec.split(","):
            cs = part.split(":")
            if len(cs) != 2:
                raise ValueError(f"unexpected custom-columns spec: {part}, expected <header>:<json-path-expr>")
            cols.append((cs[0], jp.relaxed_expression(cs[1])))
        return cls(cols, no_headers)

    @classmethod
    def from_template(cls, text: str) -> "CustomColumnsPrinter":
        lines = text.split("\n")
        if not lines or not lines[0].strip() and len(lines) < 2:
            raise ValueError("invalid template, missing header line. Expected format is one line of space separated "
                             "headers, one line of space separated column specs.")
        if len(lines) < 2:
            raise ValueError("invalid template, missing spec line. Expected format is one line of space separated "
                             "headers, one line of space separated column specs.")
        headers, specs = lines[0].split(), lines[1].split()
        if len(headers) != len(specs):
            raise ValueError(f"number of headers ({len(headers)}) and field specifications ({len(specs)}) don't match")
        return cls([(h, jp.relaxed_expression(s)) for h, s in zip(headers, specs)])

    def print(self, objs) -> str:
        lines = []
        if not self.no_headers:
            lines.append("\t".join(h for h, _ in self.columns))
        parsers = [jp.JSONPath(f"column{i}", allow_missing_keys=True).parse(spec) for i, (_, spec) in enumerate(self.columns)]
        for o in objs:
            cells = []
            for p in parsers:
                values = p.find_results(o)
                vs = [] if values and values[0] else ["<none>"]
                for arr in values:
                    vs.extend(jp.go_fmt(v) for v in arr)
                cells.append(",".join(vs))
            lines.append("\t".join(cells))
        return tabwrite("\n".join(lines) + "\n")


# ---------------------------------------------------------------------------- sorting
def natural_less(a: str, b: str) -> bool:
    """vbom.ml/util/sortorder NaturalLess: digit runs compare as numbers."""
    i = j = 0
    while i < len(a) and j < len(b):
        ca, cb = a[i], b[j]
        da, db = ca.isdigit(), cb.isdigit()
        if da != db:
            return da
        if not da:
            if ca != cb:
                return ca < cb
            i += 1
            j += 1
            continue
        while i < len(a) and a[i] == "0":
            i += 1
        while j < len(b) and b[j] == "0":
            j += 1
        ni, nj = i, j
        while i < len(a) and a[i].isdigit():
            i += 1
        while j < len(b) and b[j].isdigit():
            j += 1
        if i - ni != j - nj:
            return i - ni < j - nj
        if a[ni:i] != b[nj:j]:
            return a[ni:i] < b[nj:j]
        if ni != nj:
            return ni < nj
    return len(a) < len(b)


def _is_time(s) -> bool:
    return isinstance(s, str) and len(s) >= 20 and s[4] == "-" and s[10] == "T" and m.parse_time(s) is not None


def _less(x, y) -> bool:
    """sorting_printer.go isLess over decoded JSON (timestamps compared as times)."""
    if isinstance(x, bool) or isinstance(y, bool):
        raise ValueError(f"unsortable type: {type(x).__name__}")
    if isinstance(x, (int, float)) and isinstance(y, (int, float)):
        return x < y
    if isinstance(x, str) and isinstance(y, str):
        if _is_time(x) and _is_time(y):
            return m.parse_time(x) < m.parse_time(y)
        return natural_less(x, y)
    if isinstance(x, list) and isinstance(y, list):
        for a, b in zip(x, y):
            if not _less(a, b):
                return False
        return True
    raise ValueError(f"unsortable type: {type(x).__name__}")


def sort_objects(objs: list, field: str) -> list:
    """SortObjects + RuntimeSort: the objects ordered by the JSONPath field; objects without it
    sort first; an error when no object has the field."""
    field = jp.relaxed_expression(field)
    parser = jp.JSONPath("sorting", allow_missing_keys=True).parse(field)
    values = []
    found = False
    for o in objs:
        r = parser.find_results(o)
        v = r[0][0] if r and r[0] else None
        found = found or (r and bool(r[0]))
        values.append((v, bool(r and r[0])))
    if objs and not found:
        raise ValueError(f"couldn't find any field with path {json.dumps(field)} in the list of objects")

    def cmp(a, b):
        (va, ha), (vb, hb) = a[1], b[1]
        if not ha:
            return -1
        if not hb:
            return 1
        if _less(va, vb):
            return -1
        if _less(vb, va):
            return 1
        return 0
    order = sorted(zip(objs, values), key=functools.cmp_to_key(cmp))
    return [o for o, _ in order]
