"""`kubectl describe`: a describer per kind, in the reference's layout.

Reference: pkg/printers/internalversion/describe.go — the PrefixWriter levels (2 spaces each)
through a tabwriter (minwidth 0, padding 2); printLabelsMultiline / printAnnotationsMultiline;
DescribePodTemplate and describeContainers (ports, command, state, last state, ready, restart
count, limits/requests, probes, environment, mounts); DescribeEvents; describePod,
describeNode, describeDeployment (replica summary, strategy, conditions, Old/NewReplicaSets),
describeReplicaSet / describeReplicationController / describeDaemonSet / describeStatefulSet
(pod status counts), describeJob, describeCronJob, describeService (per-port target ports
and endpoints), describeEndpoints, describePersistentVolume (with its source),
describePersistentVolumeClaim (Mounted By), describeNamespace (resource quotas and limit
ranges), describeConfigMap, describeSecret (sizes only), describeServiceAccount,
describeIngress, describeHorizontalPodAutoscaler, describePodDisruptionBudget,
describeStorageClass, describeNetworkPolicy, describeQuota, describeLimitRange; a generic
describer for every other kind.

The fork's additions are kept: the pod's extended resources (request, affinity, assigned
device IDs) and the node's per-device health, type, memory, NUMA node and partition.
"""
from __future__ import annotations

import base64
import time

from ..api import meta as m
from .printers import (access_modes_string, age, format_endpoints, format_hosts, format_label_selector,
                       format_labels, load_balancer_status, node_gpu_summary, pod_status_reason, pv_class, tabwrite)


def _rfc1123z(ts: str | None) -> str:
    t = m.parse_time(ts)
    if t is None:
        return "<unset>"
    return time.strftime("%a, %d %b %Y %H:%M:%S +0000", time.gmtime(t))


class PrefixWriter:
    def __init__(self):
        self.lines: list[str] = []

    def write(self, level: int, text: str):
        self.lines.append("  " * level + text)

    def render(self) -> str:
        return tabwrite("\n".join(self.lines), minwidth=0, padding=2).rstrip("\n")


def _multiline(w: PrefixWriter, title: str, items: dict | None, level: int = 0):
    """printLabelsMultiline: the first entry on the title line, the rest below, sorted."""
    if not items:
        w.write(level, f"{title}:\t<none>")
        return
    keys = sorted(items)
    w.write(level, f"{title}:\t{keys[0]}={items[keys[0]]}")
    for k in keys[1:]:
        w.write(level, f"\t{k}={items[k]}")


def _header(w, o, with_ns=True):
    w.write(0, f"Name:\t{m.name_of(o)}")
    if with_ns and m.namespace_of(o):
        w.write(0, f"Namespace:\t{m.namespace_of(o)}")


def _controlled_by(o) -> str:
    ref = next((r for r in (o.get("metadata") or {}).get("ownerReferences") or [] if r.get("controller")), None)
    return f"{ref.get('kind')}/{ref.get('name')}" if ref else ""


def describe_events(w: PrefixWriter, events):
    """DescribeEvents."""
    if not events:
        w.write(0, "Events:\t<none>")
        return
    w.write(0, "Events:")
    w.write(1, "Type\tReason\tAge\tFrom\tMessage")
    w.write(1, "----\t------\t----\t----\t-------")
    for e in sorted(events, key=lambda e: e.get("lastTimestamp") or e.get("firstTimestamp") or ""):
        src = e.get("source") or {}
        frm = src.get("component", "") + (f", {src['host']}" if src.get("host") else "")
        interval = age(e.get("lastTimestamp"))
        if int(e.get("count") or 1) > 1:
            interval = f"{age(e.get('lastTimestamp'))} (x{e['count']} over {age(e.get('firstTimestamp'))})"
        w.write(1, f"{e.get('type', '')}\t{e.get('reason', '')}\t{interval}\t{frm}\t{(e.get('message') or '').strip()}")


def _ports(ports) -> str:
    return ", ".join(f"{p.get('containerPort')}/{p.get('protocol') or 'TCP'}" for p in ports or [])


def _probe(p) -> str:
    attrs = (f"delay={p.get('initialDelaySeconds', 0)}s timeout={p.get('timeoutSeconds', 1)}s "
             f"period={p.get('periodSeconds', 10)}s #success={p.get('successThreshold', 1)} "
             f"#failure={p.get('failureThreshold', 3)}")
    if "exec" in p:
        return f"exec {p['exec'].get('command')} {attrs}"
    if "httpGet" in p:
        h = p["httpGet"]
        scheme = (h.get("scheme") or "HTTP").lower()
        return f"http-get {scheme}://{h.get('host', '')}:{h.get('port')}{h.get('path', '')} {attrs}"
    if "tcpSocket" in p:
        return f"tcp-socket {p['tcpSocket'].get('host', '')}:{p['tcpSocket'].get('port')} {attrs}"
    return f"unknown {attrs}"


def _state(w, name, state):
    state = state or {}
    if "running" in state:
        w.write(2, f"{name}:\tRunning")
        w.write(3, f"Started:\t{_rfc1123z(state['running'].get('startedAt'))}")
    elif "terminated" in state:
        t = state["terminated"]
        w.write(2, f"{name}:\tTerminated")
        if t.get("reason"):
            w.write(3, f"Reason:\t{t['reason']}")
        if t.get("message"):
            w.write(3, f"Message:\t{t['message']}")
        w.write(3, f"Exit Code:\t{t.get('exitCode', 0)}")
        if t.get("signal"):
            w.write(3, f"Signal:\t{t['signal']}")
        w.write(3, f"Started:\t{_rfc1123z(t.get('startedAt'))}")
        w.write(3, f"Finished:\t{_rfc1123z(t.get('finishedAt'))}")
    else:
        w.write(2, f"{name}:\tWaiting")
        reason = (state.get("waiting") or {}).get("reason")
        if reason:
            w.write(3, f"Reason:\t{reason}")


def describe_containers(w: PrefixWriter, label: str, containers, statuses=()):
    by_name = {s.get("name"): s for s in statuses or []}
    w.write(0, f"{label}:")
    for c in containers or []:
        st = by_name.get(c.get("name"))
        w.write(1, f"{c.get('name')}:")
        if st is not None:
            w.write(2, f"Container ID:\t{st.get('containerID', '')}")
        w.write(2, f"Image:\t{c.get('image', '')}")
        if st is not None:
            w.write(2, f"Image ID:\t{st.get('imageID', '')}")
        ps = _ports(c.get("ports"))
        w.write(2, (f"Ports:\t{ps}" if "," in ps else f"Port:\t{ps or '<none>'}"))
        if c.get("command"):
            w.write(2, "Command:")
            for x in c["command"]:
                w.write(3, x)
        if c.get("args"):
            w.write(2, "Args:")
            for x in c["args"]:
                w.write(3, x)
        if st is not None:
            _state(w, "State", st.get("state"))
            if (st.get("lastState") or {}).get("terminated"):
                _state(w, "Last State", st.get("lastState"))
            w.write(2, f"Ready:\t{'True' if st.get('ready') else 'False'}")
            w.write(2, f"Restart Count:\t{st.get('restartCount', 0)}")
        res = c.get("resources") or {}
        for title, key in (("Limits", "limits"), ("Requests", "requests")):
            if res.get(key):
                w.write(2, f"{title}:")
                for k in sorted(res[key]):
                    w.write(3, f"{k}:\t{res[key][k]}")
        for title, key in (("Liveness", "livenessProbe"), ("Readiness", "readinessProbe")):
            if c.get(key):
                w.write(2, f"{title}:\t{_probe(c[key])}")
        if c.get("extendedResourceRequests"):
            w.write(2, f"Extended Resource Requests:\t{', '.join(c['extendedResourceRequests'])}")
        env = c.get("env") or []
        if not env and not c.get("envFrom"):
            w.write(2, "Environment:\t<none>")
        else:
            w.write(2, "Environment:")
            for e in env:
                if "valueFrom" in e:
                    vf = e["valueFrom"]
                    src = next(iter(vf))
                    ref = vf[src]
                    desc = {"fieldRef": lambda r: f"({r.get('apiVersion', 'v1')}:{r.get('fieldPath')})",
                            "resourceFieldRef": lambda r: f"{r.get('containerName', '')} ({r.get('resource')})",
                            "secretKeyRef": lambda r: f"<set to the key '{r.get('key')}' in secret '{r.get('name')}'>",
                            "configMapKeyRef": lambda r: f"<set to the key '{r.get('key')}' of config map '{r.get('name')}'>",
                            }.get(src, lambda r: "<unknown>")(ref)
                    w.write(3, f"{e.get('name')}:\t{desc}\tOptional: {'true' if ref.get('optional') else 'false'}"
                            if src in ("secretKeyRef", "configMapKeyRef") else f"{e.get('name')}:\t{desc}")
                else:
                    w.write(3, f"{e.get('name')}:\t{e.get('value', '')}")
            for ef in c.get("envFrom") or []:
                kind, ref = ("ConfigMap", ef["configMapRef"]) if "configMapRef" in ef else ("Secret", ef.get("secretRef") or {})
                w.write(3, f"{ref.get('name')}\t{kind}\tOptional: {'true' if ref.get('optional') else 'false'}")
        mounts = c.get("volumeMounts") or []
        if not mounts:
            w.write(2, "Mounts:\t<none>")
        else:
            w.write(2, "Mounts:")
            for vm in sorted(mounts, key=lambda x: x.get("mountPath", "")):
                flags = ["ro" if vm.get("readOnly") else "rw"]
                if vm.get("subPath"):
                    flags.append(f"path=\"{vm['subPath']}\"")
                w.write(3, f"{vm.get('mountPath')} from {vm.get('name')} ({','.join(flags)})")


def describe_volumes(w: PrefixWriter, volumes, level=0):
    if not volumes:
        w.write(level, "Volumes:\t<none>")
        return
    w.write(level, "Volumes:")
    for v in volumes:
        w.write(level + 1, f"{v.get('name')}:")
        kind = next((k for k in v if k != "name"), None)
        src = v.get(kind) or {}
        if kind == "emptyDir":
            w.write(level + 2, "Type:\tEmptyDir (a temporary directory that shares a pod's lifetime)")
            w.write(level + 2, f"Medium:\t{src.get('medium', '')}")
        elif kind == "hostPath":
            w.write(level + 2, "Type:\tHostPath (bare host directory volume)")
            w.write(level + 2, f"Path:\t{src.get('path', '')}")
            w.write(level + 2, f"HostPathType:\t{src.get('type', '')}")
        elif kind == "secret":
            w.write(level + 2, "Type:\tSecret (a volume populated by a Secret)")
            w.write(level + 2, f"SecretName:\t{src.get('secretName', '')}")
            w.write(level + 2, f"Optional:\t{'true' if src.get('optional') else 'false'}")
        elif kind == "configMap":
            w.write(level + 2, "Type:\tConfigMap (a volume populated by a ConfigMap)")
            w.write(level + 2, f"Name:\t{src.get('name', '')}")
            w.write(level + 2, f"Optional:\t{'true' if src.get('optional') else 'false'}")
        elif kind == "persistentVolumeClaim":
            w.write(level + 2, "Type:\tPersistentVolumeClaim (a reference to a PersistentVolumeClaim in the same namespace)")
            w.write(level + 2, f"ClaimName:\t{src.get('claimName', '')}")
            w.write(level + 2, f"ReadOnly:\t{'true' if src.get('readOnly') else 'false'}")
        elif kind == "downwardAPI":
            w.write(level + 2, "Type:\tDownwardAPI (a volume populated by information about the pod)")
            w.write(level + 2, "Items:")
            for it in src.get("items") or []:
                f = (it.get("fieldRef") or {}).get("fieldPath") or (it.get("resourceFieldRef") or {}).get("resource")
                w.write(level + 3, f"{f} -> {it.get('path')}")
        else:
            w.write(level + 2, f"Type:\t{kind} (unknown)")
            for k in sorted(src):
                w.write(level + 2, f"{k}:\t{src[k]}")


def describe_pod_template(w: PrefixWriter, tpl):
    """DescribePodTemplate."""
    tpl = tpl or {}
    w.write(0, "Pod Template:")
    md, sp = tpl.get("metadata") or {}, tpl.get("spec") or {}
    _multiline(w, "Labels", md.get("labels"), 1)
    if md.get("annotations"):
        _multiline(w, "Annotations", md.get("annotations"), 1)
    if sp.get("serviceAccountName"):
        w.write(1, f"Service Account:\t{sp['serviceAccountName']}")
    if sp.get("initContainers"):
        sub = PrefixWriter()
        describe_containers(sub, "Init Containers", sp["initContainers"])
        for ln in sub.lines:
            w.write(1, ln)
    sub = PrefixWriter()
    describe_containers(sub, "Containers", sp.get("containers"))
    for ln in sub.lines:
        w.write(1, ln)
    sub = PrefixWriter()
    describe_volumes(sub, sp.get("volumes"))
    for ln in sub.lines:
        w.write(1, ln)


def _pod_counts(pods) -> tuple[int, int, int, int]:
    running = waiting = succeeded = failed = 0
    for p in pods or []:
        ph = (p.get("status") or {}).get("phase")
        if ph == "Running":
            running += 1
        elif ph == "Pending":
            waiting += 1
        elif ph == "Succeeded":
            succeeded += 1
        elif ph == "Failed":
            failed += 1
    return running, waiting, succeeded, failed


def _conditions(w, conds, cols=("Type", "Status", "Reason")):
    if not conds:
        return
    w.write(0, "Conditions:")
    w.write(1, "\t".join(cols))
    w.write(1, "\t".join("-" * len(c) for c in cols))
    for c in conds:
        w.write(1, "\t".join(str(c.get(k[0].lower() + k[1:].replace(" ", ""), "")) for k in cols))


# ---------------------------------------------------------------------------- kinds
def describe_pod(pod, events=()):
    w = PrefixWriter()
    md, sp, st = pod.get("metadata") or {}, pod.get("spec") or {}, pod.get("status") or {}
    _header(w, pod)
    w.write(0, f"Node:\t{sp.get('nodeName', '') + ('/' + st['hostIP'] if st.get('hostIP') else '') or '<none>'}")
    if st.get("startTime"):
        w.write(0, f"Start Time:\t{_rfc1123z(st['startTime'])}")
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    if md.get("deletionTimestamp"):
        w.write(0, f"Status:\tTerminating (lasts {age(md['deletionTimestamp'])})")
        w.write(0, f"Termination Grace Period:\t{md.get('deletionGracePeriodSeconds', 0)}s")
    else:
        w.write(0, f"Status:\t{st.get('phase', '')}")
    if st.get("reason"):
        w.write(0, f"Reason:\t{st['reason']}")
    if st.get("message"):
        w.write(0, f"Message:\t{st['message']}")
    w.write(0, f"IP:\t{st.get('podIP', '')}")
    if _controlled_by(pod):
        w.write(0, f"Controlled By:\t{_controlled_by(pod)}")
    if sp.get("extendedResources"):
        w.write(0, "Extended Resources:")
        for pres in sp["extendedResources"]:
            lim = (pres.get("resources") or {}).get("limits") or {}
            sel = ", ".join(f"{r.get('key')} {r.get('operator')} {r.get('values') or ''}"
                            for r in (pres.get("affinity") or {}).get("required") or [])
            w.write(1, f"{pres.get('name')}:\t{', '.join(f'{k}={v}' for k, v in lim.items())}")
            w.write(2, f"Affinity:\t{sel or '<none>'}")
            w.write(2, f"Assigned:\t{', '.join(pres.get('assigned') or []) or '<not yet scheduled>'}")
    if sp.get("initContainers"):
        describe_containers(w, "Init Containers", sp["initContainers"], st.get("initContainerStatuses"))
    describe_containers(w, "Containers", sp.get("containers"), st.get("containerStatuses"))
    if st.get("conditions"):
        w.write(0, "Conditions:")
        w.write(1, "Type\tStatus")
        for c in st["conditions"]:
            w.write(1, f"{c.get('type')} \t{c.get('status')} ")
    describe_volumes(w, sp.get("volumes"))
    w.write(0, f"QoS Class:\t{st.get('qosClass', '')}")
    w.write(0, f"Node-Selectors:\t{format_labels(sp.get('nodeSelector'))}")
    tols = sp.get("tolerations") or []
    if not tols:
        w.write(0, "Tolerations:\t<none>")
    for i, t in enumerate(tols):
        s = t.get("key", "")
        if t.get("value"):
            s += "=" + t["value"]
        if t.get("effect"):
            s += ":" + t["effect"]
        if t.get("operator") == "Exists" and not t.get("value"):
            s += " op=Exists"
        if t.get("tolerationSeconds") is not None:
            s += f" for {t['tolerationSeconds']}s"
        w.write(0, ("Tolerations:\t" if i == 0 else "\t") + s)
    describe_events(w, events)
    return w.render()


def describe_node(node, pods=(), events=()):
    w = PrefixWriter()
    md, sp, st = node.get("metadata") or {}, node.get("spec") or {}, node.get("status") or {}
    _header(w, node, with_ns=False)
    from .printers import node_roles
    w.write(0, f"Roles:\t{','.join(node_roles(node)) or '<none>'}")
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    w.write(0, f"CreationTimestamp:\t{_rfc1123z(md.get('creationTimestamp'))}")
    taints = sp.get("taints") or []
    if not taints:
        w.write(0, "Taints:\t<none>")
    for i, t in enumerate(taints):
        s = f"{t.get('key')}={t.get('value', '')}:{t.get('effect')}" if t.get("value") else f"{t.get('key')}:{t.get('effect')}"
        w.write(0, ("Taints:\t" if i == 0 else "\t") + s)
    w.write(0, f"Unschedulable:\t{'true' if sp.get('unschedulable') else 'false'}")
    if st.get("conditions"):
        w.write(0, "Conditions:")
        w.write(1, "Type\tStatus\tLastHeartbeatTime\tLastTransitionTime\tReason\tMessage")
        w.write(1, "----\t------\t-----------------\t------------------\t------\t-------")
        for c in st["conditions"]:
            w.write(1, f"{c.get('type')} \t{c.get('status')} \t{_rfc1123z(c.get('lastHeartbeatTime'))} \t"
                       f"{_rfc1123z(c.get('lastTransitionTime'))} \t{c.get('reason', '')} \t{c.get('message', '')}")
    if st.get("addresses"):
        w.write(0, "Addresses:")
        for a in st["addresses"]:
            w.write(1, f"{a.get('type')}:\t{a.get('address')}")
    for title, key in (("Capacity", "capacity"), ("Allocatable", "allocatable")):
        if st.get(key):
            w.write(0, f"{title}:")
            for k in sorted(st[key]):
                w.write(1, f"{k}:\t{st[key][k]}")
    info = st.get("nodeInfo") or {}
    if info:
        w.write(0, "System Info:")
        for label, k in (("Machine ID", "machineID"), ("System UUID", "systemUUID"), ("Boot ID", "bootID"),
                         ("Kernel Version", "kernelVersion"), ("OS Image", "osImage"), ("Operating System", "operatingSystem"),
                         ("Architecture", "architecture"), ("Container Runtime Version", "containerRuntimeVersion"),
                         ("Kubelet Version", "kubeletVersion"), ("Kube-Proxy Version", "kubeProxyVersion")):
            w.write(1, f"{label}:\t{info.get(k, '')}")
    if sp.get("podCIDR"):
        w.write(0, f"PodCIDR:\t{sp['podCIDR']}")
    if sp.get("externalID"):
        w.write(0, f"ExternalID:\t{sp['externalID']}")
    cap, alloc, healthy, model = node_gpu_summary(node)
    w.write(0, f"GPUs:\t{cap} capacity / {alloc} allocatable / {healthy} healthy ({model})")
    if st.get("extendedResources"):
        w.write(0, "Extended Resources:")
        for r, dom in st["extendedResources"].items():
            w.write(1, f"{r}:")
            for did, d in sorted(((dom or {}).get("resources") or {}).items()):
                a = d.get("attributes") or {}
                w.write(2, f"{did}  {d.get('health')}  type={a.get('amd.com/gpu-type', '-')} mem={a.get('amd.com/gpu-memory', '-')}MiB "
                           f"numa={a.get('amd.com/numa-node', '-')} partition={a.get('amd.com/partition', '-')}")
    live = [p for p in pods or [] if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")]
    w.write(0, f"Non-terminated Pods:\t({len(live)} in total)")
    if live:
        w.write(1, "Namespace\tName\tCPU Requests\tMemory Requests\tGPUs")
        w.write(1, "---------\t----\t------------\t---------------\t----")
        for p in live:
            req = {}
            for c in (p.get("spec") or {}).get("containers") or []:
                for k, v in ((c.get("resources") or {}).get("requests") or {}).items():
                    req.setdefault(k, []).append(v)
            ids = [d for pr in (p.get("spec") or {}).get("extendedResources") or [] for d in pr.get("assigned") or []]
            w.write(1, f"{m.namespace_of(p)}\t{m.name_of(p)}\t{'+'.join(req.get('cpu', [])) or '0'}\t"
                       f"{'+'.join(req.get('memory', [])) or '0'}\t{','.join(ids) or '-'}")
    describe_events(w, events)
    return w.render()


def _rs_summary(rss) -> str:
    out = [f"{m.name_of(r)} ({(r.get('status') or {}).get('replicas', 0)}/{(r.get('spec') or {}).get('replicas', 0)} "
           f"replicas created)" for r in rss]
    return ", ".join(out) or "<none>"


def describe_deployment(d, rss=(), events=()):
    w = PrefixWriter()
    md, sp, st = d.get("metadata") or {}, d.get("spec") or {}, d.get("status") or {}
    _header(w, d)
    w.write(0, f"CreationTimestamp:\t{_rfc1123z(md.get('creationTimestamp'))}")
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    w.write(0, f"Selector:\t{format_label_selector(sp.get('selector'))}")
    w.write(0, f"Replicas:\t{sp.get('replicas', 1)} desired | {st.get('updatedReplicas', 0)} updated | "
               f"{st.get('replicas', 0)} total | {st.get('availableReplicas', 0)} available | "
               f"{st.get('unavailableReplicas', 0)} unavailable")
    strat = sp.get("strategy") or {}
    w.write(0, f"StrategyType:\t{strat.get('type', '')}")
    w.write(0, f"MinReadySeconds:\t{sp.get('minReadySeconds', 0)}")
    ru = strat.get("rollingUpdate")
    if ru is not None:
        w.write(0, f"RollingUpdateStrategy:\t{ru.get('maxUnavailable')} max unavailable, {ru.get('maxSurge')} max surge")
    describe_pod_template(w, sp.get("template"))
    _conditions(w, st.get("conditions"))
    from ..controllers.deployment import find_new_rs, find_old_rss
    try:
        new = find_new_rs(d, list(rss))
        old, _ = find_old_rss(d, list(rss))
        w.write(0, f"OldReplicaSets:\t{_rs_summary(old)}")
        w.write(0, f"NewReplicaSet:\t{_rs_summary([new] if new else [])}")
    except Exception:
        pass
    describe_events(w, events)
    return w.render()


def _describe_replicated(o, pods, events, replicas_line, selector, kind_extra=None):
    w = PrefixWriter()
    md, sp = o.get("metadata") or {}, o.get("spec") or {}
    _header(w, o)
    w.write(0, f"Selector:\t{selector}")
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    if _controlled_by(o):
        w.write(0, f"Controlled By:\t{_controlled_by(o)}")
    for ln in replicas_line:
        w.write(0, ln)
    r, wt, s, f = _pod_counts(pods)
    w.write(0, f"Pods Status:\t{r} Running / {wt} Waiting / {s} Succeeded / {f} Failed")
    describe_pod_template(w, sp.get("template"))
    if kind_extra:
        kind_extra(w)
    _conditions(w, (o.get("status") or {}).get("conditions"))
    describe_events(w, events)
    return w.render()


def describe_replica_set(rs, pods=(), events=()):
    sp, st = rs.get("spec") or {}, rs.get("status") or {}
    return _describe_replicated(rs, pods, events, [f"Replicas:\t{st.get('replicas', 0)} current / {sp.get('replicas', 0)} desired"],
                                format_label_selector(sp.get("selector")))


def describe_replication_controller(rc, pods=(), events=()):
    sp, st = rc.get("spec") or {}, rc.get("status") or {}
    return _describe_replicated(rc, pods, events, [f"Replicas:\t{st.get('replicas', 0)} current / {sp.get('replicas', 0)} desired"],
                                format_labels(sp.get("selector")))


def describe_daemon_set(ds, pods=(), events=()):
    sp, st = ds.get("spec") or {}, ds.get("status") or {}
    lines = [f"Node-Selector:\t{format_labels(((sp.get('template') or {}).get('spec') or {}).get('nodeSelector'))}",
             f"Desired Number of Nodes Scheduled: {st.get('desiredNumberScheduled', 0)}",
             f"Current Number of Nodes Scheduled: {st.get('currentNumberScheduled', 0)}",
             f"Number of Nodes Scheduled with Up-to-date Pods: {st.get('updatedNumberScheduled', 0)}",
             f"Number of Nodes Scheduled with Available Pods: {st.get('numberAvailable', 0)}",
             f"Number of Nodes Misscheduled: {st.get('numberMisscheduled', 0)}"]
    return _describe_replicated(ds, pods, events, lines, format_label_selector(sp.get("selector")))


def describe_stateful_set(ss, pods=(), events=()):
    sp, st = ss.get("spec") or {}, ss.get("status") or {}

    def claims(w):
        tpls = sp.get("volumeClaimTemplates") or []
        if not tpls:
            w.write(0, "Volume Claims:\t<none>")
            return
        w.write(0, "Volume Claims:")
        for t in tpls:
            w.write(1, f"Name:\t{m.name_of(t)}")
            w.write(1, f"StorageClass:\t{(t.get('spec') or {}).get('storageClassName', '')}")
            _multiline(w, "Labels", m.labels_of(t), 1)
            _multiline(w, "Annotations", m.annotations_of(t), 1)
            w.write(1, f"Capacity:\t{(((t.get('spec') or {}).get('resources') or {}).get('requests') or {}).get('storage', '')}")
            w.write(1, f"Access Modes:\t{access_modes_string((t.get('spec') or {}).get('accessModes'))}")
    return _describe_replicated(ss, pods, events,
                                [f"CreationTimestamp:\t{_rfc1123z((ss.get('metadata') or {}).get('creationTimestamp'))}",
                                 f"Replicas:\t{sp.get('replicas', 1)} desired | {st.get('replicas', 0)} total"],
                                format_label_selector(sp.get("selector")), claims)


def describe_job(job, events=()):
    w = PrefixWriter()
    md, sp, st = job.get("metadata") or {}, job.get("spec") or {}, job.get("status") or {}
    _header(w, job)
    w.write(0, f"Selector:\t{format_label_selector(sp.get('selector'))}")
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    if _controlled_by(job):
        w.write(0, f"Controlled By:\t{_controlled_by(job)}")
    w.write(0, f"Parallelism:\t{sp.get('parallelism', 1)}")
    w.write(0, f"Completions:\t{sp['completions'] if sp.get('completions') is not None else '<unset>'}")
    if st.get("startTime"):
        w.write(0, f"Start Time:\t{_rfc1123z(st['startTime'])}")
    if sp.get("activeDeadlineSeconds") is not None:
        w.write(0, f"Active Deadline Seconds:\t{sp['activeDeadlineSeconds']}s")
    w.write(0, f"Pods Statuses:\t{st.get('active', 0)} Running / {st.get('succeeded', 0)} Succeeded / {st.get('failed', 0)} Failed")
    describe_pod_template(w, sp.get("template"))
    describe_events(w, events)
    return w.render()


def describe_cron_job(cj, events=()):
    w = PrefixWriter()
    md, sp, st = cj.get("metadata") or {}, cj.get("spec") or {}, cj.get("status") or {}
    _header(w, cj)
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    w.write(0, f"Schedule:\t{sp.get('schedule', '')}")
    w.write(0, f"Concurrency Policy:\t{sp.get('concurrencyPolicy', 'Allow')}")
    w.write(0, f"Suspend:\t{'True' if sp.get('suspend') else 'False'}")
    w.write(0, f"Starting Deadline Seconds:\t{sp['startingDeadlineSeconds']}s" if sp.get("startingDeadlineSeconds") is not None
            else "Starting Deadline Seconds:\t<unset>")
    jt = (sp.get("jobTemplate") or {}).get("spec") or {}
    w.write(0, f"Selector:\t{format_label_selector(jt.get('selector'))}")
    w.write(0, f"Parallelism:\t{jt.get('parallelism', '<unset>')}")
    w.write(0, f"Completions:\t{jt.get('completions', '<unset>')}")
    describe_pod_template(w, jt.get("template"))
    w.write(0, f"Last Schedule Time:\t{_rfc1123z(st.get('lastScheduleTime'))}")
    active = st.get("active") or []
    w.write(0, f"Active Jobs:\t{', '.join(a.get('name', '') for a in active) or '<none>'}")
    describe_events(w, events)
    return w.render()


def describe_service(svc, endpoints=None, events=()):
    w = PrefixWriter()
    md, sp, st = svc.get("metadata") or {}, svc.get("spec") or {}, svc.get("status") or {}
    _header(w, svc)
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    w.write(0, f"Selector:\t{format_labels(sp.get('selector'))}")
    w.write(0, f"Type:\t{sp.get('type', 'ClusterIP')}")
    w.write(0, f"IP:\t{sp.get('clusterIP', '')}")
    if sp.get("externalIPs"):
        w.write(0, f"External IPs:\t{','.join(sp['externalIPs'])}")
    if sp.get("loadBalancerIP"):
        w.write(0, f"IP:\t{sp['loadBalancerIP']}")
    if sp.get("externalName"):
        w.write(0, f"External Name:\t{sp['externalName']}")
    ing = ((st.get("loadBalancer") or {}).get("ingress")) or []
    if ing:
        w.write(0, f"LoadBalancer Ingress:\t{', '.join(i.get('ip') or i.get('hostname', '') for i in ing)}")
    ep = endpoints or {}
    for p in sp.get("ports") or []:
        name = p.get("name") or "<unset>"
        proto = p.get("protocol") or "TCP"
        w.write(0, f"Port:\t{name}\t{p.get('port')}/{proto}")
        w.write(0, f"TargetPort:\t{p.get('targetPort', p.get('port'))}/{proto}")
        if p.get("nodePort"):
            w.write(0, f"NodePort:\t{name}\t{p['nodePort']}/{proto}")
        w.write(0, f"Endpoints:\t{format_endpoints(ep, {p.get('name', '')})}")
    w.write(0, f"Session Affinity:\t{sp.get('sessionAffinity', 'None')}")
    if sp.get("externalTrafficPolicy"):
        w.write(0, f"External Traffic Policy:\t{sp['externalTrafficPolicy']}")
    if sp.get("healthCheckNodePort"):
        w.write(0, f"HealthCheck NodePort:\t{sp['healthCheckNodePort']}")
    if sp.get("loadBalancerSourceRanges"):
        w.write(0, f"LoadBalancer Source Ranges:\t{','.join(sp['loadBalancerSourceRanges'])}")
    describe_events(w, events)
    return w.render()


def describe_endpoints(ep, events=()):
    w = PrefixWriter()
    _header(w, ep)
    _multiline(w, "Labels", m.labels_of(ep))
    _multiline(w, "Annotations", m.annotations_of(ep))
    w.write(0, "Subsets:")
    for ss in ep.get("subsets") or []:
        w.write(1, f"Addresses:\t{','.join(a.get('ip', '') for a in ss.get('addresses') or []) or '<none>'}")
        w.write(1, f"NotReadyAddresses:\t{','.join(a.get('ip', '') for a in ss.get('notReadyAddresses') or []) or '<none>'}")
        if ss.get("ports"):
            w.write(1, "Ports:")
            w.write(2, "Name\tPort\tProtocol")
            w.write(2, "----\t----\t--------")
            for p in ss["ports"]:
                w.write(2, f"{p.get('name') or '<unset>'}\t{p.get('port')}\t{p.get('protocol') or 'TCP'}")
    describe_events(w, events)
    return w.render()


PV_SOURCES = {
    "hostPath": ("HostPath (bare host directory volume)", ("path", "type")),
    "nfs": ("NFS (an NFS mount that lasts the lifetime of a pod)", ("server", "path", "readOnly")),
    "local": ("LocalVolume (a persistent volume backed by local storage on a node)", ("path",)),
    "iscsi": ("ISCSI (an ISCSI Disk resource that is attached to a kubelet's host machine and then exposed to the pod)",
              ("targetPortal", "iqn", "lun", "iscsiInterface", "fsType", "readOnly")),
    "rbd": ("RBD (a Rados Block Device mount on the host that shares a pod's lifetime)",
            ("monitors", "image", "fsType", "pool", "user", "keyring", "readOnly")),
    "cephfs": ("CephFS (a CephFS mount on the host that shares a pod's lifetime)", ("monitors", "path", "user", "readOnly")),
    "gcePersistentDisk": ("GCEPersistentDisk (a Persistent Disk resource in Google Compute Engine)",
                          ("pdName", "fsType", "partition", "readOnly")),
    "awsElasticBlockStore": ("AWSElasticBlockStore (a Persistent Disk resource in AWS)", ("volumeID", "fsType", "partition",
                                                                                        "readOnly")),
    "azureDisk": ("AzureDisk (an Azure Data Disk mount on the host and bind mount to the pod)",
                  ("diskName", "diskURI", "kind", "fsType", "cachingMode", "readOnly")),
    "csi": ("CSI (a Container Storage Interface (CSI) volume source)", ("driver", "volumeHandle", "readOnly")),
}


def describe_persistent_volume(pv, events=()):
    w = PrefixWriter()
    md, sp, st = pv.get("metadata") or {}, pv.get("spec") or {}, pv.get("status") or {}
    _header(w, pv, with_ns=False)
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    w.write(0, f"Finalizers:\t[{' '.join(md.get('finalizers') or [])}]")
    w.write(0, f"StorageClass:\t{pv_class(pv)}")
    w.write(0, f"Status:\t{st.get('phase', '')}")
    cr = sp.get("claimRef")
    w.write(0, f"Claim:\t{cr.get('namespace', '')}/{cr.get('name', '')}" if cr else "Claim:\t")
    w.write(0, f"Reclaim Policy:\t{sp.get('persistentVolumeReclaimPolicy', '')}")
    w.write(0, f"Access Modes:\t{access_modes_string(sp.get('accessModes'))}")
    if sp.get("volumeMode"):
        w.write(0, f"VolumeMode:\t{sp['volumeMode']}")
    w.write(0, f"Capacity:\t{(sp.get('capacity') or {}).get('storage', '')}")
    w.write(0, f"Message:\t{st.get('message', '')}")
    w.write(0, "Source:")
    kind = next((k for k in PV_SOURCES if k in sp), None)
    if kind is None:
        other = next((k for k in sp if isinstance(sp[k], dict) and k not in ("capacity", "claimRef", "nodeAffinity")), None)
        if other:
            w.write(1, f"Type:\t{other}")
            for k in sorted(sp[other]):
                w.write(1, f"{k}:\t{sp[other][k]}")
        else:
            w.write(1, "<unknown>")
    else:
        title, fields = PV_SOURCES[kind]
        w.write(1, f"Type:\t{title}")
        for f in fields:
            label = f[0].upper() + f[1:]
            v = sp[kind].get(f, "")
            w.write(1, f"{label}:\t{v if not isinstance(v, bool) else str(v).lower()}")
    describe_events(w, events)
    return w.render()


def describe_persistent_volume_claim(pvc, pods=(), events=()):
    w = PrefixWriter()
    md, sp, st = pvc.get("metadata") or {}, pvc.get("spec") or {}, pvc.get("status") or {}
    _header(w, pvc)
    ann = m.annotations_of(pvc).get("volume.beta.kubernetes.io/storage-class")
    w.write(0, f"StorageClass:\t{ann if ann is not None else sp.get('storageClassName', '')}")
    if md.get("deletionTimestamp"):
        w.write(0, f"Status:\tTerminating (since {_rfc1123z(md['deletionTimestamp'])})")
    else:
        w.write(0, f"Status:\t{st.get('phase', '')}")
    w.write(0, f"Volume:\t{sp.get('volumeName', '')}")
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", md.get("annotations"))
    w.write(0, f"Finalizers:\t[{' '.join(md.get('finalizers') or [])}]")
    cap = modes = ""
    if sp.get("volumeName"):
        modes = access_modes_string(st.get("accessModes"))
        cap = (st.get("capacity") or {}).get("storage", "")
    w.write(0, f"Capacity:\t{cap}")
    w.write(0, f"Access Modes:\t{modes}")
    if sp.get("volumeMode"):
        w.write(0, f"VolumeMode:\t{sp['volumeMode']}")
    users = [m.name_of(p) for p in pods or []
             if any((v.get("persistentVolumeClaim") or {}).get("claimName") == m.name_of(pvc)
                    for v in (p.get("spec") or {}).get("volumes") or [])]
    w.write(0, f"Mounted By:\t{', '.join(users) or '<none>'}")
    describe_events(w, events)
    return w.render()


def _quantity_cmp_key(r):
    return r


def describe_resource_quotas(w: PrefixWriter, quotas):
    if not quotas:
        w.write(0, "No resource quota.")
        return
    w.write(0, "Resource Quotas")
    for q in sorted(quotas, key=m.name_of):
        w.write(0, f" Name:\t{m.name_of(q)}")
        scopes = sorted((q.get("spec") or {}).get("scopes") or [])
        if scopes:
            w.write(0, f" Scopes:\t{', '.join(scopes)}")
        w.write(0, " Resource\tUsed\tHard")
        w.write(0, " --------\t---\t---")
        hard = (q.get("status") or {}).get("hard") or (q.get("spec") or {}).get("hard") or {}
        used = (q.get("status") or {}).get("used") or {}
        for r in sorted(hard):
            w.write(0, f" {r}\t{used.get(r, '0')}\t{hard[r]}")


def describe_limit_ranges(w: PrefixWriter, limits):
    if not limits:
        w.write(0, "No resource limits.")
        return
    w.write(0, "Resource Limits")
    w.write(0, " Type\tResource\tMin\tMax\tDefault Request\tDefault Limit\tMax Limit/Request Ratio")
    w.write(0, " ----\t--------\t---\t---\t---------------\t-------------\t-----------------------")
    for lr in limits:
        _limit_range_spec(w, lr.get("spec") or {}, " ")


def _limit_range_spec(w, spec, prefix):
    for item in spec.get("limits") or []:
        keys = set()
        for k in ("max", "min", "default", "defaultRequest", "maxLimitRequestRatio"):
            keys.update((item.get(k) or {}).keys())
        for r in sorted(keys):
            vals = [(item.get(k) or {}).get(r, "-") for k in ("min", "max", "defaultRequest", "default", "maxLimitRequestRatio")]
            w.write(0, f"{prefix}{item.get('type', '')}\t{r}\t" + "\t".join(str(v) for v in vals))


def describe_namespace(ns, quotas=None, limits=None):
    w = PrefixWriter()
    _header(w, ns, with_ns=False)
    _multiline(w, "Labels", m.labels_of(ns))
    _multiline(w, "Annotations", m.annotations_of(ns))
    w.write(0, f"Status:\t{(ns.get('status') or {}).get('phase', '')}")
    if quotas is not None:
        w.write(0, "")
        describe_resource_quotas(w, quotas)
    if limits is not None:
        w.write(0, "")
        describe_limit_ranges(w, limits)
    return w.render()


def describe_quota(q):
    w = PrefixWriter()
    _header(w, q)
    scopes = sorted((q.get("spec") or {}).get("scopes") or [])
    if scopes:
        w.write(0, f"Scopes:\t{', '.join(scopes)}")
    w.write(0, "Resource\tUsed\tHard")
    w.write(0, "--------\t----\t----")
    hard = (q.get("status") or {}).get("hard") or (q.get("spec") or {}).get("hard") or {}
    used = (q.get("status") or {}).get("used") or {}
    for r in sorted(hard):
        w.write(0, f"{r}\t{used.get(r, '0')}\t{hard[r]}")
    return w.render()


def describe_limit_range(lr):
    w = PrefixWriter()
    _header(w, lr)
    w.write(0, "Type\tResource\tMin\tMax\tDefault Request\tDefault Limit\tMax Limit/Request Ratio")
    w.write(0, "----\t--------\t---\t---\t---------------\t-------------\t-----------------------")
    _limit_range_spec(w, lr.get("spec") or {}, "")
    return w.render()


def describe_config_map(cm, events=()):
    w = PrefixWriter()
    _header(w, cm)
    _multiline(w, "Labels", m.labels_of(cm))
    _multiline(w, "Annotations", m.annotations_of(cm))
    w.write(0, "")
    w.write(0, "Data")
    w.write(0, "====")
    for k in sorted(cm.get("data") or {}):
        w.write(0, f"{k}:")
        w.write(0, "----")
        w.write(0, str(cm["data"][k]))
    describe_events(w, events)
    return w.render()


def describe_secret(s):
    w = PrefixWriter()
    _header(w, s)
    _multiline(w, "Labels", m.labels_of(s))
    _multiline(w, "Annotations", m.annotations_of(s))
    w.write(0, "")
    w.write(0, f"Type:\t{s.get('type', '')}")
    w.write(0, "")
    w.write(0, "Data")
    w.write(0, "====")
    for k in sorted(s.get("data") or {}):
        v = s["data"][k]
        try:
            n = len(base64.b64decode(v))
        except (ValueError, TypeError):
            n = len(v or "")
        if k == "token" and s.get("type") == "kubernetes.io/service-account-token":
            w.write(0, f"{k}:\t{base64.b64decode(v).decode(errors='replace')}")
        else:
            w.write(0, f"{k}:\t{n} bytes")
    return w.render()


def describe_service_account(sa, tokens=(), events=()):
    w = PrefixWriter()
    _header(w, sa)
    _multiline(w, "Labels", m.labels_of(sa))
    _multiline(w, "Annotations", m.annotations_of(sa))
    for title, items in (("Image pull secrets", sa.get("imagePullSecrets")), ("Mountable secrets", sa.get("secrets"))):
        names = [i.get("name", "") for i in items or []]
        if not names:
            w.write(0, f"{title}:\t<none>")
        for i, n in enumerate(names):
            w.write(0, (f"{title}:\t" if i == 0 else "\t") + n)
    names = [m.name_of(t) for t in tokens or []]
    if not names:
        w.write(0, "Tokens:\t<none>")
    for i, n in enumerate(names):
        w.write(0, ("Tokens:\t" if i == 0 else "\t") + n)
    describe_events(w, events)
    return w.render()


def describe_ingress(ing, events=()):
    w = PrefixWriter()
    sp, st = ing.get("spec") or {}, ing.get("status") or {}
    _header(w, ing)
    w.write(0, f"Address:\t{load_balancer_status(st.get('loadBalancer'), True)}")
    be = sp.get("backend")
    w.write(0, f"Default backend:\t{be.get('serviceName')}:{be.get('servicePort')}" if be else
            "Default backend:\tdefault-http-backend:80 (<none>)")
    for t in sp.get("tls") or []:
        w.write(0, "TLS:")
        w.write(1, f"{t.get('secretName', 'SNI')} terminates {','.join(t.get('hosts') or [])}")
    w.write(0, "Rules:")
    w.write(1, "Host\tPath\tBackends")
    w.write(1, "----\t----\t--------")
    for r in sp.get("rules") or []:
        w.write(1, f"{r.get('host') or '*'}\t")
        for p in ((r.get("http") or {}).get("paths")) or []:
            b = p.get("backend") or {}
            w.write(2, f"\t{p.get('path', '')} \t{b.get('serviceName')}:{b.get('servicePort')}")
    _multiline(w, "Annotations", m.annotations_of(ing))
    describe_events(w, events)
    return w.render()


def describe_hpa(hpa, events=()):
    from .printers import format_hpa_metrics
    w = PrefixWriter()
    md, sp, st = hpa.get("metadata") or {}, hpa.get("spec") or {}, hpa.get("status") or {}
    _header(w, hpa)
    _multiline(w, "Labels", md.get("labels"))
    _multiline(w, "Annotations", {k: v for k, v in (md.get("annotations") or {}).items()
                                  if not k.startswith("autoscaling.alpha.kubernetes.io/")})
    w.write(0, f"CreationTimestamp:\t{_rfc1123z(md.get('creationTimestamp'))}")
    ref = sp.get("scaleTargetRef") or {}
    w.write(0, f"Reference:\t{ref.get('kind', '')}/{ref.get('name', '')}")
    w.write(0, f"Metrics:\t( current / target )")
    for part in format_hpa_metrics(hpa).split(", "):
        w.write(1, f"resource cpu on pods  (as a percentage of request):\t{part}" if "%" in part else f"metric:\t{part}")
    w.write(0, f"Min replicas:\t{sp.get('minReplicas', '<unset>')}")
    w.write(0, f"Max replicas:\t{sp.get('maxReplicas', 0)}")
    _conditions(w, [])
    w.write(0, f"Deployment pods:\t{st.get('currentReplicas', 0)} current / {st.get('desiredReplicas', 0)} desired")
    describe_events(w, events)
    return w.render()


def describe_pdb(pdb, events=()):
    w = PrefixWriter()
    sp, st = pdb.get("spec") or {}, pdb.get("status") or {}
    _header(w, pdb)
    if sp.get("minAvailable") is not None:
        w.write(0, f"Min available:\t{sp['minAvailable']}")
    elif sp.get("maxUnavailable") is not None:
        w.write(0, f"Max unavailable:\t{sp['maxUnavailable']}")
    w.write(0, f"Selector:\t{format_label_selector(sp.get('selector'))}")
    w.write(0, "Status:")
    w.write(2, f"Allowed disruptions:\t{st.get('disruptionsAllowed', st.get('podDisruptionsAllowed', 0))}")
    w.write(2, f"Current:\t{st.get('currentHealthy', 0)}")
    w.write(2, f"Desired:\t{st.get('desiredHealthy', 0)}")
    w.write(2, f"Total:\t{st.get('expectedPods', 0)}")
    describe_events(w, events)
    return w.render()


def describe_storage_class(sc, events=()):
    w = PrefixWriter()
    _header(w, sc, with_ns=False)
    ann = m.annotations_of(sc)
    default = ann.get("storageclass.kubernetes.io/is-default-class") == "true" or \
        ann.get("storageclass.beta.kubernetes.io/is-default-class") == "true"
    w.write(0, f"IsDefaultClass:\t{'Yes' if default else 'No'}")
    _multiline(w, "Annotations", ann)
    w.write(0, f"Provisioner:\t{sc.get('provisioner', '')}")
    params = sc.get("parameters") or {}
    w.write(0, f"Parameters:\t{', '.join(f'{k}={params[k]}' for k in sorted(params)) or '<none>'}")
    w.write(0, f"ReclaimPolicy:\t{sc.get('reclaimPolicy', 'Delete')}")
    w.write(0, f"VolumeBindingMode:\t{sc.get('volumeBindingMode', 'Immediate')}")
    describe_events(w, events)
    return w.render()


def describe_network_policy(np_):
    w = PrefixWriter()
    sp = np_.get("spec") or {}
    _header(w, np_)
    w.write(0, f"Created on:\t{_rfc1123z((np_.get('metadata') or {}).get('creationTimestamp'))}")
    _multiline(w, "Labels", m.labels_of(np_))
    _multiline(w, "Annotations", m.annotations_of(np_))
    w.write(0, "Spec:")
    sel = format_label_selector(sp.get("podSelector") or {})
    w.write(1, f"PodSelector:\t{'<none> (Allowing the specific traffic to all pods in this namespace)' if sel == '<none>' else sel}")
    types = sp.get("policyTypes") or ["Ingress"]
    for t in ("Ingress", "Egress"):
        key = t.lower()
        if t not in types:
            w.write(1, f"Not affecting {t} traffic")
            continue
        rules = sp.get(key) or []
        w.write(1, f"Allowing {t.lower()} traffic:" if rules else f"Allowing {t.lower()} traffic:\n    <none> (Selected pods are isolated for {t.lower()} connectivity)")
        for i, r in enumerate(rules):
            if i:
                w.write(2, "----------")
            ports = r.get("ports") or []
            w.write(2, ("To Port: " if t == "Egress" else "To Port: ") +
                    (", ".join(f"{p.get('port', '<any>')}/{p.get('protocol', 'TCP')}" for p in ports) or "<any> (traffic allowed to all ports)"))
            peers = r.get("from" if t == "Ingress" else "to") or []
            w.write(2, ("From:" if t == "Ingress" else "To:") + ("" if peers else " <any> (traffic not restricted by source)"))
            for p in peers:
                if "podSelector" in p:
                    w.write(3, f"PodSelector: {format_label_selector(p['podSelector'])}")
                if "namespaceSelector" in p:
                    w.write(3, f"NamespaceSelector: {format_label_selector(p['namespaceSelector'])}")
                if "ipBlock" in p:
                    w.write(3, "IPBlock:")
                    w.write(4, f"CIDR: {p['ipBlock'].get('cidr')}")
                    w.write(4, f"Except: {', '.join(p['ipBlock'].get('except') or [])}")
    w.write(1, f"Policy Types: {', '.join(types)}")
    return w.render()


def describe_generic(obj, events=()):
    """The fallback for kinds without a describer: metadata, then spec and status as YAML."""
    from ..api.scheme import dump_yaml
    w = PrefixWriter()
    _header(w, obj)
    _multiline(w, "Labels", m.labels_of(obj))
    _multiline(w, "Annotations", m.annotations_of(obj))
    w.write(0, f"API Version:\t{obj.get('apiVersion', '')}")
    w.write(0, f"Kind:\t{obj.get('kind', '')}")
    text = w.render()
    rest = {k: v for k, v in obj.items() if k not in ("apiVersion", "kind", "metadata")}
    if rest:
        body = dump_yaml(rest).rstrip("\n")
        text += "\n" + "\n".join(ln for ln in body.split("\n"))
    ew = PrefixWriter()
    describe_events(ew, events)
    return text + "\n" + ew.render()


def describe(obj, events=(), **extra) -> str:
    """The describer for the object's kind; `extra` carries what it needs besides the object
    (pods, replica sets, endpoints, quotas, limit ranges, tokens)."""
    kind = obj.get("kind")
    fn = {
        "Pod": lambda: describe_pod(obj, events),
        "Node": lambda: describe_node(obj, extra.get("pods", ()), events),
        "Deployment": lambda: describe_deployment(obj, extra.get("replicasets", ()), events),
        "ReplicaSet": lambda: describe_replica_set(obj, extra.get("pods", ()), events),
        "ReplicationController": lambda: describe_replication_controller(obj, extra.get("pods", ()), events),
        "DaemonSet": lambda: describe_daemon_set(obj, extra.get("pods", ()), events),
        "StatefulSet": lambda: describe_stateful_set(obj, extra.get("pods", ()), events),
        "Job": lambda: describe_job(obj, events),
        "CronJob": lambda: describe_cron_job(obj, events),
        "Service": lambda: describe_service(obj, extra.get("endpoints"), events),
        "Endpoints": lambda: describe_endpoints(obj, events),
        "PersistentVolume": lambda: describe_persistent_volume(obj, events),
        "PersistentVolumeClaim": lambda: describe_persistent_volume_claim(obj, extra.get("pods", ()), events),
        "Namespace": lambda: describe_namespace(obj, extra.get("quotas", []), extra.get("limits", [])),
        "ResourceQuota": lambda: describe_quota(obj),
        "LimitRange": lambda: describe_limit_range(obj),
        "ConfigMap": lambda: describe_config_map(obj, events),
        "Secret": lambda: describe_secret(obj),
        "ServiceAccount": lambda: describe_service_account(obj, extra.get("tokens", ()), events),
        "Ingress": lambda: describe_ingress(obj, events),
        "HorizontalPodAutoscaler": lambda: describe_hpa(obj, events),
        "PodDisruptionBudget": lambda: describe_pdb(obj, events),
        "StorageClass": lambda: describe_storage_class(obj, events),
        "NetworkPolicy": lambda: describe_network_policy(obj),
    }.get(kind)
    return fn() if fn else describe_generic(obj, events)


async def gather_extra(c, obj) -> dict:
    """What the describer of `obj` reads besides the object (the describers' client calls)."""
    kind, ns = obj.get("kind"), m.namespace_of(obj)
    sp = obj.get("spec") or {}
    extra: dict = {}

    async def pods_matching(selector_str):
        try:
            return (await c.list("pods", ns, label_selector=selector_str))[0]
        except m.StatusError:
            return []
    if kind in ("ReplicaSet", "DaemonSet", "StatefulSet"):
        sel = format_label_selector(sp.get("selector"))
        extra["pods"] = await pods_matching(None if sel == "<none>" else sel)
    elif kind == "ReplicationController":
        sel = ",".join(f"{k}={v}" for k, v in sorted((sp.get("selector") or {}).items()))
        extra["pods"] = await pods_matching(sel or None)
    elif kind == "Deployment":
        try:
            rss, _ = await c.list("replicasets", ns)
        except m.StatusError:
            rss = []
        extra["replicasets"] = [r for r in rss if any(o.get("uid") == m.uid_of(obj)
                                                      for o in (r.get("metadata") or {}).get("ownerReferences") or [])]
    elif kind == "Service":
        extra["endpoints"] = await c.get_or_none("endpoints", m.name_of(obj), ns)
    elif kind == "PersistentVolumeClaim":
        extra["pods"] = await pods_matching(None)
    elif kind == "Node":
        try:
            extra["pods"] = (await c.list("pods", "", field_selector=f"spec.nodeName={m.name_of(obj)}"))[0]
        except m.StatusError:
            extra["pods"] = []
    elif kind == "Namespace":
        for key, res in (("quotas", "resourcequotas"), ("limits", "limitranges")):
            try:
                extra[key] = (await c.list(res, m.name_of(obj)))[0]
            except m.StatusError:
                extra[key] = None
    elif kind == "ServiceAccount":
        try:
            secrets, _ = await c.list("secrets", ns)
        except m.StatusError:
            secrets = []
        extra["tokens"] = [s for s in secrets if s.get("type") == "kubernetes.io/service-account-token" and
                           m.annotations_of(s).get("kubernetes.io/service-account.name") == m.name_of(obj)]
    return extra
