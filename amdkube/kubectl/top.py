"""kubectl top node|pod|gpu (pkg/kubectl/cmd/top_node.go, top_pod.go, pkg/kubectl/metricsutil).

`top node` / `top pod` read the resource metrics API (metrics.k8s.io/v1beta1, served by the
metrics-server through the aggregator) when the apiserver advertises it and fall back to the
kubelets' /stats/summary otherwise (the reference's Heapster path has no counterpart here).
Columns follow metricsutil.MetricsPrinter: NAME CPU(cores) CPU% MEMORY(bytes) MEMORY% for
nodes (percent of allocatable), NAME CPU(cores) MEMORY(bytes) for pods (`--containers` adds a
row per container, `-A` a NAMESPACE column, `-l` filters). `top gpu` is the amdkube addition:
per-MI355X duty cycle, VRAM and owning pod from the kubelet summaries.
"""
from __future__ import annotations

import aiohttp

from ..api import meta as m
from ..api.quantity import Quantity
from . import printers

GV = "metrics.k8s.io/v1beta1"


def _milli(q) -> int:
    return Quantity(q or "0").milli_value()


def _bytes(q) -> int:
    return Quantity(q or "0").value()


async def _metrics_available(c) -> bool:
    try:
        groups = (await c.request("GET", "/apis")).get("groups") or []
    except Exception:
        return False
    return any(g.get("name") == "metrics.k8s.io" for g in groups)


async def _summaries(c):
    """(node, /stats/summary) of every reachable kubelet."""
    nodes, _ = await c.list("nodes")
    out = []
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=10)) as s:
        for n in nodes:
            st = n.get("status") or {}
            port = ((st.get("daemonEndpoints") or {}).get("kubeletEndpoint") or {}).get("Port")
            addr = next((x["address"] for x in st.get("addresses") or [] if x.get("type") == "InternalIP"), "127.0.0.1")
            if not port:
                continue
            try:
                async with s.get(f"http://{addr}:{port}/stats/summary") as r:
                    out.append((n, await r.json()))
            except Exception:
                continue
    return out


def _cpu_str(milli: int) -> str:
    return f"{milli}m"


def _mem_str(b: int) -> str:
    return f"{b >> 20}Mi"


async def node_metrics(c, selector=None) -> list[dict]:
    if await _metrics_available(c):
        q = {"labelSelector": selector} if selector else None
        return (await c.request("GET", f"/apis/{GV}/nodes", params=q)).get("items") or []
    from ..metrics import _cpu, _mem
    out = []
    for n, summ in await _summaries(c):
        node = summ.get("node") or {}
        out.append({"metadata": {"name": m.name_of(n)},
                    "usage": {"cpu": _cpu((node.get("cpu") or {}).get("usageNanoCores", 0)),
                              "memory": _mem((node.get("memory") or {}).get("workingSetBytes", 0))}})
    return out


async def pod_metrics(c, ns: str | None, selector=None) -> list[dict]:
    if await _metrics_available(c):
        path = f"/apis/{GV}/namespaces/{ns}/pods" if ns else f"/apis/{GV}/pods"
        q = {"labelSelector": selector} if selector else None
        return (await c.request("GET", path, params=q)).get("items") or []
    from ..metrics import _cpu, _mem
    from ..api.labels import parse_selector
    pods, _ = await c.list("pods", ns)
    labels = {(m.namespace_of(p), m.name_of(p)): m.labels_of(p) for p in pods}
    sel = parse_selector(selector) if selector else None
    out = []
    for _n, summ in await _summaries(c):
        for p in summ.get("pods") or []:
            ref = p.get("podRef") or {}
            key = (ref.get("namespace", ""), ref.get("name", ""))
            if key not in labels or (sel is not None and not sel.matches(labels[key])):
                continue
            out.append({"metadata": {"name": key[1], "namespace": key[0]}, "containers": [
                {"name": ct["name"], "usage": {"cpu": _cpu((ct.get("cpu") or {}).get("usageNanoCores", 0)),
                                               "memory": _mem((ct.get("memory") or {}).get("workingSetBytes", 0))}}
                for ct in p.get("containers") or []]})
    return out


async def cmd_top(c, a):
    what = a.args[0] if a.args else "node"
    if what in ("node", "nodes", "no"):
        items = await node_metrics(c, a.selector)
        if len(a.args) > 1:
            items = [i for i in items if m.name_of(i) == a.args[1]]
            if not items:
                raise SystemExit(f'error: metrics not available yet for node "{a.args[1]}"')
        alloc = {}
        for n in (await c.list("nodes"))[0]:
            al = (n.get("status") or {}).get("allocatable") or {}
            alloc[m.name_of(n)] = (_milli(al.get("cpu")), _bytes(al.get("memory")))
        rows = [["NAME", "CPU(cores)", "CPU%", "MEMORY(bytes)", "MEMORY%"]]
        for i in sorted(items, key=m.name_of):
            cpu, mem = _milli(i["usage"]["cpu"]), _bytes(i["usage"]["memory"])
            acpu, amem = alloc.get(m.name_of(i), (0, 0))
            rows.append([m.name_of(i), _cpu_str(cpu), f"{100 * cpu // acpu}%" if acpu else "<unknown>",
                         _mem_str(mem), f"{100 * mem // amem}%" if amem else "<unknown>"])
        print(printers.table(rows))
    elif what in ("pod", "pods", "po"):
        ns = None if a.all_namespaces else (a.namespace or "default")
        items = await pod_metrics(c, ns, a.selector)
        if len(a.args) > 1:
            items = [i for i in items if m.name_of(i) == a.args[1]]
            if not items:
                raise SystemExit(f'error: metrics not available yet for pod "{ns}/{a.args[1]}"')
        head = (["NAMESPACE"] if a.all_namespaces else []) + ["POD" if a.containers else "NAME"] + \
            (["NAME"] if a.containers else []) + ["CPU(cores)", "MEMORY(bytes)"]
        rows = [head]
        for i in sorted(items, key=lambda i: (m.namespace_of(i), m.name_of(i))):
            pre = [m.namespace_of(i)] if a.all_namespaces else []
            if a.containers:
                for ct in i.get("containers") or []:
                    rows.append(pre + [m.name_of(i), ct["name"], _cpu_str(_milli(ct["usage"]["cpu"])),
                                       _mem_str(_bytes(ct["usage"]["memory"]))])
            else:
                cpu = sum(_milli(ct["usage"]["cpu"]) for ct in i.get("containers") or [])
                mem = sum(_bytes(ct["usage"]["memory"]) for ct in i.get("containers") or [])
                rows.append(pre + [m.name_of(i), _cpu_str(cpu), _mem_str(mem)])
        print(printers.table(rows))
    else:   # gpu
        rows = [["NODE", "GPU", "MODEL", "UTIL", "VRAM", "POD"]]
        for n, summ in await _summaries(c):
            owner = {}
            for p in summ.get("pods") or []:
                for ct in p.get("containers") or []:
                    for acc in ct.get("accelerators") or []:
                        owner[acc["id"]] = f"{p['podRef']['namespace']}/{p['podRef']['name']}"
            for acc in (summ.get("node") or {}).get("accelerators") or []:
                rows.append([m.name_of(n), acc["id"], acc["model"], f"{acc['dutyCycle']}%",
                             f"{acc['memoryUsed'] >> 20}Mi/{acc['memoryTotal'] >> 20}Mi", owner.get(acc["id"], "-")])
        print(printers.table(rows))
