"""amdkube dashboard: the cluster's web UI (the kubernetes-dashboard addon).

cluster/addons/dashboard deploys kubernetes-dashboard 1.8 (dashboard-controller.yaml,
dashboard-service.yaml, its RBAC and secrets): a web UI over the API — cluster overview,
workloads, pods with logs, services, events, and the scale / delete actions. The dashboard here
is one aiohttp process serving a single page (no external assets: the UI works on an offline
node) and a small JSON API that it calls:
* `GET /api/namespaces`;
* `GET /api/overview?namespace=` — nodes (readiness, CPU/memory, MI355X GPUs: capacity,
  allocatable, allocated to running pods, the GPU type label and unhealthy count), pods (phase,
  readiness, restarts, node, GPUs), Deployments / ReplicaSets / DaemonSets / StatefulSets / Jobs
  with desired and ready counts, Services, the newest events;
* `GET /api/pods/{ns}/{name}/log?container=&tailLines=` — the pods/log subresource;
* `POST /api/scale` `{kind, namespace, name, replicas}` — the scale subresource;
* `DELETE /api/pods/{ns}/{name}`;
* `GET /api/logs?q=&namespace=&pod=` — a search of the cluster log store (the Kibana role of the
  fluentd-elasticsearch addon) when --log-store-url is set.
It acts with its own credentials (service account in the addon, or --kubeconfig), as the
reference's dashboard does without a login.
"""
from __future__ import annotations

import logging
import time

from aiohttp import web

from ..api import meta as m
from ..api.quantity import Quantity

log = logging.getLogger("amdkube.dashboard")

GPU = "amd.com/gpu"
WORKLOADS = ("deployments", "replicasets", "daemonsets", "statefulsets", "jobs")
SCALABLE = {"deployment": "deployments", "replicaset": "replicasets", "statefulset": "statefulsets",
            "replicationcontroller": "replicationcontrollers"}


def _age(ts: str | None) -> str:
    if not ts:
        return ""
    try:
        import datetime
        t = datetime.datetime.strptime(ts, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=datetime.timezone.utc).timestamp()
    except ValueError:
        return ""
    s = max(0, int(time.time() - t))
    for unit, n in (("d", 86400), ("h", 3600), ("m", 60)):
        if s >= n:
            return f"{s // n}{unit}"
    return f"{s}s"


def _pod_gpus(pod: dict) -> int:
    n = 0
    for c in (pod.get("spec") or {}).get("containers") or []:
        r = c.get("resources") or {}
        v = (r.get("limits") or {}).get(GPU) or (r.get("requests") or {}).get(GPU)
        n += int(Quantity(v).value()) if v else 0
    return n


def summarize_pod(p: dict) -> dict:
    st, spec = p.get("status") or {}, p.get("spec") or {}
    cs = st.get("containerStatuses") or []
    return {"name": m.name_of(p), "namespace": m.namespace_of(p), "phase": st.get("phase", "Pending"),
            "ready": f"{sum(1 for c in cs if c.get('ready'))}/{len(spec.get('containers') or [])}",
            "restarts": sum(int(c.get("restartCount", 0)) for c in cs), "node": spec.get("nodeName", ""),
            "gpus": _pod_gpus(p), "ip": st.get("podIP", ""), "age": _age((p.get("metadata") or {}).get("creationTimestamp")),
            "containers": [c.get("name") for c in spec.get("containers") or []],
            "reason": st.get("reason") or next((c.get("state", {}).get("waiting", {}).get("reason") for c in cs
                                                if (c.get("state") or {}).get("waiting")), "")}


def summarize_node(n: dict, pods: list) -> dict:
    st = n.get("status") or {}
    cap, alloc = st.get("capacity") or {}, st.get("allocatable") or {}
    ready = next((c.get("status") == "True" for c in st.get("conditions") or [] if c.get("type") == "Ready"), False)
    used = sum(_pod_gpus(p) for p in pods if (p.get("spec") or {}).get("nodeName") == m.name_of(n)
               and (p.get("status") or {}).get("phase") in ("Pending", "Running"))
    labels = (n.get("metadata") or {}).get("labels") or {}
    return {"name": m.name_of(n), "ready": ready, "unschedulable": bool((n.get("spec") or {}).get("unschedulable")),
            "cpu": cap.get("cpu", ""), "memory": cap.get("memory", ""),
            "gpus": {"capacity": int(Quantity(cap.get(GPU, "0")).value()),
                     "allocatable": int(Quantity(alloc.get(GPU, "0")).value()), "allocated": used,
                     "unhealthy": max(0, int(Quantity(cap.get(GPU, "0")).value()) - int(Quantity(alloc.get(GPU, "0")).value())),
                     "type": labels.get("amd.com/gpu-type") or labels.get("amd.com/gpu.product-name", "")},
            "age": _age((n.get("metadata") or {}).get("creationTimestamp"))}


def summarize_workload(kind: str, o: dict) -> dict:
    spec, st = o.get("spec") or {}, o.get("status") or {}
    if kind == "daemonsets":
        desired, ready = st.get("desiredNumberScheduled", 0), st.get("numberReady", 0)
    elif kind == "jobs":
        desired, ready = spec.get("completions") or 1, st.get("succeeded", 0)
    else:
        desired, ready = spec.get("replicas", 1), st.get("readyReplicas", 0)
    return {"kind": kind, "name": m.name_of(o), "namespace": m.namespace_of(o), "desired": desired, "ready": ready or 0,
            "age": _age((o.get("metadata") or {}).get("creationTimestamp"))}


class Dashboard:
    def __init__(self, client, log_store_url: str = ""):
        self.client, self.log_store_url = client, log_store_url.rstrip("/")

    async def _list(self, resource: str, ns: str = "") -> list:
        try:
            items, _ = await self.client.list(resource, ns)
            return items
        except m.StatusError as e:
            if e.code in (403, 404):
                return []
            raise

    async def overview(self, ns: str = "") -> dict:
        nodes, pods = await self._list("nodes"), await self._list("pods", ns)
        all_pods = pods if not ns else await self._list("pods")
        work = []
        for kind in WORKLOADS:
            work += [summarize_workload(kind, o) for o in await self._list(kind, ns)]
        events = sorted(await self._list("events", ns), key=lambda e: e.get("lastTimestamp") or "", reverse=True)[:50]
        return {"nodes": [summarize_node(n, all_pods) for n in nodes],
                "pods": [summarize_pod(p) for p in sorted(pods, key=lambda p: (m.namespace_of(p), m.name_of(p)))],
                "workloads": work,
                "services": [{"name": m.name_of(s), "namespace": m.namespace_of(s), "type": (s.get("spec") or {}).get("type", "ClusterIP"),
                              "clusterIP": (s.get("spec") or {}).get("clusterIP", ""),
                              "ports": [f"{p.get('port')}/{p.get('protocol', 'TCP')}" for p in (s.get("spec") or {}).get("ports") or []]}
                             for s in await self._list("services", ns)],
                "events": [{"type": e.get("type", ""), "reason": e.get("reason", ""), "message": e.get("message", ""),
                            "object": f"{(e.get('involvedObject') or {}).get('kind', '')}/{(e.get('involvedObject') or {}).get('name', '')}",
                            "count": e.get("count", 1), "last": e.get("lastTimestamp", "")} for e in events]}

    async def scale(self, kind: str, ns: str, name: str, replicas: int) -> dict:
        resource = SCALABLE.get(kind.lower())
        if resource is None:
            raise web.HTTPBadRequest(text=f"cannot scale a {kind}")
        if replicas < 0:
            raise web.HTTPBadRequest(text="replicas must be >= 0")
        path = self.client.path(self.client.resource_info(resource), ns, name, "scale")
        sc = await self.client.request("GET", path)
        sc.setdefault("spec", {})["replicas"] = replicas
        return await self.client.request("PUT", path, body=sc)

    def app(self) -> web.Application:
        def fail(e: m.StatusError):
            return web.json_response({"error": str(e)}, status=e.code or 500)

        async def index(_r):
            return web.Response(text=PAGE, content_type="text/html")

        async def namespaces(_r):
            return web.json_response(sorted(m.name_of(n) for n in await self._list("namespaces")))

        async def overview(r):
            try:
                return web.json_response(await self.overview(r.query.get("namespace", "")))
            except m.StatusError as e:
                return fail(e)

        async def pod_log(r):
            ri = self.client.resource_info("pods")
            params = {k: r.query[k] for k in ("container", "tailLines", "previous") if r.query.get(k)}
            try:
                raw = await self.client.request("GET", self.client.path(ri, r.match_info["ns"], r.match_info["name"], "log"),
                                                params=params, raw=True)
            except m.StatusError as e:
                return fail(e)
            return web.Response(text=raw.decode(errors="replace") if isinstance(raw, bytes) else str(raw))

        async def scale(r):
            body = await r.json()
            try:
                out = await self.scale(body.get("kind", ""), body.get("namespace", "default"), body["name"], int(body["replicas"]))
            except m.StatusError as e:
                return fail(e)
            return web.json_response(out)

        async def delete_pod(r):
            try:
                await self.client.delete("pods", r.match_info["name"], r.match_info["ns"])
            except m.StatusError as e:
                return fail(e)
            return web.json_response({"deleted": f"{r.match_info['ns']}/{r.match_info['name']}"})

        async def logs(r):
            if not self.log_store_url:
                return web.json_response({"error": "no log store configured (--log-store-url)"}, status=404)
            import aiohttp
            must = []
            if r.query.get("namespace"):
                must.append({"term": {"kubernetes.namespace_name": r.query["namespace"]}})
            if r.query.get("pod"):
                must.append({"term": {"kubernetes.pod_name": r.query["pod"]}})
            if r.query.get("q"):
                must.append({"query_string": {"query": r.query["q"]}})
            q = {"query": {"bool": {"must": must}} if must else {"match_all": {}}, "size": int(r.query.get("size", 200)),
                 "sort": [{"@timestamp": "desc"}]}
            async with aiohttp.ClientSession() as s:
                async with s.post(f"{self.log_store_url}/logstash-*/_search", json=q) as resp:
                    body = await resp.json(content_type=None)
            return web.json_response([h["_source"] for h in (body.get("hits") or {}).get("hits", [])])

        a = web.Application()
        a.router.add_get("/", index)
        a.router.add_get("/healthz", lambda _r: web.Response(text="ok"))
        a.router.add_get("/api/namespaces", namespaces)
        a.router.add_get("/api/overview", overview)
        a.router.add_get("/api/pods/{ns}/{name}/log", pod_log)
        a.router.add_delete("/api/pods/{ns}/{name}", delete_pod)
        a.router.add_post("/api/scale", scale)
        a.router.add_get("/api/logs", logs)
        return a


PAGE = """<!doctype html>
<html><head><meta charset="utf-8"><title>amdkube dashboard</title>
<style>
body{font-family:sans-serif;margin:0;background:#f4f5f7;color:#222}
header{background:#1f2937;color:#fff;padding:10px 18px;display:flex;gap:16px;align-items:center}
header h1{font-size:18px;margin:0}
main{padding:14px 18px}
section{background:#fff;border-radius:6px;padding:10px 14px;margin-bottom:14px;box-shadow:0 1px 2px #0002}
h2{font-size:15px;margin:4px 0 8px}
table{border-collapse:collapse;width:100%;font-size:13px}
th,td{text-align:left;padding:4px 8px;border-bottom:1px solid #e5e7eb}
.bad{color:#b91c1c}.ok{color:#15803d}
button{font-size:12px}
pre{background:#111;color:#ddd;padding:8px;max-height:360px;overflow:auto;font-size:12px}
</style></head>
<body>
<header><h1>amdkube</h1>
<label>namespace <select id="ns"><option value="">(all)</option></select></label>
<span id="status"></span></header>
<main>
<section><h2>Nodes</h2><table id="nodes"></table></section>
<section><h2>Workloads</h2><table id="workloads"></table></section>
<section><h2>Pods</h2><table id="pods"></table></section>
<section><h2>Services</h2><table id="services"></table></section>
<section><h2>Events</h2><table id="events"></table></section>
<section><h2>Logs</h2><input id="q" placeholder="search the cluster log store"> <button onclick="searchLogs()">search</button>
<pre id="log"></pre></section>
</main>
<script>
const $ = id => document.getElementById(id);
const esc = s => String(s ?? '').replace(/[&<>"]/g, c => ({'&':'&amp;','<':'&lt;','>':'&gt;','"':'&quot;'}[c]));
function table(id, cols, rows, extra) {
  $(id).innerHTML = '<tr>' + cols.map(c => '<th>' + c[0] + '</th>').join('') + (extra ? '<th></th>' : '') + '</tr>' +
    rows.map(r => '<tr>' + cols.map(c => '<td>' + c[1](r) + '</td>').join('') + (extra ? '<td>' + extra(r) + '</td>' : '') + '</tr>').join('');
}
async function api(path, opts) { const r = await fetch(path, opts); if (!r.ok) throw new Error(await r.text()); return r; }
async function load() {
  const ns = $('ns').value;
  try {
    const o = await (await api('/api/overview?namespace=' + encodeURIComponent(ns))).json();
    table('nodes', [['name', n => esc(n.name)], ['ready', n => n.ready ? '<span class=ok>Ready</span>' : '<span class=bad>NotReady</span>'],
      ['cpu', n => esc(n.cpu)], ['memory', n => esc(n.memory)], ['GPU type', n => esc(n.gpus.type)],
      ['GPUs used/alloc/cap', n => n.gpus.allocated + '/' + n.gpus.allocatable + '/' + n.gpus.capacity],
      ['unhealthy', n => n.gpus.unhealthy ? '<span class=bad>' + n.gpus.unhealthy + '</span>' : '0'], ['age', n => esc(n.age)]], o.nodes);
    table('workloads', [['kind', w => esc(w.kind)], ['namespace', w => esc(w.namespace)], ['name', w => esc(w.name)],
      ['ready/desired', w => w.ready + '/' + w.desired], ['age', w => esc(w.age)]], o.workloads,
      w => ['deployments', 'replicasets', 'statefulsets'].includes(w.kind) ?
        '<button onclick="scale(\\'' + w.kind.slice(0, -1) + '\\',\\'' + esc(w.namespace) + '\\',\\'' + esc(w.name) + '\\',' + w.desired + ')">scale</button>' : '');
    table('pods', [['namespace', p => esc(p.namespace)], ['name', p => esc(p.name)], ['phase', p => esc(p.phase) + (p.reason ? ' (' + esc(p.reason) + ')' : '')],
      ['ready', p => esc(p.ready)], ['restarts', p => p.restarts], ['GPUs', p => p.gpus], ['node', p => esc(p.node)], ['age', p => esc(p.age)]], o.pods,
      p => '<button onclick="showLog(\\'' + esc(p.namespace) + '\\',\\'' + esc(p.name) + '\\')">logs</button> ' +
           '<button onclick="del(\\'' + esc(p.namespace) + '\\',\\'' + esc(p.name) + '\\')">delete</button>');
    table('services', [['namespace', s => esc(s.namespace)], ['name', s => esc(s.name)], ['type', s => esc(s.type)],
      ['cluster IP', s => esc(s.clusterIP)], ['ports', s => esc(s.ports.join(', '))]], o.services);
    table('events', [['type', e => esc(e.type)], ['reason', e => esc(e.reason)], ['object', e => esc(e.object)],
      ['message', e => esc(e.message)], ['count', e => e.count], ['last', e => esc(e.last)]], o.events);
    $('status').textContent = 'updated ' + new Date().toLocaleTimeString();
  } catch (e) { $('status').textContent = 'error: ' + e.message; }
}
async function showLog(ns, name) { $('log').textContent = await (await api('/api/pods/' + ns + '/' + name + '/log?tailLines=500')).text(); }
async function del(ns, name) { if (confirm('delete pod ' + ns + '/' + name + '?')) { await api('/api/pods/' + ns + '/' + name, {method: 'DELETE'}); load(); } }
async function scale(kind, ns, name, cur) {
  const n = prompt('replicas for ' + ns + '/' + name, cur); if (n === null) return;
  await api('/api/scale', {method: 'POST', headers: {'Content-Type': 'application/json'},
    body: JSON.stringify({kind, namespace: ns, name, replicas: parseInt(n)})}); load();
}
async function searchLogs() {
  const ns = $('ns').value, q = $('q').value;
  try {
    const hits = await (await api('/api/logs?q=' + encodeURIComponent(q) + '&namespace=' + encodeURIComponent(ns))).json();
    $('log').textContent = hits.map(h => h['@timestamp'] + ' ' + ((h.kubernetes || {}).pod_name || h.tag || '') + ' ' + (h.log || h.message || '')).join('');
  } catch (e) { $('log').textContent = e.message; }
}
(async () => {
  for (const n of await (await api('/api/namespaces')).json()) { const o = document.createElement('option'); o.textContent = n; $('ns').appendChild(o); }
  $('ns').onchange = load; load(); setInterval(load, 10000);
})();
</script></body></html>
"""

