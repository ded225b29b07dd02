"""Kubelet HTTP API (reference pkg/kubelet/server/server.go:260-411): /healthz (with the
syncloop check), /pods, /runningpods/, /metrics, /metrics/cadvisor (per-container
accelerator series), /stats/summary (stats/v1alpha1 incl. Accelerators[], types.go:121-122,
213-230), /spec, /containerLogs/{ns}/{pod}/{container}, /run/{ns}/{pod}/{container}
(exec-sync), the streaming endpoints /exec, /attach and /portForward (relayed WebSockets to
the runtime's streaming server, server.go:296-330 with redirect-container-streaming=false) and
/debug/pprof."""
from __future__ import annotations

import asyncio
import os
import time

from aiohttp import web

from ..runtime import spdy

from ..api import meta as m
from ..grpcdesc.cri import CRI as C
from ..utils import profiling
from ..utils.metrics import CONTENT_TYPE, render


class KubeletServer:
    """mode "full": the authenticated API on --port (debugging handlers unless
    --enable-debugging-handlers=false); "readonly": --read-only-port, unauthenticated, only the
    default handlers (server.go ListenAndServeKubeletReadOnlyServer); "healthz": --healthz-port."""

    def __init__(self, kubelet, mode: str = "full"):
        self.k = kubelet
        self.mode = mode
        mws = [kubelet.auth.middleware()] if mode == "full" and getattr(kubelet, "auth", None) is not None else []
        app = self.app = web.Application(middlewares=mws)
        app.router.add_get("/healthz", self.healthz)
        app.router.add_get("/healthz/syncloop", self.healthz)
        if mode != "healthz":
            app.router.add_get("/pods", self.pods)
            app.router.add_get("/metrics", self.metrics)
            app.router.add_get("/metrics/cadvisor", self.metrics_cadvisor)
            app.router.add_get("/stats/summary", self.summary)
            app.router.add_get("/stats/", self.summary)
            app.router.add_get("/spec/", self.spec)
            app.router.add_get("/spec", self.spec)
        if mode == "full" and getattr(getattr(kubelet, "cfg", None), "enable_debugging_handlers", True):
            app.router.add_get("/runningpods/", self.running_pods)
            app.router.add_get("/containerLogs/{ns}/{pod}/{container}", self.logs)
            app.router.add_post("/run/{ns}/{pod}/{container}", self.run)
            for meth in ("GET", "POST"):
                app.router.add_route(meth, "/exec/{ns}/{pod}/{container}", self.exec_stream)
                app.router.add_route(meth, "/attach/{ns}/{pod}/{container}", self.attach_stream)
                app.router.add_route(meth, "/portForward/{ns}/{pod}", self.port_forward)
            profiling.add_routes(app)
        self.runner = None
        self.port = None

    def _ssl(self):
        """HTTPS when a serving certificate is configured (--tls-cert-file/--tls-private-key-file
        or the rotated kubelet-server-current.pem); client certificates are requested and
        verified against --client-ca-file. A rotation reloads the chain for new handshakes."""
        cert, key = self.k.serving_cert()
        if not cert:
            return None
        import ssl
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(cert, key)
        if self.k.cfg.client_ca_file:
            ctx.load_verify_locations(self.k.cfg.client_ca_file)
            ctx.verify_mode = ssl.CERT_OPTIONAL
        self.ssl = ctx
        return ctx

    def reload_cert(self, _path=None):
        cert, key = self.k.serving_cert()
        if self.ssl is not None and cert:
            self.ssl.load_cert_chain(cert, key)

    async def start(self, host, port):
        self.runner = web.AppRunner(self.app, access_log=None)
        await self.runner.setup()
        self.ssl = None
        site = web.TCPSite(self.runner, host, port, reuse_address=True, ssl_context=self._ssl() if self.mode == "full" else None)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        if self.runner:
            await self.runner.cleanup()

    async def healthz(self, req):
        # the sync loop is healthy if a pod worker or the housekeeping pass ran recently
        if time.time() - self.k.last_sync_loop > max(120.0, 2 * self.k.cfg.sync_frequency):
            return web.Response(status=500, text="syncloop failed: no sync in the last interval")
        return web.Response(text="ok")

    async def pods(self, req):
        items = []
        for uid, p in self.k.pods.items():
            p = dict(p)
            st = self.k.status.get(uid)
            if st:
                p["status"] = st
            items.append(p)
        return web.json_response({"kind": "PodList", "apiVersion": "v1", "metadata": {}, "items": items})

    async def running_pods(self, req):
        out = []
        for s in await self.k.cri.list_pod_sandbox():
            if s.state != C.SANDBOX_READY:
                continue
            cs = await self.k.cri.list_containers(s.id)
            out.append({"metadata": {"name": s.metadata.name, "namespace": s.metadata.namespace, "uid": s.metadata.uid},
                        "spec": {"containers": [{"name": c.metadata.name, "image": c.image.image} for c in cs
                                                if c.state == C.CONTAINER_RUNNING]}})
        return web.json_response({"kind": "PodList", "apiVersion": "v1", "metadata": {}, "items": out})

    async def metrics(self, req):
        return web.Response(body=render(self.k.metrics), headers={"Content-Type": CONTENT_TYPE})

    async def metrics_cadvisor(self, req):
        return web.Response(text=await self.k.stats.render_cadvisor(), headers={"Content-Type": CONTENT_TYPE})

    def _pod_devices(self) -> list[dict]:
        """[{namespace, pod, container, devices: [ids]}] for running pods on this node."""
        from .devicemanager import container_device_requests
        out = []
        for uid, p in self.k.pods.items():
            st = self.k.status.get(uid) or {}
            if st.get("phase") != "Running":
                continue
            for c in (p.get("spec") or {}).get("containers") or []:
                ids = [d for lst in container_device_requests(p, c).values() for d in lst]
                if ids:
                    out.append({"namespace": m.namespace_of(p), "pod": m.name_of(p), "container": c["name"], "devices": ids})
        return out

    async def summary(self, req):
        return web.json_response(await self.k.stats.summary())

    async def spec(self, req):
        from ..monitoring.cadvisor import machine_info
        return web.json_response({**machine_info(), "accelerators": [dict(g) for g in (self.k.smi.gpus() if self.k.smi else [])]})

    async def _find_container(self, ns, pod, cname):
        for uid, p in self.k.pods.items():
            if m.namespace_of(p) == ns and m.name_of(p) == pod:
                rt = await self.k.runtime.pod_status(uid)
                return rt.latest(cname)
        return None

    @staticmethod
    def _flag(req, name, default=False) -> bool:
        v = req.query.get(name)
        return default if v is None else v.lower() in ("1", "true", "yes")

    async def exec_stream(self, req):
        from ..runtime.streaming import CHANNEL_PROTOCOLS, bridge
        ns, pod, cname = req.match_info["ns"], req.match_info["pod"], req.match_info["container"]
        cmd = req.query.getall("command", [])
        cs = await self._find_container(ns, pod, cname)
        if cs is None:
            return web.Response(status=404, text=f"container {cname} of pod {ns}/{pod} not found")
        if not cmd:
            return web.Response(status=400, text="command is required")
        url = await self.k.cri.exec_url(cs.id, cmd, self._flag(req, "tty"), self._flag(req, "stdin"),
                                        self._flag(req, "stdout", True), self._flag(req, "stderr", True))
        if spdy.is_upgrade(req):
            return await spdy.upgrade_proxy(req, url)
        ws = web.WebSocketResponse(protocols=CHANNEL_PROTOCOLS, max_msg_size=0)
        await ws.prepare(req)
        return await bridge(ws, url, [ws.ws_protocol or CHANNEL_PROTOCOLS[0]])

    async def attach_stream(self, req):
        from ..runtime.streaming import CHANNEL_PROTOCOLS, bridge
        ns, pod, cname = req.match_info["ns"], req.match_info["pod"], req.match_info["container"]
        cs = await self._find_container(ns, pod, cname)
        if cs is None:
            return web.Response(status=404, text=f"container {cname} of pod {ns}/{pod} not found")
        url = await self.k.cri.attach_url(cs.id, self._flag(req, "tty"), self._flag(req, "stdin"),
                                          self._flag(req, "stdout", True), self._flag(req, "stderr", True))
        if spdy.is_upgrade(req):
            return await spdy.upgrade_proxy(req, url)
        ws = web.WebSocketResponse(protocols=CHANNEL_PROTOCOLS, max_msg_size=0)
        await ws.prepare(req)
        return await bridge(ws, url, [ws.ws_protocol or CHANNEL_PROTOCOLS[0]])

    async def port_forward(self, req):
        from ..runtime.streaming import PORTFORWARD_PROTOCOLS, bridge
        ns, pod = req.match_info["ns"], req.match_info["pod"]
        ports = [int(p) for p in req.query.getall("port", []) + req.query.getall("ports", []) for p in p.split(",") if p]
        sid = None
        for uid, p in self.k.pods.items():
            if m.namespace_of(p) == ns and m.name_of(p) == pod:
                rt = await self.k.runtime.pod_status(uid)
                ready = rt.ready_sandbox()
                sid = ready[0] if ready else None
        if sid is None:
            return web.Response(status=404, text="pod sandbox not ready")
        if spdy.is_upgrade(req):          # SPDY clients name the port per stream (the `port` header)
            return await spdy.upgrade_proxy(req, await self.k.cri.port_forward_url(sid, ports))
        if not ports:
            return web.Response(status=400, text="port is required")
        url = await self.k.cri.port_forward_url(sid, ports)
        ws = web.WebSocketResponse(protocols=PORTFORWARD_PROTOCOLS, max_msg_size=0)
        await ws.prepare(req)
        return await bridge(ws, url + "?" + "&".join(f"port={p}" for p in ports), [ws.ws_protocol or PORTFORWARD_PROTOCOLS[0]])

    async def logs(self, req):
        """getContainerLogs (server.go:452-538) + GetKubeletContainerLogs (kubelet_pods.go:1216):
        query → PodLogOptions (422 when invalid), the pod and container must exist (404), the
        instance is chosen from the pod's status (validateContainerLogStatus; `previous` is the
        last terminated one), then ReadLogs streams the CRI log file."""
        from . import logs as L
        ns, pod, cname = req.match_info["ns"], req.match_info["pod"], req.match_info["container"]
        try:
            opts = L.decode_log_query(req.query)
        except ValueError:
            return web.Response(status=400, text='{"message": "Unable to decode query."}')
        if L.validate_pod_log_options(opts):
            return web.Response(status=422, text='{"message": "Invalid request."}')
        found = next(((uid, p) for uid, p in self.k.pods.items() if m.namespace_of(p) == ns and m.name_of(p) == pod), None)
        if found is None:
            return web.Response(status=404, text=f'pod "{pod}" does not exist\n')
        uid, p = found
        spec = p.get("spec") or {}
        if not any(c.get("name") == cname for c in (spec.get("containers") or []) + (spec.get("initContainers") or [])):
            return web.Response(status=404, text=f'container "{cname}" not found in pod "{pod}"\n')
        status = self.k.status.get(uid) or p.get("status") or {}
        try:
            cid = L.validate_container_log_status(pod, status, cname, bool(opts.get("previous")))
            st, _ = await self.k.cri.container_status(cid)
        except ValueError as e:
            return web.Response(status=400, text=str(e))
        except Exception as e:
            return web.Response(status=400, text=f'failed to get container status "{cid}": {e}')
        path = st.log_path
        resp = web.StreamResponse(headers={"Content-Type": "text/plain"})
        resp.enable_chunked_encoding()
        await resp.prepare(req)
        if path and os.path.exists(path):
            async def running():
                try:
                    s, _ = await self.k.cri.container_status(cid)
                except Exception:
                    return False
                return s.state == C.CONTAINER_RUNNING
            await L.read_logs(path, L.LogOptions.from_api(opts), resp.write, is_running=running,
                              state_check_period=float(getattr(self.k.cfg, "log_state_check_period", L.STATE_CHECK_PERIOD)))
        await resp.write_eof()
        return resp

    async def run(self, req):
        ns, pod, cname = req.match_info["ns"], req.match_info["pod"], req.match_info["container"]
        cs = await self._find_container(ns, pod, cname)
        if cs is None:
            return web.Response(status=404, text="container not found")
        cmd = req.query.getall("cmd", None) or (await req.text()).split()
        out, err, rc = await self.k.cri.exec_sync(cs.id, cmd, int(req.query.get("timeout", "30")))
        return web.Response(body=out + err, status=200 if rc == 0 else 500, headers={"X-Exit-Code": str(rc)})
