"""amdgpu-exporter: amd-smi → Prometheus (replaces the DCGM exporter the reference's README
promises, README.md:57, which is not in the repo — SURVEY §0.2 row 2).

Serves `/metrics` with
  * node-level series `amd_gpu_*{gpu, uuid, node, model, pod, namespace, container}`:
    utilization_percent, memory_utilization_percent (instantaneous) and their 10 s means
    utilization_avg10s_percent / memory_utilization_avg10s_percent (native background
    sampler, native/sampler_core.h), vram_used_bytes, vram_total_bytes,
    power_watts, power_limit_watts, temperature_celsius, temperature_memory_celsius,
    ecc_correctable_total, ecc_uncorrectable_total, ecc_deferred_total,
    xgmi_link_read_bytes_total / xgmi_link_write_bytes_total {peer}, health (1 = Healthy),
    process_vram_bytes {pid};
  * cAdvisor-compatible per-container series container_accelerator_{memory_total_bytes,
    memory_used_bytes,duty_cycle} (vendor/github.com/google/cadvisor/metrics/prometheus.go:275-306).
Pod/container attribution comes from the kubelet's /pods (assigned device IDs), so the
exporter works with any container runtime. Scrape config + Grafana dashboard in deploy/.
"""
from __future__ import annotations

import asyncio
import logging
import time

import aiohttp
from aiohttp import web

from ..smi import Backend, device_id
from .collector import DUTY_CYCLE_WINDOW_S, duty_cycle
from ..utils.metrics import CONTENT_TYPE

log = logging.getLogger("amdkube.exporter")


def _esc(v) -> str:
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", " ")


class Exporter:
    def __init__(self, backend: Backend, node: str = "", kubelet_url: str | None = None, ecc_threshold: int = 0):
        self.b = backend
        self.node = node
        self.kubelet_url = kubelet_url
        self.ecc_threshold = ecc_threshold
        from ..smi.health import HealthMonitor
        self.monitor = HealthMonitor(backend, ecc_threshold)     # same judgement as the device plugin
        self.gpus = backend.gpus()
        self.sampling = backend.start_sampling()
        self.scrapes = 0
        self._runner = None
        self.port = None

    async def pod_map(self) -> dict[str, tuple[str, str, str]]:
        """device id -> (namespace, pod, container) from the kubelet's running pods."""
        if not self.kubelet_url:
            return {}
        out = {}
        try:
            async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=2)) as s:
                async with s.get(self.kubelet_url.rstrip("/") + "/pods") as r:
                    pods = (await r.json()).get("items") or []
        except Exception as e:
            log.debug("kubelet /pods unavailable: %r", e)
            return {}
        from ..kubelet.devicemanager import container_device_requests
        for p in pods:
            if (p.get("status") or {}).get("phase") not in ("Running", "Pending"):
                continue
            md = p.get("metadata") or {}
            for c in (p.get("spec") or {}).get("containers") or []:
                for ids in container_device_requests(p, c).values():
                    for d in ids:
                        out[d] = (md.get("namespace", ""), md.get("name", ""), c["name"])
        return out

    def collect(self, owners: dict) -> str:
        L = []
        fam: dict[str, list[str]] = {}

        def add(name, labels: dict, value, help_=""):
            lab = ",".join(f'{k}="{_esc(v)}"' for k, v in labels.items())
            fam.setdefault(name, [help_]).append(f"{name}{{{lab}}} {value}")
        for g in self.gpus:
            did = device_id(g)
            ns, pod, ctr = owners.get(did, ("", "", ""))
            base = {"gpu": g["index"], "uuid": did, "node": self.node, "model": g.get("market_name", ""),
                    "namespace": ns, "pod": pod, "container": ctr}
            try:
                s = self.b.sample(g["index"])
                up = 1
            except Exception:
                s, up = {}, 0
            healthy = 1 if up and self.monitor.check(g["index"])[0] else 0
            add("amd_gpu_up", base, up, "1 if the GPU answered the last amd-smi query")
            add("amd_gpu_health", base, healthy,
                "1 if the GPU is schedulable (no new uncorrectable ECC/xGMI/bad-page faults since the exporter started)")
            try:
                ras = self.b.ras(g["index"]) if up else {}
            except Exception:
                ras = {}
            if "xgmi_error" in ras:
                add("amd_gpu_xgmi_error_status", base, ras["xgmi_error"], "xGMI error status (0 none, 1 error, 2 multiple)")
            for state in ("retired", "pending", "unreservable"):
                if f"bad_pages_{state}" in ras:
                    add("amd_gpu_bad_pages", dict(base, state=state), ras[f"bad_pages_{state}"],
                        "HBM pages the driver retired, has pending retirement, or could not reserve")
            add("amd_gpu_vram_total_bytes", base, int(g.get("vram_total_bytes") or 0), "Total HBM (VRAM) in bytes")
            for key, name, help_ in (("gfx_activity", "amd_gpu_utilization_percent", "GFX engine busy percent"),
                                     ("umc_activity", "amd_gpu_memory_utilization_percent", "Memory controller busy percent"),
                                     ("vram_used_bytes", "amd_gpu_vram_used_bytes", "Used HBM (VRAM) in bytes"),
                                     ("temperature_c", "amd_gpu_temperature_celsius", "Hotspot temperature"),
                                     ("temperature_mem_c", "amd_gpu_temperature_memory_celsius", "HBM temperature"),
                                     ("ecc_correctable", "amd_gpu_ecc_correctable_total", "Correctable ECC errors"),
                                     ("ecc_uncorrectable", "amd_gpu_ecc_uncorrectable_total", "Uncorrectable ECC errors"),
                                     ("ecc_deferred", "amd_gpu_ecc_deferred_total", "Deferred ECC errors")):
                if key in s:
                    add(name, base, s[key], help_)
            if self.sampling:
                try:
                    avg = self.b.average_activity(g["index"], DUTY_CYCLE_WINDOW_S)
                except Exception:
                    avg = None
                if avg:
                    add("amd_gpu_utilization_avg10s_percent", base, round(avg["gfx_activity"], 2),
                        "GFX engine busy percent, mean of the background samples over the last 10 s")
                    if "umc_activity" in avg:
                        add("amd_gpu_memory_utilization_avg10s_percent", base, round(avg["umc_activity"], 2),
                            "Memory controller busy percent, mean over the last 10 s")
            for key, name in (("power_watts", "amd_gpu_power_watts"), ("power_limit_watts", "amd_gpu_power_limit_watts")):
                if key in s:
                    v = s[key]
                    add(name, base, v / 1e6 if v > 1e5 else v, "Socket power in watts")  # some firmware reports µW
            try:
                for lk in self.b.link_metrics(g["index"]):
                    lb = dict(base, peer=lk.get("peer_bdf", ""), link=lk.get("type", ""))
                    add("amd_gpu_xgmi_link_read_bytes_total", lb, int(lk.get("read_kb", 0)) * 1024, "xGMI bytes received")
                    add("amd_gpu_xgmi_link_write_bytes_total", lb, int(lk.get("write_kb", 0)) * 1024, "xGMI bytes sent")
            except Exception:
                pass
            try:
                for pr in self.b.processes(g["index"]):
                    add("amd_gpu_process_vram_bytes", dict(base, pid=pr.get("pid")), pr.get("vram_bytes", 0), "VRAM held by a process")
            except Exception:
                pass
            if pod:
                cl = {"container_name": ctr, "pod_name": pod, "namespace": ns, "make": "amd", "model": g.get("market_name", ""),
                      "acc_id": did}
                add("container_accelerator_memory_total_bytes", cl, int(g.get("vram_total_bytes") or 0), "Total accelerator memory.")
                add("container_accelerator_memory_used_bytes", cl, int(s.get("vram_used_bytes") or 0), "Total accelerator memory allocated.")
                add("container_accelerator_duty_cycle", cl, duty_cycle(self.b, g["index"], s),
                    "Percent of time over the past sample period during which the accelerator was actively processing.")
        for name, lines in fam.items():
            L.append(f"# HELP {name} {lines[0]}")
            L.append(f"# TYPE {name} {'counter' if name.endswith('_total') else 'gauge'}")
            L.extend(lines[1:])
        return "\n".join(L) + "\n"

    async def metrics(self, req):
        t0 = time.perf_counter()
        owners = await self.pod_map()
        text = await asyncio.to_thread(self.collect, owners)
        self.scrapes += 1
        text += f"# HELP amd_gpu_exporter_scrape_duration_seconds Time to collect all GPU metrics\n" \
                f"# TYPE amd_gpu_exporter_scrape_duration_seconds gauge\n" \
                f'amd_gpu_exporter_scrape_duration_seconds{{node="{_esc(self.node)}"}} {time.perf_counter() - t0:.6f}\n'
        return web.Response(text=text, headers={"Content-Type": CONTENT_TYPE})

    async def start(self, host="0.0.0.0", port=9400):
        app = web.Application()
        app.router.add_get("/metrics", self.metrics)
        app.router.add_get("/healthz", lambda r: web.Response(text="ok"))
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, host, port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        if self._runner:
            await self._runner.cleanup()
