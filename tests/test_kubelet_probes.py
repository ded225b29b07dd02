"""Liveness/readiness end to end on an in-process node: the restart semantics of
kuberuntime_manager.go computePodActions/doBackOff and the prober workers together.

* restartPolicy Never + a failing liveness probe: the container is killed once, never
  restarted; the pod ends Failed with restartCount 0.
* restartPolicy Always + a failing liveness probe: each kill restarts the container with the
  attempt carried over (restartCount grows, lastState.terminated filled) and the restarts go
  through the back-off (CrashLoopBackOff shows up).
* an httpGet liveness probe on a *named* port against the pod IP keeps a healthy server
  running (restartCount stays 0), with its headers sent.
"""
import asyncio
import socket

from amdkube.localcluster import LocalCluster, wait_pod
from tests.conftest import run


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _failing_liveness(name, policy):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {"restartPolicy": policy, "terminationGracePeriodSeconds": 1,
                     "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "300"],
                                     "livenessProbe": {"exec": {"command": ["false"]}, "periodSeconds": 1,
                                                       "failureThreshold": 1}}]}}


def test_never_pod_failing_liveness_is_killed_once_and_fails():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False) as lc:
            c = lc.client
            await c.create(_failing_liveness("never", "Never"))
            p = await wait_pod(c, "default", "never", ("Failed",), 40)
            cs = p["status"]["containerStatuses"][0]
            assert cs["restartCount"] == 0 and "terminated" in cs["state"], cs
            await asyncio.sleep(2.5)    # no further restarts after the pod failed
            p = await c.get("pods", "never", "default")
            assert p["status"]["phase"] == "Failed" and p["status"]["containerStatuses"][0]["restartCount"] == 0
            for _ in range(50):
                ev, _ = await c.list("events", "default")
                reasons = [e["reason"] for e in ev if e["involvedObject"]["name"] == "never"]
                if "Unhealthy" in reasons and "Killing" in reasons:
                    break
                await asyncio.sleep(0.1)
            assert "Unhealthy" in reasons and reasons.count("Killing") == 1, reasons
    run(go(), 90)


def test_always_pod_failing_liveness_restarts_with_count_and_backoff():
    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False) as lc:
            c = lc.client
            lc.kubelet.runtime.backoff.default = 2.0
            await c.create(_failing_liveness("always", "Always"))
            seen_counts, crashloop, last = set(), False, None
            for _ in range(300):
                p = await c.get("pods", "always", "default")
                for cs in p["status"].get("containerStatuses") or []:
                    seen_counts.add(cs.get("restartCount", 0))
                    if ((cs.get("state") or {}).get("waiting") or {}).get("reason") == "CrashLoopBackOff":
                        crashloop = True
                    if (cs.get("restartCount", 0) >= 2 and "running" in (cs.get("state") or {})
                            and "terminated" in (cs.get("lastState") or {})):
                        last = cs
                if crashloop and max(seen_counts) >= 2 and last:
                    break
                await asyncio.sleep(0.1)
            assert max(seen_counts) >= 2, seen_counts
            assert crashloop, "restarts never went through the back-off"
            assert last["lastState"]["terminated"]["containerID"] != last.get("containerID")
            assert p["status"]["phase"] == "Running"
    run(go(), 90)


def test_named_port_http_liveness_keeps_healthy_server():
    async def go():
        port = _free_port()
        server = ("import http.server, sys\n"
                  "class H(http.server.BaseHTTPRequestHandler):\n"
                  "    def do_GET(self):\n"
                  "        ok = self.path == '/healthz' and self.headers.get('X-Probe') == 'yes'\n"
                  "        self.send_response(200 if ok else 500); self.end_headers(); self.wfile.write(b'ok')\n"
                  "    def log_message(self, *a): pass\n"
                  f"http.server.HTTPServer(('127.0.0.1', {port}), H).serve_forever()\n")
        async with LocalCluster(gpus="none", relist_period=0.2, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "web", "namespace": "default"},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["python3", "-c", server],
                                                     "ports": [{"name": "http", "containerPort": port}],
                                                     "livenessProbe": {"httpGet": {"path": "/healthz", "port": "http",
                                                                                   "httpHeaders": [{"name": "X-Probe", "value": "yes"}]},
                                                                       "periodSeconds": 1, "failureThreshold": 5,
                                                                       "initialDelaySeconds": 3, "timeoutSeconds": 5},
                                                     "readinessProbe": {"httpGet": {"path": "/healthz", "port": "http",
                                                                                    "httpHeaders": [{"name": "X-Probe", "value": "yes"}]},
                                                                        "periodSeconds": 1}}]}})
            await wait_pod(c, "default", "web", ("Running",), 30)
            ready = False
            for _ in range(300):
                p = await c.get("pods", "web", "default")
                if p["status"]["containerStatuses"][0]["ready"]:
                    ready = True
                    break
                await asyncio.sleep(0.1)
            assert ready, p["status"]
            w = lc.kubelet.probes.workers
            assert len(w) == 2
            await asyncio.sleep(4)
            assert all(x.probes >= 1 for x in w.values())
            p = await c.get("pods", "web", "default")
            cs = p["status"]["containerStatuses"][0]
            assert cs["restartCount"] == 0 and "running" in cs["state"] and cs["ready"], cs
            assert sum(x.probes for x in w.values()) >= 6
    run(go(), 90)
