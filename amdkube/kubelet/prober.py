"""Container probes: one worker task per (pod, container, probe type).

Reference pkg/kubelet/prober:
* prober.go — `probe` (:83-121: a probe with no spec is a Success, a failing or erroring probe
  is a Failure with an `Unhealthy` event), `runProbeWithRetries` (:125, maxProbeRetries = 3
  on error), `runProbe` (:147-199: exec in the container with the command expanded from the
  container's static env; HTTP GET / TCP to `status.podIP` unless a host is given; the port
  by number or by container port name), `extractPort` (:201), `findPortByName` (:224),
  `formatURL` (:235), `buildHeader` (:137);
* worker.go — `doProbe` (:141-232: no status ⇒ wait; terminal pod ⇒ stop; a new container id
  resets the result to the probe's initial value and lifts the hold; a non-running container
  is a Failure; initial delay from the container's start; success/failure thresholds over
  runs of equal results; a liveness Failure puts the worker on hold until a new container)
  and `run` (:97: a random fraction of the period first, then every period);
* prober_manager.go — AddPod/RemovePod/CleanupPods and UpdatePodStatus readiness;
* results/results_manager.go — the per-container-id result cache with change updates;
* pkg/probe/{exec,http,tcp} — exit status, HTTP 2xx/3xx (TLS not verified, `kube-probe/1.9`
  User-Agent, a `Host` header sets the request host), TCP connect.

The workers are asyncio tasks on the kubelet loop; a probe never blocks another one.
"""
from __future__ import annotations

import asyncio
import logging
import random
import time
import urllib.parse

from ..api import meta as m

log = logging.getLogger("amdkube.kubelet.prober")

LIVENESS, READINESS = "Liveness", "Readiness"
SUCCESS, FAILURE, UNKNOWN = "success", "failure", "unknown"     # pkg/probe Result
MAX_PROBE_RETRIES = 3
USER_AGENT = "kube-probe/1.9"
PROBE_DEFAULTS = {"timeoutSeconds": 1, "periodSeconds": 10, "successThreshold": 1, "failureThreshold": 3}


# ------------------------------------------------------------------ helpers
def find_port_by_name(container: dict, name: str) -> int:
    for p in container.get("ports") or []:
        if p.get("name") == name:
            return int(p.get("containerPort", 0))
    raise ValueError(f"port {name} not found")


def extract_port(param, container: dict) -> int:
    """intstr port: a number, a container port name, or a number written as a string."""
    if isinstance(param, bool) or param is None:
        raise ValueError(f"IntOrString had no kind: {param!r}")
    if isinstance(param, int):
        port = param
    else:
        try:
            port = find_port_by_name(container, str(param))
        except ValueError:
            try:
                port = int(str(param), 10)
            except ValueError:
                raise ValueError(f'strconv.Atoi: parsing "{param}": invalid syntax') from None
    if 0 < port < 65536:
        return port
    raise ValueError(f"invalid port number: {port}")


def format_url(scheme: str, host: str, port: int, path: str) -> str:
    u = urllib.parse.urlsplit(path or "")
    hostport = f"[{host}]:{port}" if ":" in host else f"{host}:{port}"
    return urllib.parse.urlunsplit((scheme, hostport, u.path, u.query, u.fragment))


def build_header(headers: list | None) -> dict[str, list[str]]:
    out: dict[str, list[str]] = {}
    for h in headers or []:
        out.setdefault(_canonical(h["name"]), []).append(h.get("value", ""))
    return out


def _canonical(name: str) -> str:
    """textproto.CanonicalMIMEHeaderKey (http.Header keys)."""
    if not name or any(c in name for c in " :\t"):
        return name
    return "-".join(p[:1].upper() + p[1:].lower() for p in name.split("-"))


def expand_only_static(cmd: list, env: list | None) -> list:
    """kubecontainer.ExpandContainerCommandOnlyStatic: $(VAR) from env entries with a literal
    value only (valueFrom is not resolved for probes)."""
    from .podcontext import expand
    mapping = {e["name"]: e.get("value", "") for e in env or [] if "valueFrom" not in e}
    return [expand(x, mapping) for x in cmd or []]


# ------------------------------------------------------------------ probers
class ExecProber:
    """pkg/probe/exec: exit 0 ⇒ success, another exit status ⇒ failure, a runner error ⇒
    unknown with the error. `runner(cid, cmd, timeout) -> (output, exit_code)`."""

    async def probe(self, runner, cid: str, cmd: list, timeout: float):
        try:
            out, code = await runner(cid, cmd, timeout)
        except Exception as e:       # grpc.RpcError, timeout, ...
            return UNKNOWN, "", e
        return (SUCCESS if code == 0 else FAILURE), out, None


class HTTPProber:
    async def probe(self, url: str, headers: dict[str, list[str]], timeout: float):
        import aiohttp
        hdrs = [(k, v) for k, vs in headers.items() for v in vs]
        if "User-Agent" not in headers:
            hdrs.append(("User-Agent", USER_AGENT))
        try:
            async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout),
                                             connector=aiohttp.TCPConnector(ssl=False, force_close=True)) as s:
                async with s.get(url, headers=hdrs, allow_redirects=True) as r:
                    body = await r.text(errors="replace")
                    if 200 <= r.status < 400:
                        return SUCCESS, body, None
                    return FAILURE, f"HTTP probe failed with statuscode: {r.status}", None
        except Exception as e:        # timeouts and connection errors are failures, not errors
            return FAILURE, str(e) or type(e).__name__, None


class TCPProber:
    async def probe(self, host: str, port: int, timeout: float):
        try:
            _, w = await asyncio.wait_for(asyncio.open_connection(host, port), timeout)
        except Exception as e:
            return FAILURE, str(e) or type(e).__name__, None
        w.close()
        return SUCCESS, "", None


class Prober:
    def __init__(self, runner=None, recorder=None):
        self.runner = runner          # async (cid, cmd, timeout) -> (output, exit code)
        self.recorder = recorder
        self.exec = ExecProber()
        self.readiness_http = HTTPProber()
        self.liveness_http = HTTPProber()
        self.tcp = TCPProber()

    async def probe(self, probe_type: str, pod: dict, status: dict, container: dict, cid: str):
        """(result, error): result True = Success, False = Failure."""
        spec = container.get("livenessProbe" if probe_type == LIVENESS else "readinessProbe")
        if spec is None:
            return True, None
        result, output, err = await self.run_with_retries(probe_type, spec, pod, status, container, cid)
        if err is not None or result != SUCCESS:
            if self.recorder is not None:
                msg = f"{probe_type} probe errored: {err}" if err is not None else f"{probe_type} probe failed: {output}"
                self.recorder.event(pod, "Warning", "Unhealthy", msg)
            return False, err
        return True, None

    async def run_with_retries(self, probe_type, spec, pod, status, container, cid, retries: int = MAX_PROBE_RETRIES):
        result, output, err = UNKNOWN, "", None
        for _ in range(retries):
            result, output, err = await self.run_probe(probe_type, spec, pod, status, container, cid)
            if err is None:
                break
        return result, output, err

    async def run_probe(self, probe_type, spec, pod, status, container, cid):
        timeout = float(spec.get("timeoutSeconds") or PROBE_DEFAULTS["timeoutSeconds"])
        if spec.get("exec") is not None:
            cmd = expand_only_static(spec["exec"].get("command"), container.get("env"))
            return await self.exec.probe(self.runner, cid, cmd, timeout)
        if spec.get("httpGet") is not None:
            h = spec["httpGet"]
            host = h.get("host") or (status or {}).get("podIP") or ""
            try:
                port = extract_port(h.get("port"), container)
            except ValueError as e:
                return UNKNOWN, "", e
            url = format_url((h.get("scheme") or "HTTP").lower(), host, port, h.get("path") or "")
            prober = self.liveness_http if probe_type == LIVENESS else self.readiness_http
            return await prober.probe(url, build_header(h.get("httpHeaders")), timeout)
        if spec.get("tcpSocket") is not None:
            t = spec["tcpSocket"]
            try:
                port = extract_port(t.get("port"), container)
            except ValueError as e:
                return UNKNOWN, "", e
            host = t.get("host") or (status or {}).get("podIP") or ""
            return await self.tcp.probe(host, port, timeout)
        md = pod.get("metadata") or {}
        return UNKNOWN, "", RuntimeError(f"Missing probe handler for {md.get('name')}_{md.get('namespace')}"
                                         f"({md.get('uid')}):{container.get('name')}")


# ------------------------------------------------------------------ results
class ResultsManager:
    """results_manager.go: container id -> last result; `on_update(cid, result, pod)` fires
    only when the cached value changes (the Updates channel)."""

    def __init__(self, on_update=None):
        self.cache: dict[str, bool] = {}
        self.on_update = on_update

    def get(self, cid: str):
        return self.cache.get(cid)

    def set(self, cid: str, result: bool, pod: dict):
        if cid not in self.cache or self.cache[cid] != result:
            self.cache[cid] = result
            if self.on_update is not None:
                self.on_update(cid, result, pod)

    def remove(self, cid: str):
        self.cache.pop(cid, None)


# ------------------------------------------------------------------ worker
class Worker:
    def __init__(self, mgr: "ProbeManager", probe_type: str, pod: dict, container: dict):
        self.mgr, self.probe_type, self.pod, self.container = mgr, probe_type, pod, container
        if probe_type == READINESS:
            self.spec = {**PROBE_DEFAULTS, **container["readinessProbe"]}
            self.results, self.initial = mgr.readiness, False
        else:
            self.spec = {**PROBE_DEFAULTS, **container["livenessProbe"]}
            self.results, self.initial = mgr.liveness, True
        for k, v in PROBE_DEFAULTS.items():      # SetDefaults_Probe: zero means the default
            if not self.spec.get(k):
                self.spec[k] = v
        self.container_id = ""
        self.last_result = None
        self.result_run = 0
        self.on_hold = False
        self._stop = asyncio.Event()
        self.task = None
        self.probes = 0

    def stop(self):
        self._stop.set()

    async def run(self):
        period = float(self.spec["periodSeconds"])
        try:
            if self.mgr.jitter:
                # worker.go:101 after a kubelet restart probes would start in lock step
                if await self._wait(random.random() * period):
                    return
            while await self.do_probe():
                if await self._wait(period):
                    break
        finally:
            if self.container_id:
                self.results.remove(self.container_id)
            self.mgr._remove_worker(self)

    async def _wait(self, secs: float) -> bool:
        try:
            await asyncio.wait_for(self._stop.wait(), secs)
            return True
        except asyncio.TimeoutError:
            return False

    async def do_probe(self) -> bool:
        """One probe; False when the worker should exit (worker.go doProbe)."""
        try:
            return await self._do_probe()
        except asyncio.CancelledError:
            raise
        except Exception as e:      # HandleCrash: a crashing probe keeps the worker going
            log.warning("probe worker %s/%s crashed: %r", m.name_of(self.pod), self.container.get("name"), e)
            return True

    async def _do_probe(self) -> bool:
        status = self.mgr.status_of(m.uid_of(self.pod))
        if status is None:
            return True
        if status.get("phase") in ("Failed", "Succeeded"):
            return False
        c = next((cs for cs in status.get("containerStatuses") or [] if cs.get("name") == self.container["name"]), None)
        if c is None or not c.get("containerID"):
            return True
        if self.container_id != c["containerID"]:
            if self.container_id:
                self.results.remove(self.container_id)
            self.container_id = c["containerID"]
            self.results.set(self.container_id, self.initial, self.pod)
            self.on_hold = False      # a new container: probe again
        if self.on_hold:
            return True
        state = c.get("state") or {}
        if "running" not in state:
            if self.container_id:
                self.results.set(self.container_id, False, self.pod)
            return "terminated" not in state or (self.pod.get("spec") or {}).get("restartPolicy") != "Never"
        started = m.parse_time((state["running"] or {}).get("startedAt"))
        if started is not None and int(time.time() - started) < int(self.spec.get("initialDelaySeconds") or 0):
            return True
        self.probes += 1
        result, err = await self.mgr.prober.probe(self.probe_type, self.pod, status, self.container, self.container_id)
        if err is not None:
            return True     # prober error: the result is thrown away
        if self.last_result == result:
            self.result_run += 1
        else:
            self.last_result, self.result_run = result, 1
        if (not result and self.result_run < int(self.spec["failureThreshold"])) or \
                (result and self.result_run < int(self.spec["successThreshold"])):
            return True
        self.results.set(self.container_id, result, self.pod)
        if self.probe_type == LIVENESS and not result:
            # stop probing a container that is about to be killed until a new one shows up
            self.on_hold = True
            self.result_run = 1
        return True


# ------------------------------------------------------------------ manager
class ProbeManager:
    """prober_manager.go. `status_of(uid)` is the status manager's latest pod status;
    `on_change(uid)` is called when a readiness result changes or a liveness result turns
    Failure (the kubelet re-syncs the pod: status readiness / kill)."""

    def __init__(self, status_of, runner=None, recorder=None, on_change=None, jitter: bool = True):
        self.status_of = status_of
        self.on_change = on_change
        self.jitter = jitter
        self.prober = Prober(runner, recorder)
        self.readiness = ResultsManager(self._readiness_update)
        self.liveness = ResultsManager(self._liveness_update)
        self.workers: dict[tuple[str, str, str], Worker] = {}

    def _readiness_update(self, cid, result, pod):
        if self.on_change is not None:
            self.on_change(m.uid_of(pod))

    def _liveness_update(self, cid, result, pod):
        if not result and self.on_change is not None:
            self.on_change(m.uid_of(pod))

    def add_pod(self, pod: dict):
        uid = m.uid_of(pod)
        for c in (pod.get("spec") or {}).get("containers") or []:
            for kind, field in ((READINESS, "readinessProbe"), (LIVENESS, "livenessProbe")):
                if c.get(field) is None:
                    continue
                key = (uid, c["name"], kind)
                if key in self.workers:
                    log.error("%s probe already exists! %s - %s", kind, m.name_of(pod), c["name"])
                    return
                w = self.workers[key] = Worker(self, kind, pod, c)
                w.task = asyncio.get_running_loop().create_task(w.run(), name=f"probe-{kind}-{c['name']}")

    def remove_pod(self, pod_or_uid):
        uid = pod_or_uid if isinstance(pod_or_uid, str) else m.uid_of(pod_or_uid)
        for key, w in list(self.workers.items()):
            if key[0] == uid:
                w.stop()

    def cleanup_pods(self, active_uids):
        keep = set(active_uids)
        for key, w in list(self.workers.items()):
            if key[0] not in keep:
                w.stop()

    def _remove_worker(self, w: Worker):
        key = (m.uid_of(w.pod), w.container["name"], w.probe_type)
        if self.workers.get(key) is w:
            del self.workers[key]

    def has_worker(self, uid: str, cname: str, kind: str) -> bool:
        return (uid, cname, kind) in self.workers

    def readiness_of(self, uid: str, pod: dict, rt) -> dict[str, bool]:
        """UpdatePodStatus: a running container is ready when its readiness result is Success,
        or when it has no readiness worker; probe results are per container id."""
        out = {}
        for c in (pod.get("spec") or {}).get("containers") or []:
            if c.get("readinessProbe") is None:
                continue
            cs = rt.latest(c["name"]) if rt is not None else None
            r = self.readiness.get(f"rocshim://{cs.id}") if cs is not None else None
            out[c["name"]] = bool(r) if r is not None else not self.has_worker(uid, c["name"], READINESS)
        return out

    def liveness_failed(self, cid: str) -> bool:
        return self.liveness.get(f"rocshim://{cid}") is False

    async def stop(self):
        ws = list(self.workers.values())
        for w in ws:
            w.stop()
        tasks = [w.task for w in ws if w.task is not None]
        if tasks:
            await asyncio.gather(*tasks, return_exceptions=True)
