"""node-problem-detector: kernel-log problems → Node conditions and Events, with an amdgpu rule set.

The reference ships NPD as a cluster addon (cluster/addons/node-problem-detector/npd.yaml:46-51
runs `/node-problem-detector --system-log-monitors=/config/kernel-monitor.json,...`), and its
node e2e test pins the system-log-monitor contract (test/e2e_node/node_problem_detector_linux.go:
112-146 the config, :244-330 the expected behaviour):

  * a monitor config names a log `plugin` (`kmsg`: /dev/kmsg records; `filelog`: a text log whose
    lines are split by the `pluginConfig` `timestamp`/`message` regexes and parsed with the Go
    `timestampFormat`; `journald`: `journalctl -k`), a `lookback`, a `bufferSize`, the event
    `source`, the default `conditions` and `rules`;
  * at start every condition is set to its default (status False, default reason/message);
  * log entries from before boot, or older than `lookback`, are ignored;
  * a `temporary` rule whose pattern matches produces one Warning Event per matching entry
    (reason = the rule's, message = the matched log text), on the Node, from `source`;
  * a `permanent` rule sets its condition True with the rule's reason and the matched text; a
    later match with the SAME reason leaves the condition alone, a different reason replaces it;
    permanent rules produce no Events of their own;
  * a pattern is matched against the newest `bufferSize` entries joined by newlines and must end
    at the newest entry (multi-line kernel traces such as hung-task reports).

MI355X addition: the amdgpu rule set (deploy/node-problem-detector/amdgpu-monitor.json) turns
ring timeouts and GPU resets into events and unrecoverable faults (failed reset, RAS poison /
uncorrectable errors, bad-page threshold, xGMI link faults) into the `AMDGPUProblem` condition.
A rule marked `"gpuFault": true` also hands the faulting device's PCI address to the AMD device
plugin (`report_gpu_fault` → `<health-state>.faults`, applied by smi/health.py on the plugin's
next tick), so the kubelet stops admitting pods onto that GPU with the kernel's words as its
`amd.com/health-reason`, not only the node's condition.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import re
import shutil
import subprocess
import time
from dataclasses import dataclass, field

from ..api import meta as m

log = logging.getLogger("amdkube.npd")

TEMPORARY, PERMANENT = "temporary", "permanent"
_BDF = re.compile(r"\b([0-9a-fA-F]{4}:[0-9a-fA-F]{2}:[0-9a-fA-F]{2}\.[0-7])\b")


# --------------------------------------------------------------------------- config
@dataclass
class Rule:
    type: str
    reason: str
    pattern: str
    condition: str = ""
    gpu_fault: bool = False
    rx: re.Pattern | None = None

    def __post_init__(self):
        if self.type not in (TEMPORARY, PERMANENT):
            raise ValueError(f"rule {self.reason!r}: type must be temporary or permanent, not {self.type!r}")
        if self.type == PERMANENT and not self.condition:
            raise ValueError(f"permanent rule {self.reason!r} names no condition")
        # NPD: "the pattern must match to the end of the buffer" (logBuffer.Match appends \z)
        self.rx = re.compile(f"(?:{self.pattern})\\Z")


@dataclass
class MonitorConfig:
    plugin: str
    log_path: str
    source: str
    lookback_s: float = 0.0
    buffer_size: int = 10
    plugin_config: dict = field(default_factory=dict)
    conditions: list[dict] = field(default_factory=list)
    rules: list[Rule] = field(default_factory=list)

    @classmethod
    def parse(cls, raw: dict) -> "MonitorConfig":
        from ..api.protobuf import parse_duration
        cfg = cls(plugin=raw.get("plugin") or "kmsg", log_path=raw.get("logPath") or "/dev/kmsg",
                  source=raw.get("source") or "kernel-monitor",
                  lookback_s=parse_duration(raw["lookback"]) / 1e9 if raw.get("lookback") else 0.0,
                  buffer_size=int(raw.get("bufferSize") or 10), plugin_config=dict(raw.get("pluginConfig") or {}),
                  conditions=[dict(c) for c in raw.get("conditions") or []],
                  rules=[Rule(type=r.get("type", ""), reason=r.get("reason", ""), pattern=r.get("pattern", ""),
                              condition=r.get("condition", ""), gpu_fault=bool(r.get("gpuFault")))
                         for r in raw.get("rules") or []])
        if cfg.plugin not in ("kmsg", "filelog", "journald"):
            raise ValueError(f"{cfg.source}: unknown log plugin {cfg.plugin!r}")
        known = {c.get("type") for c in cfg.conditions}
        for r in cfg.rules:
            if r.type == PERMANENT and r.condition not in known:
                raise ValueError(f"{cfg.source}: rule {r.reason!r} sets condition {r.condition!r} with no default")
        return cfg

    @classmethod
    def load(cls, path: str) -> "MonitorConfig":
        with open(path) as f:
            return cls.parse(json.load(f))


# --------------------------------------------------------------------------- log sources
@dataclass
class LogEntry:
    ts: float            # wall-clock seconds
    message: str


def boot_time(uptime_path: str = "/proc/uptime") -> float:
    try:
        with open(uptime_path) as f:
            return time.time() - float(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        return 0.0


def parse_kmsg_record(rec: str, boot: float) -> LogEntry | None:
    """`<prio>,<seq>,<usec since boot>,<flags>[,…];<message>` plus ` KEY=value` continuation lines."""
    head, sep, body = rec.partition(";")
    if not sep:
        return None
    parts = head.split(",")
    if len(parts) < 3:
        return None
    try:
        usec = int(parts[2])
    except ValueError:
        return None
    return LogEntry(boot + usec / 1e6, body.split("\n", 1)[0])


_GO_LAYOUT = [("January", "%B"), ("Jan", "%b"), ("Monday", "%A"), ("Mon", "%a"), ("2006", "%Y"),
              ("_2", "%d"), ("02", "%d"), ("01", "%m"), ("15", "%H"), ("03", "%I"), ("04", "%M"),
              ("05", "%S"), ("PM", "%p"), ("MST", "%Z"), ("-07:00", "%z"), ("-0700", "%z"), ("Z07:00", "%z")]


def go_layout_to_strptime(layout: str) -> str:
    """Go reference-time layouts (time.Stamp "Jan _2 15:04:05", RFC3339, …) → strptime."""
    out, i = [], 0
    while i < len(layout):
        if layout.startswith((".000000", ".999999"), i):
            out.append(".%f")
            i += 7
            continue
        for tok, fmt in _GO_LAYOUT:
            if layout.startswith(tok, i):
                out.append(fmt)
                i += len(tok)
                break
        else:
            out.append("%%" if layout[i] == "%" else layout[i])
            i += 1
    return "".join(out)


class FileLogParser:
    """The `filelog` plugin: `timestamp` regex → the time text (parsed with `timestampFormat`),
    `message` regex group 1 → the message. A year-less layout takes the current year (or the
    previous one when that would put the entry in the future)."""

    def __init__(self, plugin_config: dict):
        self.ts_rx = re.compile(plugin_config.get("timestamp") or r"^.{15}")
        self.msg_rx = re.compile(plugin_config.get("message") or r"kernel: \[.*\] (.*)")
        self.fmt = go_layout_to_strptime(plugin_config.get("timestampFormat") or "Jan _2 15:04:05")
        self.yearless = "%Y" not in self.fmt

    def parse(self, line: str) -> LogEntry | None:
        tm, mm = self.ts_rx.search(line), self.msg_rx.search(line)
        if tm is None or mm is None:
            return None
        import datetime as dt
        try:
            t = dt.datetime.strptime(tm.group(0).strip(), self.fmt)
        except ValueError:
            return None
        if self.yearless:
            now = dt.datetime.now()
            t = t.replace(year=now.year)
            if t > now + dt.timedelta(days=1):
                t = t.replace(year=now.year - 1)
        ts = t.timestamp() if t.tzinfo is None else t.astimezone().timestamp()
        return LogEntry(ts, mm.group(1) if mm.groups() else mm.group(0))


class LogWatcher:
    """Yields entries appended to the monitor's log (from the start of the log, so `lookback`
    can replay recent history; the filter drops what is too old)."""

    def __init__(self, cfg: MonitorConfig, boot: float | None = None, poll: float = 0.2):
        self.cfg, self.poll = cfg, poll
        self.boot = boot_time() if boot is None else boot
        self._fd: int | None = None
        self._f = None
        self._proc: subprocess.Popen | None = None
        self._partial = ""
        self._head = b""           # the file's first bytes, to notice a copytruncate rotation
        self._parser = FileLogParser(cfg.plugin_config) if cfg.plugin == "filelog" else None

    def open(self) -> bool:
        p = self.cfg
        try:
            if p.plugin == "kmsg":
                self._fd = os.open(p.log_path, os.O_RDONLY | os.O_NONBLOCK)
            elif p.plugin == "filelog":
                self._f = open(p.log_path, "r", errors="replace")
            else:
                jc = shutil.which("journalctl")
                if jc is None:
                    log.warning("%s: journalctl not found; the journald monitor is off", p.source)
                    return False
                since = f"-{int(p.lookback_s)}s" if p.lookback_s else "-0s"
                self._proc = subprocess.Popen([jc, "-k", "-f", "-o", "short-unix", "--no-pager", f"--since={since}"],
                                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
                os.set_blocking(self._proc.stdout.fileno(), False)
        except OSError as e:
            log.warning("%s: cannot open %s (%s); this monitor is off", p.source, p.log_path, e)
            return False
        return True

    def read(self) -> list[LogEntry]:
        out: list[LogEntry] = []
        if self._fd is not None:
            while True:
                try:
                    rec = os.read(self._fd, 8192)
                except BlockingIOError:
                    break
                except OSError:          # EPIPE: the ring overwrote records we had not read
                    continue
                if not rec:
                    break
                # /dev/kmsg returns one record per read; a plain file (tests) returns many lines
                for line in rec.decode(errors="replace").splitlines():
                    if line and not line.startswith(" "):
                        e = parse_kmsg_record(line, self.boot)
                        if e is not None:
                            out.append(e)
        elif self._f is not None:
            self._follow_rotation()
            chunk = self._f.read()
            if len(self._head) < 64:
                self._head = os.pread(self._f.fileno(), 64, 0)
            if chunk:
                text = self._partial + chunk
                lines = text.split("\n")
                self._partial = lines.pop()
                for line in lines:
                    e = self._parser.parse(line)
                    if e is not None:
                        out.append(e)
        elif self._proc is not None and self._proc.stdout is not None:
            try:
                chunk = self._proc.stdout.read() or ""
            except (BlockingIOError, TypeError):
                chunk = ""
            text = self._partial + chunk
            lines = text.split("\n")
            self._partial = lines.pop()
            for line in lines:          # "<unix.usec> host kernel: message"
                ts, _, rest = line.partition(" ")
                try:
                    t = float(ts)
                except ValueError:
                    continue
                msg = rest.split("kernel: ", 1)[1] if "kernel: " in rest else rest
                out.append(LogEntry(t, msg))
        return out

    def _follow_rotation(self):
        """A log rotated away (new inode at the path) is reopened from its start; one truncated in
        place is read again from offset 0 (what `tail -F` does for NPD's filelog plugin)."""
        try:
            st = os.stat(self.cfg.log_path)
            cur = os.fstat(self._f.fileno())
        except OSError:
            return
        if (st.st_ino, st.st_dev) != (cur.st_ino, cur.st_dev):
            rest = self._f.read()                     # whatever the old file still had
            if rest:
                self._partial += rest
            self._f.close()
            self._f = open(self.cfg.log_path, "r", errors="replace")
            self._head = b""
            return
        # truncated in place: shorter than what was read, or its first bytes are not the ones seen
        head = os.pread(self._f.fileno(), 64, 0)
        pos = self._f.tell()
        if st.st_size < pos or (self._head and head[:len(self._head)] != self._head):
            self._f.seek(0)
            self._partial = ""
            self._head = b""

    def close(self):
        if self._fd is not None:
            os.close(self._fd)
            self._fd = None
        if self._f is not None:
            self._f.close()
            self._f = None
        if self._proc is not None:
            self._proc.kill()
            self._proc.wait()
            self._proc = None


# --------------------------------------------------------------------------- GPU fault hand-off
def report_gpu_fault(health_state: str, device: str, reason: str, source: str = "node-problem-detector"):
    """Tell the AMD device plugin that owns `health_state` that `device` (PCI address or device
    ID) has an unrecoverable fault; its next health tick marks the GPU Unhealthy (sticky)."""
    os.makedirs(os.path.dirname(os.path.abspath(health_state)), exist_ok=True)
    with open(health_state + ".faults", "a") as f:
        f.write(json.dumps({"device": device, "reason": reason, "source": source, "ts": time.time()}) + "\n")


# --------------------------------------------------------------------------- the monitor
@dataclass
class Status:
    events: list[tuple[str, str]]                 # (reason, message) of temporary rules
    conditions: dict[str, dict]                   # changed conditions, by type
    gpu_faults: list[tuple[str, str]]             # (pci address, reason)


class KernelMonitor:
    """One system-log monitor: the rule engine over one log (the NPD kernel monitor)."""

    def __init__(self, cfg: MonitorConfig, now=time.time, boot: float | None = None):
        self.cfg, self.now = cfg, now
        self.boot = boot_time() if boot is None else boot
        self.buffer: list[LogEntry] = []
        self.started = now()
        self.conditions: dict[str, dict] = {c["type"]: self._default(c) for c in cfg.conditions}

    def _default(self, c: dict) -> dict:
        return {"type": c["type"], "status": "False", "reason": c.get("reason", ""), "message": c.get("message", ""),
                "transition": self.now()}

    def too_old(self, e: LogEntry) -> bool:
        if self.boot and e.ts < self.boot:
            return True
        return bool(self.cfg.lookback_s) and e.ts < self.started - self.cfg.lookback_s

    def _match(self, rule: Rule) -> list[LogEntry] | None:
        joined, starts, pos = [], [], 0
        for e in self.buffer:
            starts.append(pos)
            joined.append(e.message)
            pos += len(e.message) + 1
        text = "\n".join(joined)
        mt = rule.rx.search(text)
        if mt is None:
            return None
        first = max(i for i, s in enumerate(starts) if s <= mt.start()) if mt.start() < len(text) else len(starts) - 1
        return self.buffer[first:]

    def process(self, e: LogEntry) -> Status:
        st = Status([], {}, [])
        if self.too_old(e):
            return st
        self.buffer.append(e)
        if len(self.buffer) > self.cfg.buffer_size:
            del self.buffer[0]
        for rule in self.cfg.rules:
            hit = self._match(rule)
            if hit is None:
                continue
            msg = "\n".join(x.message for x in hit)
            if rule.type == TEMPORARY:
                st.events.append((rule.reason, msg))
            else:
                cur = self.conditions[rule.condition]
                if cur["status"] != "True" or cur["reason"] != rule.reason:
                    cur.update(status="True", reason=rule.reason, message=msg, transition=e.ts)
                    st.conditions[rule.condition] = dict(cur)
            if rule.gpu_fault:
                for bdf in dict.fromkeys(mt.group(1).lower() for mt in _BDF.finditer(msg)):
                    st.gpu_faults.append((bdf, f"{rule.reason}: {msg.splitlines()[-1][:200]}"))
        return st


class NodeProblemDetector:
    """The daemon: every monitor's log → its rule engine → Node conditions (strategic-merge
    PATCH of nodes/<name>/status, merged by condition type so the kubelet's own conditions are
    untouched, re-sent every `resync` s as a heartbeat) and Events from each monitor's source."""

    def __init__(self, client, node_name: str, configs: list[MonitorConfig], health_state: str | None = None,
                 poll: float = 0.2, resync: float = 10.0, boot: float | None = None):
        self.client, self.node_name = client, node_name
        self.health_state, self.poll, self.resync = health_state, poll, resync
        self.monitors = [KernelMonitor(c, boot=boot) for c in configs]
        self.watchers = [LogWatcher(c, boot=boot, poll=poll) for c in configs]
        self.recorders = {}
        self._task: asyncio.Task | None = None
        self._dirty = True
        self.events_sent = 0
        self.gpu_faults_reported: list[tuple[str, str]] = []

    def _node_ref(self) -> dict:
        # the reference's recorder uses the node name as UID for Node events (no namespace)
        return {"kind": "Node", "apiVersion": "v1", "metadata": {"name": self.node_name, "uid": self.node_name}}

    async def start(self):
        from ..client.record import EventRecorder
        for c in {mon.cfg.source for mon in self.monitors}:
            self.recorders[c] = EventRecorder(self.client, c, self.node_name).start()
        opened = [w.open() for w in self.watchers]
        self.monitors = [mon for mon, ok in zip(self.monitors, opened) if ok]
        self.watchers = [w for w, ok in zip(self.watchers, opened) if ok]
        await self.sync_conditions()
        self._task = asyncio.create_task(self._run(), name="node-problem-detector")
        return self

    async def stop(self):
        from ..utils import cancel_and_wait
        await cancel_and_wait([self._task])
        for w in self.watchers:
            w.close()
        for r in self.recorders.values():
            await r.stop()

    def all_conditions(self) -> list[dict]:
        now = m.now_rfc3339()
        out = []
        for mon in self.monitors:
            for c in mon.conditions.values():
                out.append({"type": c["type"], "status": c["status"], "reason": c["reason"], "message": c["message"],
                            "lastHeartbeatTime": now,
                            "lastTransitionTime": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(c["transition"]))})
        return out

    async def sync_conditions(self):
        conds = self.all_conditions()
        if not conds:
            return
        try:
            await self.client.patch("nodes", self.node_name, {"status": {"conditions": conds}}, sub="status",
                                    patch_type="application/strategic-merge-patch+json")
            self._dirty = False
        except m.StatusError as e:
            log.warning("cannot update conditions of node %s: %s", self.node_name, e)

    def step(self) -> int:
        """Drain every log once; returns how many entries were processed."""
        n = 0
        for mon, w in zip(self.monitors, self.watchers):
            for e in w.read():
                n += 1
                st = mon.process(e)
                for reason, msg in st.events:
                    self.recorders[mon.cfg.source].event(self._node_ref(), "Warning", reason, msg)
                    self.events_sent += 1
                if st.conditions:
                    self._dirty = True
                    for t, c in st.conditions.items():
                        log.warning("node condition %s=%s (%s): %s", t, c["status"], c["reason"], c["message"])
                for bdf, why in st.gpu_faults:
                    self.gpu_faults_reported.append((bdf, why))
                    if self.health_state:
                        report_gpu_fault(self.health_state, bdf, why)
        return n

    async def _run(self):
        last_sync = time.monotonic()
        while True:
            try:
                self.step()
                if self._dirty or time.monotonic() - last_sync >= self.resync:
                    await self.sync_conditions()
                    last_sync = time.monotonic()
            except asyncio.CancelledError:
                raise
            except Exception as e:   # keep watching; the next tick retries
                log.error("problem detector tick failed: %r", e)
            await asyncio.sleep(self.poll)
