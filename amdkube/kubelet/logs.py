"""Container log files: the CRI log format, and the kubelet's reader for /containerLogs.

Reference: pkg/kubelet/kuberuntime/logs/logs.go —
  * NewLogOptions (:97-119): tail/bytes default −1 (all); since = now − sinceSeconds, or
    sinceTime when that is later;
  * parseCRILog (:131-167) `<RFC3339Nano> <stdout|stderr> <tags> <content>` — a P(artial) record
    loses its trailing newline, an F(ull) one keeps it; parseDockerJSONLog (:171-186)
    `{"log", "stream", "time"}`; getParseFunc tries them in that order (:189-197);
  * logWriter (:199-262): lines older than `since` are skipped, `timestamps` prefixes the
    record's time, `limitBytes` cuts the output short (errMaximumWrite);
  * ReadLogs (:267-352): start `tail` lines before the end, parse with the function the first
    line selects, and with `follow` wait for more until the container stops running (state
    checked every 5 s, waitLogs :356-390);
pkg/util/tail/tail.go FindTailLineStartIndex (an unterminated last line does not count);
pkg/kubelet/kubelet_pods.go validateContainerLogStatus (:1165-1211, which instance `previous`
and the container's state select); pkg/apis/core/validation ValidatePodLogOptions (:4842).

Writers: rocshim hands each container's stdout and stderr to native/logpump.cpp, which writes
the CRI format. Files in no known format (rktshim's raw output, logs written before the pump
existed) are read as raw stdout lines without timestamps — an amdkube fallback, since the
reference refuses an unknown format.
"""
from __future__ import annotations

import asyncio
import calendar
import json
import os
import re
import time

from ..api import field

STDOUT, STDERR = "stdout", "stderr"
BLOCK_SIZE = 1024
STATE_CHECK_PERIOD = 5.0
_TS = re.compile(r"^(\d{4})-(\d{2})-(\d{2})T(\d{2}):(\d{2}):(\d{2})(?:\.(\d{1,9}))?(Z|[+-]\d{2}:\d{2})$")
ZERO_TIME_NS = -62135596800 * 10**9        # Go's zero time.Time, 0001-01-01T00:00:00Z


def parse_rfc3339(s: str) -> int:
    """time.Parse(time.RFC3339Nano, s) as nanoseconds since the epoch (RFC3339 without a
    fraction parses too)."""
    mt = _TS.match(s.strip())
    if not mt:
        raise ValueError(f'unexpected timestamp format "{time_format_name()}": {s!r}')
    y, mo, d, h, mi, se, frac, tz = mt.groups()
    secs = calendar.timegm((int(y), int(mo), int(d), int(h), int(mi), int(se), 0, 0, 0))
    if tz != "Z":
        sign = 1 if tz[0] == "+" else -1
        secs -= sign * (int(tz[1:3]) * 3600 + int(tz[4:6]) * 60)
    return secs * 10**9 + (int(frac.ljust(9, "0")) if frac else 0)


def time_format_name() -> str:
    return "2006-01-02T15:04:05.999999999Z07:00"


def format_rfc3339nano(ns: int) -> str:
    """Go's Format(time.RFC3339Nano) in UTC: the fraction without trailing zeros."""
    secs, frac = divmod(ns, 10**9)
    import datetime
    t = datetime.datetime(1970, 1, 1) + datetime.timedelta(seconds=secs)
    s = t.strftime("%Y-%m-%dT%H:%M:%S") if t.year >= 1000 else f"{t.year:04d}" + t.strftime("-%m-%dT%H:%M:%S")
    if frac:
        s += ("." + f"{frac:09d}").rstrip("0")
    return s + "Z"


class LogMessage:
    __slots__ = ("timestamp", "stream", "log")

    def __init__(self, timestamp: int | None = None, stream: str = "", log: bytes = b""):
        self.timestamp, self.stream, self.log = timestamp, stream, log

    def __eq__(self, o):
        return isinstance(o, LogMessage) and (self.timestamp, self.stream, self.log) == (o.timestamp, o.stream, o.log)

    def __repr__(self):
        return f"LogMessage({self.timestamp}, {self.stream!r}, {self.log!r})"


def parse_cri_log(line: bytes) -> LogMessage:
    """`2016-10-06T00:17:09.669794202Z stdout P log content 1`."""
    idx = line.find(b" ")
    if idx < 0:
        raise ValueError("timestamp is not found")
    ts = parse_rfc3339(line[:idx].decode("ascii", "replace"))
    rest = line[idx + 1:]
    idx = rest.find(b" ")
    if idx < 0:
        raise ValueError("stream type is not found")
    stream = rest[:idx].decode("ascii", "replace")
    if stream not in (STDOUT, STDERR):
        raise ValueError(f'unexpected stream type "{stream}"')
    rest = rest[idx + 1:]
    idx = rest.find(b" ")
    if idx < 0:
        raise ValueError("log tag is not found")
    partial = rest[:idx].split(b":")[0] == b"P"
    if partial and rest.endswith(b"\n"):
        rest = rest[:-1]
    return LogMessage(ts, stream, rest[idx + 1:])


def parse_docker_json_log(line: bytes) -> LogMessage:
    """`{"log":"content 1","stream":"stdout","time":"2016-10-20T18:39:20.57606443Z"}`."""
    try:
        d = json.loads(line)
    except ValueError as e:
        raise ValueError(f"failed with {e} to unmarshal log {line!r}") from None
    if not isinstance(d, dict):
        raise ValueError(f"failed to unmarshal log {line!r}")
    t = d.get("time")
    return LogMessage(parse_rfc3339(t) if t else ZERO_TIME_NS, str(d.get("stream", "")), str(d.get("log", "")).encode())


def parse_raw_log(line: bytes) -> LogMessage:
    """amdkube fallback: an untagged line is stdout with no timestamp."""
    return LogMessage(None, STDOUT, line)


PARSE_FUNCS = (parse_cri_log, parse_docker_json_log)


def get_parse_func(line: bytes, allow_raw: bool = False):
    for p in PARSE_FUNCS:
        try:
            p(line)
            return p
        except ValueError:
            continue
    if allow_raw:
        return parse_raw_log
    raise ValueError(f"unsupported log format: {line!r}")


class LogOptions:
    __slots__ = ("tail", "bytes", "since", "follow", "timestamp")

    def __init__(self, tail=-1, bytes=-1, since=None, follow=False, timestamp=False):
        self.tail, self.bytes, self.since, self.follow, self.timestamp = tail, bytes, since, follow, timestamp

    def __eq__(self, o):
        return isinstance(o, LogOptions) and all(getattr(self, k) == getattr(o, k) for k in self.__slots__)

    def __repr__(self):
        return "LogOptions(" + ", ".join(f"{k}={getattr(self, k)!r}" for k in self.__slots__) + ")"

    @classmethod
    def from_api(cls, o: dict, now_ns: int | None = None) -> "LogOptions":
        """NewLogOptions from a v1.PodLogOptions dict (tailLines, limitBytes, sinceSeconds,
        sinceTime, follow, timestamps)."""
        now_ns = time.time_ns() if now_ns is None else now_ns
        opts = cls(follow=bool(o.get("follow")), timestamp=bool(o.get("timestamps")))
        if o.get("tailLines") is not None:
            opts.tail = int(o["tailLines"])
        if o.get("limitBytes") is not None:
            opts.bytes = int(o["limitBytes"])
        if o.get("sinceSeconds") is not None:
            opts.since = now_ns - int(o["sinceSeconds"]) * 10**9
        if o.get("sinceTime"):
            st = o["sinceTime"] if isinstance(o["sinceTime"], int) else parse_rfc3339(o["sinceTime"])
            if opts.since is None or st > opts.since:
                opts.since = st
        return opts


class MaximumWrite(Exception):
    """errMaximumWrite: the byte limit was reached."""


class LogWriter:
    """newLogWriter: `stdout` / `stderr` are callables taking bytes."""

    def __init__(self, stdout, stderr, opts: LogOptions):
        self.stdout, self.stderr, self.opts = stdout, stderr, opts
        self.remain = opts.bytes if opts.bytes >= 0 else float("inf")

    def write(self, msg: LogMessage):
        since = self.opts.since
        if since is not None and msg.timestamp is not None and msg.timestamp < since:
            return
        line = msg.log
        if self.opts.timestamp and msg.timestamp is not None:
            line = format_rfc3339nano(msg.timestamp).encode() + b" " + line
        if len(line) > self.remain:
            line = line[:int(self.remain)]
        if msg.stream == STDOUT:
            self.stdout(line)
        elif msg.stream == STDERR:
            self.stderr(line)
        else:
            raise ValueError(f'unexpected stream type "{msg.stream}"')
        self.remain -= len(line)
        if self.remain <= 0:
            raise MaximumWrite()


def find_tail_line_start_index(f, n: int) -> int:
    """The offset where the last `n` lines start (an unterminated last line is not counted);
    0 for n < 0 or a file with fewer lines."""
    if n < 0:
        return 0
    size = f.seek(0, os.SEEK_END)
    left = cnt = 0
    buf = b""
    right = size
    while right > 0 and cnt <= n:
        left = max(0, right - BLOCK_SIZE)
        f.seek(left)
        buf = f.read(right - left)
        cnt += buf.count(b"\n")
        right -= BLOCK_SIZE
    while cnt > n:
        idx = buf.index(b"\n") + 1
        buf = buf[idx:]
        left += idx
        cnt -= 1
    return left


def validate_pod_log_options(o: dict) -> list:
    """ValidatePodLogOptions: field.Error list."""
    errs = []
    if o.get("tailLines") is not None and int(o["tailLines"]) < 0:
        errs.append(field.invalid("tailLines", int(o["tailLines"]), "must be greater than or equal to 0"))
    if o.get("limitBytes") is not None and int(o["limitBytes"]) < 1:
        errs.append(field.invalid("limitBytes", int(o["limitBytes"]), "must be greater than 0"))
    if o.get("sinceSeconds") is not None and o.get("sinceTime"):
        errs.append(field.forbidden("", "at most one of `sinceTime` or `sinceSeconds` may be specified"))
    elif o.get("sinceSeconds") is not None and int(o["sinceSeconds"]) < 1:
        errs.append(field.invalid("sinceSeconds", int(o["sinceSeconds"]), "must be greater than 0"))
    return errs


def decode_log_query(q) -> dict:
    """PodLogOptions from query parameters (container, follow, previous, sinceSeconds, sinceTime,
    timestamps, tailLines, limitBytes; the kubelet's legacy `tail`, with "all" = unset). A value
    that does not decode raises ValueError."""
    def flag(v):
        if v.lower() in ("1", "t", "true"):
            return True
        if v.lower() in ("0", "f", "false", ""):
            return False
        raise ValueError(v)
    o: dict = {}
    if q.get("container"):
        o["container"] = q["container"]
    for k in ("follow", "previous", "timestamps"):
        if q.get(k) is not None:
            o[k] = flag(q[k])
    tail = q.get("tail")
    if tail is not None and tail != "all":
        o["tailLines"] = int(tail)
    for k in ("tailLines", "limitBytes", "sinceSeconds"):
        if q.get(k) not in (None, ""):
            o[k] = int(q[k])
    if q.get("sinceTime"):
        parse_rfc3339(q["sinceTime"])
        o["sinceTime"] = q["sinceTime"]
    return o


def _iter_lines(data: bytes):
    start = 0
    while True:
        nl = data.find(b"\n", start)
        if nl < 0:
            return start
        yield data[start:nl + 1]
        start = nl + 1


class _Reader:
    """The parse/write loop of ReadLogs over a byte stream of whole lines."""

    def __init__(self, path: str, opts: LogOptions, stdout, stderr):
        self.path, self.opts = path, opts
        self.writer = LogWriter(stdout, stderr, opts)
        self.parse = None

    def feed(self, lines) -> bool:
        """Write each line; True once the byte limit is hit."""
        for ln in lines:
            if self.parse is None:
                self.parse = get_parse_func(ln, allow_raw=True)
            try:
                msg = self.parse(ln)
            except ValueError:
                continue      # glog.Errorf and skip, as the reference does
            try:
                self.writer.write(msg)
            except MaximumWrite:
                return True
        return False


def read_logs_sync(path: str, opts: LogOptions, stdout, stderr):
    """ReadLogs without follow."""
    with open(path, "rb") as f:
        start = find_tail_line_start_index(f, opts.tail)
        f.seek(start)
        data = f.read()
    r = _Reader(path, opts, stdout, stderr)
    lines = data.splitlines(keepends=True)
    if lines and not lines[-1].endswith(b"\n"):
        pass      # an incomplete last line is still written ("Incomplete line in log file")
    r.feed(lines)


def read_text(path: str, tail: int = -1, limit: int = -1, keep_last: int = -1) -> str:
    """The container's output as text (both streams, in file order). `limit` keeps the first
    bytes (limitBytes), `keep_last` the last ones (the circular buffer of
    readLastStringFromContainerLogs: 80 lines, 2 KiB, for the termination-message fallback)."""
    out: list[bytes] = []
    try:
        read_logs_sync(path, LogOptions(tail=tail, bytes=limit), out.append, out.append)
    except OSError:
        return ""
    data = b"".join(out)
    if keep_last >= 0:
        data = data[-keep_last:] if keep_last else b""
    return data.decode(errors="replace")


async def read_logs(path: str, opts: LogOptions, write, is_running=None, state_check_period: float = STATE_CHECK_PERIOD,
                    poll_interval: float = 0.1):
    """ReadLogs: `write(bytes)` is awaited with each batch (stdout and stderr interleaved as in
    the file, the way the kubelet hands both to one response). With `follow`, new lines are
    streamed until `is_running()` (awaited every `state_check_period` seconds without new
    output) reports the container stopped."""
    buf: list[bytes] = []
    r = _Reader(path, opts, buf.append, buf.append)
    with open(path, "rb") as f:
        f.seek(find_tail_line_start_index(f, opts.tail))
        pending = b""
        last_check = time.monotonic()
        while True:
            chunk = f.read(1 << 20)
            data = pending + chunk
            lines = list(_iter_lines(data))
            consumed = sum(len(x) for x in lines)
            pending = data[consumed:]
            if not chunk and pending and not opts.follow:
                lines.append(pending)       # an incomplete last line
                pending = b""
            done = r.feed(lines)
            if buf:
                await write(b"".join(buf))
                buf.clear()
            if done:
                return
            if chunk:
                last_check = time.monotonic()
                continue
            if not opts.follow:
                return
            if is_running is not None and time.monotonic() - last_check >= state_check_period:
                last_check = time.monotonic()
                if not await is_running():
                    # drain what the container wrote before it stopped
                    rest = pending + f.read()
                    tail_lines = list(_iter_lines(rest))
                    used = sum(len(x) for x in tail_lines)
                    if used < len(rest):
                        tail_lines.append(rest[used:])
                    r.feed(tail_lines)
                    if buf:
                        await write(b"".join(buf))
                    return
            await asyncio.sleep(poll_interval)


def parse_container_id(cid: str) -> str:
    """kubecontainer.ParseContainerID: `<type>://<id>` → id."""
    return cid.split("://", 1)[1] if "://" in cid else cid


def _container_status(statuses, name):
    return next((s for s in statuses or [] if s.get("name") == name), None)


def validate_container_log_status(pod_name: str, pod_status: dict, container_name: str, previous: bool) -> str:
    """The container ID whose log a request means; ValueError with the reference's message when
    there is none."""
    cs = _container_status(pod_status.get("containerStatuses"), container_name) or \
        _container_status(pod_status.get("initContainerStatuses"), container_name)
    if cs is None:
        raise ValueError(f'container "{container_name}" in pod "{pod_name}" is not available')
    last = (cs.get("lastState") or {}).get("terminated")
    st = cs.get("state") or {}
    waiting, running, terminated = st.get("waiting"), st.get("running"), st.get("terminated")
    if previous:
        if last is None:
            raise ValueError(f'previous terminated container "{container_name}" in pod "{pod_name}" not found')
        cid = last.get("containerID", "")
    elif running is not None:
        cid = cs.get("containerID", "")
    elif terminated is not None:
        cid = terminated.get("containerID", "")
    elif last is not None:
        cid = last.get("containerID", "")
    elif waiting is not None:
        reason = waiting.get("reason", "")
        if reason == "ErrImagePull":
            raise ValueError(f'container "{container_name}" in pod "{pod_name}" is waiting to start: image can\'t be pulled')
        if reason == "ImagePullBackOff":
            raise ValueError(f'container "{container_name}" in pod "{pod_name}" is waiting to start: '
                             "trying and failing to pull image")
        raise ValueError(f'container "{container_name}" in pod "{pod_name}" is waiting to start: {reason}')
    else:
        raise ValueError(f'container "{container_name}" in pod "{pod_name}" is waiting to start - no logs yet')
    return parse_container_id(cid)


def log_location_container(pod: dict, name: str, container: str | None) -> str:
    """registry/core/pod LogLocation's container choice (strategy.go:325-347): the only container
    when none is named; a BadRequest message otherwise."""
    spec = pod.get("spec") or {}
    conts = [c.get("name", "") for c in spec.get("containers") or []]
    inits = [c.get("name", "") for c in spec.get("initContainers") or []]
    if not container:
        if len(conts) == 1:
            return conts[0]
        if not conts:
            raise ValueError(f"a container name must be specified for pod {name}")
        msg = f"a container name must be specified for pod {name}, choose one of: [{' '.join(conts)}]"
        if inits:
            msg += f" or one of the init containers: [{' '.join(inits)}]"
        raise ValueError(msg)
    if container not in conts and container not in inits:
        raise ValueError(f"container {container} is not valid for pod {name}")
    return container
