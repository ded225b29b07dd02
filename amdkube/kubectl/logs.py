"""kubectl logs.

Reference: pkg/kubectl/cmd/logs.go (Complete :124-216 — POD or TYPE/NAME with an optional
inline CONTAINER, or -l; --follow, --previous, --timestamps, --since / --since-time,
--limit-bytes, --tail; "only one of follow (-f) or selector (-l) is allowed"), ValidatePodLogOptions
before the request, RunLogs (:231-259, every pod of a selector in turn);
cmd/util/factory_client_access.go LogsForObject — a workload or service is resolved to one of
its pods through SelectorsForObject and GetFirstPod (factory.go:290-330) ordered by
controller.ByLogging (controller_utils.go:694-723), with "Found N pods, using pod/NAME" on
stderr.

The shared argument parser gives -f to --filename and -p to --patch, so main() rewrites them
to --follow / --previous after `logs`, as the reference's own flag set has them.
"""
from __future__ import annotations

import asyncio
import functools
import sys
import time

from ..api import meta as m
from ..api.helpers import is_pod_ready
from ..api.scheme import SCHEME

USAGE = "expected POD, TYPE/NAME, or -l selector (e.g. 'kubectl logs -l app=x')"


def parse_duration_s(s: str) -> float:
    """time.ParseDuration for the --since flag (e.g. 5s, 2m, 3h, 1h30m)."""
    from ..api.protobuf import parse_duration
    return parse_duration(s) / 1e9


def _ready_time(p) -> str:
    for c in (p.get("status") or {}).get("conditions") or []:
        if c.get("type") == "Ready" and c.get("status") == "True":
            return c.get("lastTransitionTime") or ""
    return ""


def _after_or_zero(t1: str, t2: str) -> bool:
    """afterOrZero: an empty time sorts last."""
    if not t1 or not t2:
        return not t1
    return m.parse_time(t1) > m.parse_time(t2)


def _max_restarts(p) -> int:
    return max([int(c.get("restartCount") or 0) for c in (p.get("status") or {}).get("containerStatuses") or []] or [0])


def by_logging_less(a: dict, b: dict) -> bool:
    """controller.ByLogging: the pod whose logs are most useful first."""
    na, nb = (a.get("spec") or {}).get("nodeName") or "", (b.get("spec") or {}).get("nodeName") or ""
    if na != nb and (not na or not nb):
        return bool(na)
    rank = {"Running": 0, "Unknown": 1, "Pending": 2}
    pa, pb = (a.get("status") or {}).get("phase"), (b.get("status") or {}).get("phase")
    if rank.get(pa, 0) != rank.get(pb, 0):
        # an unlisted phase maps to 0 as a missing Go map key does
        return rank.get(pa, 0) < rank.get(pb, 0)
    ra, rb = is_pod_ready(a), is_pod_ready(b)
    if ra != rb:
        return ra
    if ra and rb and _ready_time(a) != _ready_time(b):
        return _after_or_zero(_ready_time(b), _ready_time(a))
    if _max_restarts(a) != _max_restarts(b):
        return _max_restarts(a) > _max_restarts(b)
    ca, cb = (a.get("metadata") or {}).get("creationTimestamp") or "", (b.get("metadata") or {}).get("creationTimestamp") or ""
    if ca != cb:
        return _after_or_zero(cb, ca)
    return False


def sort_by_logging(pods: list[dict]) -> list[dict]:
    return sorted(pods, key=functools.cmp_to_key(lambda x, y: -1 if by_logging_less(x, y) else (1 if by_logging_less(y, x) else 0)))


def selector_for_object(obj: dict) -> str:
    """SelectorsForObject: the label selector string of a controller or service."""
    from ..api.labels import SelectorError, selector_from_label_selector
    kind = obj.get("kind", "")
    sel = (obj.get("spec") or {}).get("selector")
    if kind in ("ReplicationController", "Service"):
        if not sel:
            raise ValueError(f"invalid {kind.lower()}: no selector" if kind == "ReplicationController"
                             else "invalid service provided: no selector")
        return ",".join(f"{k}={sel[k]}" for k in sorted(sel))
    if kind in ("ReplicaSet", "Deployment", "DaemonSet", "StatefulSet", "Job"):
        if not sel:
            raise ValueError(f"invalid {kind.lower()}: no selector")
        try:
            return str(selector_from_label_selector(sel))
        except SelectorError as e:
            raise ValueError(f"invalid label selector: {e}") from None
    raise ValueError(f"selector for {kind} not implemented")


async def first_pod(c, ns: str, selector: str, timeout: float) -> tuple[dict, int]:
    """GetFirstPod: the best pod of the selector by ByLogging, waiting up to `timeout` for one."""
    end = time.monotonic() + timeout
    while True:
        items, _ = await c.list("pods", ns, selector)
        if items:
            return sort_by_logging(items)[0], len(items)
        if time.monotonic() >= end:
            raise TimeoutError("timed out waiting for the condition")
        await asyncio.sleep(0.2)


def _options(a) -> dict:
    """PodLogOptions from the flags, checked as ValidatePodLogOptions does."""
    from ..kubelet.logs import parse_rfc3339, validate_pod_log_options
    o = {"previous": bool(getattr(a, "previous", False)), "timestamps": bool(getattr(a, "timestamps", False)),
         "follow": bool(getattr(a, "follow", False))}
    if getattr(a, "since_time", None):
        parse_rfc3339(a.since_time)
        o["sinceTime"] = a.since_time
    if getattr(a, "limit_bytes", 0):
        o["limitBytes"] = int(a.limit_bytes)
    if a.tail != -1:
        o["tailLines"] = int(a.tail)
    if getattr(a, "since", None):
        import math
        o["sinceSeconds"] = int(math.ceil(parse_duration_s(a.since)))
    errs = validate_pod_log_options(o)
    if errs:
        raise ValueError("; ".join(str(e) for e in errs) if len(errs) == 1 else "[" + ", ".join(str(e) for e in errs) + "]")
    return o


async def cmd_logs(c, a):
    args = list(a.args)
    container = a.container
    selector = a.selector
    if not args:
        if not selector:
            print(f"error: {USAGE}", file=sys.stderr)
            return 1
    elif len(args) == 1:
        if selector:
            print("error: only a selector (-l) or a POD name is allowed", file=sys.stderr)
            return 1
    elif len(args) == 2:
        if a.container:
            print("error: only one of -c or an inline [CONTAINER] arg is allowed", file=sys.stderr)
            return 1
        container = args[1]
    else:
        print(f"error: {USAGE}", file=sys.stderr)
        return 1
    try:
        opts = _options(a)
    except ValueError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    if selector and opts["follow"]:
        print("error: only one of follow (-f) or selector (-l) is allowed", file=sys.stderr)
        return 1
    ns = a.namespace or "default"
    if selector:
        pods = [m.name_of(p) for p in (await c.list("pods", ns, selector))[0]]
    else:
        ref = args[0]
        if "/" in ref:
            kind, name = ref.split("/", 1)
            ri = SCHEME.resolve(kind)
            if ri is None:
                print(f'error: the server doesn\'t have a resource type "{kind}"', file=sys.stderr)
                return 1
        else:
            ri, name = SCHEME.resolve("pods"), ref
        if ri.plural == "pods":
            pods = [name]
        else:
            obj = await c.get(f"{ri.plural}.{ri.group}" if ri.group else ri.plural, name, ns)
            try:
                sel = selector_for_object(obj)
                pod, n = await first_pod(c, ns, sel, float(getattr(a, "pod_running_timeout", 20.0) or 20.0))
            except (ValueError, TimeoutError) as e:
                print(f"error: {e}", file=sys.stderr)
                return 1
            if n > 1:
                print(f"Found {n} pods, using pod/{m.name_of(pod)}", file=sys.stderr)
            pods = [m.name_of(pod)]
    kw = {"previous": opts["previous"], "timestamps": opts["timestamps"], "since_seconds": opts.get("sinceSeconds"),
          "since_time": opts.get("sinceTime"), "limit_bytes": opts.get("limitBytes")}
    out = sys.stdout.buffer
    for name in pods:
        if opts["follow"]:
            async for chunk in c.stream_logs(ns, name, container, opts.get("tailLines"), **kw):
                out.write(chunk)
                out.flush()
        else:
            text = await c.logs(ns, name, container, opts.get("tailLines"), **kw)
            out.write(text.encode())
            out.flush()
    return 0


def rewrite_short_flags(argv: list[str]) -> list[str]:
    """`kubectl logs -f` / `-p` are --follow / --previous (the shared parser gives -f to
    --filename and -p to --patch); `log` is an alias of `logs`."""
    value_flags = {"-s", "--server", "--token", "--kubeconfig", "--context", "-n", "--namespace"}
    i, cmd_at = 0, None
    while i < len(argv):
        t = argv[i]
        if t in value_flags:
            i += 2
            continue
        if t.startswith("-"):
            i += 1
            continue
        cmd_at = i
        break
    if cmd_at is None or argv[cmd_at] not in ("logs", "log"):
        return argv
    out = argv[:cmd_at] + ["logs"]
    for t in argv[cmd_at + 1:]:
        if t == "-f":
            out.append("--follow")
        elif t == "-p":
            out.append("--previous")
        elif len(t) > 2 and t[0] == "-" and t[1] != "-" and set(t[1:]) <= {"f", "p"}:
            out += ["--follow" if ch == "f" else "--previous" for ch in t[1:]]
        else:
            out.append(t)
    return out


def add_arguments(sp):
    sp.add_argument("--follow", action="store_true")
    sp.add_argument("--previous", action="store_true")
    sp.add_argument("--timestamps", action="store_true")
    sp.add_argument("--since", default=None)
    sp.add_argument("--since-time", default=None)
    sp.add_argument("--limit-bytes", type=int, default=0)
    sp.add_argument("--pod-running-timeout", type=lambda s: parse_duration_s(s) if s[-1:].isalpha() else float(s),
                    default=20.0)
