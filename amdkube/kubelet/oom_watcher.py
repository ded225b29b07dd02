"""System OOM watcher: the reference's pkg/kubelet/oom_watcher.go, which streams cAdvisor's
kernel-log OOM events and records a `SystemOOM` Warning event on the Node for each.

cgroup-v2 hosts count every kernel OOM kill in /proc/vmstat `oom_kill`; the watcher polls it
and, for each increase, records one event per kill. When the kernel log is readable
(/dev/kmsg needs CAP_SYSLOG) the victim's "Killed process <pid> (<comm>)" line is added to
the message; otherwise the event carries the reference's plain text.
"""
from __future__ import annotations

import asyncio
import logging
import os
import re

log = logging.getLogger("amdkube.kubelet.oom")

SYSTEM_OOM_EVENT = "SystemOOM"
_VICTIM = re.compile(r"Killed process (\d+) \(([^)]*)\)")


def read_oom_kills(vmstat: str = "/proc/vmstat") -> int | None:
    try:
        with open(vmstat) as f:
            for line in f:
                if line.startswith("oom_kill "):
                    return int(line.split()[1])
    except (OSError, ValueError):
        pass
    return None


class KmsgReader:
    """Non-blocking reader of new kernel log records (each read returns whole records)."""

    def __init__(self, path: str = "/dev/kmsg"):
        self.fd = None
        try:
            self.fd = os.open(path, os.O_RDONLY | os.O_NONBLOCK)
        except OSError:
            self.fd = None
            return
        try:
            os.lseek(self.fd, 0, os.SEEK_END)          # only records from now on
        except OSError:
            pass                                        # a stream (tests): nothing to skip

    def victims(self) -> list[tuple[int, str]]:
        out = []
        while self.fd is not None:
            try:
                rec = os.read(self.fd, 8192)
            except BlockingIOError:
                break
            except OSError:              # EPIPE: overwritten records; keep reading
                continue
            if not rec:
                break
            mt = _VICTIM.search(rec.decode(errors="replace"))
            if mt:
                out.append((int(mt.group(1)), mt.group(2)))
        return out

    def close(self):
        if self.fd is not None:
            os.close(self.fd)
            self.fd = None


class OOMWatcher:
    def __init__(self, recorder, node_ref, vmstat: str = "/proc/vmstat", kmsg: str | None = "/dev/kmsg",
                 period: float = 1.0):
        self.recorder, self.node_ref = recorder, node_ref
        self.vmstat, self.period = vmstat, period
        self.kmsg = KmsgReader(kmsg) if kmsg else None
        self.last = read_oom_kills(vmstat)
        self.events = 0

    def poll(self) -> int:
        """Record one SystemOOM event per new kernel OOM kill; returns how many."""
        cur = read_oom_kills(self.vmstat)
        victims = self.kmsg.victims() if self.kmsg is not None else []
        if cur is None or self.last is None:
            self.last = cur
            return 0
        new, self.last = max(0, cur - self.last), cur
        for i in range(new):
            msg = "System OOM encountered"
            if i < len(victims):
                msg += f", victim process: {victims[i][1]}, pid: {victims[i][0]}"
            self.recorder.event(self.node_ref(), "Warning", SYSTEM_OOM_EVENT, msg)
        self.events += new
        return new

    async def run(self):
        if self.last is None:
            log.info("no oom_kill counter in %s; system OOM events are not reported", self.vmstat)
            return
        try:
            while True:
                await asyncio.sleep(self.period)
                self.poll()
        finally:
            if self.kmsg is not None:
                self.kmsg.close()
