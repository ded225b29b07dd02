"""Pod status generation + status manager.

Reference: pkg/kubelet/kubelet_pods.go generateAPIPodStatus/getPhase (phase from container
states and restartPolicy), convertToAPIContainerStatuses; pkg/kubelet/status/
status_manager.go:131,399 (versioned per-pod status cache, background sync to the API,
never regress a terminal phase).
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..api import meta as m
from ..utils.trace import POD_TRACE
from ..grpcdesc.cri import CRI as C

log = logging.getLogger("amdkube.kubelet.status")


def _ts(ns: int) -> str | None:
    if not ns:
        return None
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(ns / 1e9))


def _terminated(rs) -> dict:
    term = {"exitCode": rs.exit_code, "reason": rs.reason or ("Completed" if rs.exit_code == 0 else "Error"),
            "startedAt": _ts(rs.started_at), "finishedAt": _ts(rs.finished_at), "containerID": f"rocshim://{rs.id}"}
    if rs.message:
        term["message"] = rs.message
    return term


def container_status(spec_c: dict, rs, ready: bool, will_restart: bool, waiting_reason: str,
                     last_error: tuple[str, str] | None = None, prev=None) -> dict:
    """convertToAPIContainerStatuses (kubelet_pods.go:1464-1605): the newest instance is the
    state, the one before it the lastState; a container that will be restarted waits."""
    out = {"name": spec_c["name"], "image": spec_c.get("image", ""), "imageID": "", "ready": False, "restartCount": 0}
    if prev is not None and prev.state in (C.CONTAINER_EXITED, C.CONTAINER_UNKNOWN, C.CONTAINER_CREATED):
        out["lastState"] = {"terminated": _terminated(prev)}
    if rs is None:
        # reason_cache.go: a container that failed to start waits with that failure's reason
        out["state"] = {"waiting": {"reason": last_error[0], "message": last_error[1]} if last_error
                        else {"reason": waiting_reason}}
        return out
    out["restartCount"] = rs.restart_count
    out["containerID"] = f"rocshim://{rs.id}"
    out["imageID"] = rs.image_ref
    if rs.state == C.CONTAINER_RUNNING:
        out["state"] = {"running": {"startedAt": _ts(rs.started_at)}}
        out["ready"] = ready
    elif rs.state in (C.CONTAINER_EXITED, C.CONTAINER_UNKNOWN):
        term = _terminated(rs)
        if will_restart:
            out["state"] = {"waiting": {"reason": last_error[0], "message": last_error[1]} if last_error else
                            {"reason": "CrashLoopBackOff" if rs.exit_code else "Completed",
                             "message": "back-off restarting failed container"}}
            out["lastState"] = {"terminated": term}
        else:
            out["state"] = {"terminated": term}
    else:
        out["state"] = {"waiting": {"reason": "ContainerCreating"}}
    return out


def _prev(rt, name):
    lst = rt.containers.get(name) if rt is not None else None
    return lst[1] if lst and len(lst) > 1 else None


def generate_status(pod: dict, rt, node_ip: str, readiness: dict, errors: list[str], now: str,
                    reasons: dict | None = None) -> dict:
    """`reasons`: container name → (reason, message) of its last start failure."""
    reasons = reasons or {}
    spec = pod.get("spec") or {}
    old = pod.get("status") or {}
    policy = spec.get("restartPolicy", "Always")
    inits = spec.get("initContainers") or []
    conts = spec.get("containers") or []
    init_done = True
    init_failed = False
    init_statuses = []
    for ic in inits:
        rs = rt.latest(ic["name"]) if rt else None
        done = rs is not None and rs.state == C.CONTAINER_EXITED and rs.exit_code == 0
        failed = rs is not None and rs.state == C.CONTAINER_EXITED and rs.exit_code != 0
        if failed and policy == "Never":
            init_failed = True
        if not done:
            init_done = False
        init_statuses.append(container_status(ic, rs, done, failed and policy != "Never", "PodInitializing",
                                              reasons.get(ic["name"])))
    running = succeeded = failed_n = waiting = 0
    statuses = []
    all_ready = True
    for c in conts:
        rs = rt.latest(c["name"]) if rt and init_done else None
        if rs is None:
            waiting += 1
            all_ready = False
            statuses.append(container_status(c, None, False, False, "ContainerCreating" if init_done else "PodInitializing",
                                             reasons.get(c["name"]) if init_done else None))
            continue
        if rs.state == C.CONTAINER_RUNNING:
            running += 1
            # a container with a readiness probe starts unready until its first success
            # (reference prober/worker.go: readiness initialValue = results.Failure)
            ready = readiness.get(c["name"], not c.get("readinessProbe"))
            all_ready &= ready
            statuses.append(container_status(c, rs, ready, False, "", prev=_prev(rt, c["name"])))
        elif rs.state in (C.CONTAINER_EXITED, C.CONTAINER_UNKNOWN):
            all_ready = False
            if rs.exit_code == 0:
                succeeded += 1
            else:
                failed_n += 1
            restart = policy == "Always" or (policy == "OnFailure" and rs.exit_code != 0)
            statuses.append(container_status(c, rs, False, restart, "", reasons.get(c["name"]),
                                             prev=None if restart else _prev(rt, c["name"])))
        else:
            waiting += 1
            all_ready = False
            statuses.append(container_status(c, rs, False, False, "ContainerCreating"))
    # getPhase (kubelet_pods.go)
    if init_failed:
        phase = "Failed"
    elif not init_done:
        phase = "Pending"
    elif waiting and not running:
        phase = "Pending"
    elif running:
        phase = "Running"
    elif policy == "Always":
        phase = "Running"
    elif succeeded == len(conts):
        phase = "Succeeded"
    elif policy == "OnFailure":
        phase = "Running"
    else:
        phase = "Failed"
    conds = []
    for c in old.get("conditions") or []:
        if c.get("type") == "PodScheduled":
            conds.append(c)

    def cond(t, ok, reason=None):
        prev = next((c for c in old.get("conditions") or [] if c.get("type") == t), None)
        st = "True" if ok else "False"
        d = {"type": t, "status": st, "lastProbeTime": None,
             "lastTransitionTime": prev["lastTransitionTime"] if prev and prev.get("status") == st and prev.get("lastTransitionTime") else now}
        if reason and not ok:
            d["reason"] = reason
        conds.append(d)
    cond("Initialized", init_done, "ContainersNotInitialized")
    ready = phase == "Running" and all_ready and bool(conts)
    cond("ContainersReady", ready, "ContainersNotReady")
    cond("Ready", ready, "ContainersNotReady")
    pod_ip = node_ip if spec.get("hostNetwork") else (getattr(rt, "ip", "") or node_ip)
    st = {"phase": phase, "conditions": conds, "hostIP": node_ip, "podIP": pod_ip,
          "startTime": old.get("startTime") or now, "containerStatuses": statuses,
          "initContainerStatuses": init_statuses or None, "qosClass": old.get("qosClass"),
          "message": "; ".join(errors) if errors else None, "reason": None}
    return st


class StatusManager:
    """Per-pod latest status; pushes changes to the API server in the background."""

    def __init__(self, client, on_terminal=None):
        self.client = client
        self.statuses: dict[str, tuple[dict, dict]] = {}  # uid -> (pod meta ref, status)
        self.sent: dict[str, dict] = {}
        self.terminal: set[str] = set()
        self.dirty: dict[str, None] = {}
        self._wake = asyncio.Event()
        self._task = None
        self.on_terminal = on_terminal
        self.updates = 0

    def start(self):
        self._task = asyncio.create_task(self._run(), name="status-manager")
        return self

    async def stop(self):
        if self._task:
            self._task.cancel()

    def set(self, pod: dict, status: dict):
        uid = m.uid_of(pod)
        if uid in self.terminal and status.get("phase") not in ("Succeeded", "Failed"):
            return  # never regress a terminal phase
        self.statuses[uid] = ({"name": m.name_of(pod), "namespace": m.namespace_of(pod), "uid": uid}, status)
        if self.sent.get(uid) != status:
            self.dirty[uid] = None
            self._wake.set()

    def get(self, uid):
        s = self.statuses.get(uid)
        return s[1] if s else None

    def forget(self, uid):
        self.statuses.pop(uid, None)
        self.sent.pop(uid, None)
        self.dirty.pop(uid, None)
        self.terminal.discard(uid)

    async def flush(self, uid):
        """Synchronously push one pod's status (used before the final delete)."""
        if uid in self.dirty:
            self.dirty.pop(uid, None)
            await self._send(uid)

    async def _run(self):
        while True:
            await self._wake.wait()
            self._wake.clear()
            batch = list(self.dirty)
            self.dirty.clear()
            await asyncio.gather(*(self._send(uid) for uid in batch))

    async def _send(self, uid):
        ent = self.statuses.get(uid)
        if ent is None:
            return
        ref, status = ent
        if self.sent.get(uid) == status:
            return
        try:
            await self.client.patch("pods", ref["name"], {"status": status}, ref["namespace"], sub="status")
            POD_TRACE(uid, "sent_" + str(status.get("phase")))
            self.sent[uid] = status
            self.updates += 1
            if status.get("phase") in ("Succeeded", "Failed"):
                self.terminal.add(uid)
                if self.on_terminal:
                    self.on_terminal(uid)
        except m.StatusError as e:
            if m.is_not_found(e):
                self.forget(uid)
                return
            log.debug("status update for %s failed: %s", ref["name"], e)
            self.dirty[uid] = None
            asyncio.get_running_loop().call_later(0.2, self._wake.set)
        except Exception as e:
            log.debug("status update for %s failed: %r", ref["name"], e)
            self.dirty[uid] = None
            asyncio.get_running_loop().call_later(0.5, self._wake.set)
