"""Kubelet run-once mode (pkg/kubelet/runonce.go, `kubelet --runonce`): read the static pod
manifests once, run every pod without any API server, wait until each is running — syncing it
again with a doubling back-off (1 s, 10 attempts: runOnceMaxRetries / runOnceRetryDelay /
runOnceRetryDelayBackoff) — report per-pod results and exit. Used to bring up a node's own
services (and MI355X burn-in or health pods) before the control plane exists.
"""
from __future__ import annotations

import asyncio
import logging

from ..api import meta as m

log = logging.getLogger("amdkube.kubelet.runonce")

MAX_RETRIES = 10
RETRY_DELAY = 1.0
BACKOFF = 2


class NullClient:
    """The absent API server: reads find nothing, writes are dropped."""

    async def get_or_none(self, *a, **k):
        return None

    async def get(self, resource, name, *a, **k):
        raise m.StatusError(404, "NotFound", f'{resource} "{name}" not found (run-once mode has no API server)')

    async def list(self, *a, **k):
        return [], "0"

    async def create(self, obj, *a, **k):
        return obj

    async def patch(self, *a, **k):
        return {}

    async def update(self, obj, *a, **k):
        return obj

    async def delete(self, *a, **k):
        return {}

    async def request(self, *a, **k):
        return {}

    def set_client_cert(self, *a):
        pass

    async def close(self):
        pass


def _running(rt, pod) -> bool:
    """isPodRunning: the sandbox is ready and every container's newest instance is running."""
    from ..grpcdesc.cri import CRI as C
    if rt.ready_sandbox() is None:
        return False
    for c in (pod.get("spec") or {}).get("containers") or []:
        cur = rt.latest(c["name"])
        if cur is None or cur.state != C.CONTAINER_RUNNING:
            return False
    return True


async def run_pod(kubelet, pod: dict, retries: int = MAX_RETRIES, delay: float = RETRY_DELAY) -> str | None:
    """runPod: sync until running; None on success, else the last error."""
    uid = m.uid_of(pod)
    kubelet.pods[uid] = pod
    last = None
    for attempt in range(retries):
        try:
            await kubelet.sync_pod(uid)
            rt = await kubelet.runtime.pod_status(uid)
            if _running(rt, pod):
                log.info("pod %s is running", m.name_of(pod))
                return None
            last = kubelet.rejected.get(uid, ("", f"pod {m.name_of(pod)} is not running yet"))[1]
            if uid in kubelet.rejected:
                return f"rejected: {last}"
        except Exception as e:      # a failed sync is retried like a not-yet-running pod
            last = repr(e)
        log.info("pod %s not running (attempt %d): %s; retrying in %.1fs", m.name_of(pod), attempt + 1, last, delay)
        await asyncio.sleep(delay)
        delay *= BACKOFF
    return f"timeout after {retries} attempts: {last}"


async def run_once(kubelet, retries: int = MAX_RETRIES, delay: float = RETRY_DELAY) -> list[dict]:
    """kl.runOnce: all pods of the manifest directory at once; [{"pod", "error"}]."""
    pods = list(kubelet._read_manifests().values())
    kubelet._static_read = True
    results = await asyncio.gather(*(run_pod(kubelet, p, retries, delay) for p in pods))
    out = [{"pod": m.name_of(p), "error": err} for p, err in zip(pods, results)]
    for r in out:
        if r["error"]:
            log.error("failed to run pod %s: %s", r["pod"], r["error"])
    return out


async def start_standalone(kubelet):
    """The parts of Kubelet.start a run needs without an API server: runtime, device plugins."""
    import os
    os.makedirs(os.path.join(kubelet.cfg.root_dir, "pods"), exist_ok=True)
    await kubelet.cri.connect()
    await kubelet.dm.start()
    kubelet.volume_manager.start()
    if hasattr(kubelet.dm, "wait_initial_registration"):
        await kubelet.dm.wait_initial_registration(5.0)
    return kubelet
