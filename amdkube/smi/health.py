"""Device health from amd-smi RAS state, judged on NEW faults.

The reference's plugin contract only carries `health` per device (Healthy/Unhealthy); the
kubelet refuses to admit pods onto an unhealthy device but leaves running pods alone
(pkg/kubelet/cm/devicemanager/device_store.go:103-110, manager_store.go:116-118).
What counts as unhealthy is the plugin's call. A lifetime counter is the wrong signal: a part
with one uncorrectable error from last year would stay unschedulable forever, and a part
already above a threshold would hide every new error. So the monitor snapshots each GPU's RAS
state when it starts and flags:

  * uncorrectable ECC errors above `ecc_threshold` SINCE the snapshot (deferred errors too);
  * an xGMI error status that was clear at the snapshot, or new uncorrectable errors in the
    XGMI_WAFL RAS block (link errors: the multi-GPU collectives of a pod placed across this GPU
    would fail or crawl);
  * new pages pending retirement or unreservable (memory the driver could not retire);
  * the bad-page count reaching the driver's bad-page threshold (the RAS EEPROM's limit:
    the part needs service);
  * any RAS/SMI query that fails outright.

A flagged device stays Unhealthy until an operator resets it. With a `state_file` the
baselines and the sticky reasons are checkpointed (keyed by device ID, like the kubelet's
device checkpoint, pkg/kubelet/cm/devicemanager/manager_store.go), so a plugin restart keeps
judging against the ORIGINAL baseline and a faulted GPU is re-advertised Unhealthy with its
reason instead of being re-baselined into service. `amdkube gpu-health reset <id|all>` drops a
`<state_file>.reset` request that the running plugin applies on its next health tick (fresh
baseline, fault cleared). Without a state file the state lives as long as the process. The
reason is published as the `amd.com/health-reason` attribute.

Faults the RAS counters cannot see come from the kernel log: the node-problem-detector's
amdgpu rules (monitoring/problemdetector.py) append `{"device": <pci address|device id>,
"reason": …}` lines to `<state_file>.faults`; `pending_faults()` hands them to the plugin,
which makes them sticky like any other fault (`fault()`).
"""
from __future__ import annotations

import json
import logging
import os
import time

HEALTH_REASON_ATTR = "amd.com/health-reason"
log = logging.getLogger("amdkube.health")


def request_reset(state_file: str, device_ids: list[str]):
    """Ask the plugin that owns `state_file` to clear these devices' faults ("all": every one)."""
    with open(state_file + ".reset", "a") as f:
        for d in device_ids:
            f.write(d + "\n")


class HealthMonitor:
    def __init__(self, backend, ecc_threshold: int = 0, state_file: str | None = None, key_of=None):
        self.backend = backend
        self.ecc_threshold = ecc_threshold
        self.baseline: dict[int, dict] = {}
        self.sticky: dict[int, str] = {}
        self.state_file = state_file
        self.key_of = key_of or str
        self._saved: dict[str, dict] = self._load()

    # ------------------------------------------------------------------ checkpoint
    def _load(self) -> dict:
        if not self.state_file or not os.path.exists(self.state_file):
            return {}
        try:
            with open(self.state_file) as f:
                return dict((json.load(f) or {}).get("gpus") or {})
        except (OSError, ValueError) as e:
            log.error("health state %s unreadable (%s); starting from fresh baselines", self.state_file, e)
            return {}

    def _save(self):
        if not self.state_file:
            return
        os.makedirs(os.path.dirname(os.path.abspath(self.state_file)), exist_ok=True)
        tmp = self.state_file + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"gpus": self._saved}, f, sort_keys=True, default=str)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.state_file)

    def pending_resets(self) -> set[str]:
        """Device IDs (or "all") an operator asked to reset since the last call."""
        if not self.state_file:
            return set()
        req = self.state_file + ".reset"
        try:
            with open(req) as f:
                ids = {line.strip() for line in f if line.strip()}
            os.unlink(req)
            return ids
        except FileNotFoundError:
            return set()

    def pending_faults(self) -> list[dict]:
        """Faults reported from outside (the node-problem-detector) since the last call."""
        if not self.state_file:
            return []
        req = self.state_file + ".faults"
        try:
            tmp = req + f".{os.getpid()}"
            os.replace(req, tmp)              # take the whole file; a writer appending now starts a new one
        except FileNotFoundError:
            return []
        out = []
        with open(tmp) as f:
            for line in f:
                try:
                    ent = json.loads(line)
                except ValueError:
                    continue
                if isinstance(ent, dict) and ent.get("device") and ent.get("reason"):
                    out.append(ent)
        os.unlink(tmp)
        return out

    def fault(self, index: int, why: str):
        """Take a device out of service until an operator resets it (checkpointed)."""
        if index in self.sticky:
            return
        if index not in self.baseline:
            self.snapshot(index)
        self.sticky[index] = why
        ent = self._saved.setdefault(self.key_of(index), {"baseline": self.baseline.get(index) or {}})
        ent["sticky"], ent["faulted_at"] = why, time.time()
        self._save()

    def reset(self, index: int):
        """Clear a device's fault and judge it from a fresh baseline from now on."""
        self.sticky.pop(index, None)
        self.snapshot(index, fresh=True)

    def _state(self, index: int) -> dict:
        st = dict(self.backend.sample(index))
        try:
            st.update({f"ras_{k}" if not k.startswith(("xgmi_error", "bad_page")) else k: v
                       for k, v in (self.backend.ras(index) or {}).items()})
        except Exception as e:   # noqa: BLE001 — a RAS query that fails outright is itself a fault
            st["ras_error"] = str(e)
        return st

    def snapshot(self, index: int, fresh: bool = False) -> dict:
        """The baseline new faults are judged against: the checkpointed one when there is one
        (a restart keeps it and any sticky fault), else the device's state now."""
        key = self.key_of(index)
        ent = self._saved.get(key)
        if ent is not None and not fresh:
            self.baseline[index] = ent.get("baseline") or {}
            if ent.get("sticky"):
                self.sticky[index] = ent["sticky"]
            return self.baseline[index]
        try:
            self.baseline[index] = self._state(index)
        except Exception as e:   # noqa: BLE001
            self.baseline[index] = {"snapshot_error": str(e)}
        self._saved[key] = {"baseline": self.baseline[index], "sticky": "", "since": time.time()}
        self._save()
        return self.baseline[index]

    def check(self, index: int) -> tuple[bool, str]:
        if index in self.sticky:
            return False, self.sticky[index]
        if index not in self.baseline:
            self.snapshot(index)
        base = self.baseline[index]
        try:
            cur = self._state(index)
        except Exception as e:   # noqa: BLE001
            return False, f"smi query failed: {e}"
        why = self._judge(base, cur)
        if why:
            self.sticky[index] = why
            ent = self._saved.setdefault(self.key_of(index), {"baseline": base})
            ent["sticky"], ent["faulted_at"] = why, time.time()
            self._save()
            return False, why
        return True, ""

    def _judge(self, base: dict, cur: dict) -> str:
        if cur.get("ras_error"):
            return f"RAS query failed: {cur['ras_error']}"
        due = cur.get("ecc_uncorrectable", 0) - base.get("ecc_uncorrectable", 0)
        if due > self.ecc_threshold:
            return f"uncorrectable ECC errors: +{due} since the plugin started (lifetime {cur.get('ecc_uncorrectable')})"
        ddef = cur.get("ecc_deferred", 0) - base.get("ecc_deferred", 0)
        if ddef > self.ecc_threshold:
            return f"deferred ECC errors: +{ddef} since the plugin started"
        if cur.get("xgmi_error", 0) and not base.get("xgmi_error", 0):
            return "xGMI link error" if cur["xgmi_error"] == 1 else "multiple xGMI link errors"
        # the XGMI_WAFL RAS block's uncorrectable count: the same fault where the error-status
        # file is not readable (the MI355X gpurun box answers that query with INVAL)
        dx = cur.get("ras_xgmi_ecc_uncorrectable", 0) - base.get("ras_xgmi_ecc_uncorrectable", 0)
        if dx > self.ecc_threshold:
            return f"xGMI link uncorrectable errors: +{dx} since the plugin started"
        for k, what in (("bad_pages_pending", "pending retirement"), ("bad_pages_unreservable", "unreservable")):
            d = cur.get(k, 0) - base.get(k, 0)
            if d > 0:
                return f"{d} new bad page(s) {what}"
        thr = cur.get("bad_page_threshold")
        if thr and cur.get("bad_pages", 0) >= thr:
            return f"bad pages {cur['bad_pages']} reached the retirement threshold {thr}"
        return ""
