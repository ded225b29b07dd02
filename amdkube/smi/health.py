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

The checkpointed counters are only comparable while the counters they came from live: ECC and
xGMI counters restart at 0 after a reboot or a driver reload, while the state file (under
/var/lib/kubelet) survives both. The checkpoint therefore records the instance it was taken
in (the kernel boot_id and the amdgpu module's load time); when that changed, or when any
counter went DOWN, the baseline is retaken from the device's state now, keeping the sticky
reasons (a faulted GPU stays out of service until an operator resets it).

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


BOOT_ID = "/proc/sys/kernel/random/boot_id"
AMDGPU_MODULE = "/sys/module/amdgpu"
COUNTERS = ("ecc_uncorrectable", "ecc_deferred", "ecc_correctable", "ras_xgmi_ecc_uncorrectable",
            "bad_pages_pending", "bad_pages_unreservable", "bad_pages")


def instance_id(boot_id_path: str = BOOT_ID, module_path: str = AMDGPU_MODULE) -> str:
    """This boot and this load of the amdgpu driver: counters are comparable only within it."""
    try:
        with open(boot_id_path) as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    try:
        loaded = str(int(os.stat(module_path).st_ctime))
    except OSError:
        loaded = ""
    return f"{boot}/{loaded}"


def request_reset(state_file: str, device_ids: list[str]):
    """Ask the plugin that owns `state_file` to clear these devices' faults ("all": every one)."""
    with open(state_file + ".reset", "a") as f:
        for d in device_ids:
            f.write(d + "\n")


class HealthMonitor:
    def __init__(self, backend, ecc_threshold: int = 0, state_file: str | None = None, key_of=None,
                 instance=instance_id):
        self.backend = backend
        self.ecc_threshold = ecc_threshold
        self.baseline: dict[int, dict] = {}
        self.sticky: dict[int, str] = {}
        self.state_file = state_file
        self.key_of = key_of or str
        self.instance = instance() if callable(instance) else str(instance)
        self._saved_instance = None
        self._saved: dict[str, dict] = self._load()
        if self._saved and self._saved_instance != self.instance:
            log.warning("health state %s was taken in another boot or driver load (%s, now %s): "
                        "counters restarted, baselines are retaken (faults stay)", state_file,
                        self._saved_instance, self.instance)
            for ent in self._saved.values():
                ent["stale"] = True

    # ------------------------------------------------------------------ checkpoint
    def _load(self) -> dict:
        if not self.state_file or not os.path.exists(self.state_file):
            return {}
        try:
            with open(self.state_file) as f:
                doc = json.load(f) or {}
            self._saved_instance = doc.get("instance")
            return dict(doc.get("gpus") or {})
        except (OSError, ValueError) as e:
            log.error("health state %s unreadable (%s); starting from fresh baselines", self.state_file, e)
            return {}

    def _save(self):
        if not self.state_file:
            return
        os.makedirs(os.path.dirname(os.path.abspath(self.state_file)), exist_ok=True)
        tmp = self.state_file + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"gpus": self._saved, "instance": self.instance}, f, sort_keys=True, default=str)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.state_file)

    def pending_resets(self) -> set[str]:
        """Device IDs (or "all") an operator asked to reset since the last call."""
        if not self.state_file:
            return set()
        req = self.state_file + ".reset"
        tmp = req + f".{os.getpid()}"
        try:
            os.replace(req, tmp)              # take the whole file; a later request starts a new one
        except FileNotFoundError:
            return set()
        with open(tmp) as f:
            ids = {line.strip() for line in f if line.strip()}
        os.unlink(tmp)
        return ids

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
        keep = ""
        if ent is not None and not fresh:
            if ent.get("sticky"):
                self.sticky[index] = ent["sticky"]
            if not ent.get("stale"):
                self.baseline[index] = ent.get("baseline") or {}
                return self.baseline[index]
            keep = ent.get("sticky") or ""      # another boot/driver load: retake, keep the fault
        try:
            self.baseline[index] = self._state(index)
        except Exception as e:   # noqa: BLE001
            self.baseline[index] = {"snapshot_error": str(e)}
        self._saved[key] = {"baseline": self.baseline[index], "sticky": keep, "since": time.time()}
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
        if any(cur.get(k, 0) < base.get(k, 0) for k in COUNTERS if isinstance(cur.get(k, 0), (int, float))):
            # a counter went down: the driver restarted them (reload, reset) under a live plugin;
            # judge from here on
            log.warning("GPU %s RAS counters went down (%s -> %s); taking a fresh baseline", self.key_of(index),
                        {k: base.get(k) for k in COUNTERS if k in base}, {k: cur.get(k) for k in COUNTERS if k in cur})
            self.baseline[index] = cur
            self._saved[self.key_of(index)] = {"baseline": cur, "sticky": "", "since": time.time()}
            self._save()
            return True, ""
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
