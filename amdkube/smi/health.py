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

A flagged device stays Unhealthy until the plugin restarts (a fresh snapshot), the same
lifetime the reference gives a ListAndWatch health flip. The reason is kept per device and
published as the `amd.com/health-reason` attribute.
"""
from __future__ import annotations

HEALTH_REASON_ATTR = "amd.com/health-reason"


class HealthMonitor:
    def __init__(self, backend, ecc_threshold: int = 0):
        self.backend = backend
        self.ecc_threshold = ecc_threshold
        self.baseline: dict[int, dict] = {}
        self.sticky: dict[int, str] = {}

    def _state(self, index: int) -> dict:
        st = dict(self.backend.sample(index))
        try:
            st.update({f"ras_{k}" if not k.startswith(("xgmi_error", "bad_page")) else k: v
                       for k, v in (self.backend.ras(index) or {}).items()})
        except Exception as e:   # noqa: BLE001 — a RAS query that fails outright is itself a fault
            st["ras_error"] = str(e)
        return st

    def snapshot(self, index: int) -> dict:
        try:
            self.baseline[index] = self._state(index)
        except Exception as e:   # noqa: BLE001
            self.baseline[index] = {"snapshot_error": str(e)}
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
