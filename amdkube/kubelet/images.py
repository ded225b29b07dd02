"""Image garbage collection (pkg/kubelet/images/image_gc_manager.go).

Every ImageGCPeriod (5 min) the manager refreshes its image records (first detected, last
used — an image is in use while any container, running or not, references it — and size) and,
when the image filesystem is at or above --image-gc-high-threshold percent, frees
capacity × (100 − --image-gc-low-threshold) / 100 − available bytes by deleting unused images,
least recently used first (then oldest detected), skipping images younger than
--minimum-image-ttl-duration. Failing to free enough records a FreeDiskSpaceFailed event. The
eviction manager calls delete_unused() to reclaim disk under nodefs/imagefs pressure
(eviction_manager.go reclaimNodeLevelResources).
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import dataclass

log = logging.getLogger("amdkube.kubelet.images")


class ImageGCError(RuntimeError):
    pass


@dataclass
class ImageRecord:
    first_detected: float
    last_used: float
    size: int


class ImageGCManager:
    def __init__(self, cri, high: int = 85, low: int = 80, min_age: float = 120.0, clock=time.time, recorder=None,
                 node_ref=None):
        if not 0 <= high <= 100:
            raise ValueError(f"invalid HighThresholdPercent {high}, must be in range [0-100]")
        if not 0 <= low <= 100:
            raise ValueError(f"invalid LowThresholdPercent {low}, must be in range [0-100]")
        if low > high:
            raise ValueError(f"LowThresholdPercent {low} can not be higher than HighThresholdPercent {high}")
        self.cri, self.high, self.low, self.min_age, self.clock = cri, high, low, min_age, clock
        self.recorder, self.node_ref = recorder, node_ref
        self.records: dict[str, ImageRecord] = {}

    async def detect(self) -> set[str]:
        now = self.clock()
        images = await self.cri.list_images()
        conts = await self.cri.list_containers()
        in_use = {c.image_ref for c in conts} | {c.image.image for c in conts}
        ids = set()
        for img in images:
            ids.add(img.id)
            rec = self.records.get(img.id)
            if rec is None:
                rec = self.records[img.id] = ImageRecord(now, 0.0, int(img.size))
            used = img.id in in_use or any(t in in_use for t in img.repo_tags)
            if used:
                rec.last_used = now
            rec.size = int(img.size)
        for k in [k for k in self.records if k not in ids]:
            del self.records[k]
        return {i for i in ids if self.records[i].last_used == now}

    async def fs_stats(self) -> tuple[int, int]:
        """(capacity, available) of the runtime's image filesystem."""
        fss = await self.cri.image_fs_info()
        path = fss[0].storage_id.uuid if fss else "/"
        try:
            st = os.statvfs(path if os.path.isabs(path) else "/")
        except OSError:
            st = os.statvfs("/")
        return st.f_blocks * st.f_frsize, st.f_bavail * st.f_frsize

    async def free_space(self, amount: int) -> int:
        in_use = await self.detect()
        now = self.clock()
        cands = sorted(((rid, r) for rid, r in self.records.items() if rid not in in_use),
                       key=lambda x: (x[1].last_used, x[1].first_detected))
        freed = 0
        for rid, r in cands:
            if now - r.first_detected < self.min_age:
                continue            # just pulled: a container may be about to use it
            try:
                await self.cri.remove_image(rid)
            except Exception as e:
                log.debug("image %s not removed: %r", rid, e)
                continue
            self.records.pop(rid, None)
            freed += r.size
            if freed >= amount:
                break
        return freed

    def _event(self, reason: str, msg: str):
        if self.recorder is not None and self.node_ref is not None:
            self.recorder.event(self.node_ref(), "Warning", reason, msg)

    async def garbage_collect(self) -> dict:
        """GarbageCollect: above the high threshold free down to the low one. A zero capacity
        (InvalidDiskCapacity) or a shortfall (FreeDiskSpaceFailed) is an event and an error."""
        cap, avail = await self.fs_stats()
        if avail > cap:
            log.warning("available %d is larger than capacity %d", avail, cap)
            avail = cap
        if cap == 0:
            self._event("InvalidDiskCapacity", "invalid capacity 0 on image filesystem")
            raise ImageGCError("invalid capacity 0 on image filesystem")
        usage = 100 - (avail * 100) // cap
        out = {"usage_percent": usage, "freed": 0}
        if usage >= self.high:
            amount = cap * (100 - self.low) // 100 - avail
            freed = await self.free_space(amount)
            out.update(freed=freed, wanted=amount)
            if freed < amount:
                msg = (f"failed to garbage collect required amount of images. Wanted to free {amount} bytes, "
                       f"but freed {freed} bytes")
                log.warning("image GC: %s", msg)
                self._event("FreeDiskSpaceFailed", msg)
                raise ImageGCError(msg)
        return out

    async def delete_unused(self) -> int:
        """DeleteUnusedImages: every image no container uses (eviction-driven reclaim)."""
        saved, self.min_age = self.min_age, 0.0
        try:
            return await self.free_space(1 << 62)
        finally:
            self.min_age = saved
