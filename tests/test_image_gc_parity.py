"""Image garbage collection held to pkg/kubelet/images/image_gc_manager_test.go.

Every test of that file: the detectImages cases (:90-:239), freeSpace / DeleteUnusedImages (:241-:353),
GarbageCollect (:355-:418), the minimum-age case (:420) and TestValidateImageGCPolicy (:468). The fake
runtime mirrors containertest.FakeRuntime: images `image-<i>` and containers whose ImageID is the
image's ID; the image filesystem stats are injected as the reference's mock stats provider is.
"""
from __future__ import annotations

from types import SimpleNamespace as NS

import pytest

from amdkube.kubelet.images import ImageGCError, ImageGCManager
from tests.conftest import run


def image(i, size):
    return NS(id=f"image-{i}", size=size, repo_tags=[])


def container(i, named=True):
    return NS(image_ref=f"image-{i}", image=NS(image=f"image-{i}-name" if named else ""))


class FakeRuntime:
    def __init__(self, images=(), containers=()):
        self.images, self.containers = list(images), list(containers)

    async def list_images(self):
        return list(self.images)

    async def list_containers(self):
        return list(self.containers)

    async def remove_image(self, ref):
        self.images = [i for i in self.images if i.id != ref]


class Clock:
    def __init__(self, t=1000.0):
        self.t = t

    def __call__(self):
        return self.t


def manager(rt, high=90, low=80, min_age=0.0, fs=None):
    clock, events = Clock(), []
    gc = ImageGCManager(rt, high, low, min_age, clock=clock,
                        recorder=NS(event=lambda obj, typ, reason, msg: events.append((reason, msg))), node_ref=lambda: {})
    if fs is not None:
        async def fs_stats():
            if isinstance(fs, Exception):
                raise fs
            return fs
        gc.fs_stats = fs_stats
    return gc, clock, events


def test_detect_images_initial_detect():
    rt = FakeRuntime([image(0, 1024), image(1, 2048), image(2, 2048)], [container(1, named=False), container(2)])
    gc, clock, _ = manager(rt)
    run(gc.detect())
    assert len(gc.records) == 3
    assert (gc.records["image-0"].first_detected, gc.records["image-0"].last_used) == (clock.t, 0.0)
    assert gc.records["image-1"].last_used == clock.t          # a no-name image is matched by its ID
    assert gc.records["image-2"].last_used == clock.t


def test_detect_images_with_new_image():
    rt = FakeRuntime([image(0, 1024), image(1, 2048)], [container(1)])
    gc, clock, _ = manager(rt)
    t0 = clock.t
    run(gc.detect())
    rt.images = [image(0, 1024), image(1, 1024), image(2, 1024)]
    clock.t += 1
    run(gc.detect())
    assert len(gc.records) == 3
    assert (gc.records["image-0"].first_detected, gc.records["image-0"].last_used) == (t0, 0.0)
    assert gc.records["image-1"].first_detected == t0 and gc.records["image-1"].last_used == clock.t
    assert gc.records["image-2"].first_detected == clock.t and gc.records["image-2"].last_used == 0.0
    assert gc.records["image-1"].size == 1024


def test_detect_images_container_stopped():
    rt = FakeRuntime([image(0, 1024), image(1, 2048)], [container(1)])
    gc, clock, _ = manager(rt)
    run(gc.detect())
    used = gc.records["image-1"].last_used
    rt.containers = []
    clock.t += 5
    run(gc.detect())
    assert len(gc.records) == 2 and gc.records["image-0"].last_used == 0.0 and gc.records["image-1"].last_used == used


def test_detect_images_with_removed_images():
    rt = FakeRuntime([image(0, 1024), image(1, 2048)], [container(1)])
    gc, clock, _ = manager(rt)
    run(gc.detect())
    rt.images = []
    run(gc.detect())
    assert gc.records == {}


def test_free_space_images_in_use_containers_are_ignored():
    rt = FakeRuntime([image(0, 1024), image(1, 2048)], [container(1)])
    gc, _, _ = manager(rt)
    assert run(gc.free_space(2048)) == 1024 and len(rt.images) == 1


def test_delete_unused_images_remove_all_unused_images():
    rt = FakeRuntime([image(0, 1024), image(1, 2048), image(2, 2048)], [container(2)])
    gc, _, _ = manager(rt)
    assert run(gc.delete_unused()) == 3072 and len(rt.images) == 1


def test_free_space_remove_by_least_recently_used():
    rt = FakeRuntime([image(0, 1024), image(1, 2048)], [container(0), container(1)])
    gc, clock, _ = manager(rt)
    run(gc.detect())
    rt.containers = [container(1)]          # 1 more recently used than 0
    clock.t += 1
    run(gc.detect())
    rt.containers = []
    clock.t += 1
    run(gc.detect())
    assert len(gc.records) == 2
    assert run(gc.free_space(1024)) == 1024 and [i.id for i in rt.images] == ["image-1"]


def test_free_space_ties_broken_by_detected_time():
    rt = FakeRuntime([image(0, 1024)], [container(0)])
    gc, clock, _ = manager(rt)
    run(gc.detect())
    rt.images = [image(0, 1024), image(1, 2048)]
    clock.t += 1
    run(gc.detect())
    rt.containers = []
    clock.t += 1
    run(gc.detect())
    assert len(gc.records) == 2
    assert run(gc.free_space(1024)) == 2048 and [i.id for i in rt.images] == ["image-0"]


def test_garbage_collect_below_low_threshold():
    gc, _, _ = manager(FakeRuntime(), fs=(1000, 600))       # 40 % usage
    assert run(gc.garbage_collect())["freed"] == 0


def test_garbage_collect_stats_failure():
    gc, _, _ = manager(FakeRuntime(), fs=OSError("error"))
    with pytest.raises(OSError):
        run(gc.garbage_collect())


def test_garbage_collect_below_success():
    rt = FakeRuntime([image(0, 450)])
    gc, _, events = manager(rt, fs=(1000, 50))              # 95 % usage, most of it freed
    assert run(gc.garbage_collect())["freed"] == 450 and events == []


def test_garbage_collect_not_enough_freed():
    rt = FakeRuntime([image(0, 50)])
    gc, _, events = manager(rt, fs=(1000, 50))
    with pytest.raises(ImageGCError, match="Wanted to free 150 bytes, but freed 50 bytes"):
        run(gc.garbage_collect())
    assert [e[0] for e in events] == ["FreeDiskSpaceFailed"]


def test_garbage_collect_zero_capacity():
    """GarbageCollect's `invalid capacity 0 on image filesystem` (image_gc_manager.go:275)."""
    gc, _, events = manager(FakeRuntime(), fs=(0, 0))
    with pytest.raises(ImageGCError, match="invalid capacity 0"):
        run(gc.garbage_collect())
    assert [e[0] for e in events] == ["InvalidDiskCapacity"]


def test_garbage_collect_image_not_old_enough():
    rt = FakeRuntime([image(0, 1024), image(1, 2048)], [container(1)])
    gc, clock, _ = manager(rt, min_age=60.0)
    run(gc.detect())
    assert len(gc.records) == 2
    assert run(gc.free_space(1024)) == 0 and len(rt.images) == 2
    clock.t += 60.0
    assert run(gc.free_space(1024)) == 1024 and len(rt.images) == 1


@pytest.mark.parametrize("high,low,error", [
    (2, 1, None),
    (-1, 0, "invalid HighThresholdPercent -1, must be in range [0-100]"),
    (101, 0, "invalid HighThresholdPercent 101, must be in range [0-100]"),
    (0, -1, "invalid LowThresholdPercent -1, must be in range [0-100]"),
    (0, 101, "invalid LowThresholdPercent 101, must be in range [0-100]"),
    (1, 2, "LowThresholdPercent 2 can not be higher than HighThresholdPercent 1"),
])
def test_validate_image_gc_policy(high, low, error):
    if error is None:
        ImageGCManager(FakeRuntime(), high, low)
    else:
        with pytest.raises(ValueError) as e:
            ImageGCManager(FakeRuntime(), high, low)
        assert str(e.value) == error


def test_available_larger_than_capacity_is_clamped():
    """Not in the reference tests; image_gc_manager.go:269 clamps available to capacity."""
    gc, _, _ = manager(FakeRuntime(), fs=(1000, 1200))
    assert run(gc.garbage_collect())["usage_percent"] == 0
