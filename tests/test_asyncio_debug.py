"""The control plane under asyncio debug mode (PYTHONASYNCIODEBUG in tests, the
asyncio counterpart of the reference's `-race` runs): a full pod lifecycle — GPU pod admitted
with devices, running, a crash restart, deletion — through apiserver, scheduler, controllers,
kubelet, device plugin and rocshim must leave no coroutine un-awaited, no task exception
unretrieved and no callback raising into the loop's exception handler."""
import asyncio
import logging
import warnings

from amdkube.localcluster import LocalCluster, wait_pod


class _Capture(logging.Handler):
    def __init__(self):
        super().__init__(logging.WARNING)
        self.records = []

    def emit(self, record):
        self.records.append(record.getMessage())


def test_pod_lifecycle_clean_under_asyncio_debug():
    cap = _Capture()
    logging.getLogger("asyncio").addHandler(cap)
    loop_errors = []

    async def go():
        loop = asyncio.get_running_loop()
        loop.set_debug(True)
        loop.slow_callback_duration = 10.0           # report misuse, not slowness of a loaded CI box
        loop.set_exception_handler(lambda lp, ctx: loop_errors.append(ctx.get("message", "")) or lp.default_exception_handler(ctx))
        async with LocalCluster(gpus="fake", n_gpus=2, relist_period=0.2) as lc:
            await lc.wait_gpus(2)
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "g"}, "spec": {
                "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "30"],
                                "resources": {"limits": {"amd.com/gpu": "1"}}}]}}, "default")
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "crash"}, "spec": {
                "restartPolicy": "OnFailure", "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", "exit 1"]}]}},
                           "default")
            p = await wait_pod(c, "default", "g", timeout=30)
            assert p["spec"]["extendedResources"][0]["assigned"]
            for _ in range(100):
                cr = await c.get("pods", "crash", "default")
                if any((cs.get("restartCount") or 0) >= 1 for cs in (cr.get("status") or {}).get("containerStatuses") or []):
                    break
                await asyncio.sleep(0.1)
            for name in ("g", "crash"):
                await c.delete("pods", name, "default", grace=0)
            for _ in range(100):
                if not (await c.list("pods", "default"))[0]:
                    break
                await asyncio.sleep(0.1)
        await asyncio.sleep(0.2)

    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        asyncio.run(asyncio.wait_for(go(), 90), debug=True)
    logging.getLogger("asyncio").removeHandler(cap)
    never_awaited = [str(w.message) for w in caught if "was never awaited" in str(w.message)]
    assert not never_awaited, never_awaited
    bad = [r for r in cap.records if "never retrieved" in r or "was never awaited" in r or "Exception in callback" in r]
    assert not bad, bad
    assert not [e for e in loop_errors if "never retrieved" in e or "Exception in callback" in e], loop_errors
