

async def cancel_and_wait(tasks, timeout: float = 5.0):
    """Cancel background tasks and wait until they have finished, so a component's stop() leaves
    nothing pending on the loop ("Task was destroyed but it is pending" at interpreter exit)."""
    import asyncio
    tasks = [t for t in tasks if t is not None and not t.done()]
    for t in tasks:
        t.cancel()
    if tasks:
        await asyncio.wait(tasks, timeout=timeout)


async def wait_event(ev, timeout: float) -> bool:
    """`await asyncio.wait_for(ev.wait(), timeout)` without its Python 3.10 race: when the event
    fires at the moment the waiting task is cancelled, wait_for returns normally and the
    cancellation is lost, so a periodic loop never stops. asyncio.wait keeps the cancellation.
    True when the event was set, False on timeout."""
    import asyncio
    if ev.is_set():
        return True
    t = asyncio.ensure_future(ev.wait())
    try:
        done, _ = await asyncio.wait({t}, timeout=timeout)
        return bool(done)
    finally:
        if not t.done():
            t.cancel()
