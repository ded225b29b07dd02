"""/debug/pprof equivalents for asyncio components.

Reference exposes /debug/pprof/{profile,...} on the apiserver (routes/profiling.go:26-35),
kubelet and scheduler (--profiling). Here: `/debug/pprof/profile?seconds=N` runs cProfile
over the event-loop thread for N seconds and returns pstats text; `/debug/pprof/goroutine`
dumps the live asyncio tasks with their stacks.
"""
from __future__ import annotations

import asyncio
import cProfile
import io
import pstats

from aiohttp import web


async def profile_handler(request: web.Request) -> web.Response:
    secs = min(float(request.query.get("seconds", "5")), 60.0)
    pr = cProfile.Profile()
    pr.enable()
    try:
        await asyncio.sleep(secs)
    finally:
        pr.disable()
    out = io.StringIO()
    sort = request.query.get("sort", "cumulative")
    pstats.Stats(pr, stream=out).sort_stats(sort if sort in ("cumulative", "tottime", "ncalls") else "cumulative").print_stats(
        int(request.query.get("lines", "60")))
    return web.Response(text=out.getvalue())


async def tasks_handler(request: web.Request) -> web.Response:
    out = io.StringIO()
    tasks = asyncio.all_tasks()
    out.write(f"{len(tasks)} tasks\n\n")
    for t in tasks:
        out.write(f"{t.get_name()}: {t!r}\n")
        t.print_stack(limit=8, file=out)
        out.write("\n")
    return web.Response(text=out.getvalue())


def add_routes(app: web.Application):
    app.router.add_get("/debug/pprof/profile", profile_handler)
    app.router.add_get("/debug/pprof/goroutine", tasks_handler)
    app.router.add_get("/debug/pprof/", tasks_handler)
