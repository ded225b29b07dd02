"""GPU-subset selection for the scheduler: native C++ (amdkube._native._topo, see
native/topo_core.h) with an identical pure-Python reference implementation.

`select(free, k, link, numa, all_free, parent) -> (chosen, cost)` and `score(...) -> [0, 10]`.
`parent` (optional) maps each device to its physical GPU when the node runs partitioned
MI355X GPUs (CPX/QPX/DPX compute partitions); fragmentation then scores whole-GPU retention.
The Python version exists for CPU-only environments and as the numerics oracle for the
native one (tests/test_topology.py checks they agree); on a GPU node the native module
is required (AMDKUBE_REQUIRE_NATIVE=1, set by bench/smoke) and a missing build fails loudly.
"""
from __future__ import annotations

import itertools
import logging
import math
import os

log = logging.getLogger("amdkube.ops.topology")

W_NUMA, W_LINK, W_FRAG = 100.0, 10.0, 1.0
MAX_ENUM = 200000

try:
    from .._native import _topo as _native  # type: ignore
except ImportError as _e:  # pragma: no cover - exercised only without a build
    _native = None
    if os.environ.get("AMDKUBE_REQUIRE_NATIVE") == "1":
        raise ImportError(f"amdkube native topology module not built (run native/build.py): {_e}")

NATIVE = _native is not None


def _norm(link):
    mx = max((v for r in link for v in r), default=0.0)
    return [[(v / mx if mx > 0 else 0.0) for v in r] for r in link]


def _min_groups(free, numa, k):
    cnt = {}
    for d in free:
        cnt[numa[d]] = cnt.get(numa[d], 0) + 1
    need, g = k, 0
    for c in sorted(cnt.values(), reverse=True):
        if need <= 0:
            break
        need -= c
        g += 1
    return max(g, 1 if k > 0 else 0)


def _parents(parent, n):
    """Dense parent ids + largest parent size (1 = unpartitioned), as topo::make does."""
    if not parent:
        return None, 1
    if len(parent) != n:
        raise ValueError("parent must have one entry per device")
    ids, sz = {}, {}
    dense = []
    for g in parent:
        dense.append(ids.setdefault(g, len(ids)))
        sz[g] = sz.get(g, 0) + 1
    psize = max(sz.values())
    return (dense, psize) if psize > 1 else (None, 1)


def _frag(all_free, numa, chosen, parent=None, psize=1):
    taken = set(chosen)
    rem = [d for d in all_free if d not in taken]
    total = len(rem)
    if total == 0:
        return 0.0
    per = {}
    for d in rem:
        per[numa[d]] = per.get(numa[d], 0) + 1
    q = sum(c * c for c in per.values())
    fg = 1.0 - q / float(total * total)
    if parent is not None:
        pp = {}
        for d in rem:
            pp[parent[d]] = pp.get(parent[d], 0) + 1
        qp = sum(c * c for c in pp.values())
        fpar = 1.0 - qp / float(total * min(total, psize))
        return 0.5 * fg + 0.5 * max(0.0, fpar)
    pairs = sum(c // 2 for c in per.values())     # 2-GPU gangs still placeable inside one NUMA domain
    fp = 1.0 - (2.0 * pairs) / total
    return 0.75 * fg + 0.25 * max(0.0, fp)


def _cost(s, link, numa, all_free, mg, parent=None, psize=1):
    groups = len({numa[d] for d in s})
    tot, n = 0.0, 0
    for a in range(len(s)):
        for b in range(a + 1, len(s)):
            tot += link[s[a]][s[b]]
            n += 1
    mean = tot / n if n else 0.0
    return W_NUMA * (groups - mg) + W_LINK * mean + W_FRAG * _frag(all_free, numa, s, parent, psize)


def py_select(free, k, link, numa, all_free=None, parent=None):
    all_free = list(all_free) if all_free else list(free)
    parent, psize = _parents(parent, len(numa))
    if k <= 0:
        return [], 0.0
    if k > len(free):
        return [], math.inf
    link = _norm(link)
    mg = _min_groups(free, numa, k)
    sf = sorted(free)
    best, bc = [], math.inf
    if math.comb(len(sf), k) <= MAX_ENUM:
        for s in itertools.combinations(sf, k):
            c = _cost(list(s), link, numa, all_free, mg, parent, psize)
            if c < bc - 1e-12:
                bc, best = c, list(s)
        return best, bc
    seeds, seen = [], set()
    for d in sf:  # partitions of one GPU are interchangeable seeds (topo_core.h)
        if parent is not None:
            if parent[d] in seen:
                continue
            seen.add(parent[d])
        seeds.append(d)
    for seed in seeds:
        s, used = [seed], {seed}
        while len(s) < k:
            pick, pc = None, math.inf
            for d in sf:
                if d in used:
                    continue
                c = _cost(s + [d], link, numa, all_free, mg, parent, psize)
                if c < pc - 1e-12:
                    pc, pick = c, d
            s.append(pick)
            used.add(pick)
        s.sort()
        c = _cost(s, link, numa, all_free, mg, parent, psize)
        if c < bc - 1e-12:
            bc, best = c, s
    return best, bc


def py_score(free, k, link, numa, all_free=None, parent=None):
    _, c = py_select(free, k, link, numa, all_free, parent)
    if not math.isfinite(c):
        return 0.0
    groups = len(set(numa))
    mx = W_NUMA * max(0, groups - 1) + W_LINK + W_FRAG
    return max(0.0, min(10.0, 10.0 * (1.0 - c / mx)))


def select(free, k, link, numa, all_free=None, parent=None):
    if _native is not None:
        return _native.select(list(free), int(k), link, list(numa), list(all_free or []), list(parent or []))
    return py_select(free, k, link, numa, all_free, parent)


def score(free, k, link, numa, all_free=None, parent=None):
    if _native is not None:
        return _native.score(list(free), int(k), link, list(numa), list(all_free or []), list(parent or []))
    return py_score(free, k, link, numa, all_free, parent)
