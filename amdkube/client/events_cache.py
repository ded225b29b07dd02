"""Event correlation: spam filtering, aggregation of similar events, counting of identical ones.

Reference: staging/src/k8s.io/client-go/tools/record/events_cache.go —
  * getEventKey / getSpamKey (:49-81);
  * EventSourceObjectSpamFilter (:83-131): a token bucket per (source, involved object), burst
    25, refilled at 1/300 per second, in an LRU of 4096;
  * EventAggregator (:133-265): events that differ only in their message are keyed by
    EventAggregatorByReasonFunc; once 10 distinct messages were seen within 600 s of each
    other the event is replaced by one carrying "(combined from similar events): <message>";
  * eventLogger (:267-356): an identical event (or aggregate) seen before gets the earlier
    name, firstTimestamp and count + 1, with the patch that updates the stored one;
  * EventCorrelator (:358-413): aggregate → observe → filter.

The clock is a callable returning seconds, so tests can step it like clock.IntervalClock.
"""
from __future__ import annotations

import collections
import time

MAX_LRU_CACHE_ENTRIES = 4096
DEFAULT_AGGREGATE_MAX_EVENTS = 10
DEFAULT_AGGREGATE_INTERVAL_SECONDS = 600
DEFAULT_SPAM_BURST = 25
DEFAULT_SPAM_QPS = 1.0 / 300.0


def _rfc3339(t: float) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


class LRU:
    def __init__(self, n: int):
        self.n = n
        self.d: collections.OrderedDict = collections.OrderedDict()

    def get(self, k):
        if k in self.d:
            self.d.move_to_end(k)
            return self.d[k]
        return None

    def add(self, k, v):
        self.d[k] = v
        self.d.move_to_end(k)
        while len(self.d) > self.n:
            self.d.popitem(last=False)

    def __len__(self):
        return len(self.d)


def _io(ev):
    return ev.get("involvedObject") or {}


def _src(ev):
    return ev.get("source") or {}


def event_key(ev: dict) -> str:
    io, src = _io(ev), _src(ev)
    return "".join(str(x or "") for x in (src.get("component"), src.get("host"), io.get("kind"), io.get("namespace"),
                                          io.get("name"), io.get("fieldPath"), io.get("uid"), io.get("apiVersion"),
                                          ev.get("type"), ev.get("reason"), ev.get("message")))


def spam_key(ev: dict) -> str:
    io, src = _io(ev), _src(ev)
    return "".join(str(x or "") for x in (src.get("component"), src.get("host"), io.get("kind"), io.get("namespace"),
                                          io.get("name"), io.get("uid"), io.get("apiVersion")))


def aggregate_by_reason(ev: dict) -> tuple[str, str]:
    """EventAggregatorByReasonFunc: (aggregate key, local key = the message)."""
    io, src = _io(ev), _src(ev)
    return "".join(str(x or "") for x in (src.get("component"), src.get("host"), io.get("kind"), io.get("namespace"),
                                          io.get("name"), io.get("uid"), io.get("apiVersion"), ev.get("type"),
                                          ev.get("reason"))), ev.get("message", "")


def aggregate_message(ev: dict) -> str:
    """EventAggregatorByReasonMessageFunc."""
    return "(combined from similar events): " + ev.get("message", "")


def default_event_filter(ev: dict) -> bool:
    return False


class SpamFilter:
    """EventSourceObjectSpamFilter: True means drop the event."""

    def __init__(self, size=MAX_LRU_CACHE_ENTRIES, burst=DEFAULT_SPAM_BURST, qps=DEFAULT_SPAM_QPS, clock=time.time):
        self.cache = LRU(size)
        self.burst, self.qps, self.clock = burst, qps, clock

    def filter(self, ev: dict) -> bool:
        key = spam_key(ev)
        now = self.clock()
        rec = self.cache.get(key)
        if rec is None:
            tokens, last = float(self.burst), now
        else:
            tokens, last = rec
            tokens = min(float(self.burst), tokens + (now - last) * self.qps)
        drop = tokens < 1.0
        if not drop:
            tokens -= 1.0
        self.cache.add(key, (tokens, now))
        return drop


class EventAggregator:
    def __init__(self, size=MAX_LRU_CACHE_ENTRIES, key_func=aggregate_by_reason, message_func=aggregate_message,
                 max_events=DEFAULT_AGGREGATE_MAX_EVENTS, max_interval=DEFAULT_AGGREGATE_INTERVAL_SECONDS, clock=time.time):
        self.cache = LRU(size)
        self.key_func, self.message_func = key_func, message_func
        self.max_events, self.max_interval, self.clock = max_events, max_interval, clock

    def aggregate(self, ev: dict) -> tuple[dict, str]:
        """EventAggregate: (the event to record, the key the logger counts it under)."""
        now = self.clock()
        ekey = event_key(ev)
        akey, lkey = self.key_func(ev)
        rec = self.cache.get(akey)
        if rec is None or now - rec[1] > self.max_interval:
            rec = (set(), 0.0)
        keys = rec[0]
        keys.add(lkey)
        self.cache.add(akey, (keys, now))
        if len(keys) < self.max_events:
            return ev, ekey
        keys.pop()          # PopAny: the set stays at the threshold
        io = _io(ev)
        ts = _rfc3339(now)
        agg = {"apiVersion": "v1", "kind": "Event",
               "metadata": {"name": f"{io.get('name', '')}.{int(now * 1e9):x}",
                            "namespace": (ev.get("metadata") or {}).get("namespace", "")},
               "count": 1, "firstTimestamp": ts, "lastTimestamp": ts, "involvedObject": io,
               "message": self.message_func(ev), "type": ev.get("type"), "reason": ev.get("reason"),
               "source": ev.get("source")}
        return agg, akey


class EventLogger:
    def __init__(self, size=MAX_LRU_CACHE_ENTRIES, clock=time.time):
        self.cache = LRU(size)
        self.clock = clock

    def observe(self, ev: dict, key: str) -> tuple[dict, dict | None]:
        """eventObserve: the event as it should be stored, and the patch when it updates an
        earlier one (count, lastTimestamp, message)."""
        ev = {**ev, "metadata": dict(ev.get("metadata") or {})}
        last = self.cache.get(key)
        patch = None
        if last is not None and last["count"] > 0:
            ev["metadata"]["name"] = last["name"]
            if last.get("resourceVersion"):
                ev["metadata"]["resourceVersion"] = last["resourceVersion"]
            ev["firstTimestamp"] = last["firstTimestamp"]
            ev["count"] = last["count"] + 1
            patch = {"count": ev["count"], "lastTimestamp": ev.get("lastTimestamp"), "message": ev.get("message")}
        self.cache.add(key, {"count": int(ev.get("count") or 1), "firstTimestamp": ev.get("firstTimestamp"),
                             "name": ev["metadata"].get("name"), "resourceVersion": ev["metadata"].get("resourceVersion")})
        return ev, patch

    def update_state(self, ev: dict):
        md = ev.get("metadata") or {}
        self.cache.add(event_key(ev), {"count": int(ev.get("count") or 1), "firstTimestamp": ev.get("firstTimestamp"),
                                       "name": md.get("name"), "resourceVersion": md.get("resourceVersion")})


class CorrelateResult:
    __slots__ = ("event", "patch", "skip")

    def __init__(self, event=None, patch=None, skip=False):
        self.event, self.patch, self.skip = event, patch, skip


class EventCorrelator:
    def __init__(self, clock=time.time, filter_func=None):
        self.spam = SpamFilter(clock=clock)
        self.filter_func = filter_func or self.spam.filter
        self.aggregator = EventAggregator(clock=clock)
        self.logger = EventLogger(clock=clock)

    def correlate(self, ev: dict) -> CorrelateResult:
        if ev is None:
            raise ValueError("event is nil")
        agg, key = self.aggregator.aggregate(ev)
        observed, patch = self.logger.observe(agg, key)
        if self.filter_func(observed):
            return CorrelateResult(skip=True)
        return CorrelateResult(observed, patch)

    def update_state(self, ev: dict):
        self.logger.update_state(ev)
