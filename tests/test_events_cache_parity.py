"""Event correlation held to client-go tools/record/events_cache_test.go, transcribed:
TestDefaultEventFilterFunc (:131), TestEventAggregatorByReasonFunc (:139),
TestEventAggregatorByReasonMessageFunc (:160), TestEventCorrelator (:170, all nine scenarios
with clock.IntervalClock stepping), plus the recorder's sink behaviour from event_test.go
(TestEventf's counting into a patch, TestUpdateExpiredEvent: a repeat whose stored event is
gone is created again) through a real apiserver."""
import copy

import pytest

from amdkube.client import events_cache as ec
from tests.conftest import run


def ref(kind, name, ns):
    return {"kind": kind, "name": name, "namespace": ns, "uid": "C934D34AFB20242", "apiVersion": "version",
            "fieldPath": "spec.containers{mycontainer}"}


def make_event(reason, message, io):
    return {"reason": reason, "message": message, "involvedObject": copy.deepcopy(io),
            "source": {"component": "kubelet", "host": "kublet.node1"}, "count": 1, "type": "Normal", "metadata": {}}


def test_default_event_filter_func():
    assert ec.default_event_filter(make_event("end-of-world", "it was fun", ref("Pod", "pod1", "other"))) is False


def test_event_aggregator_by_reason_func():
    e1 = make_event("end-of-world", "it was fun", ref("Pod", "pod1", "other"))
    e2 = make_event("end-of-world", "it was awful", ref("Pod", "pod1", "other"))
    e3 = make_event("nevermind", "it was a bug", ref("Pod", "pod1", "other"))
    (a1, l1), (a2, l2), (a3, _) = ec.aggregate_by_reason(e1), ec.aggregate_by_reason(e2), ec.aggregate_by_reason(e3)
    assert a1 == a2 and l1 != l2 and a1 != a3


def test_event_aggregator_by_reason_message_func():
    assert ec.aggregate_message(make_event("x", "it was fun", ref("Pod", "pod1", "other"))).startswith(
        "(combined from similar events): ")


class IntervalClock:
    """clock.IntervalClock: every reading advances by the interval."""

    def __init__(self, start, step):
        self.t, self.step = start, step

    def __call__(self):
        self.t += self.step
        return self.t


FIRST = make_event("first", "i am first", ref("Pod", "my-pod", "my-ns"))
DUP = make_event("duplicate", "me again", ref("Pod", "my-pod", "my-ns"))
UNIQUE = make_event("unique", "snowflake", ref("Pod", "my-pod", "my-ns"))
SIMILAR = make_event("similar", "similar message", ref("Pod", "my-pod", "my-ns"))
SIMILAR["involvedObject"]["fieldPath"] = "spec.containers{container1}"
AGGREGATE = make_event("similar", ec.aggregate_message(SIMILAR), SIMILAR["involvedObject"])
OTHER_CONTAINER = copy.deepcopy(SIMILAR)
OTHER_CONTAINER["involvedObject"]["fieldPath"] = "spec.containers{container2}"


def events(n, tpl):
    return [copy.deepcopy(tpl) for _ in range(n)]


def unique_events(n):
    out = []
    for i in range(n):
        out.append(make_event(f"reason-{chr(i)}", f"message-{chr(i)}", ref("Pod", f"pod-{chr(i)}", f"ns-{chr(i)}")))
    return out


def similar_events(n, tpl, prefix):
    out = events(n, tpl)
    for i, e in enumerate(out):
        e["message"] = f"{prefix}-{chr(i)}-{e['message']}"
    return out


MAXE, BURST, INTERVAL = ec.DEFAULT_AGGREGATE_MAX_EVENTS, ec.DEFAULT_SPAM_BURST, ec.DEFAULT_AGGREGATE_INTERVAL_SECONDS
SCENARIOS = {
    "create-a-single-event": ([], FIRST, (FIRST, 1), 5, False),
    "the-same-event-should-just-count": (events(1, DUP), DUP, (DUP, 2), 5, False),
    "the-same-event-should-just-count-even-if-more-than-aggregate": (events(MAXE, DUP), DUP, (DUP, MAXE + 1), 30, False),
    "the-same-event-is-spam-if-happens-too-frequently": (events(BURST + 1, DUP), DUP, None, 1, True),
    "create-many-unique-events": (unique_events(30), UNIQUE, (UNIQUE, 1), 5, False),
    "similar-events-should-aggregate-event": (similar_events(MAXE - 1, SIMILAR, SIMILAR["message"]), SIMILAR,
                                              (AGGREGATE, 1), 5, False),
    "similar-events-many-times-should-count-the-aggregate": (similar_events(MAXE, SIMILAR, SIMILAR["message"]), SIMILAR,
                                                             (AGGREGATE, 2), 5, False),
    "events-from-different-containers-do-not-aggregate": (events(1, OTHER_CONTAINER), SIMILAR, (SIMILAR, 1), 5, False),
    "similar-events-whose-interval-is-greater-than-aggregate-interval-do-not-aggregate": (
        similar_events(MAXE - 1, SIMILAR, SIMILAR["message"]), SIMILAR, (SIMILAR, 1), INTERVAL, False),
}


@pytest.mark.parametrize("name", list(SCENARIOS))
def test_event_correlator(name):
    previous, new, expected, interval, skip = SCENARIOS[name]
    clock = IntervalClock(1_700_000_000.0, interval)
    c = ec.EventCorrelator(clock=clock)
    for e in copy.deepcopy(previous):
        now = ec._rfc3339(clock())
        e["firstTimestamp"] = e["lastTimestamp"] = now
        res = c.correlate(e)
        if not res.skip:
            stored = copy.deepcopy(res.event)
            stored["metadata"].setdefault("name", "stored")
            c.update_state(stored)
    new = copy.deepcopy(new)
    new["firstTimestamp"] = new["lastTimestamp"] = ec._rfc3339(clock())
    res = c.correlate(new)
    assert res.skip is skip
    if skip:
        return
    exp, count = expected
    got = res.event
    assert got["count"] == count
    assert got["message"] == exp["message"] and got["reason"] == exp["reason"]
    assert got["involvedObject"] == exp["involvedObject"] and got["source"] == exp["source"]
    if count > 1:
        assert got["firstTimestamp"] != got["lastTimestamp"] and res.patch["count"] == count
    else:
        assert got["firstTimestamp"] == got["lastTimestamp"]


def test_recorder_counts_repeats_into_one_event_and_recreates_an_expired_one():
    from amdkube.apiserver import APIServer
    from amdkube.client import Client
    from amdkube.client.record import EventRecorder

    async def go():
        srv = await APIServer().start()
        c = Client(srv.url)
        t = [1_700_000_000.0]
        rec = EventRecorder(c, "kubelet", "node1", clock=lambda: t[0])
        try:
            for i in range(3):
                t[0] += 1
                await rec.record(rec.make_event({"kind": "Pod", "namespace": "default", "name": "p", "uid": "u1",
                                                 "apiVersion": "v1"}, "Warning", "BackOff", "Back-off restarting", t[0]))
            evs, _ = await c.list("events", "default")
            assert len(evs) == 1 and evs[0]["count"] == 3 and evs[0]["firstTimestamp"] != evs[0]["lastTimestamp"]
            await c.delete("events", evs[0]["metadata"]["name"], "default")
            t[0] += 1
            await rec.record(rec.make_event({"kind": "Pod", "namespace": "default", "name": "p", "uid": "u1",
                                             "apiVersion": "v1"}, "Warning", "BackOff", "Back-off restarting", t[0]))
            evs, _ = await c.list("events", "default")
            assert len(evs) == 1 and evs[0]["count"] == 4      # TestUpdateExpiredEvent: created again, count kept
            # ten different messages of one reason become one combined event
            for i in range(12):
                t[0] += 1
                await rec.record(rec.make_event({"kind": "Pod", "namespace": "default", "name": "p", "uid": "u1",
                                                 "apiVersion": "v1"}, "Normal", "Pulling", f"pulling image {i}", t[0]))
            evs, _ = await c.list("events", "default")
            combined = [e for e in evs if e["message"].startswith("(combined from similar events)")]
            assert len(combined) == 1 and combined[0]["count"] == 3
            assert len([e for e in evs if e["reason"] == "Pulling"]) == 10
        finally:
            await c.close()
            await srv.stop()
    run(go())
