"""CronJob controller held to pkg/controller/cronjob's tests.

* cronjob_controller_test.go — TestSyncOne_RunOrNot :168, TestCleanupFinishedJobs_DeleteOrNot
  :373 and TestSyncOne_Status :609: their tables (100 cases) extracted by
  hack/extract_cronjob_cases.py into fixtures/cronjob_cases.json and replayed through
  controllers.apps.sync_one / cleanup_finished_jobs with the reference's fakes (fakeJobControl,
  fakeSJControl, fakePodControl from injection.go, record.FakeRecorder) re-expressed.
* utils_test.go — TestGetJobFromTemplate :33, TestGetParentUIDFromJob :91, TestGroupJobsByParent
  :151, TestGetRecentUnmetScheduleTimes :244 (all seven cases), transcribed.
"""
from __future__ import annotations

import copy
import json
import os

import pytest

from amdkube.api import meta as m
from amdkube.controllers import apps as CJ
from tests.conftest import run

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "cronjob_cases.json")))
T = FIX["times"]
NO_DEAD = -12345
ON_THE_HOUR = "0 * * * ?"


def ts(name_or_iso: str) -> float:
    return m.parse_time(T.get(name_or_iso, name_or_iso))


# ------------------------------------------------------------------ fakes (injection.go)
class FakeJobControl:
    def __init__(self, job=None):
        self.job, self.jobs, self.deleted, self.updated, self.err = job, [], [], [], None

    async def create_job(self, ns, job):
        if self.err:
            raise self.err
        job = copy.deepcopy(job)
        self.jobs.append(copy.deepcopy(job))
        job["metadata"]["uid"] = "test-uid"
        return job

    async def get_job(self, ns, name):
        if self.err:
            raise self.err
        return self.job

    async def update_job(self, ns, job):
        if self.err:
            raise self.err
        self.updated.append(m.name_of(job))
        return job

    async def delete_job(self, ns, name):
        if self.err:
            raise self.err
        self.deleted.append(name)


class FakeSJControl:
    def __init__(self):
        self.updates = []

    async def update_status(self, sj):
        self.updates.append(copy.deepcopy(sj))
        return copy.deepcopy(sj)


class FakePodControl:
    def __init__(self):
        self.err = None

    async def list_pods(self, ns, selector):
        if self.err:
            raise self.err
        return []

    async def delete_pod(self, ns, name):
        pass


class FakeRecorder:
    def __init__(self):
        self.events = []

    def event(self, obj, etype, reason, msg):
        self.events.append(f"{etype} {reason} {msg}")


def cron_job() -> dict:
    """cronJob(): the fixture every case starts from."""
    return {"apiVersion": "batch/v1beta1", "kind": "CronJob",
            "metadata": {"name": "mycronjob", "namespace": "snazzycats", "uid": "1a2b3c",
                         "creationTimestamp": T["justBeforeTheHour"]},
            "spec": {"schedule": "* * * * ?", "concurrencyPolicy": "Allow",
                     "jobTemplate": {"metadata": {"labels": {"a": "b"}, "annotations": {"x": "y"}},
                                     "spec": job_spec()}},
            "status": {}}


def job_spec() -> dict:
    return {"parallelism": 1, "completions": 1,
            "template": {"metadata": {"labels": {"foo": "bar"}}, "spec": {"containers": [{"image": "foo/bar"}]}}}


def new_job(uid: str) -> dict:
    return {"apiVersion": "batch/v1", "kind": "Job",
            "metadata": {"uid": uid, "name": "foobar", "namespace": "default"}, "spec": job_spec()}


def configure(sj, c):
    sj["spec"]["concurrencyPolicy"] = c["concurrencyPolicy"]
    sj["spec"]["suspend"] = c["suspend"]
    sj["spec"]["schedule"] = c["schedule"]
    if c["deadline"] != NO_DEAD:
        sj["spec"]["startingDeadlineSeconds"] = c["deadline"]


# ------------------------------------------------------------------ TestSyncOne_RunOrNot
RUN_OR_NOT = FIX["TestSyncOne_RunOrNot"]["cases"]


@pytest.mark.parametrize("c", RUN_OR_NOT, ids=[c["name"] for c in RUN_OR_NOT])
def test_sync_one_run_or_not(c):
    sj = cron_job()
    configure(sj, c)
    job, js = None, []
    if c["ranPreviously"]:
        sj["metadata"]["creationTimestamp"] = T["justBeforeThePriorHour"]
        sj["status"]["lastScheduleTime"] = T["justAfterThePriorHour"]
        job = CJ.get_job_from_template(sj, ts("justAfterThePriorHour"))
        job["metadata"]["uid"] = "1234"
        if c["stillActive"]:
            sj["status"]["active"] = [{"uid": "1234"}]
            js.append(job)
    jc, sjc, pc, rec = FakeJobControl(job), FakeSJControl(), FakePodControl(), FakeRecorder()
    run(CJ.sync_one(sj, js, ts(c["now"]), jc, sjc, pc, rec))
    assert len(jc.jobs) == (1 if c["expectCreate"] else 0)
    for j in jc.jobs:
        ref = m.controller_ref(j)
        assert (ref["apiVersion"], ref["kind"], ref["name"], ref["uid"], ref["controller"]) == \
            ("batch/v1beta1", "CronJob", "mycronjob", "1a2b3c", True)
    assert len(jc.deleted) == (1 if c["expectDelete"] else 0)
    expect_updates = 1 + (1 if c["expectCreate"] else 0)
    expected_events = (1 if c["expectCreate"] else 0) + (1 if c["expectDelete"] else 0) + c["expectedWarnings"]
    assert len(rec.events) == expected_events, rec.events
    assert sum(1 for e in rec.events if e.startswith("Warning")) == c["expectedWarnings"]
    assert len(sjc.updates[expect_updates - 1]["status"].get("active") or []) == c["expectActive"]


# ------------------------------------------------------------------ TestCleanupFinishedJobs_DeleteOrNot
CLEANUP = FIX["TestCleanupFinishedJobs_DeleteOrNot"]["cases"]


@pytest.mark.parametrize("c", CLEANUP, ids=[c["name"] for c in CLEANUP])
def test_cleanup_finished_jobs_delete_or_not(c):
    sj = cron_job()
    sj["spec"].update(concurrencyPolicy="Forbid", suspend=False, schedule=ON_THE_HOUR)
    for k in ("successfulJobsHistoryLimit", "failedJobsHistoryLimit"):
        if c[k] is not None:
            sj["spec"][k] = c[k]
    specs = [dict(zip(("StartTime", "IsFinished", "IsSuccessful", "ExpectDelete", "IsStillInActiveList"), s))
             for s in c["jobSpecs"]]
    if specs:
        sj["metadata"]["creationTimestamp"] = specs[0]["StartTime"]
        sj["status"]["lastScheduleTime"] = specs[-1]["StartTime"]
    js, to_delete, job = [], set(), None
    sj["status"]["active"] = []
    for i, s in enumerate(specs):
        job = CJ.get_job_from_template(sj, m.parse_time(s["StartTime"]))
        job["metadata"]["uid"] = str(i)
        if s["IsFinished"]:
            job["status"] = {"conditions": [{"type": "Complete" if s["IsSuccessful"] else "Failed", "status": "True"}]}
            if s["IsStillInActiveList"]:
                sj["status"]["active"].append({"uid": str(i)})
        else:
            assert not (s["IsSuccessful"] or s["IsStillInActiveList"]), "test setup error"
            sj["status"]["active"].append({"uid": str(i)})
        js.append(job)
        if s["ExpectDelete"]:
            to_delete.add(m.name_of(job))
    jc, pc, sjc, rec = FakeJobControl(job), FakePodControl(), FakeSJControl(), FakeRecorder()
    if c["name"] == "failed list pod err":
        pc.err = RuntimeError("fakePodControl err")
    run(CJ.cleanup_finished_jobs(sj, js, jc, sjc, pc, rec))
    assert set(jc.deleted) == to_delete and len(jc.deleted) == len(to_delete)
    expected_events = len(specs) if c["name"] == "failed list pod err" else len(to_delete)
    assert len(rec.events) == expected_events, rec.events
    active = len(sjc.updates[-1]["status"].get("active") or []) if sjc.updates else 0
    assert active == c["expectActive"]


# ------------------------------------------------------------------ TestSyncOne_Status
STATUS = FIX["TestSyncOne_Status"]["cases"]


def _ref(job):
    return {"kind": "Job", "namespace": m.namespace_of(job), "name": m.name_of(job), "uid": m.uid_of(job),
            "apiVersion": "batch/v1"}


@pytest.mark.parametrize("c", STATUS, ids=[c["name"] for c in STATUS])
def test_sync_one_status(c):
    finished = new_job("1")
    finished["status"] = {"conditions": [{"type": "Complete", "status": "True"}]}
    unexpected, missing = new_job("2"), new_job("3")
    sj = cron_job()
    configure(sj, c)
    if c["ranPreviously"]:
        sj["metadata"]["creationTimestamp"] = T["justBeforeThePriorHour"]
        sj["status"]["lastScheduleTime"] = T["justAfterThePriorHour"]
    else:
        assert not (c["hasFinishedJob"] or c["hasUnexpectedJob"] or c["hasMissingJob"]), "test setup error"
    jobs = []
    if c["hasFinishedJob"]:
        sj["status"]["active"] = [_ref(finished)]
        jobs.append(finished)
    if c["hasUnexpectedJob"]:
        jobs.append(unexpected)
    if c["hasMissingJob"]:
        sj["status"].setdefault("active", []).append(_ref(missing))
    if c["beingDeleted"]:
        sj["metadata"]["deletionTimestamp"] = c["now"]
    jc, sjc, pc, rec = FakeJobControl(), FakeSJControl(), FakePodControl(), FakeRecorder()
    run(CJ.sync_one(sj, jobs, ts(c["now"]), jc, sjc, pc, rec))
    expect_updates = 1 + (1 if c["expectCreate"] else 0)
    expected_events = sum(1 for k in ("expectCreate", "expectDelete", "hasFinishedJob", "hasUnexpectedJob", "hasMissingJob")
                          if c[k])
    assert len(rec.events) == expected_events, rec.events
    assert len(sjc.updates) == expect_updates
    first = sjc.updates[0]
    for flag, job in (("hasFinishedJob", finished), ("hasUnexpectedJob", unexpected), ("hasMissingJob", missing)):
        if c[flag]:
            assert not CJ.in_active_list(first, m.uid_of(job))
    if c["expectCreate"]:
        assert m.parse_time(sjc.updates[1]["status"]["lastScheduleTime"]) == ts("topOfTheHour")


# ------------------------------------------------------------------ utils_test.go
def test_get_job_from_template():
    sj = cron_job()
    sj["spec"]["jobTemplate"]["spec"] = {"activeDeadlineSeconds": 1, "manualSelector": False,
                                         "template": {"metadata": {"labels": {"foo": "bar"}},
                                                      "spec": {"containers": [{"image": "foo/bar"}]}}}
    job = CJ.get_job_from_template(sj, 0)
    assert m.name_of(job).startswith("mycronjob-")
    assert len(job["metadata"]["labels"]) == 1 and len(job["metadata"]["annotations"]) == 1
    assert m.name_of(CJ.get_job_from_template(sj, ts("topOfTheHour"))) == "mycronjob-1463652000"   # getTimeHash: Unix seconds


def test_get_parent_uid_from_job():
    j = new_job("x")
    j["status"] = {"conditions": [{"type": "Complete", "status": "True"}]}
    assert CJ.get_parent_uid_from_job(j) == ("", False)
    j["metadata"]["ownerReferences"] = [{"kind": "CronJob", "uid": "5ef034e0-1890-11e6-8935-42010af0003e", "controller": True}]
    assert CJ.get_parent_uid_from_job(j) == ("5ef034e0-1890-11e6-8935-42010af0003e", True)


def test_group_jobs_by_parent():
    uid1, uid2, uid3 = "11111111-1111-1111-1111-111111111111", "22222222-2222-2222-2222-222222222222", \
        "33333333-3333-3333-3333-333333333333"

    def job(name, ns, uid):
        j = {"metadata": {"name": name, "namespace": ns}}
        if uid:
            j["metadata"]["ownerReferences"] = [{"kind": "CronJob", "uid": uid, "controller": True}]
        return j
    assert CJ.group_jobs_by_parent([]) == {}
    got = CJ.group_jobs_by_parent([job("a", "x", uid1)])
    assert {k: [m.name_of(j) for j in v] for k, v in got.items()} == {uid1: ["a"]}
    js = [job("a", "x", uid1), job("b", "x", uid2), job("c", "x", uid1), job("d", "x", None), job("a", "y", uid3),
          job("b", "y", uid3), job("d", "y", None)]
    got = CJ.group_jobs_by_parent(js)
    assert {k: [(m.namespace_of(j), m.name_of(j)) for j in v] for k, v in got.items()} == \
        {uid1: [("x", "a"), ("x", "c")], uid2: [("x", "b")], uid3: [("y", "a"), ("y", "b")]}


def test_get_recent_unmet_schedule_times():
    t1, t2 = ts("2016-05-19T10:00:00Z"), ts("2016-05-19T11:00:00Z")
    sj = {"metadata": {"name": "mycronjob", "namespace": "default", "uid": "1a2b3c"},
          "spec": {"schedule": ON_THE_HOUR, "concurrencyPolicy": "Allow", "jobTemplate": {}}, "status": {}}

    def at(created, last=None, deadline=None):
        s = copy.deepcopy(sj)
        s["metadata"]["creationTimestamp"] = m.format_time(created)
        if last is not None:
            s["status"]["lastScheduleTime"] = m.format_time(last)
        if deadline is not None:
            s["spec"]["startingDeadlineSeconds"] = deadline
        return s
    assert CJ.get_recent_unmet_schedule_times(at(t1 - 600), t1 - 420) == []                  # 1: none needed yet
    assert CJ.get_recent_unmet_schedule_times(at(t1 - 600), t1 + 2) == [t1]                  # 2: one needed
    assert CJ.get_recent_unmet_schedule_times(at(t1 - 600, t1), t1 + 120) == []              # 3: known, none needed
    assert CJ.get_recent_unmet_schedule_times(at(t1 - 600, t1), t2 + 300) == [t2]            # 4: known, one needed
    assert CJ.get_recent_unmet_schedule_times(at(t1 - 7200, t1 - 3600), t2 + 300) == [t1, t2]   # 5: two needed
    with pytest.raises(ValueError):                                                          # 6: way ahead, no deadline
        CJ.get_recent_unmet_schedule_times(at(t1 - 7200, t1 - 3600), t2 + 10 * 86400)
    CJ.get_recent_unmet_schedule_times(at(t1 - 7200, t1 - 3600, deadline=7200), t2 + 10 * 86400)   # 7: short deadline


def test_remove_oldest_jobs_orders_by_start_time():
    jobs = []
    for name, start in (("c", "2016-05-19T03:00:00Z"), ("a", None), ("b", "2016-05-19T01:00:00Z"),
                        ("d", "2016-05-19T01:00:00Z")):
        j = new_job(name)
        j["metadata"]["name"] = name
        if start:
            j["status"] = {"startTime": start}
        jobs.append(j)
    jc = FakeJobControl()
    run(CJ.remove_oldest_jobs(cron_job(), jobs, jc, FakePodControl(), 1, FakeRecorder()))
    assert jc.deleted == ["b", "d", "c"]          # started first; equal times by name; never-started last
