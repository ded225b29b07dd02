"""Job controller at reference parity.

* TestControllerSyncJob and TestSyncJobPastDeadline of pkg/controller/job/job_controller_test.go,
  extracted by hack/extract_job_cases.py into tests/fixtures/job_cases.json, replayed against
  amdkube.controllers.job.sync_job with the reference's FakePodControl semantics
  (controller_utils.go: CreateLimit, Err — a create is recorded before the error; a delete too).
* A GPU Job past its activeDeadlineSeconds fails with DeadlineExceeded in a LocalCluster and its
  pod's amd.com/gpu is free again; a work-queue Job (completions unset); back-off timing.
"""
from __future__ import annotations

import asyncio
import json
import os
import time

import pytest

from amdkube.api import meta as m
from amdkube.controllers.job import DEFAULT_JOB_BACKOFF, MAX_JOB_BACKOFF, NewFailure, sync_job
from tests.conftest import run

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "job_cases.json")))


class FakePodControl:
    def __init__(self, err=None, limit=0):
        self.err, self.limit = err, limit
        self.templates, self.deleted, self.create_calls = [], [], 0

    async def create(self, job):
        self.create_calls += 1
        if self.limit and self.create_calls > self.limit:
            raise RuntimeError(f"Not creating pod, limit {self.limit} already reached")
        self.templates.append(job["spec"]["template"])
        if self.err:
            raise RuntimeError(self.err)

    async def delete(self, pod):
        self.deleted.append(m.name_of(pod))
        if self.err:
            raise RuntimeError(self.err)


def new_job(parallelism, completions, backoff_limit):
    """job_controller_test.go newJob: -1 leaves completions / parallelism unset."""
    spec = {"selector": {"matchLabels": {"foo": "bar"}}, "backoffLimit": backoff_limit,
            "template": {"metadata": {"labels": {"foo": "bar"}}, "spec": {"containers": [{"image": "foo/bar"}]}}}
    if completions >= 0:
        spec["completions"] = completions
    if parallelism >= 0:
        spec["parallelism"] = parallelism
    return {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "foobar", "namespace": "default", "uid": "u1"},
            "spec": spec, "status": {}}


def pods(job, n, phase, start=0):
    return [{"metadata": {"name": f"pod-{phase}-{start + i}", "namespace": "default",
                          "ownerReferences": [{"kind": "Job", "name": "foobar", "uid": "u1", "controller": True}]},
             "spec": {}, "status": {"phase": phase}} for i in range(n)]


@pytest.mark.parametrize("tc", FIX["TestControllerSyncJob"], ids=lambda c: c["name"])
def test_controller_sync_job_table(tc):
    job = new_job(tc["parallelism"], tc["completions"], tc["backoffLimit"])
    if tc["deleting"]:
        job["metadata"]["deletionTimestamp"] = m.now_rfc3339()
    plist = (pods(job, tc["pendingPods"], "Pending") + pods(job, tc["activePods"], "Running")
             + pods(job, tc["succeededPods"], "Succeeded") + pods(job, tc["failedPods"], "Failed"))
    err_msg = (tc["podControllerError"] or {}).get("error")
    pc = FakePodControl(err_msg, tc["podLimit"])
    new, forget, err = run(sync_job(job, plist, pc))
    if err_msg:
        assert err is not None, tc["name"]
    elif tc["podLimit"] == 0 or pc.create_calls < tc["podLimit"]:
        assert err is None, (tc["name"], err)
    assert forget == tc["jobKeyForget"], tc["name"]
    assert len(pc.templates) == tc["expectedCreations"], tc["name"]
    assert len(pc.deleted) == tc["expectedDeletions"], tc["name"]
    st = new["status"]
    assert (st["active"], st["succeeded"], st["failed"]) == \
        (tc["expectedActive"], tc["expectedSucceeded"], tc["expectedFailed"]), tc["name"]
    assert st.get("startTime")
    if tc["expectedCondition"]:
        assert any(c["type"] == tc["expectedCondition"] and c.get("reason", "") == tc["expectedConditionReason"]
                   for c in st["conditions"]), (tc["name"], st.get("conditions"))
    if tc["podLimit"]:
        limit, p = 0, 0
        while limit <= tc["podLimit"]:            # slow start: 1 + 2 + 4 + … create calls at most
            limit += 1 << p
            p += 1
        assert pc.create_calls <= limit


@pytest.mark.parametrize("tc", FIX["TestSyncJobPastDeadline"], ids=lambda c: c["name"])
def test_sync_job_past_deadline_table(tc):
    job = new_job(tc["parallelism"], tc["completions"], tc["backoffLimit"])
    job["spec"]["activeDeadlineSeconds"] = tc["activeDeadlineSeconds"]
    now = time.time()
    job["status"]["startTime"] = m.format_time(int(now) - tc["startTime"])
    plist = (pods(job, tc["activePods"], "Running") + pods(job, tc["succeededPods"], "Succeeded")
             + pods(job, tc["failedPods"], "Failed"))
    pc = FakePodControl()
    new, forget, err = run(sync_job(job, plist, pc, now=now))
    assert err is None and forget == tc["expectedForgetKey"]
    assert not pc.templates and len(pc.deleted) == tc["expectedDeletions"]
    st = new["status"]
    assert (st["active"], st["succeeded"], st["failed"]) == \
        (tc["expectedActive"], tc["expectedSucceeded"], tc["expectedFailed"]), tc["name"]
    assert any(c["type"] == "Failed" and c["reason"] == tc["expectedConditionReason"] for c in st["conditions"])


def test_new_failure_returns_an_error_and_failed_count_never_drops():
    """A new failure is an error (the key backs off); a failed pod that was garbage-collected
    still counts."""
    job = new_job(1, 3, 6)
    new, forget, err = run(sync_job(job, pods(job, 1, "Failed"), FakePodControl()))
    assert isinstance(err, NewFailure) and forget is False and new["status"]["failed"] == 1
    again, _, err2 = run(sync_job(new, pods(job, 1, "Running", 5), FakePodControl()))
    assert err2 is None and again["status"]["failed"] == 1


def test_backoff_schedule():
    """getBackoff: 0 on the first failure, then 10 s doubling, capped at 6 min."""
    from amdkube.controllers.job import JobController

    class Mgr:
        client = None
    jc = JobController(Mgr())
    delays = []
    for _ in range(8):
        delays.append(jc._backoff("ns/j"))
        jc.queue.limiter.when("ns/j")
    assert delays == [0.0, DEFAULT_JOB_BACKOFF, 20.0, 40.0, 80.0, 160.0, 320.0, MAX_JOB_BACKOFF]


def test_gpu_job_past_its_deadline_frees_the_gpu():
    """A GPU Job whose pod outlives activeDeadlineSeconds: the Job is Failed (DeadlineExceeded),
    its pod is deleted, and all 8 GPUs can be claimed again."""
    from amdkube.localcluster import LocalCluster, wait_pod

    async def go():
        async with LocalCluster(gpus="fake", relist_period=0.2) as lc:
            c = lc.client
            await lc.wait_gpus(8)
            job = await c.create({"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "train", "namespace": "default"},
                                  "spec": {"activeDeadlineSeconds": 2, "template": {"spec": {
                                      "restartPolicy": "Never", "containers": [{
                                          "name": "c", "image": "busybox", "command": ["sh", "-c", "sleep 60"],
                                          "resources": {"limits": {"amd.com/gpu": "8"}}}]}}}}, "default")
            assert job["spec"]["selector"]["matchLabels"]["controller-uid"] == job["metadata"]["uid"]
            deadline = time.time() + 30
            while time.time() < deadline:
                j = await c.get("jobs.batch", "train", "default")
                conds = (j.get("status") or {}).get("conditions") or []
                if any(x["type"] == "Failed" for x in conds):
                    break
                await asyncio.sleep(0.2)
            else:
                raise AssertionError("the Job never failed")
            assert conds[-1]["reason"] == "DeadlineExceeded" and j["status"]["active"] == 0
            # the 8-GPU pod is gone, so another 8-GPU pod schedules and runs
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "next", "namespace": "default"},
                            "spec": {"restartPolicy": "Never", "containers": [{
                                "name": "c", "image": "busybox", "command": ["sh", "-c", "true"],
                                "resources": {"limits": {"amd.com/gpu": "8"}}}]}})
            p = await wait_pod(c, "default", "next", ("Succeeded",), 30)
            assert len(p["spec"]["extendedResources"][0]["assigned"]) == 8
    run(go(), 90)


def test_work_queue_job_completes_after_first_success():
    """completions unset (parallelism 2): pods run until one succeeds, the Job completes when
    none is active."""
    from amdkube.localcluster import LocalCluster

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            job = await c.create({"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "wq", "namespace": "default"},
                                  "spec": {"parallelism": 2, "template": {"spec": {
                                      "restartPolicy": "Never", "containers": [{
                                          "name": "c", "image": "busybox", "command": ["sh", "-c", "true"]}]}}}}, "default")
            assert "completions" not in job["spec"] and job["spec"]["parallelism"] == 2
            deadline = time.time() + 30
            while time.time() < deadline:
                j = await c.get("jobs.batch", "wq", "default")
                if any(x["type"] == "Complete" for x in (j.get("status") or {}).get("conditions") or []):
                    break
                await asyncio.sleep(0.2)
            else:
                raise AssertionError(f"work-queue Job never completed: {j.get('status')}")
            assert j["status"]["succeeded"] >= 1 and j["status"]["active"] == 0
    run(go(), 60)
