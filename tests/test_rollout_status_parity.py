"""kubectl rollout status viewers against pkg/kubectl/rollout_status_test.go
(TestDeploymentStatusViewerStatus, TestDaemonSetStatusViewerStatus,
TestStatefulSetStatusViewerStatus, TestDaemonSetStatusViewerStatusWithWrongUpdateStrategyType)."""
from __future__ import annotations

import pytest

from amdkube.kubectl import rollout as R


def _d(gen, replicas, observed, rep, upd, avail, unavail=0):
    return {"metadata": {"name": "foo", "namespace": "bar", "generation": gen}, "spec": {"replicas": replicas},
            "status": {"observedGeneration": observed, "replicas": rep, "updatedReplicas": upd, "availableReplicas": avail,
                       "unavailableReplicas": unavail}}


@pytest.mark.parametrize("obj,msg,done", [
    (_d(0, 1, 1, 1, 0, 1), "Waiting for rollout to finish: 0 out of 1 new replicas have been updated...\n", False),
    (_d(1, 1, 1, 2, 1, 2), "Waiting for rollout to finish: 1 old replicas are pending termination...\n", False),
    (_d(1, 2, 1, 2, 2, 1, 1), "Waiting for rollout to finish: 1 of 2 updated replicas are available...\n", False),
    (_d(1, 2, 1, 2, 2, 2), 'deployment "foo" successfully rolled out\n', True),
    (_d(2, 2, 1, 2, 2, 2), "Waiting for deployment spec update to be observed...\n", False),
])
def test_deployment_status_viewer(obj, msg, done):
    assert R.deployment_status(obj, "foo") == (msg, done)


def test_deployment_status_viewer_deadline_and_revision():
    d = _d(1, 2, 1, 2, 1, 1)
    d["status"]["conditions"] = [{"type": "Progressing", "status": "False", "reason": "ProgressDeadlineExceeded"}]
    with pytest.raises(R.StatusError) as e:
        R.deployment_status(d, "foo")
    assert str(e.value) == 'deployment "foo" exceeded its progress deadline'
    d = _d(1, 2, 1, 2, 2, 2)
    d["metadata"]["annotations"] = {"deployment.kubernetes.io/revision": "3"}
    assert R.deployment_status(d, "foo", 3)[1]
    with pytest.raises(R.StatusError) as e:
        R.deployment_status(d, "foo", 2)
    assert str(e.value) == "desired revision (2) is different from the running revision (3)"


def _ds(gen, observed, upd, desired, avail, strategy="RollingUpdate"):
    return {"metadata": {"name": "foo", "namespace": "bar", "generation": gen}, "spec": {"updateStrategy": {"type": strategy}},
            "status": {"observedGeneration": observed, "updatedNumberScheduled": upd, "desiredNumberScheduled": desired,
                       "numberAvailable": avail}}


@pytest.mark.parametrize("obj,msg,done", [
    (_ds(0, 1, 0, 1, 0), "Waiting for rollout to finish: 0 out of 1 new pods have been updated...\n", False),
    (_ds(1, 1, 2, 2, 1), "Waiting for rollout to finish: 1 of 2 updated pods are available...\n", False),
    (_ds(1, 1, 2, 2, 2), 'daemon set "foo" successfully rolled out\n', True),
    (_ds(2, 1, 2, 2, 2), "Waiting for daemon set spec update to be observed...\n", False),
])
def test_daemonset_status_viewer(obj, msg, done):
    assert R.daemonset_status(obj, "foo") == (msg, done)


def test_daemonset_status_viewer_wrong_update_strategy():
    with pytest.raises(R.StatusError) as e:
        R.daemonset_status(_ds(1, 1, 2, 2, 2, "OnDelete"), "foo")
    assert str(e.value) == "Status is available only for RollingUpdate strategy type" and e.value.done


def _sts(gen, strategy, observed, replicas, ready, current, updated, cur_rev="", upd_rev=""):
    return {"metadata": {"name": "foo", "namespace": "bar", "generation": gen},
            "spec": {"replicas": replicas, "updateStrategy": strategy},
            "status": {"observedGeneration": observed, "replicas": replicas, "readyReplicas": ready, "currentReplicas": current,
                       "updatedReplicas": updated, "currentRevision": cur_rev, "updateRevision": upd_rev}}


RU = {"type": "RollingUpdate"}
PART2 = {"type": "RollingUpdate", "rollingUpdate": {"partition": 2}}


@pytest.mark.parametrize("name,obj,msg,done", [
    ("observed generation is behind", _sts(2, RU, 1, 3, 3, 3, 0), "Waiting for statefulset spec update to be observed...\n", False),
    ("no observed generation yet", _sts(1, RU, None, 3, 3, 3, 0), "Waiting for statefulset spec update to be observed...\n", False),
    ("pods not ready", _sts(1, RU, 2, 3, 2, 3, 0), "Waiting for 1 pods to be ready...\n", False),
    ("partition complete", _sts(1, PART2, 2, 3, 3, 2, 1), "partitioned roll out complete: 1 new pods have been updated...\n", True),
    ("partition in progress", _sts(1, PART2, 2, 3, 3, 3, 0),
     "Waiting for partitioned roll out to finish: 0 out of 1 new pods have been updated...\n", False),
    ("update in progress", _sts(1, RU, 2, 3, 3, 2, 1, "foo", "bar"),
     "waiting for statefulset rolling update to complete 1 pods at revision bar...\n", False),
    ("update complete", _sts(1, RU, 2, 3, 3, 3, 3, "foo", "foo"), "statefulset rolling update complete 3 pods at revision foo...\n", True),
    ("defaulted rolling update block", _sts(1, {"type": "RollingUpdate", "rollingUpdate": {"partition": 0}}, 2, 3, 3, 2, 3, "a", "b"),
     "partitioned roll out complete: 3 new pods have been updated...\n", True),
])
def test_statefulset_status_viewer(name, obj, msg, done):
    assert R.statefulset_status(obj, "foo") == (msg, done), name


def test_statefulset_status_viewer_on_delete():
    with pytest.raises(R.StatusError) as e:
        R.statefulset_status(_sts(1, {"type": "OnDelete"}, 1, 0, 1, 0, 0), "foo")
    assert str(e.value) == "OnDelete updateStrategy does not have a Status`" and e.value.done
