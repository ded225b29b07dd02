"""computePodActions parity: the tables of the reference's
pkg/kubelet/kuberuntime/kuberuntime_manager_test.go — TestComputePodActions (:777-926) and
TestComputePodActionsWithInitContainers (:950-1044), with makeBasePodAndStatus (:720) and
makeBasePodAndStatusWithInitContainers (:1046) as fixtures — plus the liveness cases the
reference leaves as a TODO (:912) decided by the same function (shouldRestartOnFailure), and
the back-off of doBackOff (:745) over flowcontrol.Backoff (backoff_test.go)."""
import copy

import pytest

from amdkube.grpcdesc.cri import CRI as C
from amdkube.kubelet.kuberuntime import (ContainerRuntimeStatus, PodActions, PodRuntimeStatus, compute_pod_actions,
                                         container_hash)
from amdkube.utils.flowcontrol import Backoff

RUNNING, EXITED = C.CONTAINER_RUNNING, C.CONTAINER_EXITED


def _cs(cid, name, state, h, exit_code=0, created=0):
    s = ContainerRuntimeStatus()
    s.id, s.name, s.state, s.hash, s.exit_code = cid, name, state, h, exit_code
    s.reason = s.message = s.image = s.image_ref = s.log_path = ""
    s.created_at, s.started_at, s.finished_at, s.restart_count = created, 0, 0, 0
    s.init, s.sandbox_id = False, "sandboxID"
    return s


def base_pod_and_status():
    pod = {"metadata": {"uid": "12345678", "name": "foo", "namespace": "foo-ns"},
           "spec": {"containers": [{"name": "foo1", "image": "busybox"}, {"name": "foo2", "image": "busybox"},
                                   {"name": "foo3", "image": "busybox"}]}}
    st = PodRuntimeStatus("12345678")
    st.sandboxes = [("sandboxID", C.SANDBOX_READY, 0, 1)]
    st.ip = "10.0.0.1"
    for i, c in enumerate(pod["spec"]["containers"]):
        st.containers[c["name"]] = [_cs(f"id{i + 1}", c["name"], RUNNING, container_hash(c))]
    return pod, st


def base_with_inits():
    pod, st = base_pod_and_status()
    pod["spec"]["initContainers"] = [{"name": "init1", "image": "bar-image"}, {"name": "init2", "image": "bar-image"},
                                     {"name": "init3", "image": "bar-image"}]
    h0 = container_hash(pod["spec"]["initContainers"][0])
    st.containers = {f"init{i}": [_cs(f"initid{i}", f"init{i}", EXITED, h0)] for i in (1, 2, 3)}
    return pod, st


def kill_map(pod, st, idx):
    out = {}
    for i in idx:
        c = pod["spec"]["containers"][i]
        out[st.latest(c["name"]).id] = (c["name"], c, "")
    return out


def _policy(p):
    return lambda pod: pod["spec"].__setitem__("restartPolicy", p)


def _exit(i, code):
    def f(st):
        cs = st.latest(f"foo{i + 1}")
        cs.state, cs.exit_code = EXITED, code
    return f


def _chain(*fs):
    def f(x):
        for g in fs:
            g(x)
    return f


def _sandbox_notready(st):
    st.sandboxes = [("sandboxID", C.SANDBOX_NOTREADY, 0, 1)]


def _no_ip(st):
    st.ip = ""


def _clear(st):
    st.sandboxes, st.containers = [], {}


def _hash(i, h):
    def f(st):
        st.latest(f"foo{i + 1}").hash = h
    return f


BP, BS = base_pod_and_status()
NO_ACTION = PodActions(sandbox_id="sandboxID")

# TestComputePodActions (:795-914)
CASES = {
    "everying is good; do nothing": (None, None, NO_ACTION),
    "start pod sandbox and all containers for a new pod":
        (None, _clear, PodActions(kill_pod=True, create_sandbox=True, attempt=0, to_start=[0, 1, 2])),
    "restart exited containers if RestartPolicy == Always":
        (_policy("Always"), _chain(_exit(0, 0), _exit(1, 111)), PodActions(sandbox_id="sandboxID", to_start=[0, 1])),
    "restart failed containers if RestartPolicy == OnFailure":
        (_policy("OnFailure"), _chain(_exit(0, 0), _exit(1, 111)), PodActions(sandbox_id="sandboxID", to_start=[1])),
    "don't restart containers if RestartPolicy == Never":
        (_policy("Never"), _chain(_exit(0, 0), _exit(1, 111)), NO_ACTION),
    "Kill pod and recreate everything if the pod sandbox is dead, and RestartPolicy == Always":
        (_policy("Always"), _sandbox_notready,
         PodActions(kill_pod=True, create_sandbox=True, sandbox_id="sandboxID", attempt=1, to_start=[0, 1, 2])),
    "Kill pod and recreate all containers (except for the succeeded one) if the pod sandbox is dead, and RestartPolicy == OnFailure":
        (_policy("OnFailure"), _chain(_sandbox_notready, _exit(1, 0)),
         PodActions(kill_pod=True, create_sandbox=True, sandbox_id="sandboxID", attempt=1, to_start=[0, 2])),
    "Kill pod and recreate all containers if the PodSandbox does not have an IP":
        (None, _no_ip, PodActions(kill_pod=True, create_sandbox=True, sandbox_id="sandboxID", attempt=1, to_start=[0, 1, 2])),
    "Kill and recreate the container if the container's spec changed":
        (_policy("Always"), _hash(1, "432423432"),
         PodActions(sandbox_id="sandboxID", to_kill=kill_map(BP, BS, [1]), to_start=[1])),
}


@pytest.mark.parametrize("desc", list(CASES))
def test_compute_pod_actions(desc):
    mpod, mst, want = CASES[desc]
    pod, st = base_pod_and_status()
    if mpod:
        mpod(pod)
    if mst:
        mst(st)
    got = compute_pod_actions(pod, st)
    assert got == want, desc


IP, IS = base_with_inits()
INIT_CASES = {
    "initialization completed; start all containers": (None, None, PodActions(sandbox_id="sandboxID", to_start=[0, 1, 2])),
    "initialization in progress; do nothing":
        (_policy("Always"), lambda st: setattr(st.latest("init3"), "state", RUNNING), NO_ACTION),
    "Kill pod and restart the first init container if the pod sandbox is dead":
        (_policy("Always"), _sandbox_notready,
         PodActions(kill_pod=True, create_sandbox=True, sandbox_id="sandboxID", attempt=1, next_init=IP["spec"]["initContainers"][0])),
    "initialization failed; restart the last init container if RestartPolicy == Always":
        (_policy("Always"), lambda st: setattr(st.latest("init3"), "exit_code", 137),
         PodActions(sandbox_id="sandboxID", next_init=IP["spec"]["initContainers"][2])),
    "initialization failed; restart the last init container if RestartPolicy == OnFailure":
        (_policy("OnFailure"), lambda st: setattr(st.latest("init3"), "exit_code", 137),
         PodActions(sandbox_id="sandboxID", next_init=IP["spec"]["initContainers"][2])),
    "initialization failed; kill pod if RestartPolicy == Never":
        (_policy("Never"), lambda st: setattr(st.latest("init3"), "exit_code", 137),
         PodActions(kill_pod=True, sandbox_id="sandboxID")),
}


@pytest.mark.parametrize("desc", list(INIT_CASES))
def test_compute_pod_actions_with_init_containers(desc):
    mpod, mst, want = INIT_CASES[desc]
    pod, st = base_with_inits()
    if mpod:
        mpod(pod)
    if mst:
        mst(st)
    assert compute_pod_actions(pod, st) == want, desc


@pytest.mark.parametrize("policy,restart", [("Always", True), ("OnFailure", True), ("Never", False)])
def test_liveness_failure_restarts_only_when_the_policy_allows(policy, restart):
    """shouldRestartOnFailure (:428) decides a liveness kill; the reference's TODO at :912."""
    pod, st = base_pod_and_status()
    pod["spec"]["restartPolicy"] = policy
    got = compute_pod_actions(pod, st, {"id2"})
    assert list(got.to_kill) == ["id2"]
    assert got.to_kill["id2"][2].startswith("Container failed liveness probe.")
    assert got.to_start == ([1] if restart else [])
    assert not got.kill_pod and not got.create_sandbox
    # a predicate over container ids works the same
    assert compute_pod_actions(pod, st, lambda cid: cid == "id2") == got


def test_single_container_never_pod_failing_liveness_is_killed_not_restarted():
    pod, st = base_pod_and_status()
    pod["spec"]["containers"] = pod["spec"]["containers"][:1]
    st.containers = {"foo1": st.containers["foo1"]}
    pod["spec"]["restartPolicy"] = "Never"
    got = compute_pod_actions(pod, st, {"id1"})
    assert got.to_start == [] and list(got.to_kill) == ["id1"]
    assert got.kill_pod     # nothing left running, nothing to start: the pod goes
    # after the kill the container is exited: Never never restarts it
    st.latest("foo1").state, st.latest("foo1").exit_code = EXITED, 137
    after = compute_pod_actions(pod, st)
    assert after.to_start == [] and after.kill_pod and not after.create_sandbox


def test_spec_change_restarts_even_under_never():
    pod, st = base_pod_and_status()
    pod["spec"]["restartPolicy"] = "Never"
    st.latest("foo3").hash = "other"
    got = compute_pod_actions(pod, st)
    assert got.to_start == [2] and list(got.to_kill) == ["id3"]
    assert "Container will be killed and recreated" in got.to_kill["id3"][2]


def test_never_pod_with_dead_sandbox_is_not_recreated():
    pod, st = base_pod_and_status()
    pod["spec"]["restartPolicy"] = "Never"
    _sandbox_notready(st)
    got = compute_pod_actions(pod, st)
    assert got.kill_pod and not got.create_sandbox and got.to_start == [] and got.next_init is None


def test_unknown_ip_is_not_a_reason_to_recreate():
    pod, st = base_pod_and_status()
    st.ip = None      # the sandbox status lookup failed: keep the sandbox
    assert compute_pod_actions(pod, st) == NO_ACTION
    pod["spec"]["hostNetwork"] = True
    st.ip = ""
    assert compute_pod_actions(pod, st) == NO_ACTION


# ---------------------------------------------------------------- back-off (backoff_test.go)
class FakeClock:
    def __init__(self, t=1000.0):
        self.t = t

    def __call__(self):
        return self.t


def test_backoff_doubles_to_the_cap_and_expires():
    """TestSlowBackoff / TestBackoffReset / TestBackoffHighWaterMark / TestIsInBackOffSinceUpdate."""
    clk = FakeClock()
    b = Backoff(1, 120, clk)
    want = 1
    for _ in range(10):
        b.next("id", clk())
        assert b.get("id") == want
        want = min(want * 2, 120)
        clk.t += 1
    clk.t += 241               # fine for longer than 2 × max: the next Next starts again
    b.next("id", clk())
    assert b.get("id") == 1
    b.reset("id")
    assert b.get("id") == 0


def test_is_in_backoff_since():
    clk = FakeClock()
    b = Backoff(1, 10, clk)
    ev = clk()
    assert not b.is_in_backoff_since("id", ev)
    b.next("id", ev)           # backoff 1 s since ev
    assert b.is_in_backoff_since("id", ev)
    clk.t += 1.5
    assert not b.is_in_backoff_since("id", ev)
    b.next("id", clk())        # 2 s
    ev2 = clk()
    clk.t += 1
    assert b.is_in_backoff_since("id", ev2) and abs(b.remaining("id", ev2) - 1.0) < 1e-9
    # an event far after the last update has expired the entry
    assert not b.is_in_backoff_since("id", clk() + 100)
    b.gc()
    clk.t += 100
    b.gc()
    assert len(b) == 0


def test_actions_helpers_compare_like_the_reference_verifyActions():
    a = PodActions(sandbox_id="s", to_kill={"x": ("n", {"name": "n"}, "m1")})
    b = PodActions(sandbox_id="s", to_kill={"x": ("n", {"name": "n"}, "other message")})
    assert a == b           # verifyActions clears the message field
    assert a != PodActions(sandbox_id="s")
    assert "to_kill" in repr(copy.copy(a))
