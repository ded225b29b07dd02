"""Prober parity: the tables of the reference's pkg/kubelet/prober/prober_test.go
(TestFormatURL, TestFindPortByName, TestGetURLParts, TestGetTCPAddrParts, TestHTTPHeaders,
TestProbe) and worker_test.go (TestDoProbe, TestInitialDelay, TestFailureThreshold,
TestSuccessThreshold, TestCleanUp, TestHandleCrash, TestOnHoldOnLivenessCheckFailure,
TestResultRunOnLivenessCheckFailure) with common_test.go's fixtures, plus the HTTP prober
against real servers (pod IP, named port, headers, User-Agent, HTTPS without verification)."""
import asyncio
import os
import ssl
import subprocess
import time

import pytest

from amdkube.api import meta as m
from amdkube.kubelet import prober as P

TEST_CONTAINER = "cOnTaInEr_NaMe"
TEST_POD_UID = "pOd_UiD"
TEST_CID = "test://cOnTaInEr_Id"


# ---------------------------------------------------------------- prober_test.go
@pytest.mark.parametrize("scheme,host,port,path,want", [
    ("http", "localhost", 93, "", "http://localhost:93"),
    ("https", "localhost", 93, "/path", "https://localhost:93/path"),
    ("http", "localhost", 93, "?foo", "http://localhost:93?foo"),
    ("https", "localhost", 93, "/path?bar", "https://localhost:93/path?bar"),
])
def test_format_url(scheme, host, port, path, want):
    assert P.format_url(scheme, host, port, path) == want


def test_format_url_ipv6_host():
    assert P.format_url("http", "fd00::1", 80, "/x") == "http://[fd00::1]:80/x"


def test_find_port_by_name():
    c = {"ports": [{"name": "foo", "containerPort": 8080}, {"name": "bar", "containerPort": 9000}]}
    assert P.find_port_by_name(c, "foo") == 8080
    with pytest.raises(ValueError):
        P.find_port_by_name(c, "baz")


URL_CASES = [
    ({"host": "", "port": -1, "path": ""}, False, "", -1, ""),
    ({"host": "", "port": "", "path": ""}, False, "", -1, ""),
    ({"host": "", "port": "-1", "path": ""}, False, "", -1, ""),
    ({"host": "", "port": "not-found", "path": ""}, False, "", -1, ""),
    ({"host": "", "port": "found", "path": ""}, True, "127.0.0.1", 93, ""),
    ({"host": "", "port": 76, "path": ""}, True, "127.0.0.1", 76, ""),
    ({"host": "", "port": "118", "path": ""}, True, "127.0.0.1", 118, ""),
    ({"host": "hostname", "port": 76, "path": "path"}, True, "hostname", 76, "path"),
]


@pytest.mark.parametrize("probe,ok,host,port,path", URL_CASES)
def test_get_url_parts(probe, ok, host, port, path):
    state = {"podIP": "127.0.0.1"}
    c = {"ports": [{"name": "found", "containerPort": 93}], "livenessProbe": {"httpGet": probe}}
    h = probe["host"] or state["podIP"]
    try:
        got = P.extract_port(probe["port"], c)
        err = None
    except ValueError as e:
        got, err = None, e
    if ok:
        assert err is None and (h, got, probe["path"]) == (host, port, path)
    else:
        assert err is not None


@pytest.mark.parametrize("port,ok,want", [(-1, False, -1), ("", False, -1), ("-1", False, -1), ("not-found", False, -1),
                                          ("found", True, 93), (76, True, 76), ("118", True, 118)])
def test_get_tcp_addr_parts(port, ok, want):
    c = {"ports": [{"name": "found", "containerPort": 93}], "livenessProbe": {"tcpSocket": {"port": port}}}
    if ok:
        assert P.extract_port(port, c) == want
    else:
        with pytest.raises(ValueError):
            P.extract_port(port, c)


@pytest.mark.parametrize("inp,out", [
    ([], {}),
    ([{"name": "X-Muffins-Or-Cupcakes", "value": "Muffins"}], {"X-Muffins-Or-Cupcakes": ["Muffins"]}),
    ([{"name": "X-Muffins-Or-Cupcakes", "value": "Muffins"}, {"name": "X-Muffins-Or-Plumcakes", "value": "Muffins!"}],
     {"X-Muffins-Or-Cupcakes": ["Muffins"], "X-Muffins-Or-Plumcakes": ["Muffins!"]}),
    ([{"name": "X-Muffins-Or-Cupcakes", "value": "Muffins"}, {"name": "X-Muffins-Or-Cupcakes", "value": "Cupcakes, too"}],
     {"X-Muffins-Or-Cupcakes": ["Muffins", "Cupcakes, too"]}),
])
def test_http_headers(inp, out):
    assert P.build_header(inp) == out


class FakeExec:
    def __init__(self, result=P.SUCCESS, err=None, crash=False):
        self.result, self.err, self.crash = result, err, crash
        self.cmds = []

    async def probe(self, runner, cid, cmd, timeout):
        if self.crash:
            raise RuntimeError("Intentional Probe crash.")
        self.cmds.append(cmd)
        return self.result, "", self.err


class FakeRecorder:
    def __init__(self):
        self.events = []

    def event(self, obj, etype, reason, message):
        self.events.append((etype, reason, message))


EXEC = {"exec": {}}
PROBE_CASES = [   # (probe, env, exec_error, expect_error, exec_result, expected, expect_command)
    (None, None, False, False, P.SUCCESS, True, None),                       # No probe
    ({}, None, False, True, P.SUCCESS, False, None),                         # No handler
    (EXEC, None, False, False, P.FAILURE, False, None),                      # Probe fails
    (EXEC, None, False, False, P.SUCCESS, True, None),                       # Probe succeeds
    (EXEC, None, False, False, P.UNKNOWN, False, None),                      # result is unknown
    (EXEC, None, True, True, P.UNKNOWN, False, None),                        # Probe has an error
    ({"exec": {"command": ["/bin/bash", "-c", "some script"]}}, None, False, False, P.SUCCESS, True,
     ["/bin/bash", "-c", "some script"]),
    ({"exec": {"command": ["/bin/bash", "-c", "some $(A) $(B)"]}}, [{"name": "A", "value": "script"}], False, False,
     P.SUCCESS, True, ["/bin/bash", "-c", "some script $(B)"]),
]


@pytest.mark.parametrize("i", range(len(PROBE_CASES)))
@pytest.mark.parametrize("ptype", [P.LIVENESS, P.READINESS])
async def test_probe(i, ptype):
    probe, env, exec_error, expect_error, exec_result, expected, expect_cmd = PROBE_CASES[i]
    rec = FakeRecorder()
    pr = P.Prober(recorder=rec)
    pr.exec = FakeExec(exec_result, RuntimeError("exec error") if exec_error else None)
    c = {"name": "c", "env": env or []}
    if probe is not None:
        c["livenessProbe" if ptype == P.LIVENESS else "readinessProbe"] = probe
    result, err = await pr.probe(ptype, {"metadata": {}}, {}, c, "test://foobar")
    assert (err is not None) == expect_error
    assert result == expected
    if not expected:
        assert rec.events and rec.events[-1][1] == "Unhealthy" and rec.events[-1][2].startswith(ptype)
    if expect_cmd:
        # the real exec prober through a command runner: the expanded command reaches it
        seen = []

        async def runner(cid, cmd, timeout):
            seen.append((cid, cmd))
            return "", 0
        pr2 = P.Prober(runner=runner)
        result, err = await pr2.probe(ptype, {"metadata": {}}, {}, c, "test://foobar")
        assert err is None and result
        assert seen == [("test://foobar", expect_cmd)]


async def test_probe_error_is_retried_three_times():
    n = []

    async def runner(cid, cmd, timeout):
        n.append(1)
        raise RuntimeError("runtime down")
    pr = P.Prober(runner=runner)
    result, err = await pr.probe(P.LIVENESS, {"metadata": {}}, {}, {"name": "c", "livenessProbe": EXEC}, "x://y")
    assert not result and err is not None and len(n) == P.MAX_PROBE_RETRIES


async def test_exec_probe_exit_status():
    async def runner(cid, cmd, timeout):
        return "boom", 3
    pr = P.Prober(runner=runner)
    assert (await pr.probe(P.READINESS, {"metadata": {}}, {}, {"name": "c", "readinessProbe": EXEC}, "x://y"))[0] is False


# ---------------------------------------------------------------- worker_test.go
def _rfc3339(t):
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


def running_status(started=None):
    return {"phase": "Running", "containerStatuses": [{
        "name": TEST_CONTAINER, "containerID": TEST_CID,
        "state": {"running": {"startedAt": _rfc3339(started if started is not None else time.time())}}}]}


def make_test_pod(ptype, spec):
    probe = {"exec": {}, **spec}
    for k, v in (("timeoutSeconds", 1), ("periodSeconds", 1), ("successThreshold", 1), ("failureThreshold", 1)):
        if not probe.get(k):
            probe[k] = v
    c = {"name": TEST_CONTAINER, ("livenessProbe" if ptype == P.LIVENESS else "readinessProbe"): probe}
    return {"metadata": {"name": "testPod", "uid": TEST_POD_UID}, "spec": {"containers": [c], "restartPolicy": "Never"}}


class Harness:
    def __init__(self):
        self.statuses = {}
        self.changes = []
        self.mgr = P.ProbeManager(self.statuses.get, on_change=self.changes.append, jitter=False)
        self.mgr.prober.exec = FakeExec(P.SUCCESS)

    def worker(self, ptype, spec=None):
        pod = make_test_pod(ptype, spec or {})
        return P.Worker(self.mgr, ptype, pod, pod["spec"]["containers"][0])

    def set_exec(self, result):
        self.mgr.prober.exec = FakeExec(result)

    def result(self, w):
        return w.results.get(w.container_id or TEST_CID)


def _status(kind):
    s = running_status()
    c = s["containerStatuses"][0]
    if kind == "pending":
        c["state"] = {"waiting": {}}
    elif kind == "terminated":
        c["state"] = {"terminated": {"startedAt": _rfc3339(time.time())}}
    elif kind == "other":
        c["name"] = "otherContainer"
    elif kind == "failed":
        s["phase"] = "Failed"
    return s


DO_PROBE = [   # (status kind, probe spec, expect continue, expect set, expected result)
    (None, {}, True, False, None),                   # No status
    ("failed", {}, False, False, None),              # Pod failed
    ("other", {}, True, False, None),                # No container status
    ("pending", {}, True, True, False),              # Container waiting
    ("terminated", {}, False, True, False),          # Container terminated
    ("running", {}, True, True, True),                # Probe successful
    ("running", {"initialDelaySeconds": -100}, True, True, True),   # Initial delay passed
]


@pytest.mark.parametrize("ptype", [P.LIVENESS, P.READINESS])
@pytest.mark.parametrize("i", range(len(DO_PROBE)))
async def test_do_probe(ptype, i):
    kind, spec, cont, is_set, want = DO_PROBE[i]
    h = Harness()
    w = h.worker(ptype, spec)
    if kind is not None:
        h.statuses[TEST_POD_UID] = _status(kind)
    assert await w.do_probe() == cont
    got = w.results.get(TEST_CID)
    assert (got is not None) == is_set
    if is_set:
        assert got == want


@pytest.mark.parametrize("ptype", [P.LIVENESS, P.READINESS])
async def test_initial_delay(ptype):
    h = Harness()
    w = h.worker(ptype, {"initialDelaySeconds": 10})
    h.statuses[TEST_POD_UID] = running_status()
    assert await w.do_probe()
    assert h.result(w) == (ptype == P.LIVENESS)      # the initial value during the delay
    h.statuses[TEST_POD_UID] = running_status(time.time() - 100)
    assert await w.do_probe()
    assert h.result(w) is True


async def test_failure_threshold():
    h = Harness()
    w = h.worker(P.READINESS, {"successThreshold": 1, "failureThreshold": 3})
    h.statuses[TEST_POD_UID] = running_status()
    for _ in range(2):
        h.set_exec(P.SUCCESS)
        for _ in range(3):
            assert await w.do_probe() and h.result(w) is True
        h.set_exec(P.FAILURE)
        for _ in range(2):
            assert await w.do_probe() and h.result(w) is True
        for _ in range(3):
            assert await w.do_probe() and h.result(w) is False


async def test_success_threshold():
    h = Harness()
    w = h.worker(P.READINESS, {"successThreshold": 3, "failureThreshold": 1})
    h.statuses[TEST_POD_UID] = running_status()
    w.results.set(TEST_CID, False, {"metadata": {}})
    for _ in range(2):
        for _ in range(2):
            assert await w.do_probe() and h.result(w) is False
        for _ in range(3):
            assert await w.do_probe() and h.result(w) is True
        h.set_exec(P.FAILURE)
        assert await w.do_probe() and h.result(w) is False
        h.set_exec(P.SUCCESS)


@pytest.mark.parametrize("ptype", [P.LIVENESS, P.READINESS])
async def test_clean_up(ptype):
    h = Harness()
    pod = make_test_pod(ptype, {})
    h.statuses[TEST_POD_UID] = running_status()
    h.mgr.add_pod(pod)
    key = (TEST_POD_UID, TEST_CONTAINER, ptype)
    w = h.mgr.workers[key]
    for _ in range(100):
        if w.results.get(TEST_CID) is True:
            break
        await asyncio.sleep(0.01)
    assert w.results.get(TEST_CID) is True
    for _ in range(10):
        w.stop()            # callable many times
    await asyncio.wait_for(w.task, 5)
    assert w.results.get(TEST_CID) is None
    assert key not in h.mgr.workers


async def test_handle_crash():
    h = Harness()
    w = h.worker(P.READINESS)
    h.statuses[TEST_POD_UID] = running_status()
    assert await w.do_probe() and h.result(w) is True
    h.mgr.prober.exec = FakeExec(crash=True)
    assert await w.do_probe()               # recovered, keeps going
    assert h.result(w) is True              # unchanged


async def test_on_hold_on_liveness_check_failure():
    h = Harness()
    w = h.worker(P.LIVENESS, {"successThreshold": 1, "failureThreshold": 1})
    st = running_status()
    h.statuses[TEST_POD_UID] = running_status()
    h.set_exec(P.FAILURE)
    assert await w.do_probe() and h.result(w) is False and w.on_hold
    assert h.changes == [TEST_POD_UID]      # the kubelet is told to kill it
    h.set_exec(P.SUCCESS)
    assert await w.do_probe() and h.result(w) is False and w.on_hold     # on hold: not probed
    st["containerStatuses"][0]["containerID"] = "test://newCont_ID"
    h.statuses[TEST_POD_UID] = st
    assert await w.do_probe()
    assert w.results.get("test://newCont_ID") is True and not w.on_hold


async def test_result_run_on_liveness_check_failure():
    h = Harness()
    w = h.worker(P.LIVENESS, {"successThreshold": 1, "failureThreshold": 3})
    h.statuses[TEST_POD_UID] = running_status()
    h.set_exec(P.SUCCESS)
    assert await w.do_probe() and h.result(w) is True and w.result_run == 1
    h.set_exec(P.FAILURE)
    assert await w.do_probe() and h.result(w) is True and w.result_run == 1
    assert await w.do_probe() and h.result(w) is True and w.result_run == 2
    assert await w.do_probe() and h.result(w) is False and w.result_run == 1     # reset for the next container


async def test_readiness_of_uses_results_then_worker_presence():
    from amdkube.kubelet.kuberuntime import ContainerRuntimeStatus, PodRuntimeStatus
    h = Harness()
    pod = make_test_pod(P.READINESS, {})
    rt = PodRuntimeStatus(TEST_POD_UID)
    cs = ContainerRuntimeStatus()
    cs.id = "abc"
    rt.containers[TEST_CONTAINER] = [cs]
    assert h.mgr.readiness_of(TEST_POD_UID, pod, rt) == {TEST_CONTAINER: True}     # no worker
    h.mgr.workers[(TEST_POD_UID, TEST_CONTAINER, P.READINESS)] = object()
    assert h.mgr.readiness_of(TEST_POD_UID, pod, rt) == {TEST_CONTAINER: False}    # worker, no result yet
    h.mgr.readiness.set("rocshim://abc", True, pod)
    assert h.mgr.readiness_of(TEST_POD_UID, pod, rt) == {TEST_CONTAINER: True}


# ---------------------------------------------------------------- real HTTP / TCP
async def _server(handler, ssl_ctx=None):
    from aiohttp import web
    app = web.Application()
    app.router.add_get("/{tail:.*}", handler)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0, ssl_context=ssl_ctx)
    await site.start()
    return runner, site._server.sockets[0].getsockname()[1]


async def test_http_probe_uses_pod_ip_named_port_and_headers():
    seen = []
    from aiohttp import web

    async def handler(req):
        seen.append((req.path_qs, dict(req.headers)))
        return web.Response(status=200 if req.path == "/healthz" else 500, text="ok")
    runner, port = await _server(handler)
    try:
        pr = P.Prober(recorder=FakeRecorder())
        c = {"name": "web", "ports": [{"name": "http", "containerPort": port}],
             "livenessProbe": {"httpGet": {"path": "/healthz?x=1", "port": "http",
                                           "httpHeaders": [{"name": "X-Custom", "value": "a"},
                                                           {"name": "host", "value": "example.test"}]}}}
        ok, err = await pr.probe(P.LIVENESS, {"metadata": {}}, {"podIP": "127.0.0.1"}, c, "x://y")
        assert ok and err is None
        path, hdrs = seen[-1]
        assert path == "/healthz?x=1"
        assert hdrs["X-Custom"] == "a" and hdrs["User-Agent"] == P.USER_AGENT and hdrs["Host"] == "example.test"
        c["livenessProbe"]["httpGet"]["path"] = "/bad"
        rec = FakeRecorder()
        pr.recorder = rec
        ok, err = await pr.probe(P.LIVENESS, {"metadata": {}}, {"podIP": "127.0.0.1"}, c, "x://y")
        assert not ok and err is None
        assert rec.events[-1] == ("Warning", "Unhealthy", "Liveness probe failed: HTTP probe failed with statuscode: 500")
        # an unknown named port is a probe error, never a probe of the wrong address
        c["livenessProbe"]["httpGet"]["port"] = "nope"
        ok, err = await pr.probe(P.LIVENESS, {"metadata": {}}, {"podIP": "127.0.0.1"}, c, "x://y")
        assert not ok and err is not None
    finally:
        await runner.cleanup()


async def test_https_probe_skips_certificate_verification(tmp_path):
    d = str(tmp_path)
    r = subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/k.pem", "-out",
                        f"{d}/c.pem", "-days", "1", "-subj", "/CN=not-the-pod"], capture_output=True, timeout=60)
    if r.returncode != 0:
        pytest.skip("openssl unavailable")
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(f"{d}/c.pem", f"{d}/k.pem")
    from aiohttp import web

    async def handler(req):
        return web.Response(text="ok")
    runner, port = await _server(handler, ctx)
    try:
        c = {"name": "web", "readinessProbe": {"httpGet": {"scheme": "HTTPS", "port": port, "path": "/"}}}
        ok, err = await P.Prober().probe(P.READINESS, {"metadata": {}}, {"podIP": "127.0.0.1"}, c, "x://y")
        assert ok and err is None
    finally:
        await runner.cleanup()


async def test_tcp_probe():
    srv = await asyncio.start_server(lambda r, w: w.close(), "127.0.0.1", 0)
    port = srv.sockets[0].getsockname()[1]
    try:
        c = {"name": "db", "ports": [{"name": "sql", "containerPort": port}], "livenessProbe": {"tcpSocket": {"port": "sql"}}}
        assert (await P.Prober().probe(P.LIVENESS, {"metadata": {}}, {"podIP": "127.0.0.1"}, c, "x://y"))[0]
    finally:
        srv.close()
        await srv.wait_closed()
    assert not (await P.Prober().probe(P.LIVENESS, {"metadata": {}}, {"podIP": "127.0.0.1"}, c, "x://y"))[0]
