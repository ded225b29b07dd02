"""kubectl label / annotate / scale / run at reference parity.

Transcribed: pkg/kubectl/cmd/label_test.go (TestValidateLabels, TestParseLabels, TestLabelFunc,
TestLabelErrors), annotate_test.go (TestValidateAnnotationOverwrites, TestParseAnnotations,
TestValidateAnnotations, TestUpdateAnnotations, TestAnnotateErrors), cmd/run_test.go
(TestGetRestartPolicy, TestGenerateService, TestRunValidations), pkg/kubectl/run_test.go
(TestGenerate, TestGeneratePod, TestGenerateDeployment, TestGenerateJob, TestGenerateCronJob*,
TestParseEnv), pkg/kubectl/scale.go's precondition errors. Then the commands through a live
cluster.
"""
from __future__ import annotations

import asyncio
import contextlib
import io

import pytest

from amdkube.api import meta as m
from amdkube.kubectl import metacmds as MC
from amdkube.kubectl import run as R
from amdkube.kubectl import scale as S
from tests.conftest import run


# ---------------------------------------------------------------------------- label
@pytest.mark.parametrize("labels,new,err", [
    ({"a": "b", "c": "d"}, {"a": "c", "d": "b"}, True),
    ({"a": "b", "c": "d"}, {"b": "d", "c": "a"}, True),
    ({"a": "b", "c": "d"}, {"b": "a", "d": "c"}, False),
    ({}, {"b": "a", "d": "c"}, False),
])
def test_validate_labels(labels, new, err):
    obj = {"metadata": {"labels": labels}}
    if err:
        with pytest.raises(MC.UsageError, match="already has a value"):
            MC.validate_no_overwrites(obj, new)
    else:
        MC.validate_no_overwrites(obj, new)


@pytest.mark.parametrize("spec,labels,remove,err", [
    (["a=b", "c=d"], {"a": "b", "c": "d"}, None, False),
    ([], {}, None, False),
    (["a=b", "c=d", "e-"], {"a": "b", "c": "d"}, ["e"], False),
    (["ab", "c=d"], None, None, True),
    (["a=b", "c=d", "a-"], None, None, True),
    (["a="], {"a": ""}, None, False),
    (["a=%^$"], None, None, True),
])
def test_parse_labels(spec, labels, remove, err):
    if err:
        with pytest.raises(MC.UsageError):
            MC.parse_labels(spec)
        return
    assert MC.parse_labels(spec) == (labels, remove)


@pytest.mark.parametrize("labels,overwrite,version,new,remove,expected,err", [
    ({"a": "b"}, False, "", {"a": "b"}, None, None, True),
    ({"a": "b"}, True, "", {"a": "c"}, None, {"labels": {"a": "c"}}, False),
    ({"a": "b"}, False, "", {"c": "d"}, None, {"labels": {"a": "b", "c": "d"}}, False),
    ({"a": "b"}, False, "2", {"c": "d"}, None, {"labels": {"a": "b", "c": "d"}, "resourceVersion": "2"}, False),
    ({"a": "b"}, False, "", {}, ["a"], {"labels": {}}, False),
    ({"a": "b", "c": "d"}, False, "", {"e": "f"}, ["a"], {"labels": {"c": "d", "e": "f"}}, False),
    (None, False, "", {"a": "b"}, None, {"labels": {"a": "b"}}, False),
])
def test_label_func(labels, overwrite, version, new, remove, expected, err):
    obj = {"metadata": {"labels": labels} if labels is not None else {}}
    if err:
        with pytest.raises(MC.UsageError):
            MC.label_func(obj, overwrite, version, new, remove)
        return
    MC.label_func(obj, overwrite, version, new, remove)
    assert obj["metadata"] == expected


def _args(*argv):
    from amdkube.kubectl import main as km
    argv = km._expose.rewrite_flags(km._logs.rewrite_short_flags(list(argv)))
    a, extra = km.parser().parse_known_args(argv)
    a.args = list(a.args) + extra
    a.command_flag = "--command" in argv
    if a.command is None:
        a.command = []
    return a


async def _kubectl(c, *argv, tail=None):
    from amdkube.kubectl import main as km
    out, err = io.StringIO(), io.StringIO()
    a = _args(*argv)
    if tail is not None:
        a.command = list(tail)
    with contextlib.redirect_stdout(out), contextlib.redirect_stderr(err):
        rc = await km.COMMANDS[a.cmd](c, a)
    return rc or 0, out.getvalue(), err.getvalue()


@pytest.mark.parametrize("cmd,args,msg", [
    ("label", [], "one or more resources must be specified"),
    ("label", ["pods"], "at least one label update is required"),
    ("label", ["pods", "-"], "at least one label update is required"),
    ("label", ["pods", "=bar"], "at least one label update is required"),
    ("label", ["pods-"], "one or more resources must be specified"),
    ("label", ["pods=bar"], "one or more resources must be specified"),
    ("label", ["pods", "app=bar"], "resource(s) were provided, but no name, label selector, or --all flag specified"),
    ("label", ["pods,deployments", "app=bar"], "resource(s) were provided, but no name, label selector, or --all flag specified"),
    ("annotate", [], "one or more resources must be specified"),
    ("annotate", ["pods"], "at least one annotation update is required"),
    ("annotate", ["pods", "-"], "at least one annotation update is required"),
    ("annotate", ["pods", "=bar"], "at least one annotation update is required"),
    ("annotate", ["pods-"], "one or more resources must be specified"),
    ("annotate", ["pods=bar"], "one or more resources must be specified"),
])
def test_label_and_annotate_errors(cmd, args, msg):
    class NoServer:
        async def list(self, *a, **k):
            raise AssertionError("no request expected")
        get = list

    rc, out, err = run(_kubectl(NoServer(), cmd, *args))
    assert rc == 1 and msg in err and out == ""


# ------------------------------------------------------------------------- annotate
@pytest.mark.parametrize("cur,new,err", [
    ({"a": "A", "b": "B"}, {"a": "a", "c": "C"}, True),
    ({"a": "A", "c": "C"}, {"b": "B", "c": "c"}, True),
    ({"a": "A", "c": "C"}, {"b": "B", "d": "D"}, False),
    ({}, {"a": "A", "b": "B"}, False),
])
def test_validate_annotation_overwrites(cur, new, err):
    obj = {"metadata": {"annotations": cur}}
    if err:
        with pytest.raises(MC.UsageError, match="--overwrite is false but found the following declared annotation"):
            MC.validate_no_annotation_overwrites(obj, new)
    else:
        MC.validate_no_annotation_overwrites(obj, new)


URL = "https://test.com/index.htm?id=123#u=user-name"
JSON = ("'{\"kind\":\"SerializedReference\",\"apiVersion\":\"v1\",\"reference\":{\"kind\":\"ReplicationController\","
        "\"namespace\":\"default\",\"name\":\"my-nginx\",\"uid\":\"c544ee78-2665-11e5-8051-42010af0c213\","
        "\"apiVersion\":\"v1\",\"resourceVersion\":\"61368\"}}'")


@pytest.mark.parametrize("args,new,remove,err", [
    (["a=b", "c=d"], {"a": "b", "c": "d"}, [], None),
    (["url=" + URL, "fake.kubernetes.io/annotation=" + JSON], {"url": URL, "fake.kubernetes.io/annotation": JSON}, [], None),
    ([], {}, [], None),
    (["a=b", "c=d", "e-"], {"a": "b", "c": "d"}, ["e"], None),
    (["ab", "c=d"], None, None, "invalid annotation format: ab"),
    (["a="], {"a": ""}, [], None),
    (["ab", "a="], None, None, "invalid annotation format: ab"),
    (["-"], None, None, "invalid annotation format: -"),
    (["=bar"], None, None, "invalid annotation format: =bar"),
])
def test_parse_annotations(args, new, remove, err):
    if err:
        with pytest.raises(MC.UsageError) as e:
            MC.parse_pairs(args, "annotation", True)
        assert str(e.value) == err
        return
    assert MC.parse_pairs(args, "annotation", True) == (new, remove)


def test_validate_annotations():
    with pytest.raises(MC.UsageError) as e:
        MC.validate_annotations(["a"], {"a": "b", "c": "d"})
    assert str(e.value) == "can not both modify and remove the following annotation(s) in the same command: a"
    with pytest.raises(MC.UsageError) as e:
        MC.validate_annotations(["a", "c"], {"a": "b", "c": "d"})
    assert str(e.value) == "can not both modify and remove the following annotation(s) in the same command: a, c"


@pytest.mark.parametrize("cur,overwrite,version,new,remove,expected,err", [
    ({"a": "b"}, False, "", {"a": "b"}, None, None, True),
    ({"a": "b"}, True, "", {"a": "c"}, None, {"annotations": {"a": "c"}}, False),
    ({"a": "b"}, False, "", {"c": "d"}, None, {"annotations": {"a": "b", "c": "d"}}, False),
    ({"a": "b"}, False, "2", {"c": "d"}, None, {"annotations": {"a": "b", "c": "d"}, "resourceVersion": "2"}, False),
    ({"a": "b"}, False, "", {}, ["a"], {"annotations": {}}, False),
    ({"a": "b", "c": "d"}, False, "", {"e": "f"}, ["a"], {"annotations": {"c": "d", "e": "f"}}, False),
    ({"a": "b", "c": "d"}, False, "", {"e": "f"}, ["g"], {"annotations": {"a": "b", "c": "d", "e": "f"}}, False),
    ({"a": "b", "c": "d"}, False, "", {}, ["e"], {"annotations": {"a": "b", "c": "d"}}, False),
    (None, False, "", {"a": "b"}, None, {"annotations": {"a": "b"}}, False),
])
def test_update_annotations(cur, overwrite, version, new, remove, expected, err):
    obj = {"metadata": {"annotations": cur} if cur is not None else {}}
    if err:
        with pytest.raises(MC.UsageError):
            MC.update_annotations(obj, overwrite, version, new, remove)
        return
    MC.update_annotations(obj, overwrite, version, new, remove)
    assert obj["metadata"] == expected


# ------------------------------------------------------------------------------ run
@pytest.mark.parametrize("inp,interactive,expected", [
    ("", False, "Always"), ("", True, "OnFailure"), ("Always", True, "Always"), ("Never", True, "Never"),
    ("Always", False, "Always"), ("Never", False, "Never"), ("foo", False, None),
])
def test_get_restart_policy(inp, interactive, expected):
    if expected is None:
        with pytest.raises(R.GenerateError):
            R.get_restart_policy(inp, interactive)
    else:
        assert R.get_restart_policy(inp, interactive) == expected


def _rc(labels, container, replicas=1):
    return {"apiVersion": "v1", "kind": "ReplicationController", "metadata": {"name": "foo", "labels": labels},
            "spec": {"replicas": replicas, "selector": labels,
                     "template": {"metadata": {"labels": labels}, "spec": {"containers": [dict({"name": "foo", "image": "someimage"}, **container)]}}}}


RUN = {"run": "foo"}
FOOBAR = {"foo": "bar", "baz": "blah"}


@pytest.mark.parametrize("params,expected", [
    ({"name": "foo", "image": "someimage", "image-pull-policy": "Always", "replicas": "1", "port": ""},
     _rc(RUN, {"imagePullPolicy": "Always"})),
    ({"name": "foo", "image": "someimage", "replicas": "1", "port": "", "env": ["a=b", "c=d"]},
     _rc(RUN, {"env": [{"name": "a", "value": "b"}, {"name": "c", "value": "d"}]})),
    ({"name": "foo", "image": "someimage", "image-pull-policy": "Never", "replicas": "1", "port": "", "args": ["bar", "baz", "blah"]},
     _rc(RUN, {"imagePullPolicy": "Never", "args": ["bar", "baz", "blah"]})),
    ({"name": "foo", "image": "someimage", "replicas": "1", "port": "", "args": ["bar", "baz", "blah"], "command": "true"},
     _rc(RUN, {"command": ["bar", "baz", "blah"]})),
    ({"name": "foo", "image": "someimage", "replicas": "1", "port": "80"}, _rc(RUN, {"ports": [{"containerPort": 80}]})),
    ({"name": "foo", "image": "someimage", "image-pull-policy": "IfNotPresent", "replicas": "1", "port": "80", "hostport": "80"},
     _rc(RUN, {"imagePullPolicy": "IfNotPresent", "ports": [{"containerPort": 80, "hostPort": 80}]})),
    ({"name": "foo", "image": "someimage", "replicas": "1", "hostport": "80"}, None),
    ({"name": "foo", "image": "someimage", "replicas": "1", "labels": "foo=bar,baz=blah"}, _rc(FOOBAR, {})),
    ({"name": "foo", "image": "someimage", "replicas": "1", "labels": "foo=bar,baz=blah", "requests": "cpu100m,memory=100Mi"}, None),
    ({"name": "foo", "image": "someimage", "replicas": "1", "labels": "foo=bar,baz=blah", "requests": "cpu=100m&memory=100Mi"}, None),
    ({"name": "foo", "image": "someimage", "replicas": "1", "labels": "foo=bar,baz=blah", "requests": "cpu="}, None),
    ({"name": "foo", "image": "someimage", "replicas": "1", "labels": "foo=bar,baz=blah", "requests": "cpu=100m,memory=100Mi",
      "limits": "cpu=400m,memory=200Mi"},
     _rc(FOOBAR, {"resources": {"limits": {"cpu": "400m", "memory": "200Mi"}, "requests": {"cpu": "100m", "memory": "100Mi"}}})),
])
def test_generate_replication_controller(params, expected):
    if expected is None:
        with pytest.raises(R.GenerateError):
            R.generate("run/v1", params)
        return
    assert R.generate("run/v1", params) == expected


def _pod(labels, container, restart="Always"):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "foo", "labels": labels},
            "spec": {"containers": [dict({"name": "foo", "image": "someimage", "imagePullPolicy": "IfNotPresent"}, **container)],
                     "dnsPolicy": "ClusterFirst", "restartPolicy": restart}}


@pytest.mark.parametrize("params,expected", [
    ({"name": "foo", "image": "someimage", "port": ""}, _pod(RUN, {})),
    ({"name": "foo", "image": "someimage", "env": ["a", "c"]}, None),
    ({"name": "foo", "image": "someimage", "image-pull-policy": "Always", "env": ["a=b", "c=d"]},
     _pod(RUN, {"imagePullPolicy": "Always", "env": [{"name": "a", "value": "b"}, {"name": "c", "value": "d"}]})),
    ({"name": "foo", "image": "someimage", "port": "80"}, _pod(RUN, {"ports": [{"containerPort": 80}]})),
    ({"name": "foo", "image": "someimage", "port": "80", "hostport": "80"}, _pod(RUN, {"ports": [{"containerPort": 80, "hostPort": 80}]})),
    ({"name": "foo", "image": "someimage", "hostport": "80"}, None),
    ({"name": "foo", "image": "someimage", "replicas": "1", "labels": "foo=bar,baz=blah"}, _pod(FOOBAR, {})),
    ({"name": "foo", "image": "someimage", "replicas": "1", "labels": "foo=bar,baz=blah", "stdin": "true"},
     _pod(FOOBAR, {"stdin": True, "stdinOnce": True})),
    ({"name": "foo", "image": "someimage", "replicas": "1", "labels": "foo=bar,baz=blah", "stdin": "true", "leave-stdin-open": "true"},
     _pod(FOOBAR, {"stdin": True})),
])
def test_generate_pod(params, expected):
    if expected is None:
        with pytest.raises(R.GenerateError):
            R.generate("run-pod/v1", params)
        return
    assert R.generate("run-pod/v1", params) == expected


FULL = {"name": "foo", "image": "someimage", "replicas": "3", "labels": "foo=bar,baz=blah", "port": "80", "hostport": "80",
        "stdin": "true", "command": "true", "args": ["bar", "baz", "blah"], "env": ["a=b", "c=d"],
        "requests": "cpu=100m,memory=100Mi", "limits": "cpu=400m,memory=200Mi"}
FULL_CTR = {"name": "foo", "image": "someimage", "stdin": True, "command": ["bar", "baz", "blah"],
            "ports": [{"containerPort": 80, "hostPort": 80}], "env": [{"name": "a", "value": "b"}, {"name": "c", "value": "d"}],
            "resources": {"limits": {"cpu": "400m", "memory": "200Mi"}, "requests": {"cpu": "100m", "memory": "100Mi"}}}


def test_generate_deployment_job_cronjob():
    for gen, api in (("deployment/v1beta1", "extensions/v1beta1"), ("deployment/apps.v1beta1", "apps/v1beta1")):
        assert R.generate(gen, FULL) == {
            "apiVersion": api, "kind": "Deployment", "metadata": {"name": "foo", "labels": FOOBAR},
            "spec": {"replicas": 3, "selector": {"matchLabels": FOOBAR},
                     "template": {"metadata": {"labels": FOOBAR}, "spec": {"containers": [FULL_CTR]}}}}
    job_params = dict(FULL, **{"leave-stdin-open": "true"})
    job_params.pop("replicas")
    assert R.generate("job/v1", job_params) == {
        "apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "foo", "labels": FOOBAR},
        "spec": {"template": {"metadata": {"labels": FOOBAR},
                              "spec": {"containers": [FULL_CTR], "restartPolicy": "Never"}}}}
    for gen, api in (("cronjob/v2alpha1", "batch/v2alpha1"), ("cronjob/v1beta1", "batch/v1beta1")):
        cj = R.generate(gen, dict(job_params, schedule="0/5 * * * ?"))
        assert cj == {"apiVersion": api, "kind": "CronJob", "metadata": {"name": "foo", "labels": FOOBAR},
                      "spec": {"schedule": "0/5 * * * ?", "concurrencyPolicy": "Allow",
                               "jobTemplate": {"spec": {"template": {"metadata": {"labels": FOOBAR},
                                                                     "spec": {"containers": [FULL_CTR], "restartPolicy": "Never"}}}}}}
    with pytest.raises(R.GenerateError, match="Parameter: schedule is required"):
        R.generate("cronjob/v1beta1", job_params)


@pytest.mark.parametrize("envs,ok", [
    (["FOO=bar", "FOO_BAR=baz", "A.B=c", "-x=y", "a=b=c", "EMPTY="], True),
    (["=novalue"], False), (["novalue"], False), (["1FOO=bar"], False),
])
def test_parse_env(envs, ok):
    if ok:
        assert [e["name"] for e in R.parse_envs(envs)] == [e.split("=", 1)[0] for e in envs]
    else:
        with pytest.raises(R.GenerateError, match="invalid env"):
            R.parse_envs(envs)


def test_generate_service():
    assert R.generate_service({"name": "foo", "port": "80"}) == {
        "apiVersion": "v1", "kind": "Service", "metadata": {"name": "foo"},
        "spec": {"selector": {"run": "foo"}, "ports": [{"port": 80, "protocol": "TCP", "targetPort": 80}]}}
    assert R.generate_service({"name": "foo", "port": "80", "labels": "app=bar"}) == {
        "apiVersion": "v1", "kind": "Service", "metadata": {"name": "foo", "labels": {"app": "bar"}},
        "spec": {"selector": {"app": "bar"}, "ports": [{"port": 80, "protocol": "TCP", "targetPort": 80}]}}
    with pytest.raises(R.GenerateError):
        R.generate_service({"name": "foo"})


@pytest.mark.parametrize("args,msg", [
    ([], "NAME is required"),
    (["test"], "--image is required"),
    (["test", "--image", "#"], "Invalid image name"),
    (["test", "--image", "busybox", "--stdin", "--replicas", "2"], "stdin requires that replicas is 1"),
    (["test", "--image", "busybox", "--rm"], "rm should only be used for attached containers"),
    (["test", "--image", "busybox", "--attach", "--dry-run"], "can't be used with attached containers options"),
    (["test", "--image", "busybox", "--stdin", "--dry-run"], "can't be used with attached containers options"),
    (["test", "--image", "busybox", "--tty", "--stdin", "--dry-run"], "can't be used with attached containers options"),
    (["test", "--image", "busybox", "--tty"], "stdin is required for containers with -t/--tty"),
    (["test", "--image", "busybox", "--expose"], "--port must be set when exposing a service"),
    (["test", "--image", "busybox", "--restart", "Never", "--replicas", "2"], "--restart=Never requires that --replicas=1, found 2"),
    (["test", "--image", "busybox", "--image-pull-policy", "Sometimes"], "invalid image pull policy: Sometimes"),
])
def test_run_validations(args, msg):
    class NoServer:
        async def request(self, *a, **k):
            raise AssertionError("no request expected")
    rc, _, err = run(_kubectl(NoServer(), "run", *args))
    assert rc == 1 and msg in err


def test_image_reference_regexp():
    for good in ("busybox", "rocm/vector-add:6.2", "registry.local:5000/ns/img@sha256:" + "a" * 64, "a_b__c-d.e"):
        assert R.REFERENCE_RE.match(good), good
    for bad in ("#", "UPPER", "img:", "-lead", "a//b"):
        assert not R.REFERENCE_RE.match(bad), bad


# ---------------------------------------------------------------------------- scale
def test_scale_preconditions():
    rc = {"kind": "ReplicationController", "metadata": {"resourceVersion": "7"}, "spec": {"replicas": 1}}
    S.validate_preconditions(rc, -1, "")
    with pytest.raises(S.PreconditionError, match="Expected replicas to be 3, was 1"):
        S.validate_preconditions(rc, 3, "")
    with pytest.raises(S.PreconditionError, match="Expected resource version to be 1, was 7"):
        S.validate_preconditions(rc, -1, "1")
    job = {"kind": "Job", "metadata": {}, "spec": {}}
    with pytest.raises(S.PreconditionError, match="Expected parallelism to be 2, was nil"):
        S.validate_preconditions(job, 2, "")


# --------------------------------------------------------------------- live cluster
def test_commands_through_the_cluster():
    from amdkube.localcluster import LocalCluster, wait_pod

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            for n in ("p1", "p2"):
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": n, "labels": {"tier": "a"}},
                                "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}, "default")
            # label: no overwrite without --overwrite; --overwrite; -l; removal of an absent key
            rc, _, err = await _kubectl(c, "label", "pods", "p1", "tier=b")
            assert rc == 1 and "'tier' already has a value (a), and --overwrite is false" in err
            rc, out, _ = await _kubectl(c, "label", "pods", "p1", "tier=b", "--overwrite")
            assert rc == 0 and out == 'pod "p1" labeled\n'
            assert m.labels_of(await c.get("pods", "p1", "default"))["tier"] == "b"
            rc, out, _ = await _kubectl(c, "label", "pods", "-l", "tier=a", "gpu=yes")
            assert out == 'pod "p2" labeled\n'
            rc, out, _ = await _kubectl(c, "label", "pod/p1", "missing-")
            assert out == 'label "missing" not found.\npod "p1" not labeled\n'
            rc, out, _ = await _kubectl(c, "label", "pods", "--all", "zone=z1")
            assert sorted(out.splitlines()) == ['pod "p1" labeled', 'pod "p2" labeled']
            rc, out, _ = await _kubectl(c, "label", "pods", "p2", "--list")
            assert "gpu=yes" in out.splitlines() and "zone=z1" in out.splitlines()
            # --resource-version is a precondition
            rv = (await c.get("pods", "p1", "default"))["metadata"]["resourceVersion"]
            with pytest.raises(m.StatusError) as e:
                await _kubectl(c, "label", "pods", "p1", "x=1", "--resource-version", str(int(rv) - 1))
            assert e.value.code == 409
            rc, out, _ = await _kubectl(c, "label", "pods", "p1", "x=1", "--resource-version", rv)
            assert out == 'pod "p1" labeled\n'
            rc, _, err = await _kubectl(c, "label", "pods", "--all", "y=1", "--resource-version", rv)
            assert rc == 1 and "--resource-version may only be used with a single resource" in err
            # annotate
            rc, out, _ = await _kubectl(c, "annotate", "pods", "p1", "note=hello")
            assert out == 'pod "p1" annotated\n'
            rc, _, err = await _kubectl(c, "annotate", "pods", "p1", "note=again")
            assert rc == 1 and "--overwrite is false but found the following declared annotation(s): 'note' already has a value (hello)" in err
            rc, out, _ = await _kubectl(c, "annotate", "pods", "p1", "note-")
            assert "note" not in m.annotations_of(await c.get("pods", "p1", "default"))
            # scale
            await c.create({"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": "rs"},
                            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "rs"}},
                                     "template": {"metadata": {"labels": {"app": "rs"}},
                                                  "spec": {"containers": [{"name": "w", "image": "busybox", "command": ["sleep", "60"]}]}}}},
                           "default")
            rc, _, err = await _kubectl(c, "scale", "rs", "rs")
            assert rc == 1 and "The --replicas=COUNT flag is required" in err
            rc, _, err = await _kubectl(c, "scale", "rs", "rs", "--replicas", "3", "--current-replicas", "2")
            assert rc == 1 and "Expected replicas to be 2, was 1" in err
            rc, out, _ = await _kubectl(c, "scale", "rs", "rs", "--replicas", "3", "--current-replicas", "1", "--timeout", "30s")
            assert rc == 0 and out == 'replicaset "rs" scaled\n'
            st = (await c.get("replicasets", "rs", "default"))["status"]
            assert st["replicas"] == 3
            rc, out, _ = await _kubectl(c, "scale", "--replicas", "0", "rs/rs", "-o", "name")
            assert out == "replicaset/rs\n"
            rc, _, err = await _kubectl(c, "scale", "pods", "p1", "--replicas", "2")
            assert rc == 1 and "no scaler has been implemented for" in err
            # run: the default generators
            rc, out, _ = await _kubectl(c, "run", "web", "--image", "busybox", "--port", "80", "--expose", "-l", "app=web",
                                        tail=["sleep", "60"])
            assert rc == 0 and out == 'service "web" created\ndeployment "web" created\n'
            d = await c.get("deployments", "web", "default")
            assert d["spec"]["template"]["spec"]["containers"][0]["args"] == ["sleep", "60"]
            assert (await c.get("services", "web", "default"))["spec"]["selector"] == {"app": "web"}
            rc, out, _ = await _kubectl(c, "run", "once", "--image", "busybox", "--restart", "Never", "--command", tail=["true"])
            assert out == 'pod "once" created\n'
            assert (await c.get("pods", "once", "default"))["spec"]["containers"][0]["command"] == ["true"]
            rc, out, _ = await _kubectl(c, "run", "batch", "--image", "busybox", "--restart", "OnFailure", tail=["true"])
            assert out == 'job "batch" created\n'
            rc, out, _ = await _kubectl(c, "run", "tick", "--image", "busybox", "--schedule", "*/5 * * * *", "--restart", "OnFailure")
            assert out == 'cronjob "tick" created\n'
            rc, out, _ = await _kubectl(c, "run", "dry", "--image", "busybox", "--restart", "Never", "--dry-run", "-o", "json")
            assert '"kind": "Pod"' in out and await c.get_or_none("pods", "dry", "default") is None
            # attached, --rm, the exit code of a Never pod
            rc, out, _ = await _kubectl(c, "run", "say", "--image", "busybox", "--restart", "Never", "--attach", "--rm",
                                        "--command", tail=["sh", "-c", "echo said; exit 3"])
            assert rc == 3 and "said" in out
            for _ in range(50):
                if await c.get_or_none("pods", "say", "default") is None:
                    break
                await asyncio.sleep(0.1)
            assert await c.get_or_none("pods", "say", "default") is None
    run(go(), 120)


def test_delete_through_the_cluster():
    from amdkube.kubectl import delete as D
    from amdkube.localcluster import LocalCluster, wait_pod

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            for n in ("a1", "a2", "b1"):
                await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": n, "labels": {"g": n[0]}},
                                "spec": {"terminationGracePeriodSeconds": 2,
                                         "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}, "default")
            rc, _, err = await _kubectl(c, "delete")
            assert rc == 1 and "You must provide one or more resources by argument or filename." in err
            rc, _, err = await _kubectl(c, "delete", "pods")
            assert rc == 1 and "resource(s) were provided, but no name, label selector, or --all flag specified" in err
            rc, out, err = await _kubectl(c, "delete", "pod", "nope")
            assert rc == 1 and 'Error from server (NotFound): pods "nope" not found' in err
            rc, out, err = await _kubectl(c, "delete", "pod", "nope", "--ignore-not-found")
            assert rc == 0 and out == "No resources found\n" and err == ""
            rc, _, err = await _kubectl(c, "delete", "pod", "a1", "--now", "--grace-period", "5")
            assert rc == 1 and "--now and --grace-period cannot be specified together" in err
            rc, out, _ = await _kubectl(c, "delete", "pods", "-l", "g=a", "-o", "name")
            assert sorted(out.split()) == ["pod/a1", "pod/a2"]
            rc, out, err = await _kubectl(c, "delete", "pod", "b1", "--grace-period", "0", "--force")
            assert rc == 0 and D.IMMEDIATE_WARNING in err and out == 'pod "b1" deleted\n'
            # a workload: its pods are gone when the command returns
            await c.create({"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": "rs"},
                            "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "rs"}},
                                     "template": {"metadata": {"labels": {"app": "rs"}},
                                                  "spec": {"terminationGracePeriodSeconds": 1, "containers": [
                                                      {"name": "w", "image": "busybox", "command": ["sleep", "60"]}]}}}},
                           "default")
            for _ in range(100):
                if len((await c.list("pods", "default", "app=rs"))[0]) == 2:
                    break
                await asyncio.sleep(0.1)
            rc, out, _ = await _kubectl(c, "delete", "rs", "rs")
            assert rc == 0 and out == 'replicaset "rs" deleted\n'
            assert (await c.list("pods", "default", "app=rs"))[0] == []
            assert await c.get_or_none("replicasets", "rs", "default") is None
            rc, out, _ = await _kubectl(c, "delete", "pods", "--all")
            assert rc == 0
    run(go(), 120)


def test_get_through_the_cluster(tmp_path):
    from amdkube.localcluster import LocalCluster

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2, with_kubelet=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "s1"}, "spec": {"ports": [{"port": 80}]}},
                           "default")
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p1"},
                            "spec": {"containers": [{"name": "c", "image": "busybox"}]}}, "default")
            done = await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "done"},
                                   "spec": {"containers": [{"name": "c", "image": "busybox"}]}}, "default")
            done["status"] = {"phase": "Succeeded"}
            await c.update_status(done)
            # several types: a table each, names with the short form, a blank line between (stderr)
            rc, out, err = await _kubectl(c, "get", "pods,svc")
            lines = out.splitlines()
            assert rc == 0 and any(x.startswith("po/p1 ") for x in lines) and any(x.startswith("svc/s1 ") for x in lines)
            assert not any(x.startswith("po/done") for x in lines)               # finished pods hidden from lists
            rc, out, _ = await _kubectl(c, "get", "pods", "-a")
            assert "done" in out
            rc, out, _ = await _kubectl(c, "get", "pods", "done")                  # named: never hidden
            assert "done" in out
            rc, out, err = await _kubectl(c, "get", "all")
            assert "svc/kubernetes" in out and "po/p1" in out
            # NotFound does not stop the others, and is reported after them
            rc, out, err = await _kubectl(c, "get", "pods", "p1", "nope")
            assert rc == 1 and "p1" in out and 'Error from server (NotFound): pods "nope" not found' in err
            rc, out, err = await _kubectl(c, "get", "pods", "nope", "--ignore-not-found")
            assert rc == 0 and out == "" and err == ""
            rc, out, err = await _kubectl(c, "get", "pods", "-l", "none=here")
            assert rc == 0 and err.strip() == "No resources found."
            # generic printers: one object when one was named, a List otherwise
            rc, out, _ = await _kubectl(c, "get", "svc", "s1", "-o", "json")
            assert '"kind": "Service"' in out and '"kind": "List"' not in out
            rc, out, _ = await _kubectl(c, "get", "svc/s1", "pod/p1", "-o", "name")
            assert out.split() == ["service/s1", "pod/p1"]
            f = tmp_path / "s.yaml"
            f.write_text("apiVersion: v1\nkind: Service\nmetadata: {name: s1}\nspec: {ports: [{port: 80}]}\n")
            rc, out, _ = await _kubectl(c, "get", "-f", str(f))
            assert rc == 0 and out.splitlines()[1].startswith("s1 ")
    run(go(), 60)


def test_standard_error_message():
    from amdkube.kubectl.main import standard_error_message
    one = m.StatusError(422, "Invalid", 'Pod "x" is invalid: spec.containers[0].image: Required value',
                        {"kind": "Pod", "name": "x", "causes": [{"message": "spec.containers[0].image: Required value"}]})
    assert standard_error_message(one) == 'The Pod "x" is invalid: spec.containers[0].image: Required value'
    two = m.StatusError(422, "Invalid", "...", {"kind": "Pod", "name": "x", "causes": [{"message": "a: Required value"},
                                                                                     {"field": "b", "message": "Invalid value: 1"}]})
    assert standard_error_message(two) == 'The Pod "x" is invalid: \n* a: Required value\n* b: Invalid value: 1'
    assert standard_error_message(m.not_found("pods", "nope")) == 'Error from server (NotFound): pods "nope" not found'


def test_exec_exit_code_and_refusal(capfd):
    from amdkube.kubectl import main as km
    from amdkube.localcluster import LocalCluster, wait_pod

    async def go():
        async with LocalCluster(gpus="none", relist_period=0.2) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"},
                            "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}, "default")
            await wait_pod(c, "default", "p", ("Running",), 30)
            base = ["-s", lc.api.url, "--token", lc.api.loopback_token, "exec"]
            rc = await asyncio.to_thread(km.main, base + ["p", "--", "sh", "-c", "echo out; exit 3"])
            rc2 = await asyncio.to_thread(km.main, base + ["nope", "--", "true"])
            return rc, rc2
    rc, rc2 = run(go(), 90)
    err = capfd.readouterr().err
    assert rc == 3 and "command terminated with exit code 3" in err
    assert rc2 == 1 and 'Error from server (NotFound): pods "nope" not found' in err


def test_expose_through_the_cluster():
    """expose_test.go TestRunExposeService's cases (services, selector/labels/name flags,
    affinity, cluster IP, headless with and without a port, name truncation, multi-port and
    multi-protocol objects), against a live apiserver."""
    from amdkube.localcluster import LocalCluster

    async def go():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "baz"},
                            "spec": {"selector": {"app": "go"}, "ports": [{"port": 1}]}}, "default")

            async def expose(*args):
                rc, out, err = await _kubectl(c, "expose", *args)
                return rc, out, err
            rc, out, _ = await expose("service", "baz", "--protocol", "UDP", "--port", "14", "--name", "foo", "--labels", "svc=test")
            assert rc == 0 and out == 'service "foo" exposed\n'
            svc = await c.get("services", "foo", "default")
            assert svc["metadata"]["labels"] == {"svc": "test"} and svc["spec"]["selector"] == {"app": "go"}
            assert svc["spec"]["ports"] == [{"protocol": "UDP", "port": 14, "targetPort": 14}]
            rc, out, _ = await expose("service", "baz", "--selector", "func=stream", "--port", "14", "--name", "foo2",
                                      "-l", "svc=test", "--type", "LoadBalancer", "--session-affinity", "ClientIP")
            s2 = await c.get("services", "foo2", "default")
            assert s2["spec"]["selector"] == {"func": "stream"} and s2["spec"]["type"] == "LoadBalancer"
            assert s2["spec"]["sessionAffinity"] == "ClientIP" and s2["spec"]["ports"][0]["protocol"] == "TCP"
            rc, out, _ = await expose("service", "baz", "--port", "14", "--name", "hl", "--cluster-ip", "None")
            assert (await c.get("services", "hl", "default"))["spec"]["clusterIP"] == "None"
            await c.create({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "hsrc"},
                            "spec": {"selector": {"app": "go"}, "clusterIP": "None"}}, "default")
            rc, out, _ = await expose("service", "hsrc", "--name", "hl2", "--cluster-ip", "None", "--dry-run", "-o", "json")
            assert '"ports": []' in out and '"clusterIP": "None"' in out
            # a pod: its labels select it, its long name is cut to 63 characters
            long = "a-name-that-is-toooo-big-for-a-service-because-it-can-only-handle-63-characters"
            await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": long, "labels": {"svc": "frompod"}},
                            "spec": {"containers": [{"name": "c", "image": "busybox",
                                                     "ports": [{"containerPort": 90}, {"containerPort": 53, "protocol": "UDP"}]}]}},
                           "default")
            rc, out, _ = await expose("pod", long)
            assert out == f'service "{long[:63]}" exposed\n'
            sp = await c.get("services", long[:63], "default")
            assert sp["spec"]["ports"] == [{"name": "port-1", "protocol": "TCP", "port": 90, "targetPort": 90},
                                           {"name": "port-2", "protocol": "UDP", "port": 53, "targetPort": 53}]
            assert sp["metadata"]["labels"] == {"svc": "frompod"}
            # a deployment with matchExpressions cannot be exposed; unexposable kinds are refused
            await c.create({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d"},
                            "spec": {"selector": {"matchLabels": {"a": "b"}, "matchExpressions": [{"key": "x", "operator": "Exists"}]},
                                     "template": {"metadata": {"labels": {"a": "b", "x": "1"}},
                                                  "spec": {"containers": [{"name": "c", "image": "busybox"}]}}}}, "default")
            rc, _, err = await expose("deployment", "d", "--port", "80")
            assert rc == 1 and "couldn't retrieve selectors via --selector flag or introspection" in err
            await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm"}, "data": {}}, "default")
            rc, _, err = await expose("configmap", "cm", "--port", "80")
            assert rc == 1 and "cannot expose a { ConfigMap}" in err
            rc, _, err = await expose("service", "baz", "--name", "noport", "--selector", "a=b", "--port", "", "--target-port", "x")
            assert rc == 0
    run(go(), 60)
