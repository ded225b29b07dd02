"""kubectl autoscale against pkg/kubectl/autoscale_test.go (TestHPAGenerate) and
cmd/autoscale.go's flag validation and kind check."""
from __future__ import annotations

import pytest

from amdkube.kubectl import autoscale as AS
from tests.conftest import run
from tests.test_kubectl_commands_parity import _kubectl

REF = {"scaleRef-kind": "kind", "scaleRef-name": "name", "scaleRef-apiVersion": "apiVersion"}


@pytest.mark.parametrize("name,params,expected,err", [
    ("valid case", {"name": "foo", "min": "1", "max": "10", "cpu-percent": "80", **REF},
     {"apiVersion": "autoscaling/v1", "kind": "HorizontalPodAutoscaler", "metadata": {"name": "foo"},
      "spec": {"scaleTargetRef": {"kind": "kind", "name": "name", "apiVersion": "apiVersion"}, "maxReplicas": 10,
               "minReplicas": 1, "targetCPUUtilizationPercentage": 80}}, None),
    ("'name' is a required parameter", {"min": "1", "max": "10", "cpu-percent": "80", **REF}, None,
     "'name' is a required parameter."),
    ("'max' is a required parameter", {"default-name": "foo", "min": "1", "cpu-percent": "80", **REF}, None,
     "'max' is a required parameter."),
    ("'max' must be greater than or equal to 'min'", {"name": "foo", "min": "10", "max": "1", "cpu-percent": "80", **REF}, None,
     "'max' must be greater than or equal to 'min'."),
    ("cpu-percent must be an integer if specified", {"name": "foo", "min": "1", "max": "10", "cpu-percent": "", **REF}, None,
     'strconv.Atoi: parsing "": invalid syntax'),
    ("'min' must be an integer if specified", {"name": "foo", "min": "foo", "max": "10", "cpu-percent": "60", **REF}, None,
     'strconv.Atoi: parsing "foo": invalid syntax'),
    ("'max' must be an integer if specified", {"name": "foo", "min": "1", "max": "bar", "cpu-percent": "90", **REF}, None,
     'strconv.Atoi: parsing "bar": invalid syntax'),
    ("negative min and cpu are left to the server", {"default-name": "foo", "min": "-1", "max": "3", "cpu-percent": "-1", **REF},
     {"apiVersion": "autoscaling/v1", "kind": "HorizontalPodAutoscaler", "metadata": {"name": "foo"},
      "spec": {"scaleTargetRef": {"kind": "kind", "name": "name", "apiVersion": "apiVersion"}, "maxReplicas": 3}}, None),
])
def test_hpa_generate(name, params, expected, err):
    if err:
        with pytest.raises(AS.GenerateError) as e:
            AS.generate_hpa(params)
        assert str(e.value) == err, name
    else:
        assert AS.generate_hpa(params) == expected, name


@pytest.mark.parametrize("lo,hi,errs", [
    (-1, -1, ["--max=MAXPODS is required and must be at least 1, max: -1"]),
    (5, 3, ["--max=MAXPODS must be larger or equal to --min=MINPODS, max: 3, min: 5"]),
    (2, 0, ["--max=MAXPODS is required and must be at least 1, max: 0",
            "--max=MAXPODS must be larger or equal to --min=MINPODS, max: 0, min: 2"]),
    (1, 1, []),
])
def test_validate_flags(lo, hi, errs):
    assert AS.validate_flags(lo, hi) == errs


def test_autoscale_through_the_cluster():
    from amdkube.localcluster import LocalCluster

    async def body():
        async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "api"},
                   "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "api"}},
                            "template": {"metadata": {"labels": {"app": "api"}}, "spec": {"containers": [{"name": "c", "image": "x"}]}}}}
            await c.create(dep, "default")
            rc, out, err = await _kubectl(c, "autoscale", "deployment", "api", "--max", "5", "--cpu-percent", "70")
            assert (rc, out) == (0, 'deployment "api" autoscaled\n'), err
            hpa = await c.get("horizontalpodautoscalers.autoscaling", "api", "default")
            assert hpa["spec"]["scaleTargetRef"] == {"kind": "Deployment", "name": "api", "apiVersion": "apps/v1"}
            assert hpa["spec"]["maxReplicas"] == 5 and hpa["spec"]["targetCPUUtilizationPercentage"] == 70
            assert "minReplicas" not in hpa["spec"] or hpa["spec"]["minReplicas"] == 1     # the server defaults it
            rc, out, err = await _kubectl(c, "autoscale", "deployment", "api", "--min", "2")
            assert rc == 1 and "--max=MAXPODS is required and must be at least 1, max: -1" in err
            await c.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm"}}, "default")
            rc, out, err = await _kubectl(c, "autoscale", "configmap", "cm", "--max", "3")
            assert rc == 1 and "cannot autoscale a ConfigMap" in err
            rc, out, err = await _kubectl(c, "autoscale", "deployment", "api", "--max", "3", "--name", "other", "--dry-run", "-o", "json")
            assert rc == 0 and '"name": "other"' in out
            assert await c.get_or_none("horizontalpodautoscalers.autoscaling", "other", "default") is None
    run(body())
