"""configmap/v1 and secret/v1 generators against pkg/kubectl/configmap_test.go,
secret_test.go, env_file_test.go and util/hash/hash_test.go (the --append-hash names are the
reference's own vectors)."""
from __future__ import annotations

import pytest

from amdkube.kubectl import generators as G


@pytest.fixture
def env_file(tmp_path):
    def make(*lines):
        p = tmp_path / "file.env"
        p.write_text("\n".join(lines))
        return str(p)
    return make


@pytest.mark.parametrize("kw,name,data,err", [
    (dict(), "foo", {}, None),
    (dict(append_hash=True), "foo-867km9574f", {}, None),
    (dict(literal_sources=["key1=value1", "key2=value2"]), "foo", {"key1": "value1", "key2": "value2"}, None),
    (dict(literal_sources=["key1=value1", "key2=value2"], append_hash=True), "foo-gcb75dd9gb",
     {"key1": "value1", "key2": "value2"}, None),
    (dict(literal_sources=["key1value1"]), None, None, "invalid literal source key1value1, expected key=value"),
    (dict(file_sources=["key1=/file=2"]), None, None, "Key names or file paths cannot contain '='."),
    (dict(file_sources=["key1==value"]), None, None, "Key names or file paths cannot contain '='."),
    (dict(literal_sources=["key1==value1"]), "foo", {"key1": "=value1"}, None),
    (dict(literal_sources=["key1==value1"], append_hash=True), "foo-bdgk9ttt7m", {"key1": "=value1"}, None),
])
def test_config_map_generate(kw, name, data, err):
    if err:
        with pytest.raises(G.GenerateError) as e:
            G.generate_config_map("foo", **kw)
        assert str(e.value) == err
    else:
        cm = G.generate_config_map("foo", **kw)
        assert (cm["metadata"]["name"], cm["data"]) == (name, data)


def test_config_map_from_env_file(env_file, monkeypatch):
    path = env_file("key1=value1", "#", "", "key2=value2")
    assert G.generate_config_map("valid_env", env_file=path)["data"] == {"key1": "value1", "key2": "value2"}
    assert G.generate_config_map("valid_env", env_file=path, append_hash=True)["metadata"]["name"] == "valid_env-2cgh8552ch"
    monkeypatch.setenv("g_key1", "1")
    monkeypatch.setenv("g_key2", "2")
    path = env_file("g_key1", "g_key2=")
    cm = G.generate_config_map("getenv", env_file=path, append_hash=True)
    assert cm["data"] == {"g_key1": "1", "g_key2": ""} and cm["metadata"]["name"] == "getenv-b4hh92hgdk"
    with pytest.raises(G.GenerateError) as e:
        G.generate_config_map("too_many_args", literal_sources=["key1=value1"], env_file=path)
    assert str(e.value) == "from-env-file cannot be combined with from-file or from-literal"
    with pytest.raises(G.GenerateError) as e:
        G.generate_config_map("invalid_key", env_file=env_file("key#1=value1"))
    assert str(e.value).startswith('"key#1" is not a valid key name: ')
    # env_file_test.go: a BOM on the first line and leading whitespace are dropped
    assert G.env_file_pairs(env_file("﻿A=1", "   B=2 ", "  # c")) == [("A", "1"), ("B", "2 ")]


def test_config_map_keys_and_directories(tmp_path):
    d = tmp_path / "dir"
    d.mkdir()
    (d / "a.conf").write_text("A")
    (d / "b.conf").write_text("B")
    (d / "sub").mkdir()
    assert G.generate_config_map("x", file_sources=[str(d)])["data"] == {"a.conf": "A", "b.conf": "B"}
    assert G.generate_config_map("x", file_sources=[f"k={d / 'a.conf'}"])["data"] == {"k": "A"}
    with pytest.raises(G.GenerateError) as e:
        G.generate_config_map("x", file_sources=[f"k={d}"])
    assert str(e.value) == "cannot give a key name for a directory path."
    with pytest.raises(G.GenerateError) as e:
        G.generate_config_map("x", literal_sources=["a=1", "a=2"])
    assert str(e.value) == "cannot add key a, another key by that name already exists: map[a:1]."
    with pytest.raises(G.GenerateError) as e:
        G.generate_config_map("x", literal_sources=["a b=1"])
    assert str(e.value).startswith('"a b" is not a valid key name for a ConfigMap: ')
    with pytest.raises(G.GenerateError) as e:
        G.generate_config_map("")
    assert str(e.value) == "name must be specified"


@pytest.mark.parametrize("source,result,err", [
    ("foo", ("foo", "foo"), None),
    ("/some/dir/foo", ("foo", "/some/dir/foo"), None),
    ("k=v", ("k", "v"), None),
    ("=v", None, "key name for file path v missing."),
    ("k=", None, "file path for key name k missing."),
    ("a=b=c", None, "Key names or file paths cannot contain '='."),
])
def test_parse_file_source(source, result, err):
    if err:
        with pytest.raises(G.GenerateError) as e:
            G.parse_file_source(source)
        assert str(e.value) == err
    else:
        assert G.parse_file_source(source) == result


@pytest.mark.parametrize("kw,name,err", [
    (dict(), "foo", None),
    (dict(append_hash=True), "foo-949tdgdkgg", None),
    (dict(type_="my-type"), "foo", None),
    (dict(type_="my-type", append_hash=True), "foo-dg474f9t76", None),
    (dict(literal_sources=["key1=value1", "key2=value2"]), "foo", None),
    (dict(literal_sources=["key1=value1", "key2=value2"], append_hash=True), "foo-tf72c228m4", None),
    (dict(literal_sources=["key1value1"]), None, "invalid literal source key1value1, expected key=value"),
    (dict(literal_sources=["key1==value1"], append_hash=True), "foo-fdcc8tkhh5", None),
])
def test_secret_generate(kw, name, err):
    if err:
        with pytest.raises(G.GenerateError) as e:
            G.generate_secret("foo", **kw)
        assert str(e.value) == err
    else:
        assert G.generate_secret("foo", **kw)["metadata"]["name"] == name


@pytest.mark.parametrize("obj,encoded,h", [
    ({"data": {}}, '{"data":{},"kind":"ConfigMap","name":""}', "42745tchd9"),
    ({"data": {"one": ""}}, '{"data":{"one":""},"kind":"ConfigMap","name":""}', "9g67k2htb6"),
    ({"data": {"two": "2", "one": "", "three": "3"}}, '{"data":{"one":"","three":"3","two":"2"},"kind":"ConfigMap","name":""}',
     "f5h7t85m9b"),
])
def test_config_map_hash(obj, encoded, h):
    assert G.encode_config_map(obj) == encoded and G.config_map_hash(obj) == h


@pytest.mark.parametrize("obj,encoded,h", [
    ({"type": "my-type", "data": {}}, '{"data":{},"kind":"Secret","name":"","type":"my-type"}', "t75bgf6ctb"),
    ({"type": "my-type", "data": {"one": ""}}, '{"data":{"one":""},"kind":"Secret","name":"","type":"my-type"}', "74bd68bm66"),
    ({"type": "my-type", "data": {"two": "Mg==", "one": "", "three": "Mw=="}},
     '{"data":{"one":"","three":"Mw==","two":"Mg=="},"kind":"Secret","name":"","type":"my-type"}', "dgcb6h9tmk"),
])
def test_secret_hash(obj, encoded, h):
    assert G.encode_secret(obj) == encoded and G.secret_hash(obj) == h


def _svc_port(name, port, target):
    return {"name": name, "protocol": "TCP", "port": port, "targetPort": target}


@pytest.mark.parametrize("name,tcp,cip,type_,ports,err", [
    ("clusterip-ok", ["456", "321:908"], "", "ClusterIP", [_svc_port("456", 456, 456), _svc_port("321-908", 321, 908)], None),
    ("clusterip-missing", None, "", "ClusterIP", None, "at least one tcp port specifier must be provided"),
    ("clusterip-none-wrong-type", [], "None", "NodePort", None, "ClusterIP=None can only be used with ClusterIP service type"),
    ("clusterip-none-ok", [], "None", "ClusterIP", [], None),
    ("clusterip-none-and-port-mapping", ["456:9898"], "None", "ClusterIP", [_svc_port("456-9898", 456, 9898)], None),
    ("loadbalancer-ok", ["456:9898"], "", "LoadBalancer", [_svc_port("456-9898", 456, 9898)], None),
    ("invalid-port", ["65536"], "None", "ClusterIP", None, "must be between 1 and 65535, inclusive"),
    ("invalid-port-mapping", ["8080:-abc"], "None", "ClusterIP", None, "must not begin or end with a hyphen"),
    ("", None, "", "", None, "name must be specified"),
    ("named-target", ["80:http"], "", "ClusterIP", [_svc_port("80-http", 80, "http")], None),
])
def test_service_common_generate(name, tcp, cip, type_, ports, err):
    if err:
        with pytest.raises(G.GenerateError) as e:
            G.generate_service(name, type_, tcp, cip)
        assert err in str(e.value)
    else:
        svc = G.generate_service(name, type_, tcp, cip)
        assert svc["metadata"] == {"name": name, "labels": {"app": name}} and svc["spec"]["ports"] == ports
        assert svc["spec"]["type"] == type_ and svc["spec"]["selector"] == {"app": name}
        assert svc["spec"].get("clusterIP", "") == cip


def test_service_external_name_and_node_port():
    svc = G.generate_service("ext", "ExternalName", external_name="db.example.com")
    assert svc["spec"]["externalName"] == "db.example.com" and svc["spec"]["ports"] == []
    with pytest.raises(G.GenerateError) as e:
        G.generate_service("ext", "ExternalName", external_name="Not_A_Name")
    assert str(e.value) == "invalid service external name Not_A_Name"
    assert G.generate_service("np", "NodePort", ["80:8080"], node_port=30080)["spec"]["ports"][0]["nodePort"] == 30080


HARD = "cpu=10,memory=10Gi,pods=10"


@pytest.mark.parametrize("name,hard,scopes,spec,err", [
    ("foo", HARD, "", {"hard": {"cpu": "10", "memory": "10Gi", "pods": "10"}}, None),           # test_valid_case
    ("", HARD, "", None, "name must be specified"),                                             # test_missing_required_param
    ("foo", HARD, "BestEffort,NotTerminating", {"hard": {"cpu": "10", "memory": "10Gi", "pods": "10"},
                                                 "scopes": ["BestEffort", "NotTerminating"]}, None),
    ("foo", HARD, "", {"hard": {"cpu": "10", "memory": "10Gi", "pods": "10"}}, None),            # empty scopes
    ("foo", HARD, "abc,", None, 'invalid resource quota scope ""'),
    ("foo", "cpu", "", None, "Invalid argument syntax cpu, expected <resource>=<value>"),
    ("foo", "cpu=ten", "", None, "quantities must match the regular expression"),
])
def test_quota_generate(name, hard, scopes, spec, err):
    if err:
        with pytest.raises(G.GenerateError) as e:
            G.generate_quota(name, hard, scopes)
        assert str(e.value).startswith(err)
    else:
        assert G.generate_quota(name, hard, scopes)["spec"] == spec


@pytest.mark.parametrize("kw,spec,err", [
    (dict(min_available="1", selector="app=rails"), {"selector": {"matchLabels": {"app": "rails"}, "matchExpressions": []},
                                                     "minAvailable": 1}, None),
    (dict(max_unavailable="50%", selector="app=rails"), {"selector": {"matchLabels": {"app": "rails"}, "matchExpressions": []},
                                                         "maxUnavailable": "50%"}, None),
    (dict(min_available="1", max_unavailable="1", selector="app=rails"), None,
     "min-available and max-unavailable cannot be both specified"),
    (dict(selector="app=rails"), None, "one of min-available or max-unavailable must be specified"),
    (dict(min_available="1"), None, "a selector must be specified"),
    (dict(min_available="1", selector="tier in (web,api),!legacy"),
     {"selector": {"matchLabels": {}, "matchExpressions": [{"key": "tier", "operator": "In", "values": ["api", "web"]},
                                                            {"key": "legacy", "operator": "DoesNotExist"}]}, "minAvailable": 1}, None),
    (dict(min_available="1", selector="app!=rails"), None, '"!=" is not a valid label selector operator'),
])
def test_pdb_v2_generate(kw, spec, err):
    if err:
        with pytest.raises(G.GenerateError) as e:
            G.generate_pdb("foo", **kw)
        assert str(e.value) == err
    else:
        assert G.generate_pdb("foo", **kw)["spec"] == spec


RB = "rbac.authorization.k8s.io"


def test_role_binding_generate():
    rb = G.generate_role_binding("RoleBinding", "foo", role="admin", users=["user2", "user1", "user1"], groups=["group1"],
                                 service_accounts=["ns1:name1"])
    assert rb["roleRef"] == {"apiGroup": RB, "kind": "Role", "name": "admin"}
    assert rb["subjects"] == [{"kind": "User", "apiGroup": RB, "name": "user1"}, {"kind": "User", "apiGroup": RB, "name": "user2"},
                              {"kind": "Group", "apiGroup": RB, "name": "group1"},
                              {"kind": "ServiceAccount", "namespace": "ns1", "name": "name1"}]
    assert G.generate_role_binding("RoleBinding", "foo", cluster_role="view")["roleRef"]["kind"] == "ClusterRole"
    for kw, err in ((dict(role="a", cluster_role="b"), "exactly one of clusterrole or role must be specified"),
                    (dict(), "exactly one of clusterrole or role must be specified"),
                    (dict(role="a", service_accounts=["ns1"]), "serviceaccount must be <namespace>:<name>"),
                    (dict(role="a", service_accounts=["ns1:"]), "serviceaccount must be <namespace>:<name>")):
        with pytest.raises(G.GenerateError) as e:
            G.generate_role_binding("RoleBinding", "foo", **kw)
        assert str(e.value) == err
    with pytest.raises(G.GenerateError) as e:
        G.generate_role_binding("RoleBinding", "", role="a")
    assert str(e.value) == "name must be specified"


def test_cluster_role_binding_generate():
    crb = G.generate_role_binding("ClusterRoleBinding", "foo", cluster_role="admin", groups=["group2", "group1"])
    assert crb["roleRef"] == {"apiGroup": RB, "kind": "ClusterRole", "name": "admin"}
    assert [s["name"] for s in crb["subjects"]] == ["group1", "group2"]
    with pytest.raises(G.GenerateError) as e:
        G.generate_role_binding("ClusterRoleBinding", "foo", role="admin")
    assert str(e.value) == "clusterrole must be specified"


def test_create_role_rules():
    """create_role_test.go TestCreateRole: one rule per group, sorted, subresources kept. amdkube
    serves Deployments from apps first, where the reference's 1.9 RESTMapper picks extensions."""
    role = G.generate_role("Role", "my-role", ["get", "watch", "list"], ["pods", "deployments.extensions", "pods/status"],
                           ["foo"])
    assert role["rules"] == [
        {"verbs": ["get", "watch", "list"], "apiGroups": [""], "resources": ["pods", "pods/status"], "resourceNames": ["foo"]},
        {"verbs": ["get", "watch", "list"], "apiGroups": ["extensions"], "resources": ["deployments"], "resourceNames": ["foo"]}]
    assert G.generate_role("Role", "r", ["get", "*", "list"], ["po"])["rules"][0] == {"verbs": ["*"], "apiGroups": [""],
                                                                                       "resources": ["pods"]}


@pytest.mark.parametrize("verbs,resources,err", [
    ([], ["pods"], "at least one verb must be specified"),
    (["get"], [], "at least one resource must be specified"),
    (["invalid-verb"], ["pods"], "invalid verb: 'invalid-verb'"),
    (["get"], [".extensions"], "resource must be specified if apiGroup/subresource specified"),
    (["use"], ["pods"], "can not perform 'use' on 'pods' in group ''"),
    (["use"], ["podsecuritypolicies.extensions"], None),
    (["bind"], ["roles.rbac.authorization.k8s.io"], None),
    (["impersonate"], ["users", "serviceaccounts", "groups"], None),
    (["impersonate"], ["nodes"], "can not perform 'impersonate' on 'nodes' in group ''"),
])
def test_create_role_validate(verbs, resources, err):
    if err:
        with pytest.raises(G.GenerateError) as e:
            G.generate_role("Role", "my-role", verbs, resources)
        assert str(e.value) == err
    else:
        G.generate_role("Role", "my-role", verbs, resources)


def test_create_cluster_role_non_resource_urls():
    cr = G.generate_role("ClusterRole", "metrics", ["get"], [], non_resource_urls=["/metrics", "/healthz"])
    assert cr["rules"] == [{"verbs": ["get"], "nonResourceURLs": ["/metrics", "/healthz"]}]


def test_docker_registry_secret():
    """secret_for_docker_registry_test.go: compact .dockerconfigjson with username, password,
    optional email and auth; the required fields and --append-hash."""
    import argparse
    import base64
    import json as _json
    from amdkube.kubectl.more import create_more
    from tests.conftest import run

    def args(**kw):
        base = dict(docker_username="test-user", docker_password="test-password", docker_email="test-user@example.org",
                    docker_server="https://index.docker.io/v1/", append_hash=False)
        base.update(kw)
        return argparse.Namespace(**base)
    sec = run(create_more(None, args(), "secret", ["docker-registry", "foo"]))
    raw = base64.b64decode(sec["data"][".dockerconfigjson"]).decode()
    auth = base64.b64encode(b"test-user:test-password").decode()
    assert raw == ('{"auths":{"https://index.docker.io/v1/":{"username":"test-user","password":"test-password",'
                   '"email":"test-user@example.org","auth":"' + auth + '"}}}')
    assert sec["type"] == "kubernetes.io/dockerconfigjson"
    no_email = _json.loads(base64.b64decode(run(create_more(None, args(docker_email=""), "secret",
                                                            ["docker-registry", "foo"]))["data"][".dockerconfigjson"]))
    assert "email" not in no_email["auths"]["https://index.docker.io/v1/"]
    hashed = run(create_more(None, args(append_hash=True), "secret", ["docker-registry", "foo"]))
    assert hashed["metadata"]["name"] == "foo-" + G.secret_hash({**sec, "metadata": {"name": "foo"}})
    for kw, msg in ((dict(docker_username=""), "username must be specified"),
                    (dict(docker_password=""), "password must be specified")):
        with pytest.raises(SystemExit) as e:
            run(create_more(None, args(**kw), "secret", ["docker-registry", "foo"]))
        assert str(e.value) == f"error: {msg}"


def test_tls_secret(tmp_path):
    """secret_for_tls_test.go: the pair must load; key and certificate are required."""
    import argparse
    import subprocess
    from amdkube.kubectl.more import create_more
    from tests.conftest import run
    crt, key = tmp_path / "tls.crt", tmp_path / "tls.key"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-subj", "/CN=test", "-days", "1",
                    "-keyout", str(key), "-out", str(crt)], check=True, capture_output=True)
    sec = run(create_more(None, argparse.Namespace(cert=str(crt), key=str(key), append_hash=False), "secret", ["tls", "foo"]))
    assert sec["type"] == "kubernetes.io/tls" and set(sec["data"]) == {"tls.crt", "tls.key"}
    for kw, msg in ((dict(cert=str(crt), key=""), "error: key must be specified"),
                    (dict(cert="", key=str(key)), "error: certificate must be specified"),
                    (dict(cert=str(key), key=str(key)), "error: failed to load key pair")):
        with pytest.raises(SystemExit) as e:
            run(create_more(None, argparse.Namespace(append_hash=False, **kw), "secret", ["tls", "foo"]))
        assert str(e.value).startswith(msg)


@pytest.mark.parametrize("kind", ["namespace", "serviceaccount"])
def test_namespace_and_serviceaccount_need_a_name(kind):
    """namespace_test.go / serviceaccount_test.go: a generator without a name fails."""
    from tests.conftest import run
    from tests.test_kubectl_commands_parity import _kubectl

    class NoServer:
        async def create(self, *a, **k):
            raise AssertionError("no request expected")
    with pytest.raises(SystemExit) as e:
        run(_kubectl(NoServer(), "create", kind))
    assert str(e.value) == "error: name must be specified"


def test_create_deployment_generator():
    """deployment_test.go: name and image required; the container is named after the image."""
    from tests.conftest import run
    from tests.test_kubectl_commands_parity import _kubectl

    class Capture:
        created = None

        async def create(self, obj, ns=""):
            Capture.created = obj
            return obj
    run(_kubectl(Capture(), "create", "deployment", "foo", "--image", "registry.example.com/team/nginx:1.13@sha256:abc"))
    ct = Capture.created["spec"]["template"]["spec"]["containers"][0]
    assert ct["name"] == "nginx" and Capture.created["spec"]["selector"] == {"matchLabels": {"app": "foo"}}
    for argv, msg in ((["create", "deployment", "foo"], "error: at least one image must be specified"),
                      (["create", "deployment", "--image", "x"], "error: name must be specified")):
        with pytest.raises(SystemExit) as e:
            run(_kubectl(Capture(), *argv))
        assert str(e.value) == msg
