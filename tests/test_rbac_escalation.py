"""RBAC privilege-escalation prevention (pkg/registry/rbac policybased storage).

Transcribed: pkg/registry/rbac/helpers_test.go TestIsOnlyMutatingGCFields and
pkg/registry/rbac/validation/rule_test.go TestDefaultRuleResolver. Then through an apiserver in
RBAC mode with token users: a namespace admin may create roles and bindings only within what
they hold, `bind` on a role lets them bind it anyway, updates are checked too, and
system:masters is never checked.
"""
from __future__ import annotations

import pytest

from amdkube.api import meta as m
from amdkube.apiserver import rbacescalation as E
from tests.conftest import run

RBAC = "rbac.authorization.k8s.io"


def _pod():
    return {"metadata": {"name": "p", "namespace": "ns", "annotations": {}}, "spec": {"restartPolicy": "Never"}}


@pytest.mark.parametrize("mutate,expected", [
    (lambda p: None, True),
    (lambda p: p["metadata"]["annotations"].update(foo="bar"), False),
    (lambda p: p["spec"].update(restartPolicy="Always"), False),
    (lambda p: p["metadata"].setdefault("ownerReferences", []).append({"name": "foo"}), True),
    (lambda p: (p["metadata"].setdefault("ownerReferences", []).append({"name": "foo"}),
                p["metadata"].update(finalizers=["final"])), True),
    (lambda p: (p["metadata"].setdefault("ownerReferences", []).append({"name": "foo"}),
                p["metadata"]["annotations"].update(foo="bar")), False),
    (lambda p: (p["metadata"].setdefault("ownerReferences", []).append({"name": "foo"}),
                p["spec"].update(restartPolicy="Always")), False),
], ids=["same", "only annotations", "only other", "only ownerRef", "ownerRef and finalizer", "and annotations", "and other"])
def test_is_only_mutating_gc_fields(mutate, expected):
    new = _pod()
    mutate(new)
    assert E.only_gc_fields(new, _pod()) is expected
    assert E.only_gc_fields(new, None) is False          # "and nil"


READ_PODS = {"verbs": ["GET", "WATCH"], "apiGroups": ["v1"], "resources": ["pods"]}
READ_SVCS = {"verbs": ["GET", "WATCH"], "apiGroups": ["v1"], "resources": ["services"]}
WRITE_NODES = {"verbs": ["PUT", "CREATE", "UPDATE"], "apiGroups": ["v1"], "resources": ["nodes"]}
ADMIN = {"verbs": ["*"], "apiGroups": ["*"], "resources": ["*"]}


class StaticRoles:
    def __init__(self):
        self.objs = {
            "roles": [{"metadata": {"namespace": "namespace1", "name": "readthings"}, "rules": [READ_PODS, READ_SVCS]}],
            "clusterroles": [{"metadata": {"name": "cluster-admin"}, "rules": [ADMIN]},
                             {"metadata": {"name": "write-nodes"}, "rules": [WRITE_NODES]}],
            "rolebindings": [{"metadata": {"namespace": "namespace1", "name": "b"},
                              "subjects": [{"kind": "User", "name": "foobar"}, {"kind": "Group", "name": "group1"}],
                              "roleRef": {"apiGroup": RBAC, "kind": "Role", "name": "readthings"}}],
            "clusterrolebindings": [{"metadata": {"name": "cb"},
                                     "subjects": [{"kind": "User", "name": "admin"}, {"kind": "Group", "name": "admin"}],
                                     "roleRef": {"apiGroup": RBAC, "kind": "ClusterRole", "name": "cluster-admin"}}]}

    def rs(self, plural, group):
        objs = self.objs[plural]

        class L:
            @staticmethod
            def list():
                return objs, "1"
        return L

    def get_object(self, plural, ns, name):
        return next((o for o in self.objs[plural] if m.name_of(o) == name and (m.namespace_of(o) or "") == ns), None)


@pytest.mark.parametrize("user,ns,rules", [
    ({"name": "foobar"}, "namespace1", [READ_PODS, READ_SVCS]),
    ({"name": "foobar"}, "namespace2", []),
    ({"name": "foobar", "groups": ["admin"]}, "", [ADMIN]),
    ({}, "", []),
])
def test_default_rule_resolver(user, ns, rules):
    assert E.RuleResolver(StaticRoles()).rules_for(user, ns) == rules


def test_compact_string():
    assert E.compact({"verbs": ["delete"], "apiGroups": [""], "resources": ["pods"]}) == \
        '{Resources:["pods"], APIGroups:[""], Verbs:["delete"]}'


def test_escalation_through_the_apiserver():
    from amdkube.client import Client
    from amdkube.localcluster import LocalCluster
    users = {"alice-token": {"name": "alice", "groups": []}, "root-token": {"name": "root", "groups": ["system:masters"]}}

    async def go():
        async with LocalCluster(gpus="none", api_kw={"authorization_mode": "RBAC", "token_auth": users},
                                with_kubelet=False, with_controllers=False) as lc:
            c = lc.client
            await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team"}})
            # alice administers RBAC objects in "team" and may read pods there
            await c.create({"apiVersion": f"{RBAC}/v1", "kind": "Role", "metadata": {"name": "rbac-admin", "namespace": "team"},
                            "rules": [{"apiGroups": [RBAC], "resources": ["roles", "rolebindings"], "verbs": ["*"]},
                                      {"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "list"]}]}, "team")
            await c.create({"apiVersion": f"{RBAC}/v1", "kind": "RoleBinding", "metadata": {"name": "alice", "namespace": "team"},
                            "subjects": [{"kind": "User", "name": "alice"}],
                            "roleRef": {"apiGroup": RBAC, "kind": "Role", "name": "rbac-admin"}}, "team")
            await c.create({"apiVersion": f"{RBAC}/v1", "kind": "ClusterRole", "metadata": {"name": "pod-deleter"},
                            "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["delete"]}]})
            alice = Client(lc.api.url, token="alice-token")
            root = Client(lc.api.url, token="root-token")
            try:
                ok = await alice.create({"apiVersion": f"{RBAC}/v1", "kind": "Role", "metadata": {"name": "reader"},
                                         "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get"]}]}, "team")
                assert m.name_of(ok) == "reader"
                with pytest.raises(m.StatusError) as e:
                    await alice.create({"apiVersion": f"{RBAC}/v1", "kind": "Role", "metadata": {"name": "deleter"},
                                        "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "delete"]}]}, "team")
                assert e.value.code == 403 and e.value.message.startswith(
                    'roles.rbac.authorization.k8s.io "deleter" is forbidden: attempt to grant extra privileges: '
                    '[PolicyRule{Resources:["pods"], APIGroups:[""], Verbs:["delete"]}] user=&{alice')
                # updates are checked: widening her own readable role
                r = await alice.get(f"roles.{RBAC}", "reader", "team")
                r["rules"][0]["verbs"] = ["get", "delete"]
                with pytest.raises(m.StatusError) as e:
                    await alice.update(r)
                assert e.value.code == 403
                # a binding to a role she does not hold
                bind = {"apiVersion": f"{RBAC}/v1", "kind": "RoleBinding", "metadata": {"name": "deleters"},
                        "subjects": [{"kind": "User", "name": "alice"}],
                        "roleRef": {"apiGroup": RBAC, "kind": "ClusterRole", "name": "pod-deleter"}}
                with pytest.raises(m.StatusError) as e:
                    await alice.create(bind, "team")
                assert e.value.code == 403 and "attempt to grant extra privileges" in e.value.message
                # `bind` on that cluster role lets her bind it anyway
                await c.create({"apiVersion": f"{RBAC}/v1", "kind": "Role", "metadata": {"name": "binder", "namespace": "team"},
                                "rules": [{"apiGroups": [RBAC], "resources": ["clusterroles"], "verbs": ["bind"],
                                           "resourceNames": ["pod-deleter"]}]}, "team")
                await c.create({"apiVersion": f"{RBAC}/v1", "kind": "RoleBinding", "metadata": {"name": "alice-binder"},
                                "subjects": [{"kind": "User", "name": "alice"}],
                                "roleRef": {"apiGroup": RBAC, "kind": "Role", "name": "binder"}}, "team")
                assert m.name_of(await alice.create(bind, "team")) == "deleters"
                # system:masters is never checked
                assert m.name_of(await root.create({"apiVersion": f"{RBAC}/v1", "kind": "ClusterRole", "metadata": {"name": "anything"},
                                                    "rules": [ADMIN]})) == "anything"
            finally:
                await alice.close()
                await root.close()
    run(go(), 60)
