"""RBAC privilege-escalation prevention on role and binding writes.

Reference: pkg/registry/rbac/escalation_check.go (EscalationAllowed: members of system:masters;
BindingAuthorized: the `bind` verb on the referenced role, checked in the binding's namespace),
pkg/registry/rbac/{role,clusterrole,rolebinding,clusterrolebinding}/policybased/storage.go
(create and update of a role need the writer to hold every rule it grants; a binding needs
`bind` on its roleRef or every rule of the referenced role; an update that only touches
ownerReferences / finalizers — IsOnlyMutatingGCFields — is always allowed) and
pkg/registry/rbac/validation/rule.go ConfirmNoEscalation + DefaultRuleResolver.RulesFor (the
writer's rules: every ClusterRoleBinding naming them, plus the RoleBindings of the namespace).
The message is the reference's: `<resource> "<name>" is forbidden: attempt to grant extra
privileges: [...] user=&{...} ownerrules=[...] ruleResolutionErrors=[]`.

Writes the apiserver makes for itself (bootstrap policy, controllers running in-process: no
user) are never checked, as a system:masters loopback client is not.
"""
from __future__ import annotations

from ..api import meta as m
from ..api.rbac import covers

GROUP = "rbac.authorization.k8s.io"
PRIVILEGED_GROUP = "system:masters"
PLURALS = ("roles", "clusterroles", "rolebindings", "clusterrolebindings")


def escalation_allowed(user: dict | None) -> bool:
    return user is None or PRIVILEGED_GROUP in (user.get("groups") or [])


def _q(xs) -> str:
    return "[" + " ".join('"' + str(x).replace("\\", "\\\\").replace('"', '\\"') + '"' for x in xs) + "]"


def compact(rule: dict) -> str:
    """PolicyRule.CompactString."""
    parts = []
    for key, label in (("resources", "Resources"), ("nonResourceURLs", "NonResourceURLs"), ("resourceNames", "ResourceNames"),
                       ("apiGroups", "APIGroups"), ("verbs", "Verbs")):
        if rule.get(key):
            parts.append(f"{label}:{_q(rule[key])}")
    return "{" + ", ".join(parts) + "}"


def _rules_str(rules) -> str:
    return "[" + " ".join("PolicyRule" + compact(r) for r in rules) + "]"


def _user_str(user: dict) -> str:
    extra = user.get("extra") or {}
    ex = "map[" + " ".join(f"{k}:[{' '.join(v)}]" for k, v in sorted(extra.items())) + "]"
    return f"&{{{user.get('name', '')} {user.get('uid', '')} [{' '.join(user.get('groups') or [])}] {ex}}}"


class RuleResolver:
    """DefaultRuleResolver over the registry's stored roles and bindings."""

    def __init__(self, registry):
        self.registry = registry

    def _list(self, plural):
        return self.registry.rs(plural, GROUP).list()[0]

    def _get(self, plural, ns, name):
        return self.registry.get_object(plural, ns, name)

    def role_ref_rules(self, ref: dict, ns: str) -> list[dict]:
        """GetRoleReferenceRules."""
        kind = (ref or {}).get("kind")
        if kind == "ClusterRole":
            obj = self._get("clusterroles", "", ref.get("name", ""))
        elif kind == "Role":
            obj = self._get("roles", ns, ref.get("name", ""))
        else:
            raise m.bad_request(f"unsupported role reference kind: {kind!r}")
        if obj is None:
            raise m.not_found("clusterroles" if kind == "ClusterRole" else "roles", ref.get("name", ""))
        return list(obj.get("rules") or [])

    def rules_for(self, user: dict, ns: str) -> list[dict]:
        from .auth import subject_matches
        out = []
        for b in self._list("clusterrolebindings"):
            if any(subject_matches(s, user, "") for s in b.get("subjects") or []):
                try:
                    out += self.role_ref_rules(b.get("roleRef"), "")
                except m.StatusError:
                    pass
        if ns:
            for b in self._list("rolebindings"):
                if m.namespace_of(b) == ns and any(subject_matches(s, user, ns) for s in b.get("subjects") or []):
                    try:
                        out += self.role_ref_rules(b.get("roleRef"), ns)
                    except m.StatusError:
                        pass
        return out


def confirm_no_escalation(resolver: RuleResolver, user: dict, ns: str, rules: list[dict], plural: str, name: str):
    owner = resolver.rules_for(user, ns)
    ok, missing = covers(owner, rules)
    if not ok:
        raise m.StatusError(403, "Forbidden", f'{plural}.{GROUP} "{name}" is forbidden: attempt to grant extra privileges: '
                            f"{_rules_str(missing)} user={_user_str(user)} ownerrules={_rules_str(owner)} "
                            "ruleResolutionErrors=[]", {"name": name, "group": GROUP, "kind": plural})


def binding_authorized(authz, user: dict, ref: dict, ns: str) -> bool:
    """BindingAuthorized: `bind` on the roleRef, in the binding's namespace."""
    from .auth import Attributes
    if authz is None:
        return False
    kind = (ref or {}).get("kind")
    if kind not in ("ClusterRole", "Role"):
        return False
    a = Attributes(user, "bind", (ref or {}).get("apiGroup", GROUP), "clusterroles" if kind == "ClusterRole" else "roles",
                   "", ns, ref.get("name", ""))
    try:
        ok, _ = authz.authorize(a)
    except Exception:
        return False
    return bool(ok)


def only_gc_fields(new: dict, old: dict | None) -> bool:
    """IsOnlyMutatingGCFields: ownerReferences / finalizers are all that changed."""
    if old is None:
        return False
    a, b = m.deepcopy(new), m.deepcopy(old)
    for obj in (a, b):
        md = obj.setdefault("metadata", {})
        for k in ("ownerReferences", "finalizers", "selfLink", "resourceVersion", "generation", "managedFields"):
            md.pop(k, None)
    return a == b


def check(registry, plural: str, ns: str, obj: dict, user: dict | None, old: dict | None = None):
    """Raise Forbidden when `user` would escalate through this role/binding write (`registry`:
    the apiserver's Registry, with the authorizer it was given)."""
    if plural not in PLURALS or escalation_allowed(user):
        return
    if old is not None and only_gc_fields(obj, old):
        return
    resolver = RuleResolver(registry)
    name = m.name_of(obj)
    if plural in ("roles", "clusterroles"):
        confirm_no_escalation(resolver, user, ns, list(obj.get("rules") or []), plural, name)
        return
    ref = obj.get("roleRef") or {}
    if binding_authorized(getattr(registry, "authorizer", None), user, ref, ns):
        return
    rules = resolver.role_ref_rules(ref, ns)
    confirm_no_escalation(resolver, user, ns, rules, plural, name)
