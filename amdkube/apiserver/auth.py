"""Authentication and authorization for the apiserver.

Reference:
  * authenticators — staging/src/k8s.io/apiserver/pkg/authentication: token file
    (--token-auth-file), service-account JWTs (pkg/serviceaccount/jwt.go: iss
    "kubernetes/serviceaccount", claims kubernetes.io/serviceaccount/{namespace,
    service-account.name, service-account.uid, secret.name}; the token is valid only while its
    secret and service account exist), bootstrap tokens
    (plugin/pkg/auth/authenticator/token/bootstrap: `<id>.<secret>` checked against secret
    kube-system/bootstrap-token-<id>, user system:bootstrap:<id>, groups
    system:bootstrappers + auth-extra-groups), anonymous (system:anonymous /
    system:unauthenticated); authenticated users get system:authenticated.
  * authorizers — union in --authorization-mode order (first "allow" wins):
    AlwaysAllow, AlwaysDeny, RBAC (plugin/pkg/auth/authorizer/rbac/rbac.go +
    pkg/registry/rbac/validation/rule.go: ClusterRoleBindings, then RoleBindings in the
    request namespace; subjects User / Group / ServiceAccount; rules match verb, apiGroup,
    resource[/subresource], resourceNames, nonResourceURLs with a trailing `*`), Node
    (plugin/pkg/auth/authorizer/node: a kubelet identity system:node:<name> in group
    system:nodes may read what a node needs and write only its own Node and the pods bound
    to it).
  * bootstrap policy — plugin/pkg/auth/authorizer/rbac/bootstrappolicy/policy.go.

Service-account tokens are signed with HS256 under the apiserver's
--service-account-key-file (the image has no RSA library; the claims and the validation
rules match the reference). RBAC decisions come from a rule index that is rebuilt lazily
when an RBAC object commits.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import time

from ..api import meta as m

SA_ISSUER = "kubernetes/serviceaccount"
SA_PREFIX = "system:serviceaccount:"


# ------------------------------------------------------------------------ JWT (HS256)
def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _unb64(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def jwt_sign(claims: dict, key: bytes) -> str:
    head = _b64(json.dumps({"alg": "HS256", "typ": "JWT"}, separators=(",", ":")).encode())
    body = _b64(json.dumps(claims, separators=(",", ":"), sort_keys=True).encode())
    sig = hmac.new(key, f"{head}.{body}".encode(), hashlib.sha256).digest()
    return f"{head}.{body}.{_b64(sig)}"


def jwt_verify(token: str, key: bytes) -> dict | None:
    try:
        head, body, sig = token.split(".")
        if json.loads(_unb64(head)).get("alg") != "HS256":
            return None
        want = hmac.new(key, f"{head}.{body}".encode(), hashlib.sha256).digest()
        if not hmac.compare_digest(want, _unb64(sig)):
            return None
        claims = json.loads(_unb64(body))
    except (ValueError, TypeError):
        return None
    if claims.get("exp") and time.time() > claims["exp"]:
        return None
    return claims


def service_account_token(key: bytes, ns: str, sa_name: str, sa_uid: str, secret_name: str) -> str:
    return jwt_sign({"iss": SA_ISSUER, "sub": f"{SA_PREFIX}{ns}:{sa_name}",
                     "kubernetes.io/serviceaccount/namespace": ns,
                     "kubernetes.io/serviceaccount/service-account.name": sa_name,
                     "kubernetes.io/serviceaccount/service-account.uid": sa_uid,
                     "kubernetes.io/serviceaccount/secret.name": secret_name}, key)


# -------------------------------------------------------------------- authentication
class Authenticator:
    def __init__(self, registry, tokens: dict | None = None, sa_key: bytes | None = None, anonymous: bool = True,
                 bootstrap_tokens: bool = True):
        self.registry, self.tokens, self.sa_key = registry, tokens or {}, sa_key
        self.anonymous, self.bootstrap = anonymous, bootstrap_tokens

    user_tokens = None   # token-file entries besides the loopback token (None: count them all)
    basic = None         # authx.BasicAuthenticator (--basic-auth-file)
    oidc = None          # authx.OIDCAuthenticator (--oidc-*)
    webhook = None       # authx.WebhookTokenAuthenticator (--authentication-token-webhook-config-file)

    @property
    def secured(self) -> bool:
        n = len(self.tokens) if self.user_tokens is None else self.user_tokens
        return n > 0 or self.sa_key is not None or any(x is not None for x in (self.basic, self.oidc, self.webhook))

    async def authenticate_token_async(self, tok: str) -> dict | None:
        """Local token authenticators first, then OIDC (tokens from its issuer), then the webhook."""
        u = self.authenticate_token(tok)
        if u is None and self.oidc is not None and self.oidc.claims_issuer(tok):
            u = await self.oidc.authenticate(tok)
        if u is None and self.webhook is not None:
            u = await self.webhook.authenticate(tok)
        return self._with_authenticated(u) if u is not None else None

    async def authenticate_async(self, headers, peercert: dict | None = None, peer_der: bytes | None = None) -> dict:
        h = headers.get("Authorization", "")
        if h.startswith("Bearer ") and (self.oidc is not None or self.webhook is not None) and \
                self._from_request_headers(headers, peercert, peer_der) is None:
            u = await self.authenticate_token_async(h[7:].strip())
            if u is None:
                raise m.unauthorized()
            return u
        return self.authenticate(headers, peercert, peer_der)

    def authenticate_token(self, tok: str) -> dict | None:
        u = self.tokens.get(tok)
        if u is not None:
            return self._with_authenticated(u)
        if self.sa_key is not None and tok.count(".") == 2:
            c = jwt_verify(tok, self.sa_key)
            if c and c.get("iss") == SA_ISSUER:
                ns = c.get("kubernetes.io/serviceaccount/namespace", "")
                sa = c.get("kubernetes.io/serviceaccount/service-account.name", "")
                sec = c.get("kubernetes.io/serviceaccount/secret.name", "")
                # the token dies with its secret or service account (jwt.go Validate lookups)
                sa_obj = self.registry.get_object("serviceaccounts", ns, sa)
                if sa_obj is None or m.uid_of(sa_obj) != c.get("kubernetes.io/serviceaccount/service-account.uid"):
                    return None
                if sec and self.registry.get_object("secrets", ns, sec) is None:
                    return None
                return self._with_authenticated({"name": f"{SA_PREFIX}{ns}:{sa}", "uid": m.uid_of(sa_obj),
                                                 "groups": ["system:serviceaccounts", f"system:serviceaccounts:{ns}"]})
        if self.bootstrap and "." in tok:
            tid, _, tsec = tok.partition(".")
            s = self.registry.get_object("secrets", "kube-system", f"bootstrap-token-{tid}")
            if s and s.get("type") == "bootstrap.kubernetes.io/token":
                d = {k: base64.b64decode(v).decode() for k, v in (s.get("data") or {}).items()}
                exp = m.parse_time(d.get("expiration"))
                if d.get("token-secret") == tsec and d.get("usage-bootstrap-authentication") == "true" and \
                        (exp is None or exp > time.time()):
                    extra = [g for g in (d.get("auth-extra-groups") or "").split(",") if g]
                    return self._with_authenticated({"name": f"system:bootstrap:{tid}", "uid": "",
                                                     "groups": ["system:bootstrappers", *extra]})
        return None

    @staticmethod
    def _with_authenticated(u: dict) -> dict:
        g = list(u.get("groups") or [])
        if "system:authenticated" not in g:
            g.append("system:authenticated")
        return dict(u, groups=g)

    @staticmethod
    def from_peer_cert(pc: dict) -> dict | None:
        """x509 request authenticator (authentication/request/x509: CommonNameUserConversion):
        a client certificate verified against --client-ca-file names the user in its CN and
        the groups in its O entries."""
        cn, groups = None, []
        for rdn in pc.get("subject") or ():
            for k, v in rdn:
                if k == "commonName":
                    cn = v
                elif k == "organizationName":
                    groups.append(v)
        return {"name": cn, "uid": "", "groups": groups} if cn else None

    requestheader: dict | None = None   # front-proxy (aggregator) authentication, see configure_requestheader

    def configure_requestheader(self, ca_file: str, allowed_names=(), username_headers=("X-Remote-User",),
                                group_headers=("X-Remote-Group",), extra_prefixes=("X-Remote-Extra-",)):
        """authentication/request/headerrequest: a client certificate issued by
        --requestheader-client-ca-file (and, with --requestheader-allowed-names, carrying one of
        those CNs) may assert the user in X-Remote-User / X-Remote-Group / X-Remote-Extra-*."""
        import ssl as _ssl
        from ..utils.crypto import x509_pem_to_der
        dec = _ssl._ssl._test_decode_cert(ca_file)
        with open(ca_file, "rb") as f:
            cas = x509_pem_to_der(f.read())
        self.requestheader = {"issuer": dec.get("subject"), "allowed": set(allowed_names or ()), "ca_der": cas,
                              "users": list(username_headers), "groups": list(group_headers), "extra": list(extra_prefixes)}

    def _from_request_headers(self, headers, peercert, peer_der: bytes | None = None) -> dict | None:
        """The peer certificate must be SIGNED by the requestheader CA (headerrequest verifies
        the chain against that pool alone): matching the issuer's name is not enough when the
        client CA carries the same subject."""
        from ..utils.crypto import x509_signed_by
        rh = self.requestheader
        if rh is None or not peercert or peercert.get("issuer") != rh["issuer"]:
            return None
        if peer_der is None or not any(x509_signed_by(peer_der, ca) for ca in rh.get("ca_der") or ()):
            return None
        cn = (self.from_peer_cert(peercert) or {}).get("name")
        if rh["allowed"] and cn not in rh["allowed"]:
            return None
        name = next((headers.get(h) for h in rh["users"] if headers.get(h)), None)
        if not name:
            return None
        getall = getattr(headers, "getall", None)
        groups = [g for h in rh["groups"] for g in ((getall(h, []) if getall else [headers.get(h)]) or []) if g]
        extra = {}
        for pre in rh["extra"]:
            for k in headers.keys():
                if k.lower().startswith(pre.lower()):
                    extra.setdefault(k[len(pre):].lower(), []).extend(getall(k, []) if getall else [headers.get(k)])
        return {"name": name, "uid": "", "groups": groups, "extra": extra}

    def authenticate(self, headers, peercert: dict | None = None, peer_der: bytes | None = None) -> dict:
        u = self._from_request_headers(headers, peercert, peer_der)
        if u is not None:
            return self._with_authenticated(u)
        h = headers.get("Authorization", "")
        if self.basic is not None and h.startswith("Basic "):
            return self._with_authenticated(self.basic.authenticate(h))
        if h.startswith("Bearer "):
            u = self.authenticate_token(h[7:].strip())
            if u is None:
                raise m.unauthorized()
            return u
        rh = self.requestheader
        if peercert and rh and peercert.get("issuer") == rh["issuer"] and not rh.get("client_ca_same"):
            peercert = None   # a front-proxy certificate is no x509 identity of its own (client-ca ≠ requestheader CA)
        if peercert:
            u = self.from_peer_cert(peercert)
            if u is not None:
                return self._with_authenticated(u)
        if self.secured and not self.anonymous:
            raise m.unauthorized()
        return {"name": "system:anonymous", "groups": ["system:unauthenticated"]}


# --------------------------------------------------------------------- authorization
class Attributes:
    __slots__ = ("user", "verb", "group", "resource", "subresource", "namespace", "name", "path", "resource_request")

    def __init__(self, user, verb, group="", resource="", subresource="", namespace="", name="", path="",
                 resource_request=True):
        self.user, self.verb, self.group, self.resource = user, verb, group, resource
        self.subresource, self.namespace, self.name, self.path = subresource, namespace, name, path
        self.resource_request = resource_request


def _has(lst, v) -> bool:
    return bool(lst) and ("*" in lst or v in lst)


def rule_allows(rule: dict, a: Attributes) -> bool:
    if not _has(rule.get("verbs") or [], a.verb):
        return False
    if not a.resource_request:
        for u in rule.get("nonResourceURLs") or []:
            if u == "*" or u == a.path or (u.endswith("*") and a.path.startswith(u[:-1])):
                return True
        return False
    if not _has(rule.get("apiGroups") or [], a.group):
        return False
    res = rule.get("resources") or []
    combined = f"{a.resource}/{a.subresource}" if a.subresource else a.resource
    if not ("*" in res or combined in res or (a.subresource and f"{a.resource}/*" in res) or
            (not a.subresource and a.resource in res) or (a.subresource and f"*/{a.subresource}" in res)):
        return False
    names = rule.get("resourceNames") or []
    return not names or a.name in names


def subject_matches(s: dict, user: dict, binding_ns: str) -> bool:
    kind = s.get("kind")
    if kind == "User":
        return s.get("name") == user.get("name")
    if kind == "Group":
        return s.get("name") in (user.get("groups") or [])
    if kind == "ServiceAccount":
        ns = s.get("namespace") or binding_ns
        return user.get("name") == f"{SA_PREFIX}{ns}:{s.get('name')}"
    return False


class RBACAuthorizer:
    name = "RBAC"

    def __init__(self, registry):
        self.registry = registry
        self._gen = 0
        self._built = -1
        self._crb: list = []
        self._rb: dict[str, list] = {}
        registry.store.commit_hooks.append(self._on_commit)

    def _on_commit(self, ev):
        k = ev.kv.key
        if k.startswith(("/registry/roles/", "/registry/clusterroles/", "/registry/rolebindings/",
                         "/registry/clusterrolebindings/")):
            self._gen += 1

    def _rebuild(self):
        reg = self.registry
        roles = {(m.namespace_of(r), m.name_of(r)): r.get("rules") or [] for r in reg.rs("roles", "rbac.authorization.k8s.io").list()[0]}
        croles = {m.name_of(r): r.get("rules") or [] for r in reg.rs("clusterroles", "rbac.authorization.k8s.io").list()[0]}

        def rules_for(ref, ns):
            if (ref or {}).get("kind") == "ClusterRole":
                return croles.get(ref.get("name"), [])
            return roles.get((ns, (ref or {}).get("name")), [])
        self._crb = [(b.get("subjects") or [], rules_for(b.get("roleRef"), ""))
                     for b in reg.rs("clusterrolebindings", "rbac.authorization.k8s.io").list()[0]]
        self._rb = {}
        for b in reg.rs("rolebindings", "rbac.authorization.k8s.io").list()[0]:
            ns = m.namespace_of(b)
            self._rb.setdefault(ns, []).append((b.get("subjects") or [], rules_for(b.get("roleRef"), ns)))
        self._built = self._gen

    def authorize(self, a: Attributes) -> tuple[bool, str]:
        if self._built != self._gen:
            self._rebuild()
        for subjects, rules in self._crb:
            if any(subject_matches(s, a.user, "") for s in subjects) and any(rule_allows(r, a) for r in rules):
                return True, "allowed by ClusterRoleBinding"
        if a.namespace:
            for subjects, rules in self._rb.get(a.namespace, ()):
                if any(subject_matches(s, a.user, a.namespace) for s in subjects) and any(rule_allows(r, a) for r in rules):
                    return True, "allowed by RoleBinding"
        return False, ""


class NodeAuthorizer:
    """A kubelet may read cluster objects it needs and write only its own node/pods/events."""
    name = "Node"
    READ = {"pods", "nodes", "services", "endpoints", "configmaps", "secrets", "persistentvolumeclaims",
            "persistentvolumes", "namespaces", "limitranges", "resourcequotas"}

    def __init__(self, registry):
        self.registry = registry

    def authorize(self, a: Attributes) -> tuple[bool, str]:
        u = a.user
        if "system:nodes" not in (u.get("groups") or []) or not u.get("name", "").startswith("system:node:"):
            return False, ""
        node = u["name"][len("system:node:"):]
        if not a.resource_request:
            return a.verb == "get" and a.path in ("/healthz", "/version", "/api", "/apis", "/openapi/v2", "/swagger.json"), ""
        if a.verb in ("get", "list", "watch") and a.resource in self.READ:
            return True, "node read"
        if a.resource == "nodes":
            if a.verb == "create" or a.name == node:
                return True, "node self"
            return False, ""
        if a.resource == "events" and a.verb in ("create", "update", "patch"):
            return True, "node events"
        if a.resource == "pods":
            if a.verb == "create" or (a.subresource == "eviction" and a.verb == "create"):
                return True, "mirror pods"
            pod = self.registry.get_object("pods", a.namespace, a.name) if a.name else None
            if pod is not None and (pod.get("spec") or {}).get("nodeName") == node:
                return True, "pod bound to node"
            return False, ""
        if a.resource == "certificatesigningrequests" and a.verb in ("create", "get", "list", "watch"):
            return True, "node CSR"
        return False, ""


class AlwaysAllow:
    name = "AlwaysAllow"

    def authorize(self, a):
        return True, ""


class AlwaysDeny:
    name = "AlwaysDeny"

    def authorize(self, a):
        return False, "AlwaysDeny"


class RBACLite:
    """amdkube's pre-RBAC mode: anonymous users are read-only, everyone else may do anything."""
    name = "RBACLite"

    def authorize(self, a):
        if "system:masters" in (a.user.get("groups") or []) or not a.user.get("name", "").startswith("system:anonymous"):
            return True, ""
        return a.verb in ("get", "list", "watch"), ""


class UnionAuthorizer:
    def __init__(self, modes: str, registry, policy_file: str | None = None, webhook_config: str | None = None,
                 webhook_authorized_ttl: float = 300.0, webhook_unauthorized_ttl: float = 30.0):
        def abac():
            from .authx import ABACAuthorizer
            if not policy_file:
                raise ValueError("authorization mode ABAC needs --authorization-policy-file")
            return ABACAuthorizer(policy_file)

        def webhook():
            from .authx import WebhookAuthorizer
            if not webhook_config:
                raise ValueError("authorization mode Webhook needs --authorization-webhook-config-file")
            return WebhookAuthorizer(webhook_config, webhook_authorized_ttl, webhook_unauthorized_ttl)
        table = {"AlwaysAllow": lambda: AlwaysAllow(), "AlwaysDeny": lambda: AlwaysDeny(), "RBAC": lambda: RBACAuthorizer(registry),
                 "Node": lambda: NodeAuthorizer(registry), "RBACLite": lambda: RBACLite(), "ABAC": abac, "Webhook": webhook}
        self.authorizers = []
        for mode in [x.strip() for x in modes.split(",") if x.strip()]:
            if mode not in table:
                raise ValueError(f"unknown authorization mode {mode!r}")
            self.authorizers.append(table[mode]())
        self.modes = [a.name for a in self.authorizers]

    def authorize(self, a: Attributes) -> tuple[bool, str]:
        if "system:masters" in (a.user.get("groups") or []):
            return True, "system:masters"
        for z in self.authorizers:
            ok, why = z.authorize(a)
            if ok:
                return True, why
        return False, ""

    async def authorize_async(self, a: Attributes) -> tuple[bool, str]:
        """The request path: authorizers that ask a remote service (Webhook) are awaited."""
        if "system:masters" in (a.user.get("groups") or []):
            return True, "system:masters"
        for z in self.authorizers:
            fn = getattr(z, "authorize_async", None)
            ok, why = (await fn(a)) if fn is not None else z.authorize(a)
            if ok:
                return True, why
        return False, ""


# ------------------------------------------------------------------ bootstrap policy
def _rule(verbs, groups, resources, names=None, urls=None):
    r = {"verbs": list(verbs)}
    if urls:
        r["nonResourceURLs"] = list(urls)
        return r
    r.update({"apiGroups": list(groups), "resources": list(resources)})
    if names:
        r["resourceNames"] = list(names)
    return r


READ = ("get", "list", "watch")
RW = ("get", "list", "watch", "create", "update", "patch", "delete", "deletecollection")
WORKLOAD_GROUPS = ("", "apps", "batch", "autoscaling", "policy")
WORKLOADS = ("pods", "pods/log", "pods/exec", "replicationcontrollers", "replicationcontrollers/scale", "services",
             "endpoints", "configmaps", "secrets", "persistentvolumeclaims", "serviceaccounts", "deployments",
             "deployments/scale", "replicasets", "replicasets/scale", "statefulsets", "statefulsets/scale", "daemonsets",
             "jobs", "cronjobs", "horizontalpodautoscalers", "poddisruptionbudgets", "events")


def bootstrap_cluster_roles() -> list[dict]:
    def cr(name, rules, **kw):
        return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                "metadata": {"name": name, "labels": {"kubernetes.io/bootstrapping": "rbac-defaults"},
                             "annotations": {"rbac.authorization.kubernetes.io/autoupdate": "true"}}, "rules": rules, **kw}
    return [
        cr("cluster-admin", [_rule(["*"], ["*"], ["*"]), _rule(["*"], [], [], urls=["*"])]),
        cr("admin", [_rule(RW, WORKLOAD_GROUPS, WORKLOADS),
                     _rule(RW, ["rbac.authorization.k8s.io"], ["roles", "rolebindings"])]),
        cr("edit", [_rule(RW, WORKLOAD_GROUPS, WORKLOADS)]),
        cr("view", [_rule(READ, WORKLOAD_GROUPS, [w for w in WORKLOADS if w not in ("secrets", "pods/exec")])]),
        cr("system:discovery", [_rule(["get"], [], [], urls=["/healthz", "/version", "/version/", "/api", "/api/*", "/apis",
                                                                  "/apis/*", "/swagger.json", "/swaggerapi", "/swaggerapi/*",
                                                                  "/openapi", "/openapi/*"])]),
        cr("system:basic-user", [_rule(["create"], ["authorization.k8s.io"], ["selfsubjectaccessreviews"])]),
        cr("system:node", [_rule(READ, [""], ["pods", "nodes", "services", "endpoints", "configmaps", "secrets",
                                                "persistentvolumeclaims", "persistentvolumes"]),
                           _rule(["create", "update", "patch", "delete"], [""], ["nodes", "nodes/status", "pods",
                                                                                 "pods/status", "pods/eviction"]),
                           _rule(["create", "update", "patch"], [""], ["events"]),
                           _rule(["create", "get", "list", "watch"], ["certificates.k8s.io"], ["certificatesigningrequests"])]),
        cr("system:node-proxier", [_rule(READ, [""], ["services", "endpoints", "nodes"]),
                                   _rule(["create", "update", "patch"], [""], ["events"])]),
        cr("system:kube-scheduler", [_rule(READ, ["", "apps", "policy", "storage.k8s.io"], ["*"]),
                                     _rule(["create"], [""], ["pods/binding", "bindings"]),
                                     _rule(["update", "patch"], [""], ["pods/status"]),
                                     _rule(["delete"], [""], ["pods"]),
                                     _rule(["create", "update", "patch"], [""], ["events"]),
                                     _rule(["get", "create", "update"], ["", "coordination.k8s.io"], ["endpoints", "leases"])]),
        cr("system:kube-controller-manager", [_rule(["*"], ["*"], ["*"])]),
        cr("system:node-bootstrapper", [_rule(["create", "get", "list", "watch"], ["certificates.k8s.io"],
                                              ["certificatesigningrequests"])]),
        cr("system:certificates.k8s.io:certificatesigningrequests:nodeclient",
           [_rule(["create"], ["certificates.k8s.io"], ["certificatesigningrequests/nodeclient"])]),
        cr("system:certificates.k8s.io:certificatesigningrequests:selfnodeclient",
           [_rule(["create"], ["certificates.k8s.io"], ["certificatesigningrequests/selfnodeclient"])]),
        # the AMD device-plugin DaemonSet reads nodes and posts events
        cr("amd.com:device-plugin", [_rule(READ, [""], ["nodes", "pods"]), _rule(["create", "patch"], [""], ["events"])]),
    ]


def bootstrap_cluster_role_bindings() -> list[dict]:
    def crb(name, role, subjects):
        return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                "metadata": {"name": name, "labels": {"kubernetes.io/bootstrapping": "rbac-defaults"}},
                "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": role},
                "subjects": subjects}
    g = lambda n: {"kind": "Group", "apiGroup": "rbac.authorization.k8s.io", "name": n}  # noqa: E731
    u = lambda n: {"kind": "User", "apiGroup": "rbac.authorization.k8s.io", "name": n}  # noqa: E731
    return [
        crb("cluster-admin", "cluster-admin", [g("system:masters")]),
        crb("system:discovery", "system:discovery", [g("system:authenticated"), g("system:unauthenticated")]),
        crb("system:basic-user", "system:basic-user", [g("system:authenticated"), g("system:unauthenticated")]),
        crb("system:node-proxier", "system:node-proxier", [u("system:kube-proxy")]),
        crb("system:kube-scheduler", "system:kube-scheduler", [u("system:kube-scheduler")]),
        crb("system:kube-controller-manager", "system:kube-controller-manager", [u("system:kube-controller-manager")]),
        crb("system:node-bootstrapper", "system:node-bootstrapper", [g("system:bootstrappers")]),
        crb("system:certificates.k8s.io:certificatesigningrequests:nodeclient",
            "system:certificates.k8s.io:certificatesigningrequests:nodeclient", [g("system:bootstrappers")]),
    ]


def ensure_bootstrap_policy(registry):
    """storage_rbac.go PostStartHook: create missing default roles and bindings."""
    for plural, objs in (("clusterroles", bootstrap_cluster_roles()), ("clusterrolebindings", bootstrap_cluster_role_bindings())):
        rs = registry.rs(plural, "rbac.authorization.k8s.io")
        for o in objs:
            if rs.storage.get(rs.key("", o["metadata"]["name"]), ignore_not_found=True) is None:
                rs.create("", o)
