"""Further apiserver authenticators and authorizers (the kube-apiserver flags of
pkg/kubeapiserver/authenticator/config.go and pkg/kubeapiserver/authorizer/config.go):

* `BasicAuthenticator` — --basic-auth-file: CSV `password,user,uid[,"group1,group2"]`,
  checked against `Authorization: Basic` (plugin/pkg/auth/authenticator/password/passwordfile).
* `WebhookTokenAuthenticator` — --authentication-token-webhook-config-file: bearer tokens no
  local authenticator knows are sent as authentication.k8s.io/v1beta1 TokenReview to the
  service named by a kubeconfig; answers are cached for --authentication-token-webhook-cache-ttl
  (plugin/pkg/auth/authenticator/token/webhook).
* `OIDCAuthenticator` — --oidc-issuer-url/--oidc-client-id/--oidc-ca-file/--oidc-username-claim/
  --oidc-username-prefix/--oidc-groups-claim/--oidc-groups-prefix: RS256 ID tokens checked
  against the issuer's JWKS (discovered from /.well-known/openid-configuration over TLS with
  the given CA), issuer, audience and expiry (plugin/pkg/auth/authenticator/token/oidc).
* `WebhookAuthorizer` — --authorization-mode=Webhook with --authorization-webhook-config-file:
  authorization.k8s.io/v1beta1 SubjectAccessReview, allowed answers cached for
  --authorization-webhook-cache-authorized-ttl and denials for ...-unauthorized-ttl
  (plugin/pkg/auth/authorizer/webhook).
* `ABACAuthorizer` — --authorization-mode=ABAC with --authorization-policy-file: one
  abac.authorization.kubernetes.io/v1beta1 Policy per line (pkg/auth/authorizer/abac).
"""
from __future__ import annotations

import base64
import csv
import hashlib
import hmac
import json
import time

from ..api import meta as m


class BasicAuthenticator:
    def __init__(self, path: str):
        self.users: dict[str, tuple[str, dict]] = {}
        with open(path) as f:
            for row in csv.reader(f):
                if len(row) < 3 or row[0].startswith("#"):
                    continue
                groups = [g.strip() for g in row[3].split(",")] if len(row) > 3 and row[3] else []
                self.users[row[1].strip()] = (row[0].strip(), {"name": row[1].strip(), "uid": row[2].strip(), "groups": groups})

    def authenticate(self, header: str) -> dict | None:
        """None when the header is no Basic credential; raises 401 for a wrong one."""
        if not header.startswith("Basic "):
            return None
        try:
            user, _, pw = base64.b64decode(header[6:].strip()).decode().partition(":")
        except (ValueError, UnicodeDecodeError):
            raise m.unauthorized()
        ent = self.users.get(user)
        if ent is None or not hmac.compare_digest(ent[0], pw):
            raise m.unauthorized()
        return dict(ent[1])


def _webhook_client(kubeconfig_path: str):
    """The webhook service from a kubeconfig (clusters[].cluster.server is the full URL)."""
    from ..client import Client
    return Client.from_kubeconfig(kubeconfig_path, timeout=30.0)


class _TTLCache:
    def __init__(self):
        self.d: dict[str, tuple[float, object]] = {}

    def get(self, k):
        hit = self.d.get(k)
        if hit is None or hit[0] < time.monotonic():
            return None
        return hit[1]

    def put(self, k, v, ttl: float):
        if ttl > 0:
            self.d[k] = (time.monotonic() + ttl, v)
            if len(self.d) > 10000:
                now = time.monotonic()
                self.d = {a: b for a, b in self.d.items() if b[0] >= now}


class WebhookTokenAuthenticator:
    def __init__(self, kubeconfig_path: str, cache_ttl: float = 120.0):
        self.client = _webhook_client(kubeconfig_path)
        self.ttl = cache_ttl
        self.cache = _TTLCache()

    async def authenticate(self, token: str) -> dict | None:
        key = hashlib.sha256(token.encode()).hexdigest()
        hit = self.cache.get(key)
        if hit is not None:
            return hit or None
        review = {"apiVersion": "authentication.k8s.io/v1beta1", "kind": "TokenReview", "spec": {"token": token}}
        resp = await self.client.request("POST", "", body=review)
        st = (resp or {}).get("status") or {}
        u = None
        if st.get("authenticated"):
            ui = st.get("user") or {}
            u = {"name": ui.get("username", ""), "uid": ui.get("uid", ""), "groups": list(ui.get("groups") or []),
                 "extra": ui.get("extra") or {}}
        self.cache.put(key, u or {}, self.ttl)
        return u


def _b64url(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


class OIDCAuthenticator:
    def __init__(self, issuer_url: str, client_id: str, ca_file: str | None = None, username_claim: str = "sub",
                 username_prefix: str | None = None, groups_claim: str | None = None, groups_prefix: str = ""):
        self.issuer, self.client_id = issuer_url.rstrip("/"), client_id
        self.username_claim, self.groups_claim, self.groups_prefix = username_claim, groups_claim, groups_prefix
        # oidc.go: a username claim other than email is prefixed with the issuer unless told otherwise
        if username_prefix is None:
            username_prefix = "" if username_claim == "email" else f"{issuer_url}#"
        self.username_prefix = "" if username_prefix == "-" else username_prefix
        self.ca_file = ca_file
        self.keys: dict[str, bytes] = {}
        self._fetched = 0.0

    def claims_issuer(self, token: str) -> str | None:
        try:
            return json.loads(_b64url(token.split(".")[1])).get("iss")
        except Exception:
            return None

    async def _refresh(self):
        from ..client import Client
        from ..utils.crypto import rsa_spki
        c = Client(self.issuer, ca_file=self.ca_file, timeout=30.0)
        try:
            disc = await c.request("GET", "/.well-known/openid-configuration")
            jwks_uri = disc["jwks_uri"]
            jc = Client(jwks_uri, ca_file=self.ca_file, timeout=30.0)
            try:
                jwks = await jc.request("GET", "")
            finally:
                await jc.close()
        finally:
            await c.close()
        keys = {}
        for k in jwks.get("keys") or []:
            if k.get("kty") == "RSA":
                n = int.from_bytes(_b64url(k["n"]), "big")
                e = int.from_bytes(_b64url(k["e"]), "big")
                keys[k.get("kid", "")] = rsa_spki(n, e)
        self.keys, self._fetched = keys, time.monotonic()

    async def authenticate(self, token: str) -> dict | None:
        from ..utils.crypto import rsa_sha256_verify
        try:
            h64, p64, s64 = token.split(".")
            header, claims, sig = json.loads(_b64url(h64)), json.loads(_b64url(p64)), _b64url(s64)
        except ValueError:
            return None
        if header.get("alg") != "RS256" or claims.get("iss", "").rstrip("/") != self.issuer:
            return None
        kid = header.get("kid", "")
        if kid not in self.keys and time.monotonic() - self._fetched > 10:
            await self._refresh()          # unknown key: the issuer may have rotated
        cands = [self.keys[kid]] if kid in self.keys else list(self.keys.values())
        signed = f"{h64}.{p64}".encode()
        if not any(rsa_sha256_verify(k, signed, sig) for k in cands):
            return None
        aud = claims.get("aud")
        if self.client_id not in (aud if isinstance(aud, list) else [aud]):
            return None
        # oidc.go:255-270 (go-oidc VerifyJWT): a token without exp never expires, so it is refused;
        # an email username needs an explicit boolean email_verified=true
        exp = claims.get("exp")
        if not isinstance(exp, (int, float)) or isinstance(exp, bool) or exp < time.time():
            return None
        if self.username_claim == "email" and claims.get("email_verified") is not True:
            return None
        name = claims.get(self.username_claim)
        if not name:
            return None
        groups = []
        if self.groups_claim:
            g = claims.get(self.groups_claim) or []
            groups = [self.groups_prefix + x for x in ([g] if isinstance(g, str) else g)]
        return {"name": f"{self.username_prefix}{name}", "uid": "", "groups": groups}


class WebhookAuthorizer:
    name = "Webhook"

    def __init__(self, kubeconfig_path: str, authorized_ttl: float = 300.0, unauthorized_ttl: float = 30.0):
        self.client = _webhook_client(kubeconfig_path)
        self.ttl_yes, self.ttl_no = authorized_ttl, unauthorized_ttl
        self.cache = _TTLCache()

    @staticmethod
    def _review(a) -> dict:
        spec = {"user": a.user.get("name", ""), "groups": list(a.user.get("groups") or [])}
        if a.user.get("extra"):
            spec["extra"] = a.user["extra"]
        if a.resource_request:
            spec["resourceAttributes"] = {"namespace": a.namespace, "verb": a.verb, "group": a.group, "resource": a.resource,
                                          "subresource": a.subresource, "name": a.name}
        else:
            spec["nonResourceAttributes"] = {"path": a.path, "verb": a.verb}
        return {"apiVersion": "authorization.k8s.io/v1beta1", "kind": "SubjectAccessReview", "spec": spec}

    def _key(self, review: dict) -> str:
        return json.dumps(review["spec"], sort_keys=True)

    def authorize(self, a) -> tuple[bool, str]:
        """Synchronous callers see cached decisions only (the request path awaits authorize_async)."""
        hit = self.cache.get(self._key(self._review(a)))
        return (True, hit[1]) if hit and hit[0] else (False, "")

    async def authorize_async(self, a) -> tuple[bool, str]:
        review = self._review(a)
        key = self._key(review)
        hit = self.cache.get(key)
        if hit is not None:
            return hit
        try:
            resp = await self.client.request("POST", "", body=review)
        except Exception as e:       # an unreachable webhook denies (and is not cached)
            return False, f"webhook authorizer unavailable: {e!r}"
        st = (resp or {}).get("status") or {}
        res = (bool(st.get("allowed")), st.get("reason", ""))
        self.cache.put(key, res, self.ttl_yes if res[0] else self.ttl_no)
        return res


class ABACAuthorizer:
    name = "ABAC"

    def __init__(self, path: str):
        self.policies = []
        with open(path) as f:
            for n, line in enumerate(f, 1):
                line = line.strip()
                if not line or line.startswith("#"):
                    continue
                try:
                    p = json.loads(line)
                except ValueError as e:
                    raise ValueError(f"{path}:{n}: {e}")
                self.policies.append(p.get("spec", p))

    @staticmethod
    def _subject_matches(p: dict, u: dict) -> bool:
        """abac.go subjectMatches: every subject field the policy sets must match (user AND
        group when both are set), and at least one must be set."""
        matched = False
        if p.get("user"):
            if p["user"] != "*" and p["user"] != u.get("name"):
                return False
            matched = True
        if p.get("group"):
            if p["group"] != "*" and p["group"] not in (u.get("groups") or []):
                return False
            matched = True
        return matched

    @classmethod
    def _matches(cls, p: dict, a) -> bool:
        if not cls._subject_matches(p, a.user):
            return False
        if p.get("readonly") and a.verb not in ("get", "list", "watch"):
            return False
        if a.resource_request:
            return all(p.get(k, "") in ("*", v) for k, v in
                       (("namespace", a.namespace), ("resource", a.resource), ("apiGroup", a.group)))
        path = p.get("nonResourcePath")
        return bool(path) and (path == "*" or path == a.path or (path.endswith("*") and a.path.startswith(path[:-1])))

    def authorize(self, a) -> tuple[bool, str]:
        for p in self.policies:
            if self._matches(p, a):
                return True, "allowed by ABAC policy"
        return False, ""
