"""Registry credentials for image pulls: the reference's pkg/credentialprovider.

* Docker config formats (config.go): `.dockercfg` (registry → {username, password, auth,
  email}) and `config.json` ({"auths": {...}}); `auth` is base64("user:password").
* Node credentials (config.go ReadDockerConfigFile / ReadDockercfgFile): the first
  config.json found in <root-dir>, the working directory, $HOME/.docker, /.docker, else the
  first .dockercfg in <root-dir>, the working directory, $HOME, /.
* Matching (keyring.go Lookup / urlsMatch): a key is a registry URL with an optional path;
  the host may use `*` globs per dot-separated part (`*.example.com`), the port must be equal
  and the key's path must be a prefix of the image's repository path. The most specific key
  is tried first (keys in reverse lexical order). Images with no registry host belong to
  Docker Hub (`index.docker.io`, also matched by `docker.io` and `https://index.docker.io/v1/`).
* Pods (secrets.go MakeDockerKeyring): credentials of the pod's imagePullSecrets
  (types kubernetes.io/dockercfg and kubernetes.io/dockerconfigjson) come before the node's.

The kubelet tries every matching credential in order and stops at the first pull that
succeeds (kuberuntime_image.go PullImage); with no match it pulls anonymously.
"""
from __future__ import annotations

import base64
import fnmatch
import json
import logging
import os
from dataclasses import dataclass

log = logging.getLogger("amdkube.credentialprovider")

DOCKER_HUB = "index.docker.io"
_HUB_ALIASES = {"docker.io", "index.docker.io", "registry-1.docker.io"}


@dataclass(frozen=True)
class AuthConfig:
    username: str = ""
    password: str = ""
    auth: str = ""
    server_address: str = ""
    email: str = ""

    def to_cri(self, C):
        return C.AuthConfig(username=self.username, password=self.password, auth=self.auth,
                            server_address=self.server_address)


def _entry(registry: str, e: dict) -> AuthConfig:
    user, pw = e.get("username", ""), e.get("password", "")
    auth = e.get("auth", "")
    if auth and not (user or pw):
        try:
            user, _, pw = base64.b64decode(auth).decode().partition(":")
        except Exception as ex:
            raise ValueError(f"invalid auth for {registry}: {ex}") from None
    if not auth and (user or pw):
        auth = base64.b64encode(f"{user}:{pw}".encode()).decode()
    return AuthConfig(user, pw, auth, registry, e.get("email", ""))


def parse_docker_config(data: dict | str | bytes) -> dict[str, AuthConfig]:
    """Either format; {"auths": {...}} is config.json, anything else .dockercfg."""
    if isinstance(data, (str, bytes)):
        data = json.loads(data)
    if not isinstance(data, dict):
        raise ValueError("docker config must be a JSON object")
    auths = data.get("auths") if isinstance(data.get("auths"), dict) else data
    return {reg: _entry(reg, e) for reg, e in auths.items() if isinstance(e, dict)}


def _split_key(key: str) -> tuple[str, str, str]:
    """registry key → (host, port, path); scheme and trailing /v1/ style suffixes dropped."""
    k = key.strip()
    if "://" in k:
        k = k.split("://", 1)[1]
    host, _, path = k.partition("/")
    path = path.strip("/")
    if path in ("v1", "v2"):
        path = ""
    host, _, port = host.partition(":")
    host = host.lower()
    if host in _HUB_ALIASES:
        host = DOCKER_HUB
    return host, port, path


def split_image(image: str) -> tuple[str, str, str]:
    """image reference → (registry host, port, repository path) (docker reference rules)."""
    ref = image.split("@", 1)[0]
    first, _, rest = ref.partition("/")
    if rest and ("." in first or ":" in first or first == "localhost"):
        host, _, port = first.partition(":")
        repo = rest
    else:
        host, port, repo = DOCKER_HUB, "", ref
        if "/" not in repo.rsplit(":", 1)[0]:
            repo = "library/" + repo
    last = repo.rsplit("/", 1)
    if ":" in last[-1]:                     # drop the tag
        repo = repo[:len(repo) - len(last[-1])] + last[-1].split(":", 1)[0]
    host = host.lower()
    if host in _HUB_ALIASES:
        host = DOCKER_HUB
    return host, port, repo


def _host_match(pattern: str, host: str) -> bool:
    pp, hp = pattern.split("."), host.split(".")
    return len(pp) == len(hp) and all(fnmatch.fnmatchcase(h, p) for p, h in zip(pp, hp))


def key_matches(key: str, image: str) -> bool:
    kh, kport, kpath = _split_key(key)
    ih, iport, ipath = split_image(image)
    if not _host_match(kh, ih) or kport != iport:
        return False
    return not kpath or ipath == kpath or ipath.startswith(kpath + "/")


class DockerKeyring:
    def __init__(self, entries: dict[str, AuthConfig] | None = None):
        self.entries: dict[str, AuthConfig] = {}
        if entries:
            self.add(entries)

    def add(self, entries: dict[str, AuthConfig]):
        self.entries.update(entries)

    def lookup(self, image: str) -> list[AuthConfig]:
        return [self.entries[k] for k in sorted(self.entries, reverse=True) if key_matches(k, image)]


class UnionKeyring:
    def __init__(self, *rings):
        self.rings = [r for r in rings if r is not None]

    def lookup(self, image: str) -> list[AuthConfig]:
        out: list[AuthConfig] = []
        for r in self.rings:
            for a in r.lookup(image):
                if a not in out:
                    out.append(a)
        return out


def node_keyring(root_dir: str = "/var/lib/kubelet") -> DockerKeyring:
    home = os.path.expanduser("~")
    for d in (root_dir, os.getcwd(), os.path.join(home, ".docker"), "/.docker"):
        p = os.path.join(d, "config.json")
        if os.path.isfile(p):
            try:
                return DockerKeyring(parse_docker_config(open(p).read()))
            except (OSError, ValueError) as e:
                log.warning("ignoring docker config %s: %s", p, e)
    for d in (root_dir, os.getcwd(), home, "/"):
        p = os.path.join(d, ".dockercfg")
        if os.path.isfile(p):
            try:
                return DockerKeyring(parse_docker_config(open(p).read()))
            except (OSError, ValueError) as e:
                log.warning("ignoring docker config %s: %s", p, e)
    return DockerKeyring()


SECRET_KEYS = {"kubernetes.io/dockerconfigjson": ".dockerconfigjson", "kubernetes.io/dockercfg": ".dockercfg"}


def secrets_keyring(secrets: list[dict]) -> DockerKeyring:
    """Credentials of image pull secrets; secrets of other types or with bad content are skipped."""
    ring = DockerKeyring()
    for s in secrets:
        key = SECRET_KEYS.get(s.get("type", ""))
        raw = (s.get("data") or {}).get(key or "")
        if not raw:
            continue
        try:
            ring.add(parse_docker_config(base64.b64decode(raw)))
        except (ValueError, TypeError) as e:
            log.warning("ignoring image pull secret %s: %s", (s.get("metadata") or {}).get("name"), e)
    return ring
