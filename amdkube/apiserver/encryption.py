"""Encryption of resources at rest (--experimental-encryption-provider-config;
staging/src/k8s.io/apiserver/pkg/server/options/encryptionconfig, pkg/storage/value).

The embedded store keeps objects in memory and persists them to its WAL and snapshot; this
transformer sits exactly there, so what reaches disk for the configured resources is
ciphertext. Configuration (kind EncryptionConfig):

    kind: EncryptionConfig
    apiVersion: v1
    resources:
    - resources: [secrets]
      providers:
      - aescbc: {keys: [{name: key1, secret: <base64 of 16/24/32 bytes>}]}
      - aesgcm: {keys: [...]}
      - identity: {}

Writes use the first provider (its first key); reads try every provider by its prefix
`k8s:enc:<provider>:v1:<key name>:` (identity: data without a prefix), so keys rotate by
adding the new key first and rewriting (every snapshot rewrites all data). AES-GCM
authenticates the storage key. secretbox needs NaCl, which this build does not link: it is
rejected at startup rather than silently skipped.
"""
from __future__ import annotations

import base64

import yaml

from ..utils import crypto


class _Provider:
    def __init__(self, kind: str, keys: list[tuple[str, bytes]]):
        self.kind, self.keys = kind, keys

    def prefix(self, name: str) -> bytes:
        return f"k8s:enc:{self.kind}:v1:{name}:".encode()

    def encrypt(self, key: str, data: bytes) -> bytes:
        if self.kind == "identity":
            return data
        name, k = self.keys[0]
        body = crypto.aes_cbc_encrypt(k, data) if self.kind == "aescbc" else crypto.aes_gcm_encrypt(k, data, key.encode())
        return self.prefix(name) + body

    def try_decrypt(self, key: str, data: bytes) -> bytes | None:
        if self.kind == "identity":
            return None if data.startswith(b"k8s:enc:") else data
        for name, k in self.keys:
            p = self.prefix(name)
            if data.startswith(p):
                blob = data[len(p):]
                return crypto.aes_cbc_decrypt(k, blob) if self.kind == "aescbc" else crypto.aes_gcm_decrypt(k, blob, key.encode())
        return None


class ResourceTransformer:
    """MVCCStore value transformer: to_disk / from_disk per storage key."""

    def __init__(self, rules: list[tuple[tuple[str, ...], list[_Provider]]]):
        self.rules = rules

    def _providers(self, key: str) -> list[_Provider] | None:
        for prefixes, providers in self.rules:
            if key.startswith(prefixes):
                return providers
        return None

    def to_disk(self, key: str, data: bytes) -> bytes:
        ps = self._providers(key)
        return ps[0].encrypt(key, data) if ps else data

    def from_disk(self, key: str, data: bytes) -> bytes:
        ps = self._providers(key)
        if not ps:
            return data
        for p in ps:
            out = p.try_decrypt(key, data)
            if out is not None:
                return out
        raise ValueError(f"no configured provider can read {key} (unknown key or provider prefix)")


def _storage_prefixes(resource: str) -> tuple[str, ...]:
    plural, _, group = resource.partition(".")
    return (f"/registry/{plural}/",) if plural else ()


def load(path: str) -> ResourceTransformer:
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    if cfg.get("kind") not in ("EncryptionConfig", "EncryptionConfiguration"):
        raise ValueError(f"{path}: expected kind EncryptionConfig, got {cfg.get('kind')!r}")
    rules = []
    for entry in cfg.get("resources") or []:
        providers = []
        for p in entry.get("providers") or []:
            if len(p) != 1:
                raise ValueError(f"{path}: each provider entry names exactly one provider, got {list(p)}")
            (kind, spec), = p.items()
            if kind == "identity":
                providers.append(_Provider("identity", []))
            elif kind in ("aescbc", "aesgcm"):
                keys = []
                for k in (spec or {}).get("keys") or []:
                    raw = base64.b64decode(k["secret"])
                    if len(raw) not in (16, 24, 32):
                        raise ValueError(f"{path}: key {k.get('name')!r} must be 16, 24 or 32 bytes")
                    keys.append((k["name"], raw))
                if not keys:
                    raise ValueError(f"{path}: provider {kind} has no keys")
                providers.append(_Provider(kind, keys))
            elif kind == "secretbox":
                raise ValueError(f"{path}: the secretbox provider needs NaCl, which this build does not include; "
                                 "use aescbc or aesgcm")
            else:
                raise ValueError(f"{path}: unknown provider {kind!r}")
        if not providers:
            raise ValueError(f"{path}: resources {entry.get('resources')} have no providers")
        prefixes = tuple(p for r in entry.get("resources") or [] for p in _storage_prefixes(r))
        rules.append((prefixes, providers))
    return ResourceTransformer(rules)
