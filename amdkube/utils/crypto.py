"""Symmetric and RSA primitives over the system libcrypto (OpenSSL 3, the library Python's own
ssl module links), for the pieces the standard library lacks: AES-CBC and AES-GCM for
encryption at rest (staging/src/k8s.io/apiserver/pkg/storage/value/encrypt/aes) and RS256
signature checks for OpenID Connect ID tokens (plugin/pkg/auth/authenticator/token/oidc).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import hashlib
import os

_lib = None


def _crypto():
    global _lib
    if _lib is None:
        path = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        lib = ctypes.CDLL(path)
        vp, cp, ip = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int
        for name, res, args in (
                ("EVP_CIPHER_CTX_new", vp, []), ("EVP_CIPHER_CTX_free", None, [vp]),
                ("EVP_aes_128_cbc", vp, []), ("EVP_aes_192_cbc", vp, []), ("EVP_aes_256_cbc", vp, []),
                ("EVP_aes_128_gcm", vp, []), ("EVP_aes_192_gcm", vp, []), ("EVP_aes_256_gcm", vp, []),
                ("EVP_CipherInit_ex", ip, [vp, vp, vp, cp, cp, ip]),
                ("EVP_CipherUpdate", ip, [vp, cp, ctypes.POINTER(ip), cp, ip]),
                ("EVP_CipherFinal_ex", ip, [vp, cp, ctypes.POINTER(ip)]),
                ("EVP_CIPHER_CTX_ctrl", ip, [vp, ip, ip, vp]),
                ("EVP_MD_CTX_new", vp, []), ("EVP_MD_CTX_free", None, [vp]), ("EVP_sha256", vp, []),
                ("d2i_PUBKEY", vp, [vp, ctypes.POINTER(cp), ctypes.c_long]), ("EVP_PKEY_free", None, [vp]),
                ("EVP_DigestVerifyInit", ip, [vp, vp, vp, vp, vp]),
                ("EVP_DigestVerify", ip, [vp, cp, ctypes.c_size_t, cp, ctypes.c_size_t]),
                ("d2i_X509", vp, [vp, ctypes.POINTER(cp), ctypes.c_long]), ("X509_free", None, [vp]),
                ("X509_get_pubkey", vp, [vp]), ("X509_verify", ip, [vp, vp]),
                ("BIO_new_mem_buf", vp, [cp, ip]), ("BIO_free", ip, [vp]),
                ("PEM_read_bio_X509", vp, [vp, vp, vp, vp])):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


_GCM_SET_IVLEN, _GCM_GET_TAG, _GCM_SET_TAG = 0x9, 0x10, 0x11


def _cipher(mode: str, key: bytes):
    bits = len(key) * 8
    if bits not in (128, 192, 256):
        raise ValueError(f"AES key must be 16, 24 or 32 bytes, got {len(key)}")
    return getattr(_crypto(), f"EVP_aes_{bits}_{mode}")()


def _run(mode: str, key: bytes, iv: bytes, data: bytes, encrypt: bool, aad: bytes = b"", tag: bytes | None = None):
    lib = _crypto()
    ctx = lib.EVP_CIPHER_CTX_new()
    try:
        enc = 1 if encrypt else 0
        if not lib.EVP_CipherInit_ex(ctx, _cipher(mode, key), None, None, None, enc):
            raise ValueError("cipher init failed")
        if mode == "gcm" and not lib.EVP_CIPHER_CTX_ctrl(ctx, _GCM_SET_IVLEN, len(iv), None):
            raise ValueError("gcm iv length")
        if not lib.EVP_CipherInit_ex(ctx, None, None, key, iv, enc):
            raise ValueError("cipher key/iv init failed")
        n = ctypes.c_int(0)
        if aad:
            if not lib.EVP_CipherUpdate(ctx, None, ctypes.byref(n), aad, len(aad)):
                raise ValueError("aad failed")
        out = ctypes.create_string_buffer(len(data) + 32)
        if not lib.EVP_CipherUpdate(ctx, out, ctypes.byref(n), data, len(data)):
            raise ValueError("cipher update failed")
        total = n.value
        if tag is not None and not lib.EVP_CIPHER_CTX_ctrl(ctx, _GCM_SET_TAG, len(tag), ctypes.c_char_p(tag)):
            raise ValueError("gcm tag")
        fin = ctypes.create_string_buffer(32)
        if not lib.EVP_CipherFinal_ex(ctx, fin, ctypes.byref(n)):
            raise ValueError("decryption failed (bad key, padding or authentication tag)")
        res = out.raw[:total] + fin.raw[:n.value]
        if mode == "gcm" and encrypt:
            t = ctypes.create_string_buffer(16)
            if not lib.EVP_CIPHER_CTX_ctrl(ctx, _GCM_GET_TAG, 16, t):
                raise ValueError("gcm tag")
            res += t.raw
        return res
    finally:
        lib.EVP_CIPHER_CTX_free(ctx)


def aes_cbc_encrypt(key: bytes, plaintext: bytes) -> bytes:
    """Random 16-byte IV || AES-CBC(PKCS#7) ciphertext (aes.go cbc transformer layout)."""
    iv = os.urandom(16)
    return iv + _run("cbc", key, iv, plaintext, True)


def aes_cbc_decrypt(key: bytes, blob: bytes) -> bytes:
    if len(blob) < 32 or len(blob) % 16:
        raise ValueError("the stored data is not a multiple of the block size")
    return _run("cbc", key, blob[:16], blob[16:], False)


def aes_gcm_encrypt(key: bytes, plaintext: bytes, aad: bytes = b"") -> bytes:
    """Random 12-byte nonce || ciphertext || 16-byte tag, authenticating `aad` (aes.go gcm)."""
    nonce = os.urandom(12)
    return nonce + _run("gcm", key, nonce, plaintext, True, aad)


def aes_gcm_decrypt(key: bytes, blob: bytes, aad: bytes = b"") -> bytes:
    if len(blob) < 12 + 16:
        raise ValueError("the stored data was shorter than the required size")
    return _run("gcm", key, blob[:12], blob[12:-16], False, aad, blob[-16:])


# ------------------------------------------------------------------------ RSA (RS256)
def _der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _der(tag: int, body: bytes) -> bytes:
    return bytes([tag]) + _der_len(len(body)) + body


def _der_int(v: int) -> bytes:
    b = v.to_bytes((v.bit_length() + 8) // 8, "big")     # a leading 0 keeps it positive
    return _der(0x02, b)


def rsa_spki(n: int, e: int) -> bytes:
    """DER SubjectPublicKeyInfo of an RSA key (what a JWK's n/e describe)."""
    alg = _der(0x30, _der(0x06, bytes.fromhex("2a864886f70d010101")) + b"\x05\x00")     # rsaEncryption, NULL
    key = _der(0x30, _der_int(n) + _der_int(e))
    return _der(0x30, alg + _der(0x03, b"\x00" + key))


def rsa_sha256_verify(spki_der: bytes, data: bytes, signature: bytes) -> bool:
    lib = _crypto()
    buf = ctypes.c_char_p(spki_der)
    pkey = lib.d2i_PUBKEY(None, ctypes.byref(buf), len(spki_der))
    if not pkey:
        raise ValueError("invalid public key")
    md = lib.EVP_MD_CTX_new()
    try:
        if lib.EVP_DigestVerifyInit(md, None, lib.EVP_sha256(), None, pkey) != 1:
            return False
        return lib.EVP_DigestVerify(md, signature, len(signature), data, len(data)) == 1
    finally:
        lib.EVP_MD_CTX_free(md)
        lib.EVP_PKEY_free(pkey)


def x509_pem_to_der(pem: bytes) -> list[bytes]:
    """Every CERTIFICATE block of a PEM bundle as DER."""
    import base64
    out, cur = [], None
    for line in pem.decode(errors="replace").splitlines():
        if line.startswith("-----BEGIN CERTIFICATE"):
            cur = []
        elif line.startswith("-----END CERTIFICATE") and cur is not None:
            out.append(base64.b64decode("".join(cur)))
            cur = None
        elif cur is not None:
            cur.append(line.strip())
    return out


def x509_signed_by(cert_der: bytes, issuer_der: bytes) -> bool:
    """True when `cert_der`'s signature verifies under `issuer_der`'s public key (X509_verify):
    the certificate was really issued by that CA, not just by one with the same subject name."""
    lib = _crypto()
    b1, b2 = ctypes.c_char_p(cert_der), ctypes.c_char_p(issuer_der)
    cert = lib.d2i_X509(None, ctypes.byref(b1), len(cert_der))
    ca = lib.d2i_X509(None, ctypes.byref(b2), len(issuer_der))
    try:
        if not cert or not ca:
            return False
        key = lib.X509_get_pubkey(ca)
        if not key:
            return False
        try:
            return lib.X509_verify(cert, key) == 1
        finally:
            lib.EVP_PKEY_free(key)
    finally:
        if cert:
            lib.X509_free(cert)
        if ca:
            lib.X509_free(ca)


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()
