"""OpenSSL EVP ChaCha20-Poly1305 via ctypes -- an independent second checker.

TEST INFRASTRUCTURE ONLY (fixture generation in tests/golden/make_golden.py,
cross-checks in tests/, optional extra CPU figure in bench.py).  libcrypto is
a system library of this image; it reproduced every transport vector the
reference pins in its insta snapshots, which is
why it is trusted to pin the multi-block sizes the reference's tests do not
cover.
"""
from __future__ import annotations

import ctypes
import ctypes.util

_lib = None
EVP_CTRL_AEAD_SET_IVLEN = 0x9
EVP_CTRL_AEAD_GET_TAG = 0x10
EVP_CTRL_AEAD_SET_TAG = 0x11


def available() -> bool:
    try:
        _crypto()
        return True
    except OSError:
        return False


def _crypto():
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = ctypes.CDLL(name)
        L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        L.EVP_chacha20_poly1305.restype = ctypes.c_void_p
        L.EVP_chacha20.restype = ctypes.c_void_p
        for f in ("EVP_EncryptInit_ex", "EVP_DecryptInit_ex"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                      ctypes.c_char_p]
        for f in ("EVP_EncryptUpdate", "EVP_DecryptUpdate"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                      ctypes.c_char_p, ctypes.c_int]
        for f in ("EVP_EncryptFinal_ex", "EVP_DecryptFinal_ex"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.OpenSSL_version.restype = ctypes.c_char_p
        L.OpenSSL_version.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def version() -> str:
    return _crypto().OpenSSL_version(0).decode()


def seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> tuple[bytes, bytes]:
    L = _crypto()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_chacha20_poly1305(), None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, 12, None) == 1
        assert L.EVP_EncryptInit_ex(ctx, None, None, key, nonce) == 1
        outl = ctypes.c_int(0)
        if aad:
            assert L.EVP_EncryptUpdate(ctx, None, ctypes.byref(outl), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(pt) + 16)
        assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(outl), pt, len(pt)) == 1
        n = outl.value
        fin = ctypes.create_string_buffer(16)
        assert L.EVP_EncryptFinal_ex(ctx, fin, ctypes.byref(outl)) == 1
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1
        return out.raw[:n], tag.raw
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def open_(key: bytes, nonce: bytes, aad: bytes, ct: bytes, tag: bytes):
    L = _crypto()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_DecryptInit_ex(ctx, L.EVP_chacha20_poly1305(), None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, 12, None) == 1
        assert L.EVP_DecryptInit_ex(ctx, None, None, key, nonce) == 1
        outl = ctypes.c_int(0)
        if aad:
            assert L.EVP_DecryptUpdate(ctx, None, ctypes.byref(outl), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(ct) + 16)
        assert L.EVP_DecryptUpdate(ctx, out, ctypes.byref(outl), ct, len(ct)) == 1
        n = outl.value
        tbuf = ctypes.create_string_buffer(bytes(tag), 16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_TAG, 16, tbuf) == 1
        fin = ctypes.create_string_buffer(16)
        ok = L.EVP_DecryptFinal_ex(ctx, fin, ctypes.byref(outl))
        return out.raw[:n] if ok > 0 else None
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    """Raw keystream block via EVP_chacha20 (IV = le32(counter) || nonce)."""
    L = _crypto()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        iv = int(counter).to_bytes(4, "little") + bytes(nonce)
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_chacha20(), None, key, iv) == 1
        out = ctypes.create_string_buffer(64)
        outl = ctypes.c_int(0)
        assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(outl), b"\0" * 64, 64) == 1
        return out.raw[:64]
    finally:
        L.EVP_CIPHER_CTX_free(ctx)
