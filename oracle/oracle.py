"""ctypes front-end of the CPU oracle (oracle/rg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
``cpu_baseline`` leg of bench.py, always as the checker / the timed CPU
baseline, never by the product package ``rustyguard_amd``.

The C code restates RFC 8439 (the algorithm of graviola 0.2.0, which the
reference calls at rustyguard-crypto/src/prim.rs:179-201) plus the WireGuard
nonce/framing glue; see the header of rg_oracle.c for the file:line map.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "librg_oracle.so")
_lib = None

DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("key_idx", "<u4")])

OK, DECRYPT_ERR, INVALID, REJECTED, UNALIGNED, NOT_DATA = range(6)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        L.rg_oracle_chacha20_block.argtypes = [u8p, ctypes.c_uint32, u8p, u8p]
        L.rg_oracle_poly1305.argtypes = [u8p, u8p, ctypes.c_size_t, u8p]
        L.rg_oracle_aead_seal.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p]
        L.rg_oracle_aead_open.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p]
        L.rg_oracle_aead_open.restype = ctypes.c_int
        L.rg_oracle_seal_batch.argtypes = [u8p, u8p, u8p, u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_int]
        L.rg_oracle_open_batch.argtypes = [u8p, u8p, ctypes.c_size_t, u8p, u8p, u8p, ctypes.c_int]
        L.rg_oracle_hchacha20.argtypes = [u8p, u8p, u8p]
        L.rg_oracle_blake2s.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        L.rg_oracle_mac_verify_batch.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, u8p,
                                                 ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, u8p]
        L.rg_oracle_xaead_seal.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p]
        L.rg_oracle_xaead_open.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p]
        L.rg_oracle_xaead_open.restype = ctypes.c_int
        L.rg_oracle_open_batch_rx.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, u8p, u8p,
                                              u8p]
        L.rg_oracle_mix64.argtypes = [ctypes.c_uint64]
        L.rg_oracle_mix64.restype = ctypes.c_uint64
        L.rg_oracle_synth_fill.argtypes = [u8p, u8p, u8p, ctypes.c_size_t, ctypes.c_uint64]
        L.rg_openssl_available.restype = ctypes.c_int
        L.rg_openssl_version.restype = ctypes.c_char_p
        L.rg_openssl_seal_batch.argtypes = [u8p, u8p, u8p, u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_int]
        L.rg_openssl_seal_batch.restype = ctypes.c_int
        L.rg_openssl_open_batch.argtypes = [u8p, u8p, ctypes.c_size_t, u8p, u8p, ctypes.c_int]
        L.rg_openssl_open_batch.restype = ctypes.c_int
        L.rg_cpu_bench.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p, u8p, u8p, ctypes.c_size_t, u8p,
                                   ctypes.c_double, u8p, ctypes.c_int, u8p]
        L.rg_cpu_bench.restype = ctypes.c_int
        L.rg_cpu_time_one.argtypes = [ctypes.c_int, u8p, ctypes.c_uint32, ctypes.c_uint64, u8p]
        L.rg_cpu_time_one.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, (bytes, bytearray)):
        a = np.frombuffer(bytes(a), dtype=np.uint8)
    return a.ctypes.data_as(ctypes.c_void_p)


def _u8(b) -> np.ndarray:
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def wg_nonce(counter: int) -> bytes:
    """rustyguard-crypto/src/prim.rs:32-36."""
    return b"\0" * 4 + int(counter).to_bytes(8, "little")


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    out = np.zeros(64, np.uint8)
    lib().rg_oracle_chacha20_block(_ptr(_u8(key)), counter, _ptr(_u8(nonce)), _ptr(out))
    return out.tobytes()


def poly1305(key: bytes, msg: bytes) -> bytes:
    out = np.zeros(16, np.uint8)
    m = _u8(msg) if msg else np.zeros(1, np.uint8)
    lib().rg_oracle_poly1305(_ptr(_u8(key)), _ptr(m), len(msg), _ptr(out))
    return out.tobytes()


def aead_seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> tuple[bytes, bytes]:
    """Core::chacha20poly1305_enc (prim.rs:179-188): returns (ciphertext, tag)."""
    buf = _u8(pt) if pt else np.zeros(1, np.uint8)
    a = _u8(aad) if aad else np.zeros(1, np.uint8)
    tag = np.zeros(16, np.uint8)
    lib().rg_oracle_aead_seal(_ptr(_u8(key)), _ptr(_u8(nonce)), _ptr(a), len(aad), _ptr(buf), len(pt), _ptr(tag))
    return buf.tobytes()[: len(pt)], tag.tobytes()


def aead_open(key: bytes, nonce: bytes, aad: bytes, ct: bytes, tag: bytes):
    """Core::chacha20poly1305_dec (prim.rs:190-201): plaintext or None on DecryptionError."""
    buf = _u8(ct) if ct else np.zeros(1, np.uint8)
    a = _u8(aad) if aad else np.zeros(1, np.uint8)
    rc = lib().rg_oracle_aead_open(_ptr(_u8(key)), _ptr(_u8(nonce)), _ptr(a), len(aad), _ptr(buf), len(ct),
                                   _ptr(_u8(tag)))
    return None if rc != 0 else buf.tobytes()[: len(ct)]


def blake2s(msg: bytes, key: bytes = b"", outlen: int = 32) -> bytes:
    """RFC 7693 BLAKE2s (Core::blake2s_hash / blake2s_mac, rustyguard-crypto/src/prim.rs:118-131)."""
    out = np.zeros(32, np.uint8)
    m = _u8(msg) if msg else np.zeros(1, np.uint8)
    k = _u8(key) if key else np.zeros(1, np.uint8)
    lib().rg_oracle_blake2s(_ptr(out), outlen, _ptr(k), len(key), _ptr(m), len(msg))
    return out[:outlen].tobytes()


def mac_verify_batch(keys: np.ndarray, which: int, desc: np.ndarray, buf: np.ndarray):
    """HasMac::verify_mac1 (which=1) / verify_mac2 (which=2) per handshake message; key_idx
    0xFFFFFFFE scans every key (wg-proxy).  Returns (status u8[n], matched key u32[n])."""
    assert desc.dtype == DESC_DTYPE and buf.dtype == np.uint8
    keys = np.ascontiguousarray(keys, np.uint8)
    n = len(desc)
    status = np.zeros(max(n, 1), np.uint8)
    kout = np.zeros(max(n, 1), np.uint32)
    lib().rg_oracle_mac_verify_batch(_ptr(keys), keys.shape[1], keys.shape[0], which, _ptr(desc), n, _ptr(buf),
                                     len(buf), _ptr(status), _ptr(kout))
    return status[:n], kout[:n]


def hchacha20(key: bytes, nonce16: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    lib().rg_oracle_hchacha20(_ptr(_u8(key)), _ptr(_u8(nonce16)), _ptr(out))
    return out.tobytes()


def xaead_seal(key: bytes, nonce24: bytes, aad: bytes, pt: bytes) -> tuple[bytes, bytes]:
    """XChaCha20-Poly1305 (Core::xchacha20poly1305_enc, prim.rs:202-212): (ciphertext, tag)."""
    buf = _u8(pt).copy() if pt else np.zeros(1, np.uint8)
    tag = np.zeros(16, np.uint8)
    a = _u8(aad) if aad else np.zeros(1, np.uint8)
    lib().rg_oracle_xaead_seal(_ptr(_u8(key)), _ptr(_u8(nonce24)), _ptr(a), len(aad), _ptr(buf), len(pt), _ptr(tag))
    return buf[:len(pt)].tobytes(), tag.tobytes()


def xaead_open(key: bytes, nonce24: bytes, aad: bytes, ct: bytes, tag: bytes):
    """Plaintext, or None on a tag mismatch (CryptoError::DecryptionError)."""
    buf = _u8(ct).copy() if ct else np.zeros(1, np.uint8)
    a = _u8(aad) if aad else np.zeros(1, np.uint8)
    rc = lib().rg_oracle_xaead_open(_ptr(_u8(key)), _ptr(_u8(nonce24)), _ptr(a), len(aad), _ptr(buf), len(ct),
                                    _ptr(_u8(tag)))
    return None if rc != 0 else buf[:len(ct)].tobytes()


def seal_batch(keys: np.ndarray, receivers, desc: np.ndarray, counters: np.ndarray, buf: np.ndarray,
               nthreads: int = 1, status: np.ndarray | None = None) -> None:
    """In-place batched seal over the include/rg_aead.h buffer contract."""
    assert desc.dtype == DESC_DTYPE and buf.dtype == np.uint8
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    counters = np.ascontiguousarray(counters, dtype=np.uint64)
    rec = None if receivers is None else np.ascontiguousarray(receivers, dtype=np.uint32)
    lib().rg_oracle_seal_batch(_ptr(keys), _ptr(rec), _ptr(desc), _ptr(counters), len(desc), _ptr(buf),
                               _ptr(status), nthreads)


def open_batch(keys: np.ndarray, desc: np.ndarray, buf: np.ndarray, nthreads: int = 1):
    """In-place batched open; returns (status u8[n], counters u64[n])."""
    assert desc.dtype == DESC_DTYPE and buf.dtype == np.uint8
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n = len(desc)
    status = np.zeros(max(n, 1), np.uint8)
    ctr = np.zeros(max(n, 1), np.uint64)
    lib().rg_oracle_open_batch(_ptr(keys), _ptr(desc), n, _ptr(buf), _ptr(status), _ptr(ctr), nthreads)
    return status[:n], ctr[:n]


def open_batch_rx(keys: np.ndarray, receivers, desc: np.ndarray, buf: np.ndarray):
    """In-place open resolving each frame's session from its header receiver (session s has receiver
    receivers[s] and key row s); returns (status u8[n], counters u64[n], key_idx u32[n])."""
    assert desc.dtype == DESC_DTYPE and buf.dtype == np.uint8
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    rec = np.ascontiguousarray(receivers, np.uint32)
    idx = np.arange(len(rec), dtype=np.uint32)
    n = len(desc)
    status = np.zeros(max(n, 1), np.uint8)
    ctr = np.zeros(max(n, 1), np.uint64)
    kout = np.zeros(max(n, 1), np.uint32)
    lib().rg_oracle_open_batch_rx(_ptr(keys), _ptr(rec), _ptr(idx), len(rec), _ptr(desc), n, _ptr(buf),
                                  _ptr(status), _ptr(ctr), _ptr(kout))
    return status[:n], ctr[:n], kout[:n]


def mix64(x: int) -> int:
    return int(lib().rg_oracle_mix64(x))


def synth_fill(buf: np.ndarray, desc: np.ndarray, inner_len: np.ndarray, seed: int) -> None:
    inner = np.ascontiguousarray(inner_len, dtype=np.uint32)
    lib().rg_oracle_synth_fill(_ptr(buf), _ptr(desc), _ptr(inner), len(desc), seed)


# ---- OpenSSL EVP ChaCha20-Poly1305 batches (CPU baseline "CPU-B", oracle/rg_openssl_batch.c)
def openssl_available() -> bool:
    return bool(lib().rg_openssl_available())


def openssl_version() -> str:
    return lib().rg_openssl_version().decode()


def openssl_seal_batch(keys, receivers, desc, counters, buf, nthreads=1, status=None):
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    counters = np.ascontiguousarray(counters, dtype=np.uint64)
    rec = None if receivers is None else np.ascontiguousarray(receivers, dtype=np.uint32)
    rc = lib().rg_openssl_seal_batch(_ptr(keys), _ptr(rec), _ptr(desc), _ptr(counters), len(desc), _ptr(buf),
                                     _ptr(status), nthreads)
    if rc != 0:
        raise RuntimeError("libcrypto.so.3 not available")


def openssl_open_batch(keys, desc, buf, nthreads=1):
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    status = np.zeros(max(len(desc), 1), np.uint8)
    rc = lib().rg_openssl_open_batch(_ptr(keys), _ptr(desc), len(desc), _ptr(buf), _ptr(status), nthreads)
    if rc != 0:
        raise RuntimeError("libcrypto.so.3 not available")
    return status[: len(desc)]


def cpu_bench(impl: str, nthreads: int, keys, receivers, desc, counters, buf, seconds: float, cpus=None,
              local: bool = False):
    """CPU baseline harness (rg_openssl_batch.c rg_cpu_bench): a persistent pool of `nthreads` workers
    seals then opens its slice of the sample in rounds for `seconds`; impl "port" (the C restatement) or
    "openssl" (EVP, one cipher context per worker, re-keyed per packet) or "openssl-keyed-once" (the key
    installed only when it changes: the study's measure of the re-key's cost).  cpus: one CPU per worker to pin
    it to; local: each worker works on its own first-touched copy of its slice (written back at the end).
    Returns (elapsed_s, rounds)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    counters = np.ascontiguousarray(counters, dtype=np.uint64)
    rec = None if receivers is None else np.ascontiguousarray(receivers, dtype=np.uint32)
    out = np.zeros(3, np.float64)
    cp = None if cpus is None else np.ascontiguousarray(list(cpus)[:nthreads], dtype=np.int32)
    if cp is not None and len(cp) < nthreads:
        raise ValueError("cpu_bench: fewer CPUs than threads")
    code = {"port": 0, "openssl": 1, "openssl-keyed-once": 2}[impl]
    rc = lib().rg_cpu_bench(code, nthreads, _ptr(keys), _ptr(rec), _ptr(desc),
                            _ptr(counters), len(desc), _ptr(buf), seconds, _ptr(cp), 1 if local else 0, _ptr(out))
    if rc != 0:
        raise RuntimeError(f"rg_cpu_bench({impl}, {nthreads}) failed: {rc}")
    if out[2] != 0:
        raise RuntimeError(f"rg_cpu_bench({impl}): {int(out[2])} packets failed to seal or open")
    return float(out[0]), int(out[1])


def time_one(impl: str, key: bytes, P: int, iters: int) -> tuple[float, float]:
    """BASELINE config 1 on one thread: mean ns of one seal and one open of a single P-byte
    transport frame (impl "port": the C restatement, "openssl": EVP re-keyed per packet)."""
    out = np.zeros(2, np.float64)
    rc = lib().rg_cpu_time_one(1 if impl == "openssl" else 0, _ptr(_u8(key)), P, iters, _ptr(out))
    if rc != 0:
        raise RuntimeError(f"rg_cpu_time_one({impl}) failed: {rc}")
    return float(out[0]), float(out[1])
