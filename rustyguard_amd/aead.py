"""Host-side mirror of the reference's transport AEAD interface over librg_aead.

Reference interface -> this module
  CryptoPrimatives::chacha20poly1305_enc/_dec (prim.rs:82-95, 179-201)
                                         -> Engine.chacha20poly1305_enc/_dec
  CryptoPrimatives::xchacha20poly1305_enc/_dec (prim.rs:97-110, 202-224)
                                         -> Engine.xchacha20poly1305_enc/_dec
  EncryptionKey {new, encrypt, counter}   (prim.rs:376-399) -> EncryptionKey
  DecryptionKey {new, decrypt}            (prim.rs:401-437) -> DecryptionKey
  AntiReplay {would_accept, mark_seen}    (anti_replay.rs:25-64) -> AntiReplay
  CryptoError::{DecryptionError, Rejected} (rustyguard-crypto/src/lib.rs:43-48)
                                         -> DecryptionError / Rejected exceptions
  batched hot path                        -> Engine.seal_dev/open_dev (device
                                             tensors), seal_host/open_host (numpy)
  Sessions send/recv of data frames       -> Sessions.send_batch / recv_batch

Every call goes through the HIP library; there is no CPU path here.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib
from .workloads import DESC_DTYPE

PKT_OK, PKT_DECRYPT_ERR, PKT_INVALID, PKT_REJECTED, PKT_UNALIGNED, PKT_NOT_DATA, PKT_PENDING = range(7)
RECV_AUTHENTICATED, RECV_KEEPALIVE = 1, 2
KEY_SCAN = 0xFFFFFFFE  # rg_mac_verify_batch_dev: try every key
KEY_SKIP = 0xFFFFFFFF
REKEY_AFTER_MESSAGES = 1 << 60
REJECT_AFTER_MESSAGES = (1 << 64) - 1 - (1 << 13)
WINDOW_SIZE = 1984


class CryptoError(Exception):
    pass


class DecryptionError(CryptoError):
    """CryptoError::DecryptionError"""


class Rejected(CryptoError):
    """CryptoError::Rejected"""


def _vp(x):
    """Pointer of a numpy array / torch tensor / bytes-like (None passes through)."""
    if x is None:
        return None
    if hasattr(x, "data_ptr"):
        return ctypes.c_void_p(x.data_ptr())
    if isinstance(x, np.ndarray):
        return x.ctypes.data_as(ctypes.c_void_p)
    if isinstance(x, bytearray):
        return ctypes.cast((ctypes.c_char * len(x)).from_buffer(x), ctypes.c_void_p)
    raise TypeError(type(x))


def _stream_handle(stream):
    if stream is None:
        import torch

        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


def _ndesc(desc) -> int:
    """Descriptor count of a device tensor holding rg_pkt_desc rows (16 bytes each)."""
    nb = _nbytes(desc)
    assert nb % 16 == 0, "descriptor tensor must hold whole 16-byte rg_pkt_desc rows"
    return nb // 16


def _nbytes(t) -> int:
    if hasattr(t, "numel"):
        return t.numel() * t.element_size()
    return t.nbytes


class Engine:
    """One rg_ctx: a HIP device plus its staging buffers (one per process/GPU)."""

    def __init__(self, device: int = 0, library=None):
        """library: the loaded C library (default: the product librg_aead.so; tests of the test hooks pass
        _lib.lib_test())."""
        self._L = library if library is not None else lib()
        h = ctypes.c_void_p()
        self._check(self._L.rg_create(device, ctypes.byref(h)), "rg_create")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._L.rg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def library(self):
        return self._L

    def _check(self, rc: int, what: str) -> int:
        return check(rc, what, self._L)

    def set_lanes_per_packet(self, lanes: int):
        self._check(self._L.rg_set_lanes_per_packet(self._h, lanes), "rg_set_lanes_per_packet")

    def set_staged(self, kernel: int):
        """Kernel family: -1 = automatic by batch size (default), 0 = pipelined lane kernel,
        1/2 = LDS-staged tile kernel with that many 64-byte chunks per window."""
        self._check(self._L.rg_set_staged(self._h, kernel), "rg_set_staged")

    def kernel_for(self, n: int) -> int:
        """The kernel family a batch of n packets runs on (rg_get_kernel)."""
        return self._check(self._L.rg_get_kernel(self._h, n), "rg_get_kernel")

    def last_kernel(self) -> int:
        """The kernel family the most recent batched launch ran (rg_last_kernel; -1 before any)."""
        return self._L.rg_last_kernel(self._h)

    def set_plan(self, mode):
        """Size-class planner before the batched kernels: 0/False off, 1/True on, 2 auto (default)."""
        self._check(self._L.rg_set_plan(self._h, int(mode)), "rg_set_plan")

    def set_segments(self, k: int):
        """Segments per packet for the tile kernels: 0 = automatic, 1/2/4 = forced."""
        self._check(self._L.rg_set_segments(self._h, k), "rg_set_segments")

    def set_debug_mode(self, mode: int):
        """Diagnostics: 1 = compute-only seal, 2 = memory-only seal, 3 = stamps, 4/5/6 = non-temporal
        loads / stores / both on the pipelined kernel (outputs invalid except in mode 3)."""
        self._check(self._L.rg_set_debug_mode(self._h, mode), "rg_set_debug_mode")

    def set_debug_buffer(self, tensor):
        """Diagnostics: device buffer receiving per-wave stamps (include/rg_aead.h)."""
        self._check(self._L.rg_set_debug_buffer(self._h, _vp(tensor) if tensor is not None else None),
              "rg_set_debug_buffer")

    def set_host_slice(self, nbytes: int):
        """Byte span of one host-pipeline slice (rg_set_host_slice; default 8 MiB)."""
        self._check(self._L.rg_set_host_slice(self._h, nbytes), "rg_set_host_slice")

    def set_wait_timeout(self, ms: int):
        """Limit of every host wait of the library, in ms (rg_set_wait_timeout; default 10 000)."""
        self._check(self._L.rg_set_wait_timeout(self._h, ms), "rg_set_wait_timeout")

    def set_wg_per_cu(self, wg: int):
        self._check(self._L.rg_set_wg_per_cu(self._h, wg), "rg_set_wg_per_cu")

    def lanes_per_packet(self, n: int) -> int:
        return self._check(self._L.rg_get_lanes_per_packet(self._h, n), "rg_get_lanes_per_packet")

    # ---------------------------------------------------- device-resident
    def seal_dev(self, keys, receivers, desc, counters, buf, status, stream=None):
        """Enqueue a batched seal on `stream`; all tensors on this device.  status (uint8, one per packet) is
        required: RG_PKT_OK there is the proof that the packet was sealed (ABI 6)."""
        n = _ndesc(desc)
        nkeys = _nbytes(keys) // 32
        self._check(self._L.rg_seal_batch_dev(self._h, _vp(keys), _vp(receivers), nkeys, _vp(desc), _vp(counters), n,
                                        _vp(buf), _nbytes(buf), _vp(status), _stream_handle(stream)),
              "rg_seal_batch_dev")

    def open_dev(self, keys, desc, buf, status, counters_out=None, stream=None):
        n = _ndesc(desc)
        nkeys = _nbytes(keys) // 32
        self._check(self._L.rg_open_batch_dev(self._h, _vp(keys), nkeys, _vp(desc), n, _vp(buf), _nbytes(buf),
                                        _vp(status), _vp(counters_out), _stream_handle(stream)),
              "rg_open_batch_dev")

    def open_dev_rx(self, keys, rx_table, desc, buf, status, counters_out=None, key_idx_out=None, stream=None):
        """Open frames straight off the wire: sessions resolved on the device from each header's receiver
        index through rx_table (an rx_table() array moved to this device)."""
        n = _ndesc(desc)
        nkeys = _nbytes(keys) // 32
        cap = _nbytes(rx_table) // 8
        self._check(self._L.rg_open_batch_dev_rx(self._h, _vp(keys), nkeys, _vp(rx_table), cap, _vp(desc), n, _vp(buf),
                                           _nbytes(buf), _vp(status), _vp(counters_out), _vp(key_idx_out),
                                           _stream_handle(stream)), "rg_open_batch_dev_rx")

    def mac_verify_dev(self, keys, which: int, desc, buf, status, key_idx_out=None, stream=None):
        """HasMac::verify_mac1 (which=1, 32-byte keys) / verify_mac2 (which=2, 16-byte cookies) for a batch
        of handshake messages; key_idx KEY_SCAN tries every key (wg-proxy)."""
        n = _ndesc(desc)
        key_len = 32 if which == 1 else 16
        nkeys = _nbytes(keys) // key_len
        self._check(self._L.rg_mac_verify_batch_dev(self._h, _vp(keys), key_len, nkeys, which, _vp(desc), n, _vp(buf),
                                              _nbytes(buf), _vp(status), _vp(key_idx_out), _stream_handle(stream)),
              "rg_mac_verify_batch_dev")

    def synth_fill_dev(self, desc, inner_len, buf, seed: int, stream=None):
        n = _ndesc(desc)
        self._check(self._L.rg_synth_fill_dev(self._h, _vp(desc), _vp(inner_len), n, _vp(buf), _nbytes(buf), seed,
                                        _stream_handle(stream)), "rg_synth_fill_dev")

    # -------------------------------------------------------- host memory
    def seal_host(self, keys: np.ndarray, receivers, desc: np.ndarray, counters: np.ndarray, buf: np.ndarray):
        assert desc.dtype == DESC_DTYPE and buf.dtype == np.uint8 and buf.flags.c_contiguous
        keys = np.ascontiguousarray(keys, np.uint8)
        counters = np.ascontiguousarray(counters, np.uint64)
        rec = None if receivers is None else np.ascontiguousarray(receivers, np.uint32)
        status = np.zeros(max(len(desc), 1), np.uint8)
        self._check(self._L.rg_seal_batch_host(self._h, _vp(keys), _vp(rec), keys.size // 32, _vp(desc), _vp(counters),
                                         len(desc), _vp(buf), buf.nbytes, _vp(status)), "rg_seal_batch_host")
        return status[: len(desc)]

    def open_host(self, keys: np.ndarray, desc: np.ndarray, buf: np.ndarray):
        assert desc.dtype == DESC_DTYPE and buf.dtype == np.uint8 and buf.flags.c_contiguous
        keys = np.ascontiguousarray(keys, np.uint8)
        n = len(desc)
        status = np.zeros(max(n, 1), np.uint8)
        ctr = np.zeros(max(n, 1), np.uint64)
        self._check(self._L.rg_open_batch_host(self._h, _vp(keys), keys.size // 32, _vp(desc), n, _vp(buf), buf.nbytes,
                                         _vp(status), _vp(ctr)), "rg_open_batch_host")
        return status[:n], ctr[:n]

    # --------------------------------------------- per-message drop-in
    def chacha20poly1305_enc(self, key: bytes, nonce: bytes, aad: bytes, payload: bytearray) -> bytes:
        """Core::chacha20poly1305_enc: encrypts `payload` in place, returns the tag."""
        assert len(key) == 32 and len(nonce) == 12
        tag = bytearray(16)
        k, nz, a = bytearray(key), bytearray(nonce), bytearray(aad or b"\0")
        self._check(self._L.rg_chacha20poly1305_enc(self._h, _vp(k), _vp(nz), _vp(a), len(aad), _vp(payload) if payload
                                              else None, len(payload), _vp(tag)), "rg_chacha20poly1305_enc")
        return bytes(tag)

    def xchacha20poly1305_enc(self, key: bytes, nonce: bytes, aad: bytes, payload: bytearray) -> bytes:
        """Core::xchacha20poly1305_enc (prim.rs:202-212, the cookie AEAD): in place, returns the tag."""
        assert len(key) == 32 and len(nonce) == 24
        tag = bytearray(16)
        k, nz, a = bytearray(key), bytearray(nonce), bytearray(aad or b"\0")
        self._check(self._L.rg_xchacha20poly1305_enc(self._h, _vp(k), _vp(nz), _vp(a), len(aad), _vp(payload) if payload
                                               else None, len(payload), _vp(tag)), "rg_xchacha20poly1305_enc")
        return bytes(tag)

    def xchacha20poly1305_dec(self, key: bytes, nonce: bytes, aad: bytes, payload: bytearray, tag: bytes) -> None:
        """Core::xchacha20poly1305_dec (prim.rs:214-224): decrypts in place or raises DecryptionError."""
        assert len(key) == 32 and len(nonce) == 24 and len(tag) == 16
        k, nz, a, t = bytearray(key), bytearray(nonce), bytearray(aad or b"\0"), bytearray(tag)
        rc = self._check(self._L.rg_xchacha20poly1305_dec(self._h, _vp(k), _vp(nz), _vp(a), len(aad), _vp(payload)
                                                    if payload else None, len(payload), _vp(t)),
                   "rg_xchacha20poly1305_dec")
        if rc == PKT_DECRYPT_ERR:
            raise DecryptionError()

    def chacha20poly1305_dec(self, key: bytes, nonce: bytes, aad: bytes, payload: bytearray, tag: bytes) -> None:
        """Core::chacha20poly1305_dec: decrypts in place or raises DecryptionError."""
        assert len(key) == 32 and len(nonce) == 12 and len(tag) == 16
        k, nz, a, t = bytearray(key), bytearray(nonce), bytearray(aad or b"\0"), bytearray(tag)
        rc = self._check(self._L.rg_chacha20poly1305_dec(self._h, _vp(k), _vp(nz), _vp(a), len(aad), _vp(payload) if payload
                                                   else None, len(payload), _vp(t)), "rg_chacha20poly1305_dec")
        if rc == PKT_DECRYPT_ERR:
            raise DecryptionError()


def nonce(counter: int) -> bytes:
    """prim.rs:32-36: 00000000 || le64(counter)."""
    return b"\0" * 4 + int(counter).to_bytes(8, "little")


# ---------------------------------------------------------------- AntiReplay
class _ReplayStruct(ctypes.Structure):
    _fields_ = [("bitmap", ctypes.c_uint64 * 32), ("last", ctypes.c_uint64)]


class AntiReplay:
    """rustyguard_utils::anti_replay::AntiReplay, backed by the C implementation."""

    def __init__(self, _ptr=None):
        if _ptr is None:
            self._s = _ReplayStruct()
            self._p = ctypes.cast(ctypes.byref(self._s), ctypes.c_void_p)
            lib().rg_antireplay_init(self._p)
        else:
            self._p = ctypes.c_void_p(_ptr)

    def would_accept(self, n: int) -> bool:
        return bool(lib().rg_antireplay_would_accept(self._p, n))

    def mark_seen(self, n: int) -> None:
        lib().rg_antireplay_mark_seen(self._p, n)


class EncryptionKey:
    """prim.rs:376-399: seal with nonce(counter), counter += 1."""

    def __init__(self, engine: Engine, key: bytes):
        self.engine, self.key, self._counter = engine, bytes(key), 0

    def encrypt(self, payload: bytearray) -> bytes:
        n = self._counter
        self._counter += 1
        return self.engine.chacha20poly1305_enc(self.key, nonce(n), b"", payload)

    def counter(self) -> int:
        return self._counter


class DecryptionKey:
    """prim.rs:401-437: replay gate -> open -> mark_seen only on success."""

    def __init__(self, engine: Engine, key: bytes):
        self.engine, self.key, self.replay = engine, bytes(key), AntiReplay()

    def decrypt(self, counter: int, payload_and_tag: bytearray) -> bytearray:
        if not self.replay.would_accept(counter):
            raise Rejected()
        if len(payload_and_tag) < 16:
            raise DecryptionError()
        body = bytearray(payload_and_tag[:-16])
        self.engine.chacha20poly1305_dec(self.key, nonce(counter), b"", body, bytes(payload_and_tag[-16:]))
        payload_and_tag[:-16] = body
        self.replay.mark_seen(counter)
        return body


# ------------------------------------------------------------------ Sessions
class Group:
    """rg_group: one calling thread driving several GPUs (one context per entry of `devices`; a device
    may repeat).  Host-memory batches are split into contiguous ranges of about equal AEAD work, one per
    context; the library runs each context's pipeline on a worker thread of its own and returns when all
    are done (include/rg_aead.h, "several GPUs, one thread")."""

    def __init__(self, devices, library=None):
        self._L = library if library is not None else lib()
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        check(self._L.rg_group_create(devs, len(devices), ctypes.byref(h)), "rg_group_create", self._L)
        self._h = h
        self.devices = list(devices)

    @property
    def handle(self):
        return self._h

    @property
    def library(self):
        return self._L

    def __len__(self):
        return len(self.devices)

    def close(self):
        if getattr(self, "_h", None):
            self._L.rg_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def ctx(self, i: int):
        """Handle of the i-th context (for per-context knobs through the C ABI)."""
        return ctypes.c_void_p(self._L.rg_group_ctx(self._h, i))

    def engine(self, i: int) -> "Engine":
        """An Engine view of the i-th context (not owning it: the group destroys its contexts)."""
        return _ContextView(self, i)

    def seal_host(self, keys: np.ndarray, receivers, desc: np.ndarray, counters: np.ndarray, buf: np.ndarray):
        assert desc.dtype == DESC_DTYPE and buf.dtype == np.uint8 and buf.flags.c_contiguous
        keys = np.ascontiguousarray(keys, np.uint8)
        counters = np.ascontiguousarray(counters, np.uint64)
        rec = None if receivers is None else np.ascontiguousarray(receivers, np.uint32)
        status = np.zeros(max(len(desc), 1), np.uint8)
        check(self._L.rg_seal_batch_host_multi(self._h, _vp(keys), _vp(rec), keys.size // 32, _vp(desc),
                                               _vp(counters), len(desc), _vp(buf), buf.nbytes, _vp(status)),
              "rg_seal_batch_host_multi", self._L)
        return status[: len(desc)]

    def open_host(self, keys: np.ndarray, desc: np.ndarray, buf: np.ndarray):
        assert desc.dtype == DESC_DTYPE and buf.dtype == np.uint8 and buf.flags.c_contiguous
        keys = np.ascontiguousarray(keys, np.uint8)
        n = len(desc)
        status = np.zeros(max(n, 1), np.uint8)
        ctr = np.zeros(max(n, 1), np.uint64)
        check(self._L.rg_open_batch_host_multi(self._h, _vp(keys), keys.size // 32, _vp(desc), n, _vp(buf),
                                               buf.nbytes, _vp(status), _vp(ctr)), "rg_open_batch_host_multi", self._L)
        return status[:n], ctr[:n]

    @staticmethod
    def shards(shards, seal: bool):
        """The rg_dev_shard array of `shards` (one dict per context: keys, receivers, desc, counters, buf,
        status, counters_out, stream -- tensors on that context's device), built once for repeated calls."""
        assert len(shards) > 0
        return _shard_array(shards, seal=seal)

    def seal_dev(self, shards):
        """rg_seal_batch_dev_multi: one shard per context (a list of dicts or a Group.shards array), enqueued
        on each shard's stream without waiting."""
        arr = shards if isinstance(shards, ctypes.Array) else _shard_array(shards, seal=True)
        assert len(arr) == len(self.devices)
        check(self._L.rg_seal_batch_dev_multi(self._h, ctypes.cast(arr, ctypes.c_void_p)), "rg_seal_batch_dev_multi",
              self._L)

    def open_dev(self, shards):
        arr = shards if isinstance(shards, ctypes.Array) else _shard_array(shards, seal=False)
        assert len(arr) == len(self.devices)
        check(self._L.rg_open_batch_dev_multi(self._h, ctypes.cast(arr, ctypes.c_void_p)), "rg_open_batch_dev_multi",
              self._L)


class _ContextView(Engine):
    """Engine methods on a context owned by a Group."""

    def __init__(self, group: Group, i: int):
        h = group._L.rg_group_ctx(group.handle, i)
        if not h:
            raise _lib.RgError(f"group has no context {i}")
        self._L, self._h, self.device, self._group = group.library, ctypes.c_void_p(h), group.devices[i], group

    def close(self):
        self._h = None  # the group owns the context


class _DevShard(ctypes.Structure):
    """rg_dev_shard (include/rg_aead.h)."""
    _fields_ = [("keys", ctypes.c_void_p), ("receivers", ctypes.c_void_p), ("nkeys", ctypes.c_uint32),
                ("desc", ctypes.c_void_p), ("counters", ctypes.c_void_p), ("n", ctypes.c_size_t),
                ("buf", ctypes.c_void_p), ("buf_len", ctypes.c_size_t), ("status", ctypes.c_void_p),
                ("counters_out", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


def _shard_array(shards, seal: bool):
    arr = (_DevShard * len(shards))()
    for k, sh in enumerate(shards):
        x = arr[k]
        p = lambda t: _vp(t).value if t is not None else None  # noqa: E731
        x.keys = p(sh["keys"])
        x.nkeys = _nbytes(sh["keys"]) // 32
        x.desc = p(sh["desc"])
        x.n = _ndesc(sh["desc"])
        x.buf = p(sh["buf"])
        x.buf_len = _nbytes(sh["buf"])
        x.status = p(sh.get("status"))
        x.stream = _stream_handle(sh.get("stream")).value
        if seal:
            x.receivers = p(sh.get("receivers"))
            x.counters = p(sh["counters"])
        else:
            x.counters_out = p(sh.get("counters_out"))
    return arr


def split_batch(desc: np.ndarray, parts: int, open_: bool = False) -> np.ndarray:
    """rg_split_batch: bounds[0..parts] of the group split (contiguous ranges of about equal work)."""
    assert desc.dtype == DESC_DTYPE
    b = np.zeros(parts + 1, np.uint64)
    check(lib().rg_split_batch(_vp(desc), len(desc), int(open_), parts, _vp(b)), "rg_split_batch")
    return b.astype(np.int64)


class Sessions:
    """Transport half of rustyguard_core::Sessions (batched, host frames).  On a Group the host-frame
    batches run on every GPU of the group (rg_sessions_create_group)."""

    def __init__(self, engine, capacity: int = 64):
        self.engine = engine
        self._L = engine.library
        h = ctypes.c_void_p()
        if isinstance(engine, Group):
            self._check(self._L.rg_sessions_create_group(engine.handle, capacity, ctypes.byref(h)),
                        "rg_sessions_create_group")
        else:
            self._check(self._L.rg_sessions_create(engine.handle, capacity, ctypes.byref(h)), "rg_sessions_create")
        self._h = h

    def _check(self, rc: int, what: str) -> int:
        return check(rc, what, self._L)

    def __del__(self):
        try:
            if self._h:
                self._L.rg_sessions_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def insert(self, local_id: int, remote_id: int, send_key: bytes, recv_key: bytes, peer: int | None = None) -> int:
        """Install a transport session; `peer` (an id of the caller's) makes the sessions of one peer share
        its endpoint record (PeerState.endpoint, rustyguard-core/src/lib.rs:160-181)."""
        sk, rk = bytearray(send_key), bytearray(recv_key)
        if peer is not None:
            return self._check(self._L.rg_sessions_insert_peer(self._h, local_id, remote_id, _vp(sk), _vp(rk), peer),
                               "rg_sessions_insert_peer")
        return self._check(self._L.rg_sessions_insert(self._h, local_id, remote_id, _vp(sk), _vp(rk)), "rg_sessions_insert")

    def remove(self, slot: int):
        self._check(self._L.rg_sessions_remove(self._h, slot), "rg_sessions_remove")

    def lookup(self, local_id: int) -> int | None:
        rc = self._L.rg_sessions_lookup(self._h, local_id)
        return None if rc < 0 else rc

    def send_counter(self, slot: int) -> int:
        return int(self._L.rg_sessions_send_counter(self._h, slot))

    def set_send_counter(self, slot: int, counter: int):
        self._check(self._L.rg_sessions_set_send_counter(self._h, slot, counter), "rg_sessions_set_send_counter")

    def replay(self, slot: int) -> AntiReplay:
        return AntiReplay(_ptr=self._L.rg_sessions_replay(self._h, slot))

    def send_batch(self, slots, desc: np.ndarray, buf: np.ndarray):
        slots = np.ascontiguousarray(slots, np.uint32)
        n = len(desc)
        status = np.zeros(max(n, 1), np.uint8)
        rekey = np.zeros(max(n, 1), np.uint8)
        self._check(self._L.rg_send_batch(self._h, _vp(slots), _vp(desc), n, _vp(buf), buf.nbytes, _vp(status), _vp(rekey)),
              "rg_send_batch")
        return status[:n], rekey[:n]

    def recv_batch(self, desc: np.ndarray, buf: np.ndarray, src=None, flags: bool = False):
        """Sessions::recv_message for a batch of data frames; with src (one opaque source tag per
        frame) the authenticated ones move their session's endpoint (decrypt_packet,
        rustyguard-core/src/lib.rs:664-679).  Returns (status, slots) or, with flags=True,
        (status, slots, flags) where flags holds RECV_AUTHENTICATED / RECV_KEEPALIVE bits."""
        n = len(desc)
        status = np.zeros(max(n, 1), np.uint8)
        slots = np.zeros(max(n, 1), np.uint32)
        fl = np.zeros(max(n, 1), np.uint8)
        srcs = None if src is None else np.ascontiguousarray(src, np.uint64)
        self._check(self._L.rg_recv_batch_ex(self._h, _vp(desc), n, _vp(buf), buf.nbytes, _vp(srcs), _vp(status),
                                     _vp(slots), _vp(fl)), "rg_recv_batch_ex")
        return (status[:n], slots[:n], fl[:n]) if flags else (status[:n], slots[:n])

    def send_batch_dev(self, slots, desc, buf, status, stream=None):
        """rg_send_batch_dev: device frames / descriptors (torch tensors), host slots; enqueued on
        `stream`, returns the rekey flags (host) without waiting for the GPU."""
        slots = np.ascontiguousarray(slots, np.uint32)
        n = _ndesc(desc)
        rekey = np.zeros(max(n, 1), np.uint8)
        self._check(self._L.rg_send_batch_dev(self._h, _vp(slots), _vp(desc), n, _vp(buf), _nbytes(buf), _vp(status),
                                      _vp(rekey), _stream_handle(stream)), "rg_send_batch_dev")
        return rekey[:n]

    def recv_batch_dev(self, desc, buf, status, stream=None):
        """rg_recv_batch_dev: enqueue the GPU half of a device-resident receive; finish it with
        recv_batch_dev_finish."""
        self._check(self._L.rg_recv_batch_dev(self._h, _vp(desc), _ndesc(desc), _vp(buf), _nbytes(buf), _vp(status),
                                      _stream_handle(stream)), "rg_recv_batch_dev")

    def recv_batch_dev_finish(self, n: int, src=None):
        """rg_recv_batch_dev_finish: the in-order anti-replay pass of the pending device receive.
        Returns (status, slots, flags) as host arrays."""
        status = np.zeros(max(n, 1), np.uint8)
        slots = np.zeros(max(n, 1), np.uint32)
        fl = np.zeros(max(n, 1), np.uint8)
        srcs = None if src is None else np.ascontiguousarray(src, np.uint64)
        self._check(self._L.rg_recv_batch_dev_finish(self._h, _vp(srcs), _vp(status), _vp(slots), _vp(fl)),
              "rg_recv_batch_dev_finish")
        return status[:n], slots[:n], fl[:n]

    def set_time(self, now_ns: int):
        """The table's clock (Sessions::turn's state.now), monotonic nanoseconds."""
        self._L.rg_sessions_set_time(self._h, int(now_ns))

    def endpoint(self, slot: int):
        """Source tag of the session's last authenticated packet, or None."""
        out = ctypes.c_uint64()
        rc = self._L.rg_sessions_endpoint(self._h, slot, ctypes.byref(out))
        if rc == -4:  # RG_ENOTFOUND
            return None
        self._check(rc, "rg_sessions_endpoint")
        return int(out.value)

    def peer_endpoint(self, peer: int):
        """Source tag of the peer's last authenticated packet (any of its sessions), or None."""
        out = ctypes.c_uint64()
        rc = self._L.rg_peer_endpoint(self._h, peer, ctypes.byref(out))
        if rc == -4:  # RG_ENOTFOUND
            return None
        self._check(rc, "rg_peer_endpoint")
        return int(out.value)

    def keepalive(self, slot: int):
        """rg_sessions_keepalive: the Keepalive timer entry with its destination -- the peer's endpoint
        (time.rs:135) when a keepalive is due, else None.  Raises when due with no endpoint known."""
        out = ctypes.c_uint64()
        rc = self._check(self._L.rg_sessions_keepalive(self._h, slot, ctypes.byref(out)), "rg_sessions_keepalive")
        return int(out.value) if rc == 1 else None

    def keepalive_due(self, slot: int) -> bool:
        """The Keepalive timer entry (time.rs:114-141): clears the pending flag; True when a keepalive
        (an empty payload through send_batch) should go out now."""
        return bool(self._check(self._L.rg_sessions_keepalive_due(self._h, slot), "rg_sessions_keepalive_due"))


def rx_table(receivers, key_idx, cap: int | None = None) -> np.ndarray:
    """Receiver-index table for open_dev_rx (rg_rx_table_build): uint32 [cap, 2] of (receiver, key_idx),
    cap a power of two >= 2 n (default: the smallest)."""
    rec = np.ascontiguousarray(receivers, np.uint32)
    idx = np.ascontiguousarray(key_idx, np.uint32)
    if cap is None:
        cap = 1 << max(1, int(2 * len(rec) - 1).bit_length())
    table = np.zeros((cap, 2), np.uint32)
    check(lib().rg_rx_table_build(_vp(rec), _vp(idx), len(rec), _vp(table), cap), "rg_rx_table_build")
    return table


def rx_find(table: np.ndarray, receiver: int) -> int:
    """Host lookup in an rx_table(): key index or -1."""
    return int(lib().rg_rx_table_find(_vp(table), table.shape[0], receiver))


def numa_node(engine) -> int:
    """rg_numa_node: the host NUMA node closest to the engine's (or group context's) GPU, -1 if unknown."""
    return int(engine.library.rg_numa_node(engine.handle))


def _node_free_bytes(node: int):
    """MemFree of a NUMA node (sysfs), or None when unreadable."""
    try:
        with open(f"/sys/devices/system/node/node{node}/meminfo") as f:
            for line in f:
                if "MemFree:" in line:
                    return int(line.split()[-2]) * 1024
    except (OSError, ValueError, IndexError):
        return None
    return None


def placed_host_buffer(group: "Group", desc: np.ndarray, nbytes: int, open_: bool = False):
    """A frame buffer for a host batch over `group`, placed for it (include/rg_aead.h, NUMA placement): an
    anonymous mapping whose part k -- the frames of rg_split_batch's part k -- is bound to context k's NUMA
    node (rg_numa_bind) and first-touched there, then the whole buffer pinned (rg_host_register).  Returns
    (uint8 array, placement list).  The pin is dropped when the array's buffer is collected."""
    import mmap
    import weakref

    L = group.library
    n = len(desc)
    mm = mmap.mmap(-1, max(nbytes, 1), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    arr = np.frombuffer(mm, np.uint8)
    p = arr.ctypes.data
    bounds = split_batch(desc, len(group), open_) if n else np.zeros(len(group) + 1, np.int64)
    placement = []
    for k in range(len(group)):
        lo, hi = int(bounds[k]), int(bounds[k + 1])
        node = numa_node(group.engine(k))
        part = {"context": k, "device": group.devices[k], "numa_node": node, "packets": hi - lo, "bound": False}
        if hi > lo:
            a = int(desc["offset"][lo])
            last = int(np.argmax(desc["offset"][lo:hi])) + lo
            b = min(nbytes, int(desc["offset"][last]) + int(desc["len"][last]) + (0 if open_ else 32))
            part["bytes"] = b - a
            free = _node_free_bytes(node) if node >= 0 else None
            # a strict bind on a node without the room would leave the first touch to the OOM killer: bind
            # only with twice the part free there (else the pages land where the kernel puts them)
            if node >= 0 and b > a and (free is None or free >= 2 * (b - a)):
                part["bound"] = L.rg_numa_bind(ctypes.c_void_p(p + a), b - a, node) == 0
            elif free is not None:
                part["unbound_reason"] = f"node {node} has {free >> 20} MiB free"
        placement.append(part)
    arr[:] = 0  # first touch: each part's pages on its node
    check(L.rg_host_register(ctypes.c_void_p(p), arr.nbytes), "rg_host_register", L)

    def _release(lib=L, ptr=p, m=mm):
        lib.rg_host_unregister(ctypes.c_void_p(ptr))

    weakref.finalize(arr, _release)
    return arr, placement


def host_alloc(nbytes: int) -> np.ndarray:
    """Pinned host buffer (hipHostMalloc) viewed as uint8; freed with the array's owner."""
    p = lib().rg_host_alloc(nbytes)
    if not p:
        raise _lib.RgError("rg_host_alloc failed")
    buf = (ctypes.c_uint8 * nbytes).from_address(p)
    arr = np.frombuffer(buf, dtype=np.uint8)
    import weakref

    weakref.finalize(buf, lib().rg_host_free, ctypes.c_void_p(p))
    return arr
