"""ctypes binding of librg_aead.so (include/rg_aead.h).

There is deliberately no CPU fallback: if the HIP library is missing or fails
to load, every entry point raises.  (The CPU oracle under oracle/ is test
infrastructure and is never imported from this package.)
"""
from __future__ import annotations

import ctypes
import os

from . import build as _build

_lib = None
_test_lib = None

c_u8p = ctypes.c_void_p
c_vp = ctypes.c_void_p
c_size = ctypes.c_size_t
c_u32 = ctypes.c_uint32
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int

# name -> (restype, argtypes); mirrors include/rg_aead.h one to one
SIGNATURES = {
    "rg_abi_version": (c_int, []),
    "rg_last_error": (ctypes.c_char_p, []),
    "rg_create": (c_int, [c_int, ctypes.POINTER(c_vp)]),
    "rg_destroy": (None, [c_vp]),
    "rg_seal_batch_dev": (c_int, [c_vp, c_u8p, c_vp, c_u32, c_vp, c_vp, c_size, c_u8p, c_size, c_u8p, c_vp]),
    "rg_open_batch_dev": (c_int, [c_vp, c_u8p, c_u32, c_vp, c_size, c_u8p, c_size, c_u8p, c_vp, c_vp]),
    "rg_set_lanes_per_packet": (c_int, [c_vp, c_int]),
    "rg_get_lanes_per_packet": (c_int, [c_vp, c_size]),
    "rg_set_wg_per_cu": (c_int, [c_vp, c_int]),
    "rg_set_debug_mode": (c_int, [c_vp, c_int]),
    "rg_set_staged": (c_int, [c_vp, c_int]),
    "rg_mac_verify_batch_dev": (c_int, [c_vp, c_vp, ctypes.c_uint32, ctypes.c_uint32, c_int, c_vp, c_size, c_vp,
                                        c_size, c_vp, c_vp, c_vp]),
    "rg_rx_table_build": (c_int, [c_vp, c_vp, c_size, c_vp, ctypes.c_uint32]),
    "rg_rx_table_find": (ctypes.c_int64, [c_vp, ctypes.c_uint32, ctypes.c_uint32]),
    "rg_open_batch_dev_rx": (c_int, [c_vp, c_vp, ctypes.c_uint32, c_vp, ctypes.c_uint32, c_vp, c_size, c_vp, c_size,
                                     c_vp, c_vp, c_vp, c_vp]),
    "rg_get_kernel": (c_int, [c_vp, c_size]),
    "rg_last_kernel": (c_int, [c_vp]),
    "rg_set_plan": (c_int, [c_vp, c_int]),
    "rg_set_segments": (c_int, [c_vp, c_int]),
    "rg_set_debug_buffer": (c_int, [c_vp, c_vp]),
    "rg_seal_batch_host": (c_int, [c_vp, c_u8p, c_vp, c_u32, c_vp, c_vp, c_size, c_u8p, c_size, c_u8p]),
    "rg_open_batch_host": (c_int, [c_vp, c_u8p, c_u32, c_vp, c_size, c_u8p, c_size, c_u8p, c_vp]),
    "rg_host_alloc": (c_vp, [c_size]),
    "rg_host_free": (None, [c_vp]),
    "rg_chacha20poly1305_enc": (c_int, [c_vp, c_u8p, c_u8p, c_u8p, c_size, c_u8p, c_size, c_u8p]),
    "rg_chacha20poly1305_dec": (c_int, [c_vp, c_u8p, c_u8p, c_u8p, c_size, c_u8p, c_size, c_u8p]),
    "rg_xchacha20poly1305_enc": (c_int, [c_vp, c_u8p, c_u8p, c_u8p, c_size, c_u8p, c_size, c_u8p]),
    "rg_xchacha20poly1305_dec": (c_int, [c_vp, c_u8p, c_u8p, c_u8p, c_size, c_u8p, c_size, c_u8p]),
    "rg_antireplay_init": (None, [c_vp]),
    "rg_antireplay_would_accept": (c_int, [c_vp, c_u64]),
    "rg_antireplay_mark_seen": (None, [c_vp, c_u64]),
    "rg_sessions_create": (c_int, [c_vp, c_u32, ctypes.POINTER(c_vp)]),
    "rg_sessions_destroy": (None, [c_vp]),
    "rg_sessions_insert": (c_int, [c_vp, c_u32, c_u32, c_u8p, c_u8p]),
    "rg_sessions_remove": (c_int, [c_vp, c_u32]),
    "rg_sessions_lookup": (c_int, [c_vp, c_u32]),
    "rg_sessions_send_counter": (c_u64, [c_vp, c_u32]),
    "rg_sessions_set_send_counter": (c_int, [c_vp, c_u32, c_u64]),
    "rg_sessions_replay": (c_vp, [c_vp, c_u32]),
    "rg_send_batch": (c_int, [c_vp, c_vp, c_vp, c_size, c_u8p, c_size, c_u8p, c_u8p]),
    "rg_recv_batch": (c_int, [c_vp, c_vp, c_size, c_u8p, c_size, c_u8p, c_vp]),
    "rg_recv_batch_ex": (c_int, [c_vp, c_vp, c_size, c_u8p, c_size, c_vp, c_u8p, c_vp, c_u8p]),
    "rg_sessions_set_time": (None, [c_vp, c_u64]),
    "rg_sessions_endpoint": (c_int, [c_vp, c_u32, c_vp]),
    "rg_sessions_keepalive_due": (c_int, [c_vp, c_u32]),
    "rg_send_batch_dev": (c_int, [c_vp, c_vp, c_vp, c_size, c_vp, c_size, c_vp, c_u8p, c_vp]),
    "rg_recv_batch_dev": (c_int, [c_vp, c_vp, c_size, c_vp, c_size, c_vp, c_vp]),
    "rg_recv_batch_dev_finish": (c_int, [c_vp, c_vp, c_u8p, c_vp, c_u8p]),
    "rg_synth_fill_dev": (c_int, [c_vp, c_vp, c_vp, c_size, c_u8p, c_size, c_u64, c_vp]),
    "rg_sessions_insert_peer": (c_int, [c_vp, c_u32, c_u32, c_u8p, c_u8p, c_u32]),
    "rg_peer_endpoint": (c_int, [c_vp, c_u32, c_vp]),
    "rg_sessions_keepalive": (c_int, [c_vp, c_u32, c_vp]),
    "rg_group_create": (c_int, [c_vp, c_int, ctypes.POINTER(c_vp)]),
    "rg_group_destroy": (None, [c_vp]),
    "rg_group_size": (c_int, [c_vp]),
    "rg_group_ctx": (c_vp, [c_vp, c_int]),
    "rg_split_batch": (c_int, [c_vp, c_size, c_int, c_int, c_vp]),
    "rg_seal_batch_host_multi": (c_int, [c_vp, c_u8p, c_vp, c_u32, c_vp, c_vp, c_size, c_u8p, c_size, c_u8p]),
    "rg_open_batch_host_multi": (c_int, [c_vp, c_u8p, c_u32, c_vp, c_size, c_u8p, c_size, c_u8p, c_vp]),
    "rg_seal_batch_dev_multi": (c_int, [c_vp, c_vp]),
    "rg_open_batch_dev_multi": (c_int, [c_vp, c_vp]),
    "rg_sessions_create_group": (c_int, [c_vp, c_u32, ctypes.POINTER(c_vp)]),
    "rg_set_host_slice": (c_int, [c_vp, c_size]),
    "rg_set_wait_timeout": (c_int, [c_vp, c_u32]),
    "rg_numa_node": (c_int, [c_vp]),
    "rg_numa_bind": (c_int, [c_vp, c_size, c_int]),
    "rg_host_register": (c_int, [c_vp, c_size]),
    "rg_host_unregister": (c_int, [c_vp]),
}

# include/rg_aead_test.h: exported by the test library (librg_aead_test.so) only
TEST_SIGNATURES = {
    "rg_debug_read_arena": (c_int, [c_vp, c_int, c_vp, c_size]),
    "rg_debug_fail_reserve": (None, [c_int]),
    "rg_debug_plan_handoff": (None, [c_int]),
    "rg_debug_lose_completions": (None, [c_int]),
    "rg_debug_wait_selftest": (c_int, [c_u32, c_u32, c_vp, c_vp]),
    "rg_debug_last_wipe": (ctypes.c_int64, [c_vp, c_size, c_vp]),
    "rg_debug_secret_state": (c_int, [c_vp, c_int, c_vp, c_vp]),
}


class RgError(RuntimeError):
    pass


def lib_path() -> str:
    return _build.LIB


def _load(path: str, sigs: dict, build_if_missing: bool, partial: bool = False):
    """partial: an experimental build (RG_AEAD_LIB) may predate the newest entry points; those are left
    unbound instead of failing the load (the in-tree libraries must export every one)."""
    if not os.path.exists(path):
        if not build_if_missing:
            raise RgError(f"{os.path.basename(path)} missing at {path}; run python -m rustyguard_amd.build")
        _build.build()
    L = ctypes.CDLL(path)
    for name, (res, args) in sigs.items():
        if partial and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def lib(build_if_missing: bool = True):
    """Load librg_aead.so (the product library); raise loudly if it cannot be loaded."""
    global _lib
    if _lib is None:
        path = os.environ.get("RG_AEAD_LIB") or _build.LIB  # override: experimental builds only
        _lib = _load(path, SIGNATURES, build_if_missing, partial=path != _build.LIB)
    return _lib


def lib_test(build_if_missing: bool = True):
    """Load librg_aead_test.so: the product kernels plus the test hooks of include/rg_aead_test.h.
    Only the tests that check key wiping and allocation failures use it; its contexts are its own
    (a handle of one library is never passed to the other)."""
    global _test_lib
    if _test_lib is None:
        _test_lib = _load(_build.TEST_LIB, {**SIGNATURES, **TEST_SIGNATURES}, build_if_missing)
    return _test_lib


def check(rc: int, what: str, L=None) -> int:
    if rc < 0:
        err = (L or lib()).rg_last_error()
        raise RgError(f"{what} failed ({rc}): {err.decode() if err else ''}")
    return rc
