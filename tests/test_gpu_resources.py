"""Resource handling of the C ABI.

- A context whose creation fails part way gives back everything it had allocated (rg_create's failure
  path releases through the buffers' owners; round 4 deleted the context and leaked its device memory).
- Key material in device memory is wiped in stream order: a key-table regrow waits for the buffer's own
  readers only, never for the whole device (round 4 called hipDeviceSynchronize before every wipe, so a
  regrow stalled every stream, the caller's unrelated torch work included).  The reference zeroizes keys on
  drop (rustyguard-crypto/src/prim.rs:227-231)."""
import ctypes
import time

import numpy as np
import pytest
import torch

from oracle import oracle
from rustyguard_amd import _lib, aead
from rustyguard_amd.workloads import DESC_DTYPE

pytestmark = pytest.mark.gpu

ALLOCS_IN_CREATE = 5  # rg_create: the flattened kernel's store sink, the device planner's pool, 3 slot pools


def _free_bytes() -> int:
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info(0)[0]


def test_failed_create_releases_what_it_allocated():
    """rg_debug_fail_reserve(k) fails the k-th allocation inside rg_create; for every k the call fails
    cleanly, and 8 rounds over every k leave the device's free memory where it was (the store sink alone
    is CUs x 16 KiB = 4 MiB: 32 leaked sinks would show as 128 MiB)."""
    L = _lib.lib_test()
    aead.Engine(0, library=L).close()  # warm: the runtime's own first-use allocations
    for k in range(1, ALLOCS_IN_CREATE + 1):  # one failing round first (allocator caches settle)
        L.rg_debug_fail_reserve(k)
        with pytest.raises(_lib.RgError):
            aead.Engine(0, library=L)
        L.rg_debug_fail_reserve(0)
    before = _free_bytes()
    for _ in range(8):
        for k in range(1, ALLOCS_IN_CREATE + 1):
            L.rg_debug_fail_reserve(k)
            try:
                with pytest.raises(_lib.RgError):
                    aead.Engine(0, library=L)
            finally:
                L.rg_debug_fail_reserve(0)
    after = _free_bytes()
    assert before - after < (16 << 20), f"failed rg_create calls leaked {(before - after) >> 20} MiB"
    e = aead.Engine(0, library=L)  # and a normal create still works
    e.close()


def _mac_batch(rng, nkeys, n=2000):
    from test_gpu_parity import _handshake_batch  # tests/ is on sys.path (pytest rootdir import)

    keys = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    desc, buf = _handshake_batch(rng, n, keys, 32, 1)
    desc["key_idx"][::3] = aead.KEY_SCAN
    want, wkey = oracle.mac_verify_batch(keys, 1, desc, buf)
    return keys, desc, buf, want, wkey


def test_key_table_regrow_waits_for_no_other_stream():
    """A call that regrows the context's MAC key-state table (more keys than before) returns, and its own
    stream completes, while an unrelated stream of the same device is still busy: the wipe of the old
    table is ordered behind that table's readers only (events), zeroed and freed on the call's stream."""
    eng = aead.Engine(0)
    rng = np.random.default_rng(71)
    s = torch.cuda.Stream()
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    small = _mac_batch(rng, 4)
    big = _mac_batch(rng, 200)  # 200 x 32 B > the 4 KiB first block: a real regrow
    args = []
    for keys, desc, buf, _, _ in (small, big):
        args.append((dev(keys), dev(desc.view(np.uint8).reshape(-1, 16)), dev(buf),
                     torch.zeros(len(desc), dtype=torch.uint8, device="cuda"),
                     torch.zeros(len(desc), dtype=torch.int32, device="cuda")))
    torch.cuda.synchronize()
    eng.mac_verify_dev(args[0][0], 1, args[0][1], args[0][2], args[0][3], args[0][4], stream=s)  # a small table first
    torch.cuda.synchronize()
    busy = torch.cuda.Stream()
    with torch.cuda.stream(busy):
        torch.cuda._sleep(int(6e8))  # ~300 ms of spinning on another stream
    done = torch.cuda.Event()
    done.record(busy)
    t0 = time.perf_counter()
    eng.mac_verify_dev(args[1][0], 1, args[1][1], args[1][2], args[1][3], args[1][4], stream=s)  # regrow: 4 -> 200 key states
    call_s = time.perf_counter() - t0
    s.synchronize()
    own_s = time.perf_counter() - t0
    still_busy = not done.query()
    torch.cuda.synchronize()
    assert still_busy, (f"the regrowing call or its stream waited for an unrelated stream "
                        f"(call {call_s * 1e3:.1f} ms, own stream done after {own_s * 1e3:.1f} ms)")
    for (keys, desc, buf, want, wkey), a in zip((small, big), args):
        assert list(a[3].cpu().numpy()) == list(want)
        assert list(a[4].cpu().numpy().view(np.uint32)) == list(wkey)
    eng.close()


def test_host_path_key_table_regrow_matches_oracle(engine):
    """The host path's key table (rg_seal_batch_host) regrown between calls (3 -> 40 -> 3 -> 200 keys):
    every batch still seals bit-exactly (the new table is uploaded on the upload stream after the old
    one's wipe; a slice's kernel runs only after its upload)."""
    rng = np.random.default_rng(72)
    for nk in (3, 40, 3, 200):
        n = 500
        desc = np.zeros(n, DESC_DTYPE)
        desc["len"] = rng.choice([0, 64, 576, 1504], n)
        desc["offset"] = np.concatenate([[0], np.cumsum(desc["len"][:-1].astype(np.uint64) + 32)])
        desc["key_idx"] = rng.integers(0, nk, n)
        kt = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
        rec = rng.integers(0, 2**32, nk, dtype=np.uint64).astype(np.uint32)
        ctr = rng.integers(0, 2**40, n, dtype=np.uint64)
        buf = rng.integers(0, 256, int(desc["offset"][-1]) + 1600, dtype=np.uint8)
        want = buf.copy()
        oracle.seal_batch(kt, rec, desc, ctr, want)
        st = engine.seal_host(kt, rec, desc, ctr, buf)
        assert (st == 0).all() and np.array_equal(buf, want), nk


def _mac_args(eng, batch):
    keys, desc, buf, want, wkey = batch
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    return (dev(keys), dev(desc.view(np.uint8).reshape(-1, 16)), dev(buf),
            torch.zeros(len(desc), dtype=torch.uint8, device="cuda"),
            torch.zeros(len(desc), dtype=torch.int32, device="cuda"))


def _mac_ok(args, batch):
    _, _, _, want, wkey = batch
    return (list(args[3].cpu().numpy()) == list(want)
            and list(args[4].cpu().numpy().view(np.uint32)) == list(wkey))


def _state(L, eng, which=2):
    retired, users = ctypes.c_uint32(), ctypes.c_uint32()
    cap = L.rg_debug_secret_state(eng.handle, which, ctypes.byref(retired), ctypes.byref(users))
    return cap, retired.value, users.value


def _last_wipe(L, nbytes=4096):
    buf = np.full(nbytes, 0xCC, np.uint8)
    wipes = ctypes.c_uint64()
    m = L.rg_debug_last_wipe(buf.ctypes.data_as(ctypes.c_void_p), nbytes, ctypes.byref(wipes))
    return buf[:m], wipes.value


def test_regrow_and_destroy_leave_no_key_bytes():
    """the old MAC key-state block is zeroed before it is freed -- read back from the device
    between its wipe and its free (test hook) -- on a regrow and again on rg_destroy."""
    L = _lib.lib_test()
    eng = aead.Engine(0, library=L)
    rng = np.random.default_rng(73)
    small, big = _mac_batch(rng, 4), _mac_batch(rng, 200)  # 200 x 32 B > the 4 KiB first block: a regrow
    a = _mac_args(eng, small)
    eng.mac_verify_dev(*a[:1], 1, *a[1:])
    torch.cuda.synchronize()
    _, w0 = _last_wipe(L)
    b = _mac_args(eng, big)
    eng.mac_verify_dev(*b[:1], 1, *b[1:])
    torch.cuda.synchronize()
    blk, w1 = _last_wipe(L)
    assert w1 == w0 + 1 and len(blk) == 4096 and not blk.any(), (w0, w1, blk[:16])
    assert _mac_ok(a, small) and _mac_ok(b, big)
    eng.close()
    blk, w2 = _last_wipe(L)
    assert w2 >= w1 + 1 and len(blk) > 0 and not blk.any()


def test_captured_key_states_are_not_freed_under_the_graph():
    """a MAC verify captured into a graph reads the context's key-state block; a later
    regrow outside the capture must not free that block under the graph.  The block is retired (kept until
    rg_destroy), and replaying the graph after the regrow still gives the oracle's verdicts."""
    L = _lib.lib_test()
    eng = aead.Engine(0, library=L)
    rng = np.random.default_rng(74)
    small, big = _mac_batch(rng, 4), _mac_batch(rng, 200)
    a = _mac_args(eng, small)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.mac_verify_dev(*a[:1], 1, *a[1:], stream=s)  # warm: the 4 KiB block exists before the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        eng.mac_verify_dev(*a[:1], 1, *a[1:])
    torch.cuda.synchronize()
    assert _state(L, eng)[0] == 1  # captured
    b = _mac_args(eng, big)
    eng.mac_verify_dev(*b[:1], 1, *b[1:])  # regrow outside the capture
    torch.cuda.synchronize()
    cap, retired, _ = _state(L, eng)
    assert cap == 0 and retired == 1
    a[3].zero_()
    a[4].zero_()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert _mac_ok(a, small) and _mac_ok(b, big)
    _, w0 = _last_wipe(L)
    del g
    eng.close()  # the retired block and the current one: both wiped, then freed
    blk, w1 = _last_wipe(L)
    assert w1 >= w0 + 2 and not blk.any()


def test_key_state_events_do_not_grow_with_streams():
    """a caller making a fresh stream per call no longer grows the list of stream events that
    guard the key-state block (completed ones are dropped)."""
    L = _lib.lib_test()
    eng = aead.Engine(0, library=L)
    rng = np.random.default_rng(75)
    small = _mac_batch(rng, 4, n=64)
    a = _mac_args(eng, small)
    for _ in range(24):
        s = torch.cuda.Stream()
        eng.mac_verify_dev(*a[:1], 1, *a[1:], stream=s)
        s.synchronize()
    assert _state(L, eng)[2] <= 2
    assert _mac_ok(a, small)
    eng.close()
