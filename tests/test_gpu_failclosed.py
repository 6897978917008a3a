"""Fail-closed statuses.

Round 5 once left a whole batch unsealed with its statuses untouched: the planner read a stale
finished-workgroup count, no workgroup found itself last, the pipelined kernel got no schedule -- and a
status array that happened to hold zeros read RG_PKT_OK for every packet.  For open that is ciphertext
handed up as authenticated, and the reference moves the replay window and the endpoint only after the AEAD
verifies (rustyguard-core/src/lib.rs:659-662, rustyguard-crypto/src/prim.rs:419-433).

The test library's hooks (include/rg_aead_test.h) recreate the lost hand-off on purpose:
  rg_debug_plan_handoff(1)  the planner's finished-workgroup count starts stale (no schedule is handed over)
  rg_debug_plan_handoff(2)  the tile kernel's grid-wide pool starts past its end (pooled tiles never taken)
and the assertions are the contract of include/rg_aead.h: no packet the kernel never finished reads OK, a
host call reports RG_EDEVICE, the replay pass marks nothing seen, no endpoint moves -- and the context
works again once the hook is off.  Also here: a second stream on a busy context is refused, seal requires
a status array, and bounded waits turn a lost completion into an error."""
import ctypes
import time

import numpy as np
import pytest
import torch

from oracle import oracle
from rustyguard_amd import _lib, aead, workloads
from rustyguard_amd.aead import Engine, Sessions
from rustyguard_amd.workloads import DESC_DTYPE

pytestmark = pytest.mark.gpu

PENDING = aead.PKT_PENDING


@pytest.fixture(scope="module")
def L():
    return _lib.lib_test()


@pytest.fixture
def teng(L):
    e = Engine(0, library=L)
    yield e
    L.rg_debug_plan_handoff(0)
    L.rg_debug_lose_completions(0)
    torch.cuda.synchronize()
    e.close()


def _vp(a):
    return aead._vp(a)


def _frames(sizes, rng):
    desc = np.zeros(len(sizes), DESC_DTYPE)
    off = 0
    for i, p in enumerate(sizes):
        desc[i] = (off, p, 0)
        off += p + 32
    buf = np.zeros(off + 64, np.uint8)
    for d in desc:
        buf[d["offset"] + 16: d["offset"] + 16 + d["len"]] = rng.integers(0, 256, d["len"], dtype=np.uint8)
    return desc, buf


def _pair(eng, seed=3):
    rng = np.random.default_rng(seed)
    k1, k2 = rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    a, b = Sessions(eng, 4), Sessions(eng, 4)
    sa = a.insert(0x1111, 0x2222, k1, k2)
    sb = b.insert(0x2222, 0x1111, k2, k1)
    return a, b, sa, sb


def _sealed_for_a(b, sb, n, rng):
    """n frames sealed by B to A (the hook off), as A receives them."""
    desc, buf = _frames(list(rng.integers(1, 40, n) * 16), rng)
    st, _ = b.send_batch([sb] * n, desc, buf)
    assert (st == 0).all()
    od = desc.copy()
    od["len"] += 32
    return od, buf


def _planned_pipe(eng):
    eng.set_staged(0)
    eng.set_plan(1)


def _recv_raw(L, a, desc, buf, src):
    """rg_recv_batch_ex without the wrapper's raise: (rc, status, slots, flags)."""
    n = len(desc)
    status = np.full(n, 0, np.uint8)  # zeros: what a fail-open library would have left as "OK"
    slots = np.zeros(n, np.uint32)
    fl = np.full(n, 0xAA, np.uint8)
    rc = L.rg_recv_batch_ex(a._h, _vp(desc), n, _vp(buf), buf.nbytes, _vp(src), _vp(status), _vp(slots), _vp(fl))
    return rc, status, slots, fl


def test_lost_handoff_host_recv_fails_closed(L, teng):
    """Host-frame receive over the planned pipelined kernel with the planner's hand-off lost: RG_EDEVICE,
    every status RG_PKT_PENDING, no flag, the window untouched (every counter still accepted), no endpoint,
    every frame still the ciphertext that arrived.  With the hook off the same batch is accepted."""
    a, b, sa, sb = _pair(teng)
    _planned_pipe(teng)
    rng = np.random.default_rng(5)
    desc, buf = _sealed_for_a(b, sb, 300, rng)
    arrived = buf.copy()
    src = np.arange(len(desc), dtype=np.uint64) + 77
    L.rg_debug_plan_handoff(1)
    rc, st, sl, fl = _recv_raw(L, a, desc, buf, src)
    L.rg_debug_plan_handoff(0)
    assert rc == -2, (rc, L.rg_last_error())
    assert (st == PENDING).all(), np.unique(st)
    assert not fl.any()
    assert np.array_equal(buf, arrived)
    assert a.endpoint(sa) is None
    r = a.replay(sa)
    assert all(r.would_accept(c) for c in range(300))
    # the context recovers: the same frames are accepted now
    st2, _, fl2 = a.recv_batch(desc, buf, src=src, flags=True)
    assert (st2 == aead.PKT_OK).all() and (fl2 & aead.RECV_AUTHENTICATED).all()
    assert a.endpoint(sa) == int(src[-1])
    assert not r.would_accept(0)


def test_lost_handoff_device_recv_fails_closed(L, teng):
    """rg_recv_batch_dev + _finish with the hand-off lost: finish reports RG_EDEVICE, the host and device
    status arrays read RG_PKT_PENDING, nothing is marked seen, no endpoint moves, the frames are unchanged."""
    a, b, sa, sb = _pair(teng, seed=4)
    _planned_pipe(teng)
    rng = np.random.default_rng(6)
    desc, buf = _sealed_for_a(b, sb, 200, rng)
    n = len(desc)
    dd = torch.from_numpy(desc.view(np.uint8).reshape(-1, 16).copy()).cuda()
    db = torch.from_numpy(buf.copy()).cuda()
    dst = torch.zeros(n, dtype=torch.uint8, device="cuda")
    src = np.arange(n, dtype=np.uint64) + 5
    L.rg_debug_plan_handoff(1)
    a.recv_batch_dev(dd, db, dst)
    status = np.zeros(n, np.uint8)
    slots = np.zeros(n, np.uint32)
    fl = np.full(n, 0xAA, np.uint8)
    rc = L.rg_recv_batch_dev_finish(a._h, _vp(src), _vp(status), _vp(slots), _vp(fl))
    L.rg_debug_plan_handoff(0)
    torch.cuda.synchronize()
    assert rc == -2 and b"never finished" in L.rg_last_error()
    assert (status == PENDING).all() and not fl.any()
    assert (dst.cpu().numpy() == PENDING).all()
    assert np.array_equal(db.cpu().numpy(), buf)
    assert a.endpoint(sa) is None
    assert all(a.replay(sa).would_accept(c) for c in range(n))
    a.recv_batch_dev(dd, db, dst)
    st2, _, _ = a.recv_batch_dev_finish(n, src=src)
    assert (st2 == aead.PKT_OK).all()


def test_lost_handoff_device_seal_leaves_pending(L, teng):
    """A device seal over the planned pipelined kernel with the hand-off lost: every status RG_PKT_PENDING
    (the array held zeros before), every frame still plaintext; the host seal reports RG_EDEVICE."""
    _planned_pipe(teng)
    w = workloads.uniform(3000, 576, name="t")
    from rustyguard_amd.device import DeviceBatch

    bt = DeviceBatch(teng, w)
    bt.fill()
    torch.cuda.synchronize()
    plain = bt.host_buf()
    bt.status.zero_()
    torch.cuda.synchronize()
    L.rg_debug_plan_handoff(1)
    bt.seal()
    torch.cuda.synchronize()
    L.rg_debug_plan_handoff(0)
    assert (bt.status.cpu().numpy()[: w.n] == PENDING).all()
    assert np.array_equal(bt.host_buf(), plain)
    # host memory: the call fails and says so
    hb = plain.copy()
    L.rg_debug_plan_handoff(1)
    st = np.zeros(w.n, np.uint8)
    rc = L.rg_seal_batch_host(teng.handle, _vp(w.keys), _vp(w.receivers), 1, _vp(w.desc), _vp(w.counters), w.n,
                              _vp(hb), hb.nbytes, _vp(st))
    L.rg_debug_plan_handoff(0)
    assert rc == -2 and (st == PENDING).all()
    # recovered
    bt.seal()
    torch.cuda.synchronize()
    want = plain.copy()
    oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, want)
    assert (bt.status.cpu().numpy()[: w.n] == 0).all() and np.array_equal(bt.host_buf(), want)


@pytest.mark.parametrize("plan", [0, 1])
def test_lost_pool_tiles_never_read_ok(L, teng, plan):
    """The tile kernel's grid-wide pool (its last eighth of deal rounds, from 8 rounds on: 1 Mi packets)
    started past its end: the pooled tiles are never taken.  Every packet that reads OK is sealed exactly
    as the oracle seals it, every other one reads RG_PKT_PENDING with its frame untouched, and some are
    pending (the hook took effect)."""
    teng.set_staged(2)
    teng.set_plan(plan)
    n = 1 << 20
    w = workloads.uniform(n, 0, name="tiny")  # P = 0: 32-byte frames (key block + tag only)
    from rustyguard_amd.device import DeviceBatch

    bt = DeviceBatch(teng, w)
    bt.buf.fill_(0x5A)
    bt.status.zero_()
    torch.cuda.synchronize()
    before = bt.host_buf()
    L.rg_debug_plan_handoff(2)
    bt.seal()
    torch.cuda.synchronize()
    L.rg_debug_plan_handoff(0)
    st = bt.status.cpu().numpy()[:n]
    got = bt.host_buf()
    want = before.copy()
    oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, want)
    ok = st == 0
    assert set(np.unique(st)) <= {0, PENDING}
    assert (~ok).sum() > 0, "the hook did not take effect"
    frames_got = got.reshape(n, 32)
    assert np.array_equal(frames_got[ok], want.reshape(n, 32)[ok])
    assert np.array_equal(frames_got[~ok], before.reshape(n, 32)[~ok])


def test_every_family_writes_every_status(engine):
    """The launches without a preset (the pipelined kernel in array order, the flattened kernel) deal each
    packet to a lane by index alone: with the status array preset to a sentinel, no sentinel survives a
    seal or an open in any family."""
    rng = np.random.default_rng(9)
    n = 5000
    sizes = rng.integers(0, 95, n) * 16
    desc, buf = _frames(list(sizes), rng)
    desc["key_idx"] = 0
    keys = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    rec = np.array([7], np.uint32)
    ctr = np.arange(n, dtype=np.uint64)
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
    for fam, plan in ((0, 0), (0, 1), (3, 0), (3, 1), (2, 0), (2, 1), (-1, 2)):
        engine.set_staged(fam)
        engine.set_plan(plan)
        b = dev(buf)
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        engine.seal_dev(dev(keys), dev(rec.view(np.int32)), dev(desc.view(np.uint8).reshape(-1, 16)),
                        dev(ctr.view(np.int64)), b, st)
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 0).all(), (fam, plan)
        od = desc.copy()
        od["len"] += 32
        st.fill_(0xEE)
        engine.open_dev(dev(keys), dev(od.view(np.uint8).reshape(-1, 16)), b, st)
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 0).all(), (fam, plan)
    engine.set_staged(-1)
    engine.set_plan(2)


def test_seal_requires_status(engine):
    """ABI 6: a device seal without a status array is refused (nothing enqueued)."""
    w = workloads.uniform(8, 64, name="t")
    from rustyguard_amd.device import DeviceBatch

    bt = DeviceBatch(engine, w)
    with pytest.raises(_lib.RgError, match="status is required"):
        engine.seal_dev(bt.keys, bt.receivers, bt.desc_seal, bt.counters, bt.buf, None)


def test_second_stream_on_busy_context_is_refused(engine):
    """A batch on stream 2 while the context's batch on stream 1 is still in flight is refused with
    RG_EINVAL and nothing is enqueued; once stream 1 has drained, stream 2 is accepted."""
    w = workloads.uniform(4096, 1500, name="t")
    from rustyguard_amd.device import DeviceBatch

    bt = DeviceBatch(engine, w)
    bt.fill()
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        torch.cuda._sleep(int(4e8))  # ~200 ms of spinning ahead of the seal
    bt.seal(stream=s1)
    bt.status.fill_(0xEE)  # (current stream: runs before the seal on s1 has started)
    with pytest.raises(_lib.RgError, match="context busy"):
        bt.open(stream=s2)
    s1.synchronize()
    torch.cuda.synchronize()
    bt.open(stream=s2)
    torch.cuda.synchronize()
    assert (bt.status.cpu().numpy()[: w.n] == 0).all()


def test_lost_completion_times_out_and_fails_closed(L, teng):
    """Every library wait is bounded: with completions lost (hook), a host seal returns RG_EDEVICE "timed
    out" after about the limit, with every status RG_PKT_PENDING; with the hook off the context works again
    (the slices the failed call left in flight are waited for and discarded)."""
    teng.set_wait_timeout(300)
    w = workloads.uniform(2000, 1500, name="t")
    buf = np.zeros(w.buf_bytes, np.uint8)
    oracle.synth_fill(buf, w.desc, w.inner_len, w.data_seed)
    plain = buf.copy()
    L.rg_debug_lose_completions(1)
    st = np.zeros(w.n, np.uint8)
    t0 = time.perf_counter()
    rc = L.rg_seal_batch_host(teng.handle, _vp(w.keys), _vp(w.receivers), 1, _vp(w.desc), _vp(w.counters), w.n,
                              _vp(buf), buf.nbytes, _vp(st))
    el = time.perf_counter() - t0
    L.rg_debug_lose_completions(0)
    assert rc == -2 and b"timed out" in L.rg_last_error(), L.rg_last_error()
    assert (st == PENDING).all()
    assert 0.25 < el < 10, el
    torch.cuda.synchronize()
    hb = plain.copy()
    st2 = teng.seal_host(w.keys, w.receivers, w.desc, w.counters, hb)
    want = plain.copy()
    oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, want)
    assert (st2 == 0).all() and np.array_equal(hb, want)
