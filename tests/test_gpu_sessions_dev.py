"""Device-resident session batches (rg_send_batch_dev / rg_recv_batch_dev[_finish]) against the
host-memory session path (rg_send_batch / rg_recv_batch_ex), which test_gpu_sessions.py pins to
the reference's sequential semantics (rustyguard-core/src/lib.rs:249-297, :605-681;
rustyguard-crypto/src/prim.rs:376-437).  Two tables with identical state run the same batch, one
per path: statuses, slots, flags, endpoints, counters and every frame byte must agree."""
import numpy as np
import pytest
import torch

from rustyguard_amd import _lib, aead
from rustyguard_amd.aead import Engine, Sessions
from rustyguard_amd.workloads import DESC_DTYPE

pytestmark = pytest.mark.gpu


def _keys(seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(4)]


def _twins(engine, now=0):
    """(host table, device table) of the same A side, and B (the peer) for sealing test traffic."""
    k_ab, k_ba, k_ac, k_ca = _keys(7)
    tabs = []
    for _ in range(2):
        a = Sessions(engine, 8)
        a.set_time(now)
        sa = a.insert(0x1111, 0x2222, k_ab, k_ba)
        sc = a.insert(0x3333, 0x4444, k_ac, k_ca)
        tabs.append(a)
    b = Sessions(engine, 8)
    b.set_time(now)
    sb = b.insert(0x2222, 0x1111, k_ba, k_ab)
    return tabs[0], tabs[1], b, sa, sc, sb


def _frames(sizes, rng):
    desc = np.zeros(len(sizes), DESC_DTYPE)
    off = 0
    for i, p in enumerate(sizes):
        desc[i] = (off, p, 0)
        off += (p + 32 + 15) // 16 * 16
    buf = np.zeros(off + 64, np.uint8)
    for d in desc:
        buf[d["offset"] + 16: d["offset"] + 16 + d["len"]] = rng.integers(0, 256, d["len"], dtype=np.uint8)
    return desc, buf


def _dev(a):
    """Device copy; descriptor arrays as [n, 16] byte rows (so slicing keeps whole rows)."""
    b = np.ascontiguousarray(a).view(np.uint8)
    if a.dtype == DESC_DTYPE:
        b = b.reshape(-1, 16)
    return torch.from_numpy(b).cuda()


def test_send_batch_dev_matches_host(engine):
    ah, ad, b, sa, sc, sb = _twins(engine)
    rng = np.random.default_rng(11)
    sizes = [16, 1504, 0, 576, 64, 1504, 32, 16, 48]
    slots = [sa, sa, sc, sa, 7, sc, sa, sc, sa]  # slot 7: no session
    desc, buf = _frames(sizes, rng)
    ah.set_send_counter(sc, aead.REKEY_AFTER_MESSAGES - 1)
    ad.set_send_counter(sc, aead.REKEY_AFTER_MESSAGES - 1)
    hb = buf.copy()
    st_h, rk_h = ah.send_batch(slots, desc, hb)
    db, dd = _dev(buf), _dev(desc)
    dst = torch.full((len(sizes),), 0xEE, dtype=torch.uint8, device="cuda")
    rk_d = ad.send_batch_dev(slots, dd, db, dst)
    torch.cuda.synchronize()
    assert list(dst.cpu().numpy()) == list(st_h)
    assert list(rk_d) == list(rk_h) and rk_d.any()
    assert np.array_equal(db.cpu().numpy(), hb)
    for s in (sa, sc):
        assert ad.send_counter(s) == ah.send_counter(s)


def test_send_batch_dev_two_in_flight_and_reject_after_time(engine):
    ah, ad, b, sa, sc, sb = _twins(engine)
    rng = np.random.default_rng(12)
    desc, buf = _frames([64] * 300, rng)
    hb = buf.copy()
    db, dd = _dev(buf), _dev(desc)
    s = torch.cuda.Stream()
    half = [sa] * 150 + [sc] * 150
    # three back-to-back sends on one stream (the third reuses the first's staging)
    for _ in range(3):
        ah.send_batch(half, desc, hb)
        ad.send_batch_dev(half, dd, db, torch.zeros(300, dtype=torch.uint8, device="cuda"), stream=s)
    torch.cuda.synchronize()
    assert np.array_equal(db.cpu().numpy(), hb)
    assert ad.send_counter(sa) == ah.send_counter(sa) == 450
    # should_expire (lib.rs:207-209): 181 s after the session started nothing is sealed
    for t in (ah, ad):
        t.set_time(181 * 10**9)
    st_h, _ = ah.send_batch([sa], desc[:1], hb)
    dst = torch.zeros(1, dtype=torch.uint8, device="cuda")
    ad.send_batch_dev([sa], dd[:1], db, dst)
    torch.cuda.synchronize()
    assert st_h[0] == aead.PKT_REJECTED and dst.item() == aead.PKT_REJECTED
    assert np.array_equal(db.cpu().numpy(), hb)


def _recv_batch(b, sb, rng):
    """B seals 40 frames to A; the receive batch holds them shuffled, with duplicates, forgeries,
    an unknown receiver, a handshake message, bad lengths and a header-only frame."""
    n = 40
    sizes = list(rng.integers(0, 95, n) * 16)
    desc, buf = _frames(sizes, rng)
    st, _ = b.send_batch([sb] * n, desc, buf)
    assert (st == 0).all()
    od = desc.copy()
    od["len"] += 32
    order = list(rng.permutation(n)) + [3, 7, 7, 12]
    forged = {5, 11, 12}
    parts, rdesc = [], []
    off = 0

    def put(frame):
        nonlocal off
        w = len(frame)
        parts.append((off, frame))
        rdesc.append((off, w, 0))
        off += (w + 15) // 16 * 16

    for k, i in enumerate(order):
        o, w = int(od[i]["offset"]), int(od[i]["len"])
        fr = buf[o:o + w].copy()
        if i in forged and k < n:
            fr[w - 1] ^= 0x40
        put(fr)
    hdr = lambda t, r, c: np.frombuffer(np.array([t, r], np.uint32).tobytes() + np.uint64(c).tobytes(), np.uint8)  # noqa: E731
    put(np.concatenate([hdr(4, 0x9999, 0), np.zeros(32, np.uint8)]))  # unknown receiver
    put(np.concatenate([hdr(1, 0, 0), np.zeros(132, np.uint8)]))       # handshake init (148 B)
    put(np.concatenate([hdr(4, 0x1111, 3), np.zeros(24, np.uint8)]))  # W = 40: not 16-B framed
    put(hdr(4, 0x1111, 3))                                             # header only, replayed counter
    put(hdr(4, 0x1111, 500))                                           # header only, fresh counter
    put(np.concatenate([hdr(7, 0x1111, 0), np.zeros(32, np.uint8)]))  # unknown type
    ob = np.zeros(off + 64, np.uint8)
    for o, fr in parts:
        ob[o:o + len(fr)] = fr
    return np.array(rdesc, DESC_DTYPE), ob


def test_recv_batch_dev_matches_host(engine):
    ah, ad, b, sa, sc, sb = _twins(engine, now=5 * 10**9)
    rng = np.random.default_rng(13)
    rdesc, ob = _recv_batch(b, sb, rng)
    n = len(rdesc)
    src = np.arange(n, dtype=np.uint64) + 1000
    for step in range(2):  # the second pass replays the whole batch against the advanced window
        for t in (ah, ad):
            t.set_time((30 + step) * 10**9)  # sent + 10 s < now: keepalive flags on the first accept
        hb = ob.copy()
        st_h, sl_h, fl_h = ah.recv_batch(rdesc, hb, src=src, flags=True)
        db, dd = _dev(ob), _dev(rdesc)
        dst = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        ad.recv_batch_dev(dd, db, dst)
        st_d, sl_d, fl_d = ad.recv_batch_dev_finish(n, src=src)
        torch.cuda.synchronize()
        assert list(st_d) == list(st_h)
        assert list(dst.cpu().numpy()) == list(st_h)
        assert list(sl_d) == list(sl_h)
        assert list(fl_d) == list(fl_h)
        assert np.array_equal(db.cpu().numpy(), hb)
        assert ad.endpoint(sa) == ah.endpoint(sa)
        if step == 0:
            assert (st_h == aead.PKT_OK).sum() >= 30
            assert (st_h == aead.PKT_REJECTED).sum() >= 4
            assert np.count_nonzero(fl_h & aead.RECV_KEEPALIVE) == 1
        else:
            assert not (st_h == aead.PKT_OK).any()
    # both windows ended in the same state
    for c in range(0, 600, 7):
        assert ah.replay(sa).would_accept(c) == ad.replay(sa).would_accept(c)


def test_recv_batch_dev_pending_rules(engine):
    ah, ad, b, sa, sc, sb = _twins(engine)
    rng = np.random.default_rng(14)
    rdesc, ob = _recv_batch(b, sb, rng)
    db, dd = _dev(ob), _dev(rdesc)
    dst = torch.zeros(len(rdesc), dtype=torch.uint8, device="cuda")
    with pytest.raises(_lib.RgError):
        ad.recv_batch_dev_finish(len(rdesc))  # nothing pending
    ad.recv_batch_dev(dd, db, dst)
    with pytest.raises(_lib.RgError):
        ad.recv_batch_dev(dd, db, dst)  # one pending batch per table
    with pytest.raises(_lib.RgError):
        ad.insert(0x5555, 0x6666, bytes(32), bytes(32))  # tables are frozen while pending
    ad.recv_batch_dev_finish(len(rdesc))
    # a session added afterwards is seen by the next device call
    k = _keys(9)
    s2 = ad.insert(0x7777, 0x8888, k[0], k[1])
    b2 = Sessions(engine, 4)
    t2 = b2.insert(0x8888, 0x7777, k[1], k[0])
    desc, buf = _frames([64, 576], rng)
    b2.send_batch([t2, t2], desc, buf)
    od = desc.copy()
    od["len"] += 32
    db2, dd2 = _dev(buf), _dev(od)
    dst2 = torch.zeros(2, dtype=torch.uint8, device="cuda")
    ad.recv_batch_dev(dd2, db2, dst2)
    st, sl, fl = ad.recv_batch_dev_finish(2)
    assert list(st) == [0, 0] and list(sl) == [s2, s2]


def test_recv_batch_dev_failed_setup_leaves_no_pending_batch():
    """An allocation that fails inside rg_recv_batch_dev (forced by rg_debug_fail_reserve: the k-th
    allocation after the hook is armed) leaves no pending batch behind -- finish reports none, and
    neither the window nor the frames moved: the next receive matches the host path on a twin table."""
    L = _lib.lib_test()  # rg_debug_fail_reserve lives in the test library only
    engine = Engine(0, library=L)
    failed = 0
    try:
        for k in range(1, 12):
            ah, ad, b, sa, sc, sb = _twins(engine)
            rng = np.random.default_rng(20 + k)
            rdesc, ob = _recv_batch(b, sb, rng)
            n = len(rdesc)
            db, dd = _dev(ob), _dev(rdesc)
            dst = torch.zeros(n, dtype=torch.uint8, device="cuda")
            L.rg_debug_fail_reserve(k)
            try:
                ad.recv_batch_dev(dd, db, dst)
                ok = True
            except _lib.RgError:
                ok = False
            L.rg_debug_fail_reserve(0)
            torch.cuda.synchronize()
            if ok:
                ad.recv_batch_dev_finish(n)
                continue
            failed += 1
            with pytest.raises(_lib.RgError):
                ad.recv_batch_dev_finish(n)  # no pending batch: no replay pass over stale staging
            assert np.array_equal(db.cpu().numpy(), ob)  # nothing was opened
            hb = ob.copy()
            st_h, sl_h = ah.recv_batch(rdesc, hb)
            ad.recv_batch_dev(dd, db, dst)
            st_d, sl_d, _ = ad.recv_batch_dev_finish(n)
            torch.cuda.synchronize()
            assert list(st_d) == list(st_h) and list(sl_d) == list(sl_h)
            assert np.array_equal(db.cpu().numpy(), hb)
    finally:
        L.rg_debug_fail_reserve(0)
    assert failed >= 6  # the staging reserves (and the table mirrors) were all exercised
