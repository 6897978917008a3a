"""One thread driving several contexts (rg_group, include/rg_aead.h "several GPUs, one thread") and the
per-peer endpoint record (rg_sessions_insert_peer).

The reference's host is one thread owning one Sessions (rustyguard-core/src/lib.rs:349-352); a group
splits each batch into contiguous ranges over its contexts and runs their pipelines for that thread (since
round 5 on one library worker thread per context).
Packets are independent, so every result must equal the one-context / oracle result
byte for byte.  The groups: N = 2 and 4 contexts on device 0 (one GPU runs every code path: streams,
splits, the round-robin issue, the gather) and, on a box with several GPUs, one context on each
visible device and contexts alternating over devices 0 and 1 (per-device streams,
hipSetDevice switching and pinned buffers of another device's context then run too)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import oracle
from rustyguard_amd import aead, workloads
from rustyguard_amd.aead import Engine, Group, Sessions
from rustyguard_amd.workloads import DESC_DTYPE

pytestmark = pytest.mark.gpu
S = 1_000_000_000
NDEV = torch.cuda.device_count()  # counting devices does not initialise the GPU on this image

GROUPS = {"2x dev0": [0, 0], "4x dev0": [0, 0, 0, 0],
          "all devices": list(range(NDEV)), "alternating 0,1": [0, 1, 0, 1]}


@pytest.fixture(scope="module", params=list(GROUPS))
def group(request):
    devs = GROUPS[request.param]
    if max(devs, default=0) >= NDEV or (request.param == "all devices" and NDEV < 2):
        pytest.skip(f"needs {max(devs) + 1 if devs else 2} GPUs, {NDEV} visible")
    g = Group(devs)
    yield g
    g.close()


def _hip():
    for name in ("libamdhip64.so.7", "libamdhip64.so.6", "libamdhip64.so"):
        try:
            return ctypes.CDLL(name)  # the runtime torch already loaded (same soname)
        except OSError:
            continue
    raise OSError("libamdhip64 not found")


def hip_get_device() -> int:
    d = ctypes.c_int(-1)
    assert _hip().hipGetDevice(ctypes.byref(d)) == 0
    return d.value


def _ragged(rng, n, keys=5):
    """A mixed batch: IMIX-like sizes, keepalives (P = 0), several keys, 16-byte gaps between frames."""
    sizes = rng.choice([0, 16, 64, 576, 1504, 2048], size=n, p=[0.05, 0.15, 0.3, 0.25, 0.2, 0.05])
    desc = np.zeros(n, DESC_DTYPE)
    off = 0
    for i, p in enumerate(sizes):
        desc[i] = (off, p, rng.integers(0, keys))
        off += p + 32 + 16 * int(rng.integers(0, 3))
    buf = rng.integers(0, 256, off + 256, dtype=np.uint8)
    kt = rng.integers(0, 256, (keys, 32), dtype=np.uint8)
    rec = rng.integers(0, 2**32, keys, dtype=np.uint64).astype(np.uint32)
    ctr = rng.integers(0, 2**40, n, dtype=np.uint64)
    return kt, rec, desc, ctr, buf


def test_group_host_seal_open_match_the_oracle(group):
    rng = np.random.default_rng(len(group))
    kt, rec, desc, ctr, buf = _ragged(rng, 3000)
    want = buf.copy()
    oracle.seal_batch(kt, rec, desc, ctr, want)
    got = buf.copy()
    st = group.seal_host(kt, rec, desc, ctr, got)
    assert (st == 0).all() and np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    ow = want.copy()
    so_w, co_w = oracle.open_batch(kt, od, ow)
    so, co = group.open_host(kt, od, got)
    assert (so_w == 0).all() and np.array_equal(so, so_w) and np.array_equal(got, ow)
    assert np.array_equal(co, co_w) and np.array_equal(co, ctr)
    # a forged tag in every part of the split: statuses and bytes as the oracle's (frames left as they came)
    sealed = want.copy()
    bnd = aead.split_batch(od, len(group), open_=True)
    for k in range(len(group)):
        i = int(bnd[k])
        if i < len(od):
            sealed[int(od[i]["offset"]) + int(od[i]["len"]) - 1] ^= 1
    ow2, got2 = sealed.copy(), sealed.copy()
    so_w2, _ = oracle.open_batch(kt, od, ow2)
    so2, _ = group.open_host(kt, od, got2)
    assert (so_w2 == 1).sum() == len(group) and np.array_equal(so2, so_w2) and np.array_equal(got2, ow2)


def test_group_host_large_batch_spans_many_slices(group):
    """config 2 sized batch: every context runs several 16 MiB pipeline slices, interleaved round-robin."""
    w = workloads.build("cfg2")
    buf = np.zeros(w.buf_bytes, np.uint8)
    oracle.synth_fill(buf, w.desc, w.inner_len, w.data_seed)
    plain = buf.copy()
    st = group.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)
    assert (st == 0).all()
    ref = plain.copy()
    sub = slice(0, w.n, 997)  # the oracle on a sample of packets (bit-exact per packet)
    d = w.desc[sub].copy()
    oracle.seal_batch(w.keys, w.receivers, d, w.counters[sub], ref)
    for k in range(0, len(d)):
        o, p = int(d[k]["offset"]), int(d[k]["len"]) + 32
        assert np.array_equal(buf[o:o + p], ref[o:o + p]), k
    so, co = group.open_host(w.keys, w.open_desc(), buf)
    assert (so == 0).all() and np.array_equal(co, w.counters)
    pay = np.zeros(len(buf), bool)  # the payload bytes are back to the plaintext (headers and tags stay)
    for o, p in zip(w.desc["offset"].astype(np.int64), w.desc["len"].astype(np.int64)):
        pay[o + 16:o + 16 + p] = True
    assert np.array_equal(buf[pay], plain[pay])


def test_group_device_shards(group):
    """rg_seal_batch_dev_multi / rg_open_batch_dev_multi: one shard per context (here all on device 0,
    each with its own tensors and stream), enqueued from one thread without waiting."""
    rng = np.random.default_rng(77)
    kt, rec, desc, ctr, buf = _ragged(rng, 2000)
    b = aead.split_batch(desc, len(group))
    want = buf.copy()
    oracle.seal_batch(kt, rec, desc, ctr, want)
    devs = group.devices
    streams = [torch.cuda.Stream(device=devs[k]) for k in range(len(group))]
    shards = []
    for k in range(len(group)):
        d = desc[b[k]:b[k + 1]].copy()
        dv = f"cuda:{devs[k]}"
        shards.append({"keys": torch.from_numpy(kt.reshape(-1)).to(dv), "receivers": torch.from_numpy(rec).to(dv),
                       "desc": torch.from_numpy(d.view(np.uint8)).to(dv),
                       "counters": torch.from_numpy(ctr[b[k]:b[k + 1]].copy()).to(dv),
                       "buf": torch.from_numpy(buf.copy()).to(dv),
                       "status": torch.full((max(len(d), 1),), 0xEE, dtype=torch.uint8, device=dv),
                       "stream": streams[k]})
    _sync_all(devs)
    group.seal_dev(shards)
    _sync_all(devs)
    fams = [group.engine(k).last_kernel() for k in range(len(group))]
    for k, sh in enumerate(shards):
        got = sh["buf"].cpu().numpy()
        st = sh["status"].cpu().numpy()[: b[k + 1] - b[k]]
        bad = [i for i in range(b[k], b[k + 1]) if not np.array_equal(
            got[int(desc[i]["offset"]):int(desc[i]["offset"]) + int(desc[i]["len"]) + 32],
            want[int(desc[i]["offset"]):int(desc[i]["offset"]) + int(desc[i]["len"]) + 32])]
        assert (st == 0).all() and not bad, (f"shard {k} of {len(group)} [{b[k]}, {b[k + 1]}) family {fams[k]}: "
                                             f"statuses {np.unique(st, return_counts=True)}, {len(bad)} frames "
                                             f"differ, first {bad[:8]}, sizes {[int(desc[i]['len']) for i in bad[:8]]}")
    for k, sh in enumerate(shards):
        od = sh["desc"].cpu().numpy().view(DESC_DTYPE).copy()
        od["len"] += 32
        sh["desc"] = torch.from_numpy(od.view(np.uint8)).to(f"cuda:{devs[k]}")
        sh["counters_out"] = torch.zeros(len(od), dtype=torch.int64, device=f"cuda:{devs[k]}")
    _sync_all(devs)
    group.open_dev(shards)
    _sync_all(devs)
    for k, sh in enumerate(shards):
        assert (sh["status"].cpu().numpy()[: b[k + 1] - b[k]] == 0).all()
        assert np.array_equal(sh["counters_out"].cpu().numpy().astype(np.uint64), ctr[b[k]:b[k + 1]])
        got = sh["buf"].cpu().numpy()
        for i in range(b[k], b[k + 1]):
            o, p = int(desc[i]["offset"]), int(desc[i]["len"]) + 32
            assert np.array_equal(got[o + 16:o + p - 16], buf[o + 16:o + p - 16]), i


def _sync_all(devs):
    for d in sorted(set(devs)):
        torch.cuda.synchronize(d)


def test_group_calls_leave_the_current_device_selected(group):
    """every group call selects each context's device in turn and puts the caller's
    current HIP device back (hipGetDevice read through the HIP runtime itself, not torch's view of it),
    whichever device the caller had selected -- also after a call that fails."""
    rng = np.random.default_rng(3)
    kt, rec, desc, ctr, buf = _ragged(rng, 600)
    od = desc.copy()
    od["len"] += 32
    for cur in sorted(set(group.devices)):
        torch.cuda.set_device(cur)
        assert hip_get_device() == cur
        group.seal_host(kt, rec, desc, ctr, buf)
        assert hip_get_device() == cur, "seal_host_multi"
        group.open_host(kt, od, buf)
        assert hip_get_device() == cur, "open_host_multi"
        a = Sessions(group, 4)
        s0 = a.insert(1, 2, bytes(range(32)), bytes(range(32, 64)))
        a.send_batch([s0] * 3, desc[:3].copy(), buf.copy())
        assert hip_get_device() == cur, "send_batch on a group"
        bad = (aead._DevShard * len(group))()
        for x in bad:
            x.n = 1  # one packet, no buffers: refused by the shard check before anything runs
        with pytest.raises(Exception):
            group.seal_dev(bad)
        assert hip_get_device() == cur, "failed seal_dev_multi"
        del a
    torch.cuda.set_device(0)


def test_dev_multi_checks_every_shard_before_enqueuing(group):
    """a bad argument in the LAST shard is refused before shard 0 is enqueued (its statuses stay
    at the sentinel), and the error names the shard."""
    from rustyguard_amd import _lib

    rng = np.random.default_rng(4)
    kt, rec, desc, ctr, buf = _ragged(rng, 200)
    shards = []
    for k, dv in enumerate(group.devices):
        t = f"cuda:{dv}"
        shards.append({"keys": torch.from_numpy(kt.reshape(-1)).to(t), "receivers": torch.from_numpy(rec).to(t),
                       "desc": torch.from_numpy(desc.view(np.uint8)).to(t), "counters": torch.from_numpy(ctr).to(t),
                       "buf": torch.from_numpy(buf.copy()).to(t),
                       "status": torch.full((len(desc),), 0xEE, dtype=torch.uint8, device=t),
                       "stream": torch.cuda.Stream(device=dv)})
    arr = Group.shards(shards, True)
    arr[len(group) - 1].counters = None  # seal needs counters
    _sync_all(group.devices)
    with pytest.raises(_lib.RgError) as ei:
        group.seal_dev(arr)
    assert f"shard {len(group) - 1}" in str(ei.value) and "nothing enqueued" in str(ei.value)
    _sync_all(group.devices)
    for sh in shards:
        assert (sh["status"] == 0xEE).all().item(), "a shard ran although the call was refused"
    group.seal_dev(Group.shards(shards, True))  # the same shards, valid: every one runs
    _sync_all(group.devices)
    for sh in shards:
        assert (sh["status"] == 0).all().item()


def _keys(seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(4)]


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


def test_group_sessions_match_one_context(group, engine):
    """A session table on a group (rg_sessions_create_group) gives the single-context table's results:
    counters reserved in array order before the split, the anti-replay pass after the gather --
    duplicates, forgeries and in-batch replays included."""
    k_ab, k_ba, k_ac, k_ca = _keys(5)
    rng = np.random.default_rng(9)
    tabs = []
    for e in (engine, group):
        a = Sessions(e, 8)
        sa = a.insert(0x1111, 0x2222, k_ab, k_ba)
        sc = a.insert(0x3333, 0x4444, k_ac, k_ca)
        tabs.append((a, sa, sc))
    b = Sessions(engine, 8)
    sb = b.insert(0x2222, 0x1111, k_ba, k_ab)
    sizes = list(rng.choice([0, 16, 64, 576, 1504], size=700))
    slots = [tabs[0][1] if x % 3 else tabs[0][2] for x in range(700)]
    desc, buf = _frames(sizes, rng)
    outs = []
    for a, sa, sc in tabs:
        fr = buf.copy()
        st, rk = a.send_batch(slots, desc, fr)
        outs.append((st, fr))
        assert a.send_counter(sa) == sum(1 for s in slots if s == sa)
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    # B -> A traffic with replays and a forgery, received by both A tables
    bdesc, bbuf = _frames([64] * 50 + [1504] * 50, rng)
    st, _ = b.send_batch([sb] * 100, bdesc, bbuf)
    od = bdesc.copy()
    od["len"] += 32
    idx = np.concatenate([np.arange(100), [5, 17, 5, 99]])  # in-batch replays, each its own datagram
    rd = np.zeros(len(idx), DESC_DTYPE)
    rbuf = np.zeros(int((od["len"][idx].astype(np.int64) + 16).sum()) + 64, np.uint8)
    off = 0
    for k, i in enumerate(idx):
        o, w = int(od[i]["offset"]), int(od[i]["len"])
        rbuf[off:off + w] = bbuf[o:o + w]
        rd[k] = (off, w, 0)
        off += (w + 15) // 16 * 16
    forged = int(rd[40]["offset"]) + int(rd[40]["len"]) - 1
    res = []
    for a, sa, sc in tabs:
        fr = rbuf.copy()
        fr[forged] ^= 1
        st, sl, fl = a.recv_batch(rd.copy(), fr, src=np.arange(len(rd), dtype=np.uint64) + 1000, flags=True)
        res.append((st, sl, fl, fr, a.endpoint(sa)))
    for x, y in zip(res[0], res[1]):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    assert res[0][0][40] == aead.PKT_DECRYPT_ERR and list(res[0][0][100:]) == [aead.PKT_REJECTED] * 4


def test_group_sessions_refuse_device_frames(group):
    a = Sessions(group, 4)
    s0 = a.insert(1, 2, bytes(32), bytes(32))
    d = torch.zeros(16, dtype=torch.uint8, device="cuda")
    with pytest.raises(Exception):
        a.send_batch_dev([s0], d, torch.zeros(64, dtype=torch.uint8, device="cuda"))


def test_peer_endpoint_survives_a_rekey(engine):
    """peer.endpoint is per peer (rustyguard-core/src/lib.rs:670-671) and the
    Keepalive timer sends to it (time.rs:135).  After a rekey (a new session slot of the same peer) the
    new slot reports the endpoint the old one authenticated, and a due keepalive carries that address."""
    k1, k2, k3, k4 = _keys(11)
    rng = np.random.default_rng(12)
    a, b = Sessions(engine, 8), Sessions(engine, 8)
    PEER = 42
    s_old = a.insert(0x10, 0x20, k1, k2, peer=PEER)
    b_old = b.insert(0x20, 0x10, k2, k1)
    assert a.endpoint(s_old) is None and a.peer_endpoint(PEER) is None
    desc, buf = _frames([64], rng)
    assert (b.send_batch([b_old], desc, buf)[0] == 0).all()
    od = desc.copy()
    od["len"] += 32
    st, _ = a.recv_batch(od.copy(), buf.copy(), src=np.array([555], np.uint64))
    assert st[0] == 0 and a.endpoint(s_old) == 555 and a.peer_endpoint(PEER) == 555
    # rekey: a new session of the same peer (new ids, new keys); nothing authenticated on it yet
    s_new = a.insert(0x11, 0x21, k3, k4, peer=PEER)
    b_new = b.insert(0x21, 0x11, k4, k3)
    assert a.endpoint(s_new) == 555
    # a genuine packet on the OLD session from a roamed address moves the peer's endpoint for both
    desc2, buf2 = _frames([16], rng)
    assert (b.send_batch([b_old], desc2, buf2)[0] == 0).all()
    od2 = desc2.copy()
    od2["len"] += 32
    st, _ = a.recv_batch(od2.copy(), buf2.copy(), src=np.array([556], np.uint64))
    assert st[0] == 0 and a.endpoint(s_new) == 556 and a.endpoint(s_old) == 556
    # the keepalive of the new session goes to the peer's endpoint once the session has been quiet
    a.set_time(11 * S)
    assert a.keepalive(s_new) == 556
    a.set_time(11 * S)
    desc3, buf3 = _frames([0], rng)
    assert (a.send_batch([s_new], desc3, buf3)[0] == 0).all()  # the keepalive itself resets `sent`
    assert a.keepalive(s_new) is None
    # a session without a peer keeps its own endpoint, as before
    s_own = a.insert(0x12, 0x22, k1, k3)
    assert a.endpoint(s_own) is None
    _ = b_new


def test_keepalive_without_endpoint_is_an_error(engine):
    k1, k2, _, _ = _keys(13)
    a = Sessions(engine, 4)
    s = a.insert(0x30, 0x40, k1, k2, peer=7)
    a.set_time(11 * S)
    with pytest.raises(Exception):
        a.keepalive(s)  # due, but the peer never authenticated a packet


@pytest.mark.parametrize("use_group", [False, True])
def test_host_batch_in_any_frame_order(use_group, engine, group):
    """Frames handed over in an order other than their offsets (more than one 16 MiB pipeline slice): the
    library runs them in offset order so that no slice's byte span takes in another's frames, and returns
    statuses and counters in the caller's order."""
    rng = np.random.default_rng(31)
    n = 20000
    desc = np.zeros(n, DESC_DTYPE)
    desc["len"] = 1504
    desc["offset"] = np.arange(n, dtype=np.uint64) * 1536
    desc["key_idx"] = rng.integers(0, 3, n)
    perm = rng.permutation(n)
    desc = desc[perm].copy()
    kt = rng.integers(0, 256, (3, 32), dtype=np.uint8)
    rec = np.arange(3, dtype=np.uint32) + 7
    ctr = rng.integers(0, 2**50, n, dtype=np.uint64)
    buf = rng.integers(0, 256, n * 1536, dtype=np.uint8)
    want = buf.copy()
    oracle.seal_batch(kt, rec, desc, ctr, want)
    runner = group if use_group else engine
    got = buf.copy()
    st = runner.seal_host(kt, rec, desc, ctr, got)
    assert (st == 0).all() and np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    got[int(od[7]["offset"]) + 100] ^= 4  # one forged frame, reported at its caller index
    so, co = runner.open_host(kt, od, got)
    assert so[7] == aead.PKT_DECRYPT_ERR and (np.delete(so, 7) == 0).all()
    assert np.array_equal(np.delete(co, 7), np.delete(ctr, 7))


def test_group_host_call_survives_failing_allocations():
    """Round 5 runs each context's host pipeline on a worker thread of the library.  A group host call whose
    k-th allocation fails (rg_debug_fail_reserve, test library) -- in the calling thread while the key tables
    go up (k <= 6 here: three contexts, a key table and a receiver table each), or in some context's worker
    while it reserves its slot buffers -- returns an error (the first failing context's, carried over to the
    calling thread), leaves no worker behind, and the same group's next call seals every frame bit-exactly."""
    from rustyguard_amd import _lib

    L = _lib.lib_test()
    rng = np.random.default_rng(91)
    n = 24000
    desc = np.zeros(n, DESC_DTYPE)
    desc["len"] = 1504
    desc["offset"] = np.arange(n, dtype=np.uint64) * 1536
    desc["key_idx"] = rng.integers(0, 3, n)
    kt = rng.integers(0, 256, (3, 32), dtype=np.uint8)
    rec = np.arange(3, dtype=np.uint32) + 11
    ctr = rng.integers(0, 2**50, n, dtype=np.uint64)
    base = rng.integers(0, 256, n * 1536, dtype=np.uint8)
    want = base.copy()
    oracle.seal_batch(kt, rec, desc, ctr, want)
    for k in (1, 4, 7, 12, 19, 30):
        g = Group([0, 0, 0], library=L)
        try:
            for i in range(3):
                g.engine(i).set_host_slice(2 << 20)  # ~12 MiB per context: six 2 MiB slices, all three slots used
            L.rg_debug_fail_reserve(k)
            try:
                with pytest.raises(_lib.RgError):
                    g.seal_host(kt, rec, desc, ctr, base.copy())
            finally:
                L.rg_debug_fail_reserve(0)
            got = base.copy()
            st = g.seal_host(kt, rec, desc, ctr, got)
            assert (st == 0).all() and np.array_equal(got, want), f"after a failure at allocation {k}"
        finally:
            g.close()


def test_group_host_calls_alternate_threaded_and_inline(group):
    """Round 5: a group call drives its contexts from worker threads when some context's part spans more
    than two slices and from the calling thread otherwise.  Calls of both kinds, alternating on one group
    (slots, key tables and events reused across the switch), each seal then open bit-exactly."""
    rng = np.random.default_rng(93)
    kt = rng.integers(0, 256, (4, 32), dtype=np.uint8)
    rec = np.arange(4, dtype=np.uint32) + 5
    for c in range(len(group)):
        group.engine(c).set_host_slice(2 << 20)  # the large batches span several slices on every context
    try:
        _alternate(group, rng, kt, rec)
    finally:
        for c in range(len(group)):
            group.engine(c).set_host_slice(8 << 20)


def _alternate(group, rng, kt, rec):
    for i, n in enumerate([30000, 300, 26000, 40, 28000]):
        desc = np.zeros(n, DESC_DTYPE)
        desc["len"] = 1504
        desc["offset"] = np.arange(n, dtype=np.uint64) * 1536
        desc["key_idx"] = rng.integers(0, 4, n)
        ctr = rng.integers(0, 2**50, n, dtype=np.uint64)
        buf = rng.integers(0, 256, n * 1536, dtype=np.uint8)
        want = buf.copy()
        oracle.seal_batch(kt, rec, desc, ctr, want)
        got = buf.copy()
        st = group.seal_host(kt, rec, desc, ctr, got)
        assert (st == 0).all() and np.array_equal(got, want), f"call {i} ({n} packets)"
        od = desc.copy()
        od["len"] += 32
        so, co = group.open_host(kt, od, got)
        assert (so == 0).all() and np.array_equal(co, ctr), f"open {i}"
        for k in (0, n // 2, n - 1):
            o = int(desc["offset"][k]) + 16
            assert np.array_equal(got[o:o + 1504], buf[o:o + 1504]), f"open {i} packet {k}"


def test_numa_placed_buffer_round_trip():
    """Round 6: rg_numa_node names a node (or -1), and a frame buffer placed for a group
    -- each context's part bound to its context's node (rg_numa_bind), first-touched, pinned
    (rg_host_register) -- seals and opens bit-exactly against the oracle through the group."""
    g = Group([0, 0])
    try:
        for k in range(2):
            assert aead.numa_node(g.engine(k)) >= -1
        w = workloads.uniform(3000, 576, name="t")
        buf, placement = aead.placed_host_buffer(g, w.desc, w.buf_bytes)
        assert [p["context"] for p in placement] == [0, 1] and sum(p["packets"] for p in placement) == w.n
        rng = np.random.default_rng(5)
        buf[:] = rng.integers(0, 256, buf.nbytes, dtype=np.uint8)
        plain = buf.copy()
        want = plain.copy()
        oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, want)
        st = g.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)
        assert (st == 0).all() and np.array_equal(buf, want)
        st2, _ = g.open_host(w.keys, w.open_desc(), buf)
        assert (st2 == 0).all()
    finally:
        g.close()


def test_create_leaves_no_hip_error_pending():
    """rg_create's NUMA query: this runtime answers hipDeviceAttributeHostNumaId with an error, and a failed
    query stays the thread's last HIP error, which the next launch (ours, or PyTorch's checks) then reported
    as its own failure.  rg_create clears it and reads the node from sysfs."""
    eng = Engine(0)
    try:
        assert _hip().hipGetLastError() == 0
        assert aead.numa_node(eng) >= -1
        x = torch.arange(1024, device="cuda")
        assert int((x + 1).sum().item()) == 1024 * 1025 // 2
    finally:
        eng.close()
