"""Batched transport send/recv (rg_send_batch / rg_recv_batch) vs the reference semantics.

Reference behaviour modelled packet by packet, in order:
  send: PeerState::encrypt_message/force_encrypt (rustyguard-core/src/lib.rs:249-297):
        should_reject (counter >= REJECT_AFTER_MESSAGES), P % 16 == 0, n = counter++,
        header {4, receiver, n}, rekey when counter >= REKEY_AFTER_MESSAGES (:564-570)
  recv: Sessions::recv_message / decrypt_packet (:605-681) and
        DecryptionKey::decrypt (rustyguard-crypto/src/prim.rs:414-437):
        alignment, type, length, receiver -> session, would_accept, open, mark_seen.
"""
import numpy as np
import pytest

from oracle import oracle
from rustyguard_amd import aead
from rustyguard_amd.aead import Sessions
from rustyguard_amd.workloads import DESC_DTYPE

pytestmark = pytest.mark.gpu


def _frames(sizes, rng, align=16):
    desc = np.zeros(len(sizes), DESC_DTYPE)
    off = 0
    for i, p in enumerate(sizes):
        desc[i] = (off, p, 0)
        off += (p + 32 + align - 1) // align * align
    buf = np.zeros(off + 64, np.uint8)
    for d in desc:
        buf[d["offset"] + 16: d["offset"] + 16 + d["len"]] = rng.integers(0, 256, d["len"], dtype=np.uint8)
    return desc, buf


@pytest.fixture
def pair(engine):
    rng = np.random.default_rng(42)
    k_ab, k_ba = rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    k_ac, k_ca = rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    a, b = Sessions(engine, 8), Sessions(engine, 8)
    # A's session with B: A receives on id 0x1111, B receives on id 0x2222
    sa = a.insert(0x1111, 0x2222, k_ab, k_ba)
    sb = b.insert(0x2222, 0x1111, k_ba, k_ab)
    sc = a.insert(0x3333, 0x4444, k_ac, k_ca)
    return a, b, sa, sb, sc, (k_ab, k_ba, k_ac)


def test_send_assigns_counters_in_order_and_frames(pair):
    a, b, sa, sb, sc, keys = pair
    rng = np.random.default_rng(1)
    sizes = [16, 1504, 0, 576, 64, 1504, 32]
    slots = [sa, sa, sc, sa, sc, sa, sa]
    desc, buf = _frames(sizes, rng)
    plain = buf.copy()
    st, rekey = a.send_batch(slots, desc, buf)
    assert (st == 0).all() and not rekey.any()
    assert a.send_counter(sa) == 5 and a.send_counter(sc) == 2
    # byte-exact against the oracle with the counters EncryptionKey would assign
    want = plain.copy()
    ctr = {sa: 0, sc: 0}
    for i, (d, s) in enumerate(zip(desc, slots)):
        key = keys[0] if s == sa else keys[2]
        rec = 0x2222 if s == sa else 0x4444
        one = np.zeros(1, DESC_DTYPE)
        one[0] = d
        oracle.seal_batch(np.frombuffer(key, np.uint8).reshape(1, 32), np.array([rec], np.uint32), one,
                          np.array([ctr[s]], np.uint64), want)
        ctr[s] += 1
    assert np.array_equal(buf, want)


def test_send_rejects_bad_lengths_unknown_and_exhausted(pair):
    a, b, sa, sb, sc, keys = pair
    rng = np.random.default_rng(2)
    desc, buf = _frames([16, 17, 16, 16], rng)
    a.set_send_counter(sc, aead.REJECT_AFTER_MESSAGES)
    before = buf.copy()
    st, _ = a.send_batch([sa, sa, 7, sc], desc, buf)
    assert list(st) == [aead.PKT_OK, aead.PKT_INVALID, aead.PKT_REJECTED, aead.PKT_REJECTED]
    assert a.send_counter(sa) == 1  # only the sealed packet consumed a counter
    for i in (1, 2, 3):
        o, w = int(desc[i]["offset"]), int(desc[i]["len"]) + 32
        assert np.array_equal(buf[o:o + w], before[o:o + w])


def test_rekey_flag_at_threshold(pair):
    a, b, sa, sb, sc, keys = pair
    rng = np.random.default_rng(3)
    desc, buf = _frames([16] * 3, rng)
    a.set_send_counter(sa, aead.REKEY_AFTER_MESSAGES - 2)
    st, rekey = a.send_batch([sa] * 3, desc, buf)
    assert (st == 0).all()
    assert list(rekey) == [0, 1, 1]  # counter() >= 2^60 after the 2nd seal (lib.rs:564)


def _model_recv(window_state, frames_meta):
    """Sequential reference semantics for already-authenticated-or-not frames."""
    out = []
    for ok_tag, ctr in frames_meta:
        if not window_state.would_accept(ctr):
            out.append(aead.PKT_REJECTED)
        elif not ok_tag:
            out.append(aead.PKT_DECRYPT_ERR)
        else:
            window_state.mark_seen(ctr)
            out.append(aead.PKT_OK)
    return out


def test_roundtrip_duplicates_replays_and_forgeries(pair):
    a, b, sa, sb, sc, keys = pair
    rng = np.random.default_rng(4)
    n = 40
    sizes = list(rng.integers(0, 95, n) * 16)
    desc, buf = _frames(sizes, rng)
    plain = buf.copy()
    st, _ = a.send_batch([sa] * n, desc, buf)
    assert (st == 0).all()
    sealed = buf.copy()
    od = desc.copy()
    od["len"] += 32
    # batch 1: all frames, in a shuffled order, with duplicates and forgeries
    order = list(rng.permutation(n)) + [3, 7, 7]
    forged = {5, 11}
    ob = np.zeros(sum(int(od[i]["len"]) for i in order) + 16 * len(order), np.uint8)
    rdesc = np.zeros(len(order), DESC_DTYPE)
    off = 0
    meta = []
    for k, i in enumerate(order):
        o, w = int(od[i]["offset"]), int(od[i]["len"])
        ob[off:off + w] = sealed[o:o + w]
        if i in forged and k < n:
            ob[off + w - 1] ^= 0x40
        rdesc[k] = (off, w, 0)
        meta.append((not (i in forged and k < n), int(i)))
        off += (w + 15) // 16 * 16
    frames_before = ob.copy()
    st, slots = b.recv_batch(rdesc, ob)
    model = aead.AntiReplay()
    want = _model_recv(model, meta)
    assert list(st) == want
    assert (slots[st == 0] == sb).all()
    for k, i in enumerate(order):
        o, w = int(rdesc[k]["offset"]), int(rdesc[k]["len"])
        if st[k] == aead.PKT_OK:
            src = int(desc[i]["offset"])
            assert np.array_equal(ob[o + 16:o + w - 16], plain[src + 16: src + 16 + int(desc[i]["len"])])
        else:  # DecryptionError, or Rejected (in-batch duplicate): never left decrypted
            assert st[k] in (aead.PKT_DECRYPT_ERR, aead.PKT_REJECTED)
            assert np.array_equal(ob[o:o + w], frames_before[o:o + w])  # untouched
    assert (st == aead.PKT_REJECTED).sum() >= 2  # the duplicated 3 and 7 reach the post-pass
    # a forged copy did not burn its counter: the genuine frame is accepted later
    g = np.zeros(int(od[5]["len"]) + 16, np.uint8)
    g[:int(od[5]["len"])] = sealed[int(od[5]["offset"]): int(od[5]["offset"]) + int(od[5]["len"])]
    gd = np.zeros(1, DESC_DTYPE)
    gd[0] = (0, int(od[5]["len"]), 0)
    st2, _ = b.recv_batch(gd, g)
    assert st2[0] == aead.PKT_OK
    model.mark_seen(5)
    # batch 2: replay everything -> rejected by the window and left untouched; counter 11 was
    # only ever seen forged, so its forged copy reaches the tag check again (DECRYPT_ERR)
    ob2 = frames_before.copy()
    st3, _ = b.recv_batch(rdesc, ob2)
    want3 = _model_recv(model, meta)
    assert list(st3) == want3
    assert set(want3) == {aead.PKT_REJECTED, aead.PKT_DECRYPT_ERR}
    assert np.array_equal(ob2, frames_before)


def test_recv_dispatch_checks(pair):
    a, b, sa, sb, sc, keys = pair
    buf = np.zeros(512, np.uint8)
    desc = np.zeros(5, DESC_DTYPE)
    # unknown receiver id
    buf[0:4] = [4, 0, 0, 0]
    buf[4:8] = [0x99, 0, 0, 0]
    desc[0] = (0, 48, 0)
    # handshake init type -> routed to the control plane
    buf[64:68] = [1, 0, 0, 0]
    desc[1] = (64, 148, 0)
    # unaligned frame
    desc[2] = (232, 48, 0)
    buf[232:236] = [4, 0, 0, 0]
    # length not a multiple of 16
    buf[320:324] = [4, 0, 0, 0]
    buf[324:328] = [0x22, 0x22, 0, 0]
    desc[3] = (320, 40, 0)
    # header only: no room for a tag
    buf[384:388] = [4, 0, 0, 0]
    buf[388:392] = [0x22, 0x22, 0, 0]
    desc[4] = (384, 16, 0)
    # unknown message types are Error::InvalidMessage (lib.rs:627); 1-3 go to the control plane
    types = [0, 2, 3, 5, 0xFF, 0x104]
    extra = np.zeros(len(types), DESC_DTYPE)
    big = np.zeros(512 + 64 * len(types), np.uint8)
    big[:512] = buf
    for k, t in enumerate(types):
        o = 512 + 64 * k
        big[o:o + 4] = np.frombuffer(np.uint32(t).tobytes(), np.uint8)
        extra[k] = (o, 48, 0)
    st, slots = b.recv_batch(np.concatenate([desc, extra]), big)
    assert list(st) == [aead.PKT_REJECTED, aead.PKT_NOT_DATA, aead.PKT_UNALIGNED, aead.PKT_INVALID,
                        aead.PKT_DECRYPT_ERR, aead.PKT_INVALID, aead.PKT_NOT_DATA, aead.PKT_NOT_DATA,
                        aead.PKT_INVALID, aead.PKT_INVALID, aead.PKT_INVALID]


def test_per_message_key_objects(engine):
    """EncryptionKey / DecryptionKey mirror prim.rs:376-437 (the handshake test's transport half)."""
    import json
    import os

    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_snapshots.json")))
    k1 = bytes.fromhex(g["transport_seals"][0]["key"])
    ek, dk = aead.EncryptionKey(engine, k1), aead.DecryptionKey(engine, k1)
    for v in (g["transport_seals"][0], g["transport_seals"][2]):
        msg = bytearray.fromhex(v["plaintext"])
        tag = ek.encrypt(msg)
        assert (msg.hex(), tag.hex()) == (v["ciphertext"], v["tag"])
        pt = dk.decrypt(v["counter"], msg + tag)
        assert pt.hex() == v["plaintext"]
        with pytest.raises(aead.Rejected):
            dk.decrypt(v["counter"], bytearray.fromhex(v["ciphertext"] + v["tag"]))
    assert ek.counter() == 2
    with pytest.raises(aead.DecryptionError):
        dk.decrypt(5, bytearray(8))


def test_window_shift_inside_a_batch_rejects_and_restores(pair):
    """Packet j is accepted iff its tag verifies and would_accept(n_j) holds after packets 0..j-1
    (AntiReplay, rustyguard-utils/src/anti_replay.rs:25-64): a high counter accepted first pushes a
    low one out of the 1984-counter window.  The reference rejects that packet before decrypting
    (prim.rs:420-423), so its frame must come back exactly as it arrived."""
    a, b, sa, sb, sc, keys = pair
    rng = np.random.default_rng(9)
    desc, buf = _frames([64, 64], rng)
    st, _ = a.send_batch([sa], desc[:1], buf)  # counter 0
    a.set_send_counter(sa, 5000)
    st2, _ = a.send_batch([sa], desc[1:], buf)  # counter 5000
    assert (st == 0).all() and (st2 == 0).all()
    od = desc.copy()
    od["len"] += 32
    rd = od[[1, 0]].copy()  # 5000 first, then 0 (5000 - 0 >= 1984: too old once 5000 is seen)
    before = buf.copy()
    st3, _ = b.recv_batch(rd, buf)
    assert list(st3) == [aead.PKT_OK, aead.PKT_REJECTED]
    o, w = int(od[0]["offset"]), int(od[0]["len"])
    assert np.array_equal(buf[o:o + w], before[o:o + w])


S = 1_000_000_000  # ns


def test_keepalive_flag_and_timer(pair):
    """decrypt_packet (rustyguard-core/src/lib.rs:664-678): once the session has not sent for more than
    KEEPALIVE_TIMEOUT (10 s), the first authenticated packet asks for a keepalive and marks one pending;
    later packets do not until the Keepalive timer runs (time.rs:114-141), which fires only while the
    session is still quiet; a send resets the clock."""
    a, b, sa, sb, sc, keys = pair
    rng = np.random.default_rng(21)
    desc, buf = _frames([16] * 6, rng)
    st, _ = a.send_batch([sa] * 6, desc, buf)
    assert (st == 0).all()
    od = desc.copy()
    od["len"] += 32

    def recv(idx, now):
        b.set_time(now)
        d = od[idx].copy()
        fr = buf.copy()
        return b.recv_batch(d, fr, src=np.full(len(idx), 7, np.uint64), flags=True)

    st, _, fl = recv([0], 5 * S)  # B inserted at t=0 has sent nothing since: 5 s < 10 s
    assert st[0] == 0 and fl[0] == aead.RECV_AUTHENTICATED
    st, _, fl = recv([1, 2], 11 * S)  # quiet for 11 s: the first packet asks, the second finds it pending
    assert list(st) == [0, 0]
    assert list(fl) == [aead.RECV_AUTHENTICATED | aead.RECV_KEEPALIVE, aead.RECV_AUTHENTICATED]
    st, _, fl = recv([3], 12 * S)
    assert fl[0] == aead.RECV_AUTHENTICATED  # still pending
    b.set_time(13 * S)
    assert b.keepalive_due(sb)  # the timer: still quiet -> send an empty packet
    kd, kb = _frames([0], rng)
    st, _ = b.send_batch([sb], kd, kb)  # the keepalive itself (P = 0) resets `sent`
    assert st[0] == 0
    st, _, fl = recv([4], 14 * S)
    assert fl[0] == aead.RECV_AUTHENTICATED  # sent 1 s ago
    st, _, fl = recv([5], 30 * S)  # the timer cleared `pending`; quiet again for > 10 s
    assert fl[0] == aead.RECV_AUTHENTICATED | aead.RECV_KEEPALIVE


def test_endpoint_moves_only_on_authenticated_packets(pair):
    """The reference's recv_message fuzz invariant (fuzz/fuzz_targets/recv_message.rs:70-122) and
    whitepaper §6.5: forged or replayed packets from another source never redirect the endpoint."""
    a, b, sa, sb, sc, keys = pair
    rng = np.random.default_rng(22)
    desc, buf = _frames([64, 64], rng)
    st, _ = a.send_batch([sa, sa], desc, buf)
    od = desc.copy()
    od["len"] += 32
    assert b.endpoint(sb) is None
    fr = buf.copy()
    st, _ = b.recv_batch(od[:1].copy(), fr, src=np.array([100], np.uint64))
    assert st[0] == 0 and b.endpoint(sb) == 100
    forged = buf.copy()
    o, w = int(od[1]["offset"]), int(od[1]["len"])
    forged[o + w - 1] ^= 1
    st, _, fl = b.recv_batch(od[1:].copy(), forged, src=np.array([666], np.uint64), flags=True)
    assert st[0] == aead.PKT_DECRYPT_ERR and fl[0] == 0 and b.endpoint(sb) == 100
    replay = buf.copy()
    st, _, fl = b.recv_batch(od[:1].copy(), replay, src=np.array([667], np.uint64), flags=True)
    assert st[0] == aead.PKT_REJECTED and fl[0] == 0 and b.endpoint(sb) == 100
    st, _ = b.recv_batch(od[1:].copy(), buf.copy(), src=np.array([101], np.uint64))
    assert st[0] == 0 and b.endpoint(sb) == 101  # roaming: a genuine packet from a new address


def test_send_rejects_after_reject_after_time(pair):
    """should_expire (rustyguard-core/src/lib.rs:207-209): 180 s after the session started, send refuses."""
    a, b, sa, sb, sc, keys = pair
    rng = np.random.default_rng(23)
    desc, buf = _frames([16, 16], rng)
    a.set_time(180 * S)
    st, _ = a.send_batch([sa], desc[:1].copy(), buf)
    assert st[0] == 0  # started + 180 s is not < now
    a.set_time(180 * S + 1)
    st, _ = a.send_batch([sa], desc[1:].copy(), buf)
    assert st[0] == aead.PKT_REJECTED
