"""GPU parity: the HIP path (through the C ABI) against the pinned CPU oracle.

Bit-exact comparisons everywhere (integer/byte work).  Small and medium
batches are compared byte-for-byte with the oracle run live on the same
inputs; the full BASELINE configurations are compared through SHA-256 of the
sealed frames against tests/golden/config_digests.json (computed by the
oracle, spot-checked with OpenSSL) plus the open round-trip property.
"""
import hashlib

import numpy as np
import pytest

from conftest import load_golden
from oracle import oracle
from rustyguard_amd import _lib, aead, workloads
from rustyguard_amd.workloads import DESC_DTYPE

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _random_batch(rng, n, nkeys=3, sizes=None, stride=None, counters=None):
    if sizes is None:
        sizes = rng.integers(0, 129, n) * 16  # P in [0, 2048], multiples of 16
    sizes = np.asarray(sizes, np.int64)
    desc = np.zeros(n, DESC_DTYPE)
    W = sizes + 32
    if stride:
        desc["offset"] = np.arange(n, dtype=np.uint64) * stride
        total = n * stride
    else:
        gaps = rng.integers(0, 3, n) * 16  # holes between frames
        off = np.concatenate([[0], np.cumsum(W + gaps)[:-1]]).astype(np.uint64)
        desc["offset"] = off
        total = int(off[-1] + W[-1] + 64)
    desc["len"] = sizes
    desc["key_idx"] = rng.integers(0, nkeys, n)
    keys = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    rec = rng.integers(0, 2**32, nkeys, dtype=np.uint64).astype(np.uint32)
    if counters is None:
        counters = rng.integers(0, 2**62, n, dtype=np.uint64)
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    return keys, rec, desc, np.asarray(counters, np.uint64), buf


def _gpu_seal(engine, keys, rec, desc, counters, buf):
    b = _dev(buf)
    st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
    engine.seal_dev(_dev(keys), None if rec is None else _dev(rec.view(np.int32)),
                    _dev(desc.view(np.uint8).reshape(-1, 16)), _dev(counters.view(np.int64)), b, st)
    torch.cuda.synchronize()
    return b.cpu().numpy(), st.cpu().numpy()


def _gpu_open(engine, keys, desc_open, buf):
    b = _dev(buf)
    st = torch.zeros(len(desc_open), dtype=torch.uint8, device="cuda")
    co = torch.zeros(len(desc_open), dtype=torch.int64, device="cuda")
    engine.open_dev(_dev(keys), _dev(desc_open.view(np.uint8).reshape(-1, 16)), b, st, co)
    torch.cuda.synchronize()
    return b.cpu().numpy(), st.cpu().numpy(), co.cpu().numpy().view(np.uint64)


# kernel configurations every parity test runs under: the library default
# (automatic kernel choice), the pipelined lane kernel with the size-class
# plan or in array order with K segments per packet, and the LDS-staged tile
# kernel with G-chunk windows, the planner on/off and 1/2/4 segments per
# packet (0 = automatic)
MODES = [("auto",), ("pipe", 0), ("pipe", 1), ("pipe", 2), ("pipe", 4),
         ("tile", 2, 2, 0), ("tile", 2, 1, 0), ("tile", 1, 1, 1), ("tile", 2, 1, 2), ("tile", 2, 1, 4),
         ("tile", 2, 0, 1), ("tile", 2, 0, 2), ("tile", 1, 0, 4), ("tile", 1, 1, 0),
         ("flat", 1), ("flat", 0), ("flat", 2)]


def _configure(engine, mode):
    _reset(engine)
    if mode[0] == "pipe":  # ("pipe", 0): size-class plan; ("pipe", K): array order, K segments
        engine.set_staged(0)
        engine.set_plan(1 if mode[1] == 0 else 0)
        if mode[1]:
            engine.set_lanes_per_packet(mode[1])
    elif mode[0] == "tile":
        _, g, plan, k = mode
        engine.set_staged(g)
        engine.set_plan(plan)
        engine.set_segments(k)
    elif mode[0] == "flat":  # ("flat", plan): flattened chunk stream, units planned / by count / auto
        engine.set_staged(3)
        engine.set_plan(mode[1])


def _reset(engine):
    """library defaults"""
    engine.set_staged(-1)
    engine.set_plan(2)
    engine.set_segments(0)
    engine.set_lanes_per_packet(0)


def _mode_id(m):
    if m[0] == "auto":
        return "auto"
    if m[0] == "pipe":
        return f"pipe{m[1]}" if m[1] else "pipe_plan"
    if m[0] == "flat":
        return f"flat_p{m[1]}"
    return f"tile_g{m[1]}_p{m[2]}_k{m[3]}"


# ------------------------------------------------------------ reference pins
def test_reference_snapshots_per_message(engine):
    """CryptoPrimatives drop-in reproduces the reference's insta snapshots."""
    g = load_golden("reference_snapshots.json")
    for v in g["transport_seals"]:
        key = bytes.fromhex(v["key"])
        buf = bytearray.fromhex(v["plaintext"])
        tag = engine.chacha20poly1305_enc(key, aead.nonce(v["counter"]), b"", buf)
        assert buf.hex() == v["ciphertext"] and tag.hex() == v["tag"]
        engine.chacha20poly1305_dec(key, aead.nonce(v["counter"]), b"", buf, tag)
        assert buf.hex() == v["plaintext"]


def test_xchacha_per_message(engine):
    """Core::xchacha20poly1305_{enc,dec} (cookie replies, rustyguard-crypto/src/lib.rs:50-70) on the GPU
    against tests/golden/xchacha.json; a forged tag leaves the payload untouched."""
    for v in load_golden("xchacha.json")["seals"]:
        key, nonce, aad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["aad"])
        buf = bytearray.fromhex(v["plaintext"])
        tag = engine.xchacha20poly1305_enc(key, nonce, aad, buf)
        assert buf.hex() == v["ciphertext"] and tag.hex() == v["tag"]
        if buf:
            with pytest.raises(aead.DecryptionError):
                engine.xchacha20poly1305_dec(key, nonce, aad, buf, bytes([tag[0] ^ 0x40]) + tag[1:])
            assert buf.hex() == v["ciphertext"]
        engine.xchacha20poly1305_dec(key, nonce, aad, buf, tag)
        assert buf.hex() == v["plaintext"]


@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
def test_reference_framed_packet_batch(engine, mode):
    """rustyguard-core snapshot-3: the full 48-byte framed data packet."""
    _configure(engine, mode)
    v = load_golden("reference_snapshots.json")["framed_packets"][0]
    keys = np.frombuffer(bytes.fromhex(v["key"]), np.uint8).reshape(1, 32)
    pt = np.frombuffer(bytes.fromhex(v["plaintext"]), np.uint8)
    desc = np.zeros(1, DESC_DTYPE)
    desc["len"] = len(pt)
    buf = np.zeros(len(pt) + 32, np.uint8)
    buf[16:16 + len(pt)] = pt
    out, st = _gpu_seal(engine, keys, np.array([v["receiver"]], np.uint32), desc,
                        np.array([v["counter"]], np.uint64), buf)
    assert st[0] == aead.PKT_OK
    assert out.tobytes().hex() == v["frame"]
    od = desc.copy()
    od["len"] = len(buf)
    back, st, ctr = _gpu_open(engine, keys, od, out)
    assert st[0] == aead.PKT_OK and ctr[0] == v["counter"]
    assert np.array_equal(back[16:32], pt)
    forged = out.copy()
    forged[v["tamper_byte"]] ^= 1
    back, st, _ = _gpu_open(engine, keys, od, forged)
    assert st[0] == aead.PKT_DECRYPT_ERR
    assert np.array_equal(back, forged)  # untouched on failure
    _reset(engine)


def test_per_message_openssl_vectors(engine):
    g = load_golden("openssl_vectors.json")
    for v in g["wg_transport"][::3] + g["general_aad"]:
        key = bytes.fromhex(v["key"])
        nz = bytes.fromhex(v["nonce"]) if "nonce" in v else aead.nonce(v["counter"])
        aad = bytes.fromhex(v.get("aad", ""))
        buf = bytearray.fromhex(v["plaintext"])
        tag = engine.chacha20poly1305_enc(key, nz, aad, buf)
        assert buf.hex() == v["ciphertext"] and tag.hex() == v["tag"]
        engine.chacha20poly1305_dec(key, nz, aad, buf, tag)
        assert buf.hex() == v["plaintext"]
        if len(buf):
            bad = bytearray(tag)
            bad[0] ^= 0x80
            ct = bytearray.fromhex(v["ciphertext"])
            with pytest.raises(aead.DecryptionError):
                engine.chacha20poly1305_dec(key, nz, aad, ct, bytes(bad))
            assert ct.hex() == v["ciphertext"]


@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
def test_batch_openssl_transport_vectors(engine, mode):
    """Every 16-aligned OpenSSL transport vector, sealed in one batch."""
    _configure(engine, mode)
    vs = [v for v in load_golden("openssl_vectors.json")["wg_transport"] if (len(v["plaintext"]) // 2) % 16 == 0]
    n = len(vs)
    P = np.array([len(v["plaintext"]) // 2 for v in vs])
    desc = np.zeros(n, DESC_DTYPE)
    desc["offset"] = np.concatenate([[0], np.cumsum(P + 32)[:-1]])
    desc["len"] = P
    desc["key_idx"] = np.arange(n)
    keys = np.stack([np.frombuffer(bytes.fromhex(v["key"]), np.uint8) for v in vs])
    ctr = np.array([v["counter"] for v in vs], np.uint64)
    buf = np.zeros(int((P + 32).sum()), np.uint8)
    for d, v in zip(desc, vs):
        buf[d["offset"] + 16: d["offset"] + 16 + d["len"]] = np.frombuffer(bytes.fromhex(v["plaintext"]), np.uint8)
    out, st = _gpu_seal(engine, keys, None, desc, ctr, buf)
    assert (st == aead.PKT_OK).all()
    for d, v in zip(desc, vs):
        o, p = int(d["offset"]), int(d["len"])
        assert out[o + 16: o + 16 + p].tobytes().hex() == v["ciphertext"]
        assert out[o + 16 + p: o + 32 + p].tobytes().hex() == v["tag"]
    _reset(engine)


# ------------------------------------------------------- oracle differential
@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
@pytest.mark.parametrize("seed", [1, 2])
def test_random_batches_vs_oracle(engine, mode, seed):
    _configure(engine, mode)
    rng = np.random.default_rng(seed)
    n = 3000
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=5)
    ctr[:4] = [0, 0xFFFFFFFF, 0x100000000, 2**64 - 1]
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8)
    got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st == aead.PKT_OK).all()
    assert np.array_equal(got, want)
    # open the sealed frames back
    od = desc.copy()
    od["len"] += 32
    back, st, co = _gpu_open(engine, keys, od, got)
    assert (st == aead.PKT_OK).all()
    assert np.array_equal(co, ctr)
    for d in desc[:200]:
        o, p = int(d["offset"]), int(d["len"])
        assert np.array_equal(back[o + 16: o + 16 + p], buf[o + 16: o + 16 + p])
    _reset(engine)


@pytest.mark.parametrize("wg", [1, 2, 3])
def test_planned_pipe_residency_vs_oracle(engine, wg):
    """The planned pipelined path deals its work-ordered tiles in snake order over CUs x wg_per_cu x 4
    waves (default 2 per CU): mixed sizes, invalid and skipped descriptors at 1, 2 and 3 resident
    workgroups per CU give the oracle's bytes and statuses."""
    _reset(engine)
    engine.set_staged(0)
    engine.set_plan(1)
    engine.set_wg_per_cu(wg)
    try:
        rng = np.random.default_rng(50 + wg)
        n = 20000
        sizes = rng.choice([64, 576, 1504, 0, 16, 2048], n, p=[0.5, 0.3, 0.1, 0.04, 0.04, 0.02])
        keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=4, sizes=sizes)
        want = buf.copy()
        wst = np.zeros(n, np.uint8)
        oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8, status=wst)
        got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
        assert np.array_equal(st, wst) and np.array_equal(got, want)
        od = desc.copy()
        od["len"] += 32
        od["len"][5::89] = 31  # not a whole number of 16-byte blocks: invalid after the header check
        skip = np.zeros(n, bool)
        skip[::97] = True  # RG_KEY_SKIP: rejected and untouched (the oracle never sees these frames)
        want_open = got.copy()
        wst = np.full(n, aead.PKT_REJECTED, np.uint8)
        wco = np.zeros(n, np.uint64)
        wst[~skip], wco[~skip] = oracle.open_batch(keys, od[~skip], want_open, nthreads=8)
        od["key_idx"][skip] = aead.KEY_SKIP
        back, st, co = _gpu_open(engine, keys, od, got)
        assert np.array_equal(st, wst) and np.array_equal(back, want_open)
        ok = wst == aead.PKT_OK
        assert np.array_equal(co[ok], wco[ok])
    finally:
        engine.set_wg_per_cu(0)
        _reset(engine)


@pytest.mark.parametrize("mix", ["imix", "half_1504_64", "576_1504", "spread"])
def test_schedule_targets_vs_oracle(engine, mix):
    """Size mixes whose best segment target differs (schedule_classes picks among multiples of the mean
    work per SIMD by the estimated makespan): the planned pipelined path gives the oracle's bytes."""
    _reset(engine)
    engine.set_staged(0)
    engine.set_plan(1)
    try:
        rng = np.random.default_rng(77)
        n = 40000
        if mix == "imix":
            sizes = rng.choice([64, 576, 1504], n, p=[7 / 12, 4 / 12, 1 / 12])
        elif mix == "half_1504_64":
            sizes = rng.choice([64, 1504], n)
        elif mix == "576_1504":
            sizes = rng.choice([576, 1504], n)
        else:
            sizes = rng.integers(0, 129, n) * 16
        keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=2, sizes=sizes)
        want = buf.copy()
        oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8)
        got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
        assert (st == aead.PKT_OK).all() and np.array_equal(got, want)
        od = desc.copy()
        od["len"] += 32
        want_open = got.copy()
        wst, wco = oracle.open_batch(keys, od, want_open, nthreads=8)
        back, st, co = _gpu_open(engine, keys, od, got)
        assert (wst == aead.PKT_OK).all() and np.array_equal(st, wst) and np.array_equal(co, wco)
        assert np.array_equal(back, want_open)
    finally:
        _reset(engine)


@pytest.mark.parametrize("rounds", [1.02, 2.5, 16.5])
@pytest.mark.parametrize("plan", [0, 1])
def test_tile_dynamic_deal_vs_oracle(engine, rounds, plan):
    """The tile kernel's dynamic deal (unsegmented classes, rg_tile.hip): a workgroup's tiles taken by
    whichever of its eight waves is free, over several deal rounds with a partial last one (from two rounds
    the last eighth from the grid-wide pool), five forged frames; seal and open bit-exact against the
    oracle."""
    engine.set_staged(2)
    engine.set_plan(plan)
    engine.set_segments(1)
    rng = np.random.default_rng(53)
    waves = 8 * torch.cuda.get_device_properties(0).multi_processor_count
    n = int(rounds * waves * 64) + 13
    sizes = rng.integers(0, 9, n) * 16  # P in [0, 128]: many tiles, a quick oracle
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=4, sizes=sizes)
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8)
    got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st == aead.PKT_OK).all()
    assert np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    forged = rng.choice(n, size=5, replace=False)
    tampered = got.copy()
    for j in forged:  # last tag byte
        tampered[int(od[j]["offset"]) + int(od[j]["len"]) - 1] ^= 0x01
    back, st, co = _gpu_open(engine, keys, od, tampered)
    ok = np.ones(n, bool)
    ok[forged] = False
    assert (st[ok] == aead.PKT_OK).all() and (st[forged] == aead.PKT_DECRYPT_ERR).all()
    assert np.array_equal(co, ctr)
    for j in forged:
        o, w = int(od[j]["offset"]), int(od[j]["len"])
        assert np.array_equal(back[o:o + w], tampered[o:o + w])
    for i in np.nonzero(ok)[0][::97]:
        o, p = int(desc[i]["offset"]), int(desc[i]["len"])
        assert np.array_equal(back[o + 16: o + 16 + p], buf[o + 16: o + 16 + p])
    _reset(engine)


@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
def test_large_payload_mix_vs_oracle(engine, mode):
    """Every size class of the planner (up to the 1 MiB payload limit), shuffled with small packets,
    then opened back; one large frame forged to check the segmented restore path."""
    _configure(engine, mode)
    rng = np.random.default_rng(31)
    big = [1 << 20, 65520, 40000 // 16 * 16, 16384, 4096 + 16, 2048, 1040, 1024]
    sizes = np.array(big + list(rng.integers(0, 100, 200) * 16))
    rng.shuffle(sizes)
    n = len(sizes)
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=3, sizes=sizes)
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8)
    got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st == aead.PKT_OK).all()
    assert np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    j = int(np.argmax(sizes))
    tampered = got.copy()
    tampered[int(od[j]["offset"]) + 16 + int(sizes[j]) // 2] ^= 0x10
    back, st, co = _gpu_open(engine, keys, od, tampered)
    ok = np.ones(n, bool)
    ok[j] = False
    assert (st[ok] == aead.PKT_OK).all() and st[j] == aead.PKT_DECRYPT_ERR
    o, w = int(od[j]["offset"]), int(od[j]["len"])
    assert np.array_equal(back[o:o + w], tampered[o:o + w])
    for i in np.nonzero(ok)[0][::7]:
        o, p = int(desc[i]["offset"]), int(desc[i]["len"])
        assert np.array_equal(back[o + 16: o + 16 + p], buf[o + 16: o + 16 + p])
    _reset(engine)


@pytest.mark.parametrize("per_unit", [400, 80])
@pytest.mark.parametrize("plan", [0, 1])
def test_flat_subunits_vs_oracle(engine, plan, per_unit):
    """The flattened kernel stages at most kFlatMaxPk (128) packets of a unit in LDS at a time:
    400 Ki small packets (keepalives P = 0 and 16/64/128-byte payloads) put ~400 packets in each of
    the 1024 units, so every wave runs several sub-units; forged frames in the middle of them.  With
    ~80 packets per unit the key blocks of packets 64 and up come from lane quads (rg_flat.hip), and
    some forged frames sit there (open: tag - s computed on the quad)."""
    engine.set_staged(3)
    engine.set_plan(plan)
    rng = np.random.default_rng(77)
    n = per_unit * 1024
    sizes = rng.choice(np.array([0, 16, 64, 128]), n, p=[0.4, 0.3, 0.2, 0.1])
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=4, sizes=sizes, stride=160)
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8)
    got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st == aead.PKT_OK).all()
    assert np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    forged = rng.choice(n, 50, replace=False)
    tampered = got.copy()
    for i in forged:
        tampered[int(od[i]["offset"]) + int(od[i]["len"]) - 1] ^= 1
    back, st, co = _gpu_open(engine, keys, od, tampered)
    bad = np.zeros(n, bool)
    bad[forged] = True
    assert (st[~bad] == aead.PKT_OK).all() and (st[bad] == aead.PKT_DECRYPT_ERR).all()
    assert np.array_equal(co, ctr)
    for i in forged:
        o, w = int(od[i]["offset"]), int(od[i]["len"])
        assert np.array_equal(back[o:o + w], tampered[o:o + w])
    for i in np.nonzero(~bad)[0][::97]:
        o, p = int(desc[i]["offset"]), int(desc[i]["len"])
        assert np.array_equal(back[o + 16: o + 16 + p], buf[o + 16: o + 16 + p])
    _reset(engine)


def test_flat_whole_groups_vs_oracle(engine):
    """The flattened kernel forced (rg_set_staged 3) on more than 1024 packets per unit: units are then
    whole 1024-packet groups (rg_flat.hip, the third unit rule), each wave runs eight or more 128-packet
    sub-units.  1 Mi + 5000 small packets (keepalives, 16 and 64 bytes), every byte and status against the
    oracle, and the open of the result with forged tags."""
    engine.set_staged(3)
    engine.set_plan(0)
    rng = np.random.default_rng(1025)
    n = 1024 * 1024 + 5000
    sizes = rng.choice(np.array([0, 16, 64]), n, p=[0.2, 0.4, 0.4])
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=2, sizes=sizes, stride=96)
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8)
    got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st == aead.PKT_OK).all()
    assert np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    forged = rng.choice(n, 64, replace=False)
    tampered = got.copy()
    for i in forged:
        tampered[int(od[i]["offset"]) + int(od[i]["len"]) - 1] ^= 1
    back, st, co = _gpu_open(engine, keys, od, tampered)
    bad = np.zeros(n, bool)
    bad[forged] = True
    assert (st[~bad] == aead.PKT_OK).all() and (st[bad] == aead.PKT_DECRYPT_ERR).all()
    assert np.array_equal(co, ctr)
    for i in forged:
        o, w = int(od[i]["offset"]), int(od[i]["len"])
        assert np.array_equal(back[o:o + w], tampered[o:o + w])
    for i in np.nonzero(~bad)[0][::997]:
        o, p = int(desc[i]["offset"]), int(desc[i]["len"])
        assert np.array_equal(back[o + 16: o + 16 + p], buf[o + 16: o + 16 + p])
    _reset(engine)


@pytest.mark.parametrize("plan", [0, 1])
def test_flat_far_and_empty_descriptors_vs_oracle(engine, plan):
    """Round 4: in the flattened chunk stream every packet holds at least one chunk step; a packet with no
    payload block (P = 0 keepalive, a descriptor that failed its checks) gets one step whose loads read a
    safe address and whose stores are dropped.  Descriptors far past the arena (offset 2^40, 2^63), short
    and unaligned ones sit between valid frames of 0..1504 bytes: statuses and every byte against the
    oracle, open of the sealed batch, forged tags restored."""
    engine.set_staged(3)
    engine.set_plan(plan)
    rng = np.random.default_rng(404)
    n = 3000
    sizes = rng.choice(np.array([0, 16, 64, 576, 1504]), n, p=[0.2, 0.2, 0.3, 0.2, 0.1])
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=3, sizes=sizes)
    bad = rng.choice(n, 60, replace=False)
    kinds = [(1 << 40, 64), (1 << 63, 16), (8, 16), (0, 17)]
    for j, i in enumerate(bad):
        o, p = kinds[j % len(kinds)]
        desc[i]["offset"], desc[i]["len"] = o if o else int(desc[i]["offset"]), p
    good = np.ones(n, bool)
    good[bad] = False
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc[good], ctr[good], want, nthreads=8)
    got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st[good] == aead.PKT_OK).all() and (st[bad] == aead.PKT_INVALID).all()
    assert np.array_equal(got, want)
    od = desc.copy()
    od["len"][good] += 32
    forged = rng.choice(np.nonzero(good)[0], 30, replace=False)
    tampered = got.copy()
    for i in forged:
        tampered[int(od[i]["offset"]) + int(od[i]["len"]) - 1] ^= 1
    back, st, co = _gpu_open(engine, keys, od, tampered)
    want_back = tampered.copy()
    wst, wctr = oracle.open_batch(keys, od[good], want_back, nthreads=8)
    assert np.array_equal(st[good], wst) and (st[bad] != aead.PKT_OK).all()
    assert (wst[np.searchsorted(np.nonzero(good)[0], forged)] == oracle.DECRYPT_ERR).all()
    assert np.array_equal(back, want_back)
    _reset(engine)


def test_flat_coop_search_skewed_quarters_vs_oracle(engine):
    """Round 5's one-barrier search: every wave reads its own two cut points out of the workgroup's shared
    prefix, from whichever quarter of the 4096-packet group holds each target.  Here each group's first
    quarter holds only 1504-byte packets and the other three only keepalives and 16-byte packets, so most
    units lie in quarter 0 (a few packets each), the cut points between the last of those and the next
    cross the quarter boundary, and the remaining units hold several hundred packets each (sub-units of
    kFlatMaxPk, staged one after another).  Seal and open, every byte and status against the oracle."""
    import torch

    n = 65536
    units = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    if (units * 4096) % n or ((units * 4096) // n) % 4:
        pytest.skip("the cooperative search does not apply at this CU count")
    engine.set_staged(3)
    engine.set_plan(1)
    rng = np.random.default_rng(505)
    pos = np.arange(n) % 4096
    sizes = np.where(pos < 1024, 1504, rng.choice([0, 16], n))
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=2, sizes=sizes)
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8)
    got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st == aead.PKT_OK).all()
    assert np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    back, st, co = _gpu_open(engine, keys, od, got)
    want_back = want.copy()
    wst, wctr = oracle.open_batch(keys, od, want_back, nthreads=8)
    assert (wst == 0).all() and (st == aead.PKT_OK).all() and np.array_equal(co, wctr)
    assert np.array_equal(back, want_back)
    _reset(engine)


@pytest.mark.parametrize("n", [4096, 16384, 65536, 131072])
def test_flat_coop_search_vs_oracle(engine, n):
    """When n is a multiple of 4096 and the units of a 4096-packet group are a multiple of four (CUs x 4
    units), the four waves of a workgroup cut their units together (rg_flat.hip, A.coop): ~4, 16, 64 and
    128 packets per unit here (the last with sub-units and lane-quad key blocks).  Random sizes 0..2048 B
    over three keys, descriptors that fail their checks (far offsets, unaligned lengths) among them (round
    5), 40 forged frames: every byte and status against the oracle."""
    import torch

    units = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    if (units * 4096) % n or ((units * 4096) // n) % 4:
        pytest.skip("the cooperative search does not apply at this CU count")
    engine.set_staged(3)
    engine.set_plan(1)
    rng = np.random.default_rng(n)
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=3)
    bad = rng.choice(n, 24, replace=False)
    for j, i in enumerate(bad):
        if j % 2:
            desc[i]["offset"] = 1 << 40
        else:
            desc[i]["len"] = 17
    good = np.ones(n, bool)
    good[bad] = False
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc[good], ctr[good], want, nthreads=8)
    got, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st[good] == aead.PKT_OK).all() and (st[bad] == aead.PKT_INVALID).all()
    assert np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    forged = rng.choice(np.nonzero(good)[0], 40, replace=False)
    tampered = got.copy()
    for i in forged:
        tampered[int(od[i]["offset"]) + int(od[i]["len"]) - 1] ^= 1
    back, st, co = _gpu_open(engine, keys, od, tampered)  # all n descriptors: the cooperative deal again
    want_back = tampered.copy()
    wst, wctr = oracle.open_batch(keys, od[good], want_back, nthreads=8)
    assert np.array_equal(st[good], wst) and (st[bad] != aead.PKT_OK).all()
    assert (wst[np.searchsorted(np.nonzero(good)[0], forged)] == oracle.DECRYPT_ERR).all()
    assert np.array_equal(co[good][wst == 0], wctr[wst == 0])
    assert np.array_equal(back, want_back)
    _reset(engine)


@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
def test_open_failures_leave_frames_untouched(engine, mode):
    _configure(engine, mode)
    rng = np.random.default_rng(9)
    n = 512
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=2, sizes=rng.integers(1, 96, n) * 16)
    oracle.seal_batch(keys, rec, desc, ctr, buf)
    od = desc.copy()
    od["len"] += 32
    sealed = buf.copy()
    # tamper every 3rd packet at a random byte of payload or tag
    bad = np.arange(0, n, 3)
    for i in bad:
        o, w = int(od[i]["offset"]), int(od[i]["len"])
        buf[o + int(rng.integers(16, w))] ^= 1 << int(rng.integers(0, 8))
    tampered = buf.copy()
    back, st, _ = _gpu_open(engine, keys, od, buf)
    want_st, _ = oracle.open_batch(keys, od, tampered.copy())
    assert np.array_equal(st, want_st)
    assert (st[bad] == aead.PKT_DECRYPT_ERR).all()
    for i in bad:
        o, w = int(od[i]["offset"]), int(od[i]["len"])
        assert np.array_equal(back[o:o + w], tampered[o:o + w])
    good = np.setdiff1d(np.arange(n), bad)
    assert (st[good] == aead.PKT_OK).all()
    _reset(engine)


@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
def test_open_malformed_statuses_match_oracle(engine, mode):
    _configure(engine, mode)
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 256, (2, 32), dtype=np.uint8)
    buf = np.zeros(4096, np.uint8)
    cases = [  # (offset, W, type, key_idx)
        (0, 48, 4, 0),        # decrypt error (random tag)
        (64, 47, 4, 0),       # W % 16 != 0 -> InvalidMessage
        (128, 3, 4, 0),       # shorter than the type word
        (192, 16, 4, 0),      # header only -> DecryptionError (no tag)
        (256, 64, 1, 0),      # handshake init type -> not data
        (520, 48, 4, 0),      # unaligned
        (640, 32, 4, 0),      # empty payload + random tag -> DecryptionError
        (704, 48, 4, 0xFFFFFFFF),  # skipped by the host
        (4080, 48, 4, 0),     # runs past the arena
        (768, 48, 0, 0),      # type 0 -> InvalidMessage (lib.rs:627)
        (832, 48, 5, 0),      # type 5 -> InvalidMessage
        (896, 48, 0xFF, 0),   # type 0xFF -> InvalidMessage
        (960, 48, 2, 0),      # handshake response -> not data
        (1024, 64, 3, 0),     # cookie reply -> not data
        (1088, 48, 0x104, 0), # type word 0x104: the whole LE u32 is compared -> InvalidMessage
    ]
    desc = np.zeros(len(cases), DESC_DTYPE)
    for i, (o, w, t, k) in enumerate(cases):
        desc[i] = (o, w, k)
        if o + 4 <= len(buf):
            buf[o:o + 4] = np.frombuffer(np.uint32(t).tobytes(), np.uint8)
            buf[o + 8:o + 16] = rng.integers(0, 256, 8, dtype=np.uint8)
    checked = [0, 1, 2, 3, 4, 5, 6, 9, 10, 11, 12, 13, 14]
    want, wctr = oracle.open_batch(keys, desc[checked], buf.copy())
    back, st, co = _gpu_open(engine, keys, desc, buf)
    assert list(st[checked]) == list(want)
    assert st[7] == aead.PKT_REJECTED and st[8] == aead.PKT_INVALID
    assert list(st) == [1, 2, 2, 1, 5, 4, 1, 3, 2, 2, 2, 2, 5, 5, 2]
    _reset(engine)


@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
def test_seal_rejects_bad_descriptors(engine, mode):
    _configure(engine, mode)
    keys = np.zeros((1, 32), np.uint8)
    desc = np.zeros(4, DESC_DTYPE)
    desc[0] = (0, 17, 0)      # P % 16 != 0
    desc[1] = (8, 16, 0)      # unaligned
    desc[2] = (64, 16, 3)     # key out of range
    desc[3] = (4000, 512, 0)  # past the end
    buf = np.arange(4096, dtype=np.uint32).astype(np.uint8)
    out, st = _gpu_seal(engine, keys, None, desc, np.zeros(4, np.uint64), buf)
    assert list(st) == [aead.PKT_INVALID] * 4
    assert np.array_equal(out, buf)
    _reset(engine)


@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
def test_empty_payload_keepalive(engine, mode):
    """Keepalive seals an empty payload (rustyguard-core/src/time.rs:131): 32-byte frame."""
    _configure(engine, mode)
    keys = np.frombuffer(bytes(range(32)), np.uint8).reshape(1, 32)
    desc = np.zeros(1, DESC_DTYPE)
    buf = np.zeros(32, np.uint8)
    out, st = _gpu_seal(engine, keys, np.array([7], np.uint32), desc, np.array([5], np.uint64), buf)
    want = buf.copy()
    oracle.seal_batch(keys, np.array([7], np.uint32), desc, np.array([5], np.uint64), want)
    assert np.array_equal(out, want)
    _reset(engine)


def test_host_path_matches_oracle(engine):
    rng = np.random.default_rng(11)
    n = 20000
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=7)
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc, ctr, want, nthreads=8)
    got = buf.copy()
    st = engine.seal_host(keys, rec, desc, ctr, got)
    assert (st == aead.PKT_OK).all() and np.array_equal(got, want)
    od = desc.copy()
    od["len"] += 32
    st, co = engine.open_host(keys, od, got)
    assert (st == aead.PKT_OK).all() and np.array_equal(co, ctr)
    assert np.array_equal(got[16:16 + int(desc[0]["len"])], buf[16:16 + int(desc[0]["len"])])


def test_host_path_pinned_buffer_matches_oracle(engine):
    """The caller's frames in pinned host memory (rg_host_alloc): downloads are host_store_kernel writes
    over the link, not copies.  Several slices, and a last frame with P % 16 != 0 (INVALID by the
    rg_aead.h contract, left as it came) whose bytes still lie in the last slice's span, so that the span
    ends off a 16-byte boundary (the kernel's byte tail)."""
    rng = np.random.default_rng(23)
    n = 6000
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=5)
    desc[-1]["len"] = 40  # the span's end is 8 bytes past a 16-byte boundary
    want = buf.copy()
    oracle.seal_batch(keys, rec, desc[:-1], ctr[:-1], want, nthreads=8)
    got = aead.host_alloc(len(buf))
    got[:] = buf
    engine.set_host_slice(1 << 20)
    try:
        st = engine.seal_host(keys, rec, desc, ctr, got)
        assert st[-1] == aead.PKT_INVALID and (st[:-1] == aead.PKT_OK).all()
        assert np.array_equal(got, want)
        od = desc[:-1].copy()
        od["len"] += 32
        ow = want.copy()
        so_w, co_w = oracle.open_batch(keys, od, ow)
        so, co = engine.open_host(keys, od, got)
        assert (so == aead.PKT_OK).all() and np.array_equal(so, so_w) and np.array_equal(co, co_w)
        assert np.array_equal(got, ow)
    finally:
        engine.set_host_slice(8 << 20)
        del got


# ------------------------------------------------------- full configurations
@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg4"])
def test_full_config_digest(engine, name):
    from rustyguard_amd.device import DeviceBatch

    dig = load_golden("config_digests.json")[name]
    w = workloads.build(name)
    assert w.n == dig["n"] and w.buf_bytes == dig["buf_bytes"]
    b = DeviceBatch(engine, w)
    b.fill()
    torch.cuda.synchronize()
    assert hashlib.sha256(b.host_buf().tobytes()).hexdigest() == dig["plain_sha256"]
    for mode in MODES:
        _configure(engine, mode)
        b.fill()
        b.seal()
        torch.cuda.synchronize()
        assert (b.status[: w.n] == 0).all().item()
        assert hashlib.sha256(b.host_buf().tobytes()).hexdigest() == dig["sealed_sha256"], mode
        b.open()
        torch.cuda.synchronize()
        assert (b.status[: w.n] == 0).all().item()
        assert torch.equal(b.counters_out[: w.n], b.counters)
        assert hashlib.sha256(b.host_buf().tobytes()).hexdigest() != dig["sealed_sha256"]
        # plaintext restored except the framing (header + tag) written by seal
        hb = b.host_buf()
        plain = np.zeros_like(hb)
        oracle.synth_fill(plain, w.desc, w.inner_len, w.data_seed)
        for d in w.desc[:: max(1, w.n // 500)]:
            o, p = int(d["offset"]), int(d["len"])
            assert np.array_equal(hb[o + 16:o + 16 + p], plain[o + 16:o + 16 + p])
    _reset(engine)


@pytest.mark.parametrize("rank", [0, 7])
def test_cfg5_shard_digest(engine, rank):
    """BASELINE config 5 as one rank of 8 runs it: 1 Mi x 1500-B packets, one key, counters and
    payload bytes of global packets [rank * 1 Mi, (rank + 1) * 1 Mi) (workloads.shard), sealed and
    opened on the GPU under the automatic kernel choice and the pipelined kernel, against the
    oracle's SHA-256 digests (tests/golden/cfg5_digests.json)."""
    from rustyguard_amd.device import DeviceBatch

    g = load_golden("cfg5_digests.json")
    dig = g[f"rank{rank}"]
    w = workloads.build("cfg5", rank, g["world"])
    assert w.n == dig["n"] and w.buf_bytes == dig["buf_bytes"] and int(w.counters[0]) == dig["first_counter"]
    b = DeviceBatch(engine, w)
    b.fill()
    torch.cuda.synchronize()
    assert hashlib.sha256(b.host_buf().tobytes()).hexdigest() == dig["plain_sha256"]
    for staged in (-1, 0):
        engine.set_staged(staged)
        b.fill()
        b.seal()
        torch.cuda.synchronize()
        assert (b.status[: w.n] == 0).all().item()
        assert hashlib.sha256(b.host_buf().tobytes()).hexdigest() == dig["sealed_sha256"], staged
        b.open()
        torch.cuda.synchronize()
        assert (b.status[: w.n] == 0).all().item()
        assert torch.equal(b.counters_out[: w.n], b.counters)
        assert hashlib.sha256(b.host_buf().tobytes()).hexdigest() == dig["opened_sha256"], staged
    del b
    torch.cuda.empty_cache()
    _reset(engine)


@pytest.mark.parametrize("mode", MODES, ids=_mode_id)
def test_frames_past_2_and_4_gib(engine, mode):
    """Byte offsets with bit 31 / bit 32 set (large device arenas, BASELINE config 5 on one GPU)."""
    _configure(engine, mode)
    rng = np.random.default_rng(99)
    marks = [0, 1 << 31, 1 << 32, 3 << 31]
    offs = []
    for m in marks:
        base = max(0, m - 1536 * 40)
        offs += [base + 1536 * k for k in range(80)]
    n = len(offs)
    P = rng.integers(0, 95, n) * 16
    desc = np.zeros(n, DESC_DTYPE)
    desc["offset"] = offs
    desc["len"] = P
    desc["key_idx"] = rng.integers(0, 2, n)
    keys = rng.integers(0, 256, (2, 32), dtype=np.uint8)
    rec = np.array([7, 9], np.uint32)
    ctr = rng.integers(0, 2**40, n, dtype=np.uint64)
    total = offs[-1] + 1536 + 64
    buf = torch.zeros(total, dtype=torch.uint8, device="cuda")
    frames = []
    for i in range(n):
        f = rng.integers(0, 256, int(P[i]) + 32, dtype=np.uint8)
        frames.append(f)
        buf[offs[i]: offs[i] + len(f)] = _dev(f)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.seal_dev(_dev(keys), _dev(rec.view(np.int32)), _dev(desc.view(np.uint8).reshape(-1, 16)),
                    _dev(ctr.view(np.int64)), buf, st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    for i in range(n):
        ref = frames[i].copy()
        one = np.zeros(1, DESC_DTYPE)
        one[0] = (0, P[i], desc["key_idx"][i])
        oracle.seal_batch(keys, rec, one, ctr[i:i + 1], ref)
        got = buf[offs[i]: offs[i] + len(ref)].cpu().numpy()
        assert np.array_equal(got, ref), (i, offs[i])
    od = desc.copy()
    od["len"] += 32
    ctr_out = torch.zeros(n, dtype=torch.int64, device="cuda")
    engine.open_dev(_dev(keys), _dev(od.view(np.uint8).reshape(-1, 16)), buf, st, ctr_out)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert np.array_equal(ctr_out.cpu().numpy().view(np.uint64), ctr)
    for i in range(0, n, 7):
        got = buf[offs[i] + 16: offs[i] + 16 + int(P[i])].cpu().numpy()
        assert np.array_equal(got, frames[i][16:16 + int(P[i])])
    del buf
    torch.cuda.empty_cache()
    _reset(engine)


# ------------------------------------------------- device-side receiver lookup
@pytest.mark.parametrize("mode", [("auto",), ("pipe", 0), ("tile", 2, 1, 0)], ids=_mode_id)
def test_open_with_device_receiver_lookup(engine, mode):
    _configure(engine, mode)
    rng = np.random.default_rng(21)
    nses, n = 6, 400
    keys, rec, desc, ctr, buf = _random_batch(rng, n, nkeys=nses)
    rec = np.unique(rng.integers(1, 2**32, 3 * nses, dtype=np.uint64).astype(np.uint32))[:nses]
    sealed, st = _gpu_seal(engine, keys, rec, desc, ctr, buf)
    assert (st == 0).all()
    dopen = desc.copy()
    dopen["len"] = desc["len"] + 32
    dopen["key_idx"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)  # ignored by the rx path
    wire = sealed.copy()
    pick = rng.permutation(n)
    unknown, data_type, forged = pick[:12], pick[12:20], pick[20:28]
    for i in unknown:  # receiver without a session: header is not authenticated -> Error::Rejected
        wire[desc["offset"][i] + 4:desc["offset"][i] + 8] = np.frombuffer(np.uint32(0xA5A5A5A5).tobytes(), np.uint8)
    for i in data_type:
        wire[desc["offset"][i]] = 1  # handshake initiation -> routed elsewhere
    for i in forged:
        wire[desc["offset"][i] + 16 + desc["len"][i]] ^= 0x80  # tag bit flip -> DecryptionError
    table = aead.rx_table(rec, np.arange(nses, dtype=np.uint32))
    want, wctr, wkey = oracle.open_batch_rx(keys, rec, dopen, wire.copy())
    b = _dev(wire)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    co = torch.zeros(n, dtype=torch.int64, device="cuda")
    ko = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.open_dev_rx(_dev(keys), _dev(table), _dev(dopen.view(np.uint8).reshape(-1, 16)), b, st, co, ko)
    torch.cuda.synchronize()
    st, back, ko = st.cpu().numpy(), b.cpu().numpy(), ko.cpu().numpy().view(np.uint32)
    assert list(st) == list(want)
    assert (co.cpu().numpy().view(np.uint64) == wctr).all()
    resolved = (st == 0) | (st == 1)
    assert (ko[resolved] == wkey[resolved]).all()
    assert (st[unknown] == aead.PKT_REJECTED).all() and (st[data_type] == 5).all() and (st[forged] == 1).all()
    ok = st == 0
    assert ok.sum() == n - 28
    assert (ko[ok] == desc["key_idx"][ok]).all() and (ko[unknown] == 0xFFFFFFFF).all()
    for i in np.nonzero(ok)[0]:  # plaintext back in place, byte for byte
        o, P = int(desc["offset"][i]), int(desc["len"][i])
        assert (back[o + 16:o + 16 + P] == buf[o + 16:o + 16 + P]).all()
    for i in np.nonzero(~ok)[0]:  # rejected frames are left as they came
        o, W = int(dopen["offset"][i]), int(dopen["len"][i])
        assert (back[o:o + W] == wire[o:o + W]).all()
    _reset(engine)


def test_receiver_lookup_check_order(engine):
    """Crafted frames pin the reference's order: Unaligned / InvalidMessage / not-data before the
    session lookup, Rejected (unknown receiver) before DecryptionError (too short for a tag)."""
    _reset(engine)
    keys = np.zeros((1, 32), np.uint8)
    table = aead.rx_table([77], [0])
    buf = np.zeros(1024, np.uint8)
    cases = [  # (offset, W, type, receiver) -> status
        (8, 48, 4, 77, aead.PKT_UNALIGNED),
        (64, 40, 4, 99, aead.PKT_INVALID),        # not whole 16-byte segments: before the lookup
        (128, 48, 1, 99, 5),                      # not a data message: before the lookup
        (192, 16, 4, 99, aead.PKT_REJECTED),      # unknown session beats "no room for a tag"
        (256, 16, 4, 77, 1),                      # known session, no tag -> DecryptionError
        (320, 48, 4, 99, aead.PKT_REJECTED),
        (384, 48, 4, 77, 1),                      # random tag
    ]
    desc = np.zeros(len(cases), DESC_DTYPE)
    for i, (o, w, t, r, _) in enumerate(cases):
        desc[i] = (o, w, 0)
        buf[o:o + 4] = np.frombuffer(np.uint32(t).tobytes(), np.uint8)
        buf[o + 4:o + 8] = np.frombuffer(np.uint32(r).tobytes(), np.uint8)
    st = torch.zeros(len(cases), dtype=torch.uint8, device="cuda")
    engine.open_dev_rx(_dev(keys), _dev(table), _dev(desc.view(np.uint8).reshape(-1, 16)), _dev(buf), st)
    torch.cuda.synchronize()
    assert list(st.cpu().numpy()) == [c[4] for c in cases]


# ------------------------------------------------------ handshake MAC checks
def _handshake_batch(rng, n, keys, key_len, which):
    """n handshake messages (init 148 B / response 92 B, 16-byte aligned) whose mac field is valid for a
    random key; returns desc (key_idx = the signing key), buf."""
    sizes = rng.choice([148, 92], n)
    off = np.concatenate([[0], np.cumsum((sizes + 15) // 16 * 16)[:-1]]).astype(np.uint64)
    buf = rng.integers(0, 256, int(off[-1]) + 160, dtype=np.uint8)
    desc = np.zeros(n, DESC_DTYPE)
    desc["offset"], desc["len"] = off, sizes
    desc["key_idx"] = rng.integers(0, len(keys), n)
    for i in range(n):
        o, L = int(off[i]), int(sizes[i])
        cov = L - (32 if which == 1 else 16)
        mac = oracle.blake2s(buf[o:o + cov].tobytes(), keys[desc["key_idx"][i]].tobytes(), 16)
        buf[o + cov:o + cov + 16] = np.frombuffer(mac, np.uint8)
    return desc, buf


@pytest.mark.parametrize("which", [1, 2])
def test_mac_verify_batch_vs_oracle(engine, which):
    """HasMac::verify_mac1 / verify_mac2 (rustyguard-crypto/src/lib.rs:138-158) on the GPU against the
    oracle: given keys, the wg-proxy peer scan (RG_KEY_SCAN), wrong keys and forged macs."""
    rng = np.random.default_rng(30 + which)
    key_len = 32 if which == 1 else 16
    keys = rng.integers(0, 256, (24, key_len), dtype=np.uint8)
    desc, buf = _handshake_batch(rng, 1500, keys, key_len, which)
    pick = rng.permutation(len(desc))
    desc["key_idx"][pick[:500]] = aead.KEY_SCAN
    desc["key_idx"][pick[500:600]] = (desc["key_idx"][pick[500:600]] + 1) % len(keys)  # wrong peer
    for i in pick[600:700]:  # forged mac byte
        buf[int(desc["offset"][i]) + int(desc["len"][i]) - (32 if which == 1 else 16) + 3] ^= 0x10
    want, wkey = oracle.mac_verify_batch(keys, which, desc, buf)
    st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
    ko = torch.zeros(len(desc), dtype=torch.int32, device="cuda")
    engine.mac_verify_dev(_dev(keys), which, _dev(desc.view(np.uint8).reshape(-1, 16)), _dev(buf), st, ko)
    torch.cuda.synchronize()
    st, ko = st.cpu().numpy(), ko.cpu().numpy().view(np.uint32)
    assert list(st) == list(want) and list(ko) == list(wkey)
    assert (st[pick[600:700]] == aead.PKT_REJECTED).all() and (st[pick[500:600]] == aead.PKT_REJECTED).all()
    assert (st[pick[:500]] == 0).all()


def test_mac_verify_key_table_regrow_on_a_busy_stream(engine):
    """the context's device copy of the MAC key states is wiped and regrown when a call brings
    more keys; two calls back to back on one non-blocking stream, the second with a larger key table, must
    not let the regrow (wipe before free) touch the states the first call's kernel is still reading.
    Both verdicts against the oracle, all scanned (RG_KEY_SCAN: every message reads every key)."""
    rng = np.random.default_rng(61)
    s = torch.cuda.Stream()
    runs = []
    for nk in (8, 64):
        keys = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
        desc, buf = _handshake_batch(rng, 4000, keys, 32, 1)
        desc["key_idx"][::2] = aead.KEY_SCAN
        for i in range(0, len(desc), 7):
            buf[int(desc["offset"][i]) + int(desc["len"][i]) - 29] ^= 0x10
        want, wkey = oracle.mac_verify_batch(keys, 1, desc, buf)
        with torch.cuda.stream(s):
            dk, dd, db = _dev(keys), _dev(desc.view(np.uint8).reshape(-1, 16)), _dev(buf)
            st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
            ko = torch.zeros(len(desc), dtype=torch.int32, device="cuda")
        s.synchronize()
        runs.append((dk, dd, db, st, ko, want, wkey))
    for dk, dd, db, st, ko, _, _ in runs:  # enqueued back to back, no synchronisation between them
        engine.mac_verify_dev(dk, 1, dd, db, st, ko, stream=s)
    s.synchronize()
    for _, _, _, st, ko, want, wkey in runs:
        assert list(st.cpu().numpy()) == list(want)
        assert list(ko.cpu().numpy().view(np.uint32)) == list(wkey)


@pytest.mark.parametrize("which", [1, 2])
def test_mac_verify_any_length(engine, which):
    """The batch MAC check at every message length 32..300 (covered part empty, not a multiple of 4, on
    and across 64-byte block edges) plus the descriptor checks (short, unaligned, out of range), against
    the oracle."""
    rng = np.random.default_rng(40 + which)
    key_len = 32 if which == 1 else 16
    tail = 32 if which == 1 else 16
    keys = rng.integers(0, 256, (5, key_len), dtype=np.uint8)
    sizes = np.arange(32, 301)
    off = np.concatenate([[0], np.cumsum((sizes + 15) // 16 * 16)[:-1]]).astype(np.uint64)
    buf = rng.integers(0, 256, int(off[-1]) + 320, dtype=np.uint8)
    desc = np.zeros(len(sizes) + 4, DESC_DTYPE)
    desc["offset"][: len(sizes)], desc["len"][: len(sizes)] = off, sizes
    desc["key_idx"][: len(sizes)] = rng.integers(0, len(keys), len(sizes))
    for i, L in enumerate(sizes):
        o, cov = int(off[i]), int(L) - tail
        if i % 3 == 2:
            continue  # left unsigned: rejected
        mac = oracle.blake2s(buf[o:o + cov].tobytes(), keys[desc["key_idx"][i]].tobytes(), 16)
        buf[o + cov:o + cov + 16] = np.frombuffer(mac, np.uint8)
    desc["key_idx"][: len(sizes)][rng.random(len(sizes)) < 0.3] = aead.KEY_SCAN
    end = len(buf)
    desc[len(sizes):] = [(0, 31, 0), (8, 148, 0), (end - 64, 148, 0), (0, 148, len(keys) + 3)]
    want, wkey = oracle.mac_verify_batch(keys, which, desc, buf)
    st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
    ko = torch.zeros(len(desc), dtype=torch.int32, device="cuda")
    engine.mac_verify_dev(_dev(keys), which, _dev(desc.view(np.uint8).reshape(-1, 16)), _dev(buf), st, ko)
    torch.cuda.synchronize()
    st, ko = st.cpu().numpy(), ko.cpu().numpy().view(np.uint32)
    assert list(st) == list(want) and list(ko) == list(wkey)
    assert (st[: len(sizes)][np.arange(len(sizes)) % 3 != 2] == 0).all()
    assert list(st[len(sizes):]) == [aead.PKT_INVALID, aead.PKT_UNALIGNED, aead.PKT_INVALID, aead.PKT_REJECTED]


def test_mac_verify_reference_snapshot(engine):
    """The reference's mac_snapshot (prim.rs:483-489) checked on the GPU in mac1 form: a message whose
    bytes [len-32, len-16) are blake2s_mac(key, first len-32 bytes) verifies under the snapshot's key,
    found by the peer scan, and is rejected under any other key."""
    m = load_golden("blake2s.json")["reference_mac_snapshot"]
    msg = bytes.fromhex(m["msg"]) + bytes.fromhex(m["mac"]) + bytes(16)  # the 16-byte mac2 slot follows
    buf = np.zeros(80, np.uint8)
    buf[:len(msg)] = np.frombuffer(msg, np.uint8)
    key = np.frombuffer(bytes.fromhex(m["key"]), np.uint8)
    keys = np.stack([key[::-1].copy(), key])  # row 1 is the snapshot's key
    desc = np.zeros(2, DESC_DTYPE)
    desc[0] = (0, len(msg), aead.KEY_SCAN)
    desc[1] = (0, len(msg), 0)
    st = torch.zeros(2, dtype=torch.uint8, device="cuda")
    ko = torch.zeros(2, dtype=torch.int32, device="cuda")
    engine.mac_verify_dev(_dev(keys), 1, _dev(desc.view(np.uint8).reshape(-1, 16)), _dev(buf), st, ko)
    torch.cuda.synchronize()
    assert list(st.cpu().numpy()) == [0, aead.PKT_REJECTED] and ko.cpu().numpy()[0] == 1


def test_mac1_on_reference_handshake_messages(engine):
    """The reference's recorded handshake initiation (148 B) and response (92 B) from its test
    `snapshot` (rustyguard-core/src/snapshots/rustyguard_core__tests__snapshot{,-2}.snap) pass
    HasMac::verify_mac1 (rustyguard-crypto/src/lib.rs:142-148) on the GPU under their receivers'
    mac1 keys (re-derived by tests/golden/make_handshake.py), are found by the wg-proxy peer scan
    among decoy keys, and fail with any bit of the covered bytes or of the mac1 field flipped."""
    g = load_golden("handshake_vectors.json")["handshake_macs"]
    msgs = [bytes.fromhex(g["initiation"]), bytes.fromhex(g["response"])]
    real = [bytes.fromhex(g["initiation_mac1_key"]), bytes.fromhex(g["response_mac1_key"])]
    rng = np.random.default_rng(8)
    keys = np.stack([rng.integers(0, 256, 32, dtype=np.uint8) for _ in range(6)])
    keys[2] = np.frombuffer(real[0], np.uint8)
    keys[5] = np.frombuffer(real[1], np.uint8)
    frames, desc_rows = [], []
    off = 0
    for mi, msg in enumerate(msgs):
        for variant in ("ok", "scan", "body", "mac"):
            b = bytearray(msg)
            if variant == "body":
                b[5] ^= 0x01  # sender index byte, covered by mac1
            if variant == "mac":
                b[len(b) - 32] ^= 0x80  # first byte of the mac1 field
            frames.append((off, bytes(b)))
            key = aead.KEY_SCAN if variant == "scan" else (2 if mi == 0 else 5)
            desc_rows.append((off, len(b), key))
            off += (len(b) + 15) // 16 * 16
    buf = np.zeros(off, np.uint8)
    for o, b in frames:
        buf[o:o + len(b)] = np.frombuffer(b, np.uint8)
    desc = np.array(desc_rows, DESC_DTYPE)
    st = torch.zeros(len(desc), dtype=torch.uint8, device="cuda")
    ko = torch.zeros(len(desc), dtype=torch.int32, device="cuda")
    engine.mac_verify_dev(_dev(keys), 1, _dev(desc.view(np.uint8).reshape(-1, 16)), _dev(buf), st, ko)
    torch.cuda.synchronize()
    R = aead.PKT_REJECTED
    assert list(st.cpu().numpy()) == [0, 0, R, R, 0, 0, R, R]
    k = ko.cpu().numpy()
    assert k[1] == 2 and k[5] == 5  # the scan names the receiver's key


def test_aead_with_aad_reference_handshake_snapshot(engine):
    """The per-message drop-in with a non-empty AAD against the reference's own bytes: resp.empty of
    its test `handshake` (rustyguard-crypto/src/snapshots/rustyguard_crypto__tests__handshake-3.snap)
    is ChaCha20-Poly1305(K, nonce 0, AAD = the transcript hash, empty payload); K and the hash are
    re-derived by tests/golden/make_handshake.py (which also reproduces the snapshot's transport
    keys).  Opening accepts it; a flipped AAD bit is a DecryptionError."""
    v = load_golden("handshake_vectors.json")["aead_with_aad"]
    key, nonce, aad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["aad"])
    empty = bytearray()
    tag = engine.chacha20poly1305_enc(key, nonce, aad, empty)
    assert tag.hex() == v["tag"]
    engine.chacha20poly1305_dec(key, nonce, aad, bytearray(), tag)
    bad = bytearray(aad)
    bad[31] ^= 1
    with pytest.raises(aead.DecryptionError):
        engine.chacha20poly1305_dec(key, nonce, bytes(bad), bytearray(), tag)


def test_aead_reference_initiation_fields(engine):
    """The per-message drop-in at lengths that are not multiples of 16, with a 32-byte AAD, against the
    reference's own bytes: encrypted_static (P = 32) and encrypted_timestamp (P = 12) of the recorded
    148-byte initiation (rustyguard-core/src/snapshots/rustyguard_core__tests__snapshot.snap; sealed by
    encrypt_handshake_init, rustyguard-crypto/src/lib.rs:287-344), keys and transcript hashes
    re-derived by tests/golden/make_handshake.py.  Seal reproduces them, open restores the plaintext,
    and a flipped AAD, ciphertext or tag bit is a DecryptionError that leaves the payload untouched."""
    g = load_golden("handshake_vectors.json")["initiation_aead"]
    for name in ("encrypted_static", "encrypted_timestamp"):
        v = g[name]
        key, nz, aad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["aad"])
        buf = bytearray.fromhex(v["plaintext"])
        tag = engine.chacha20poly1305_enc(key, nz, aad, buf)
        assert buf.hex() == v["ciphertext"] and tag.hex() == v["tag"], name
        engine.chacha20poly1305_dec(key, nz, aad, buf, tag)
        assert buf.hex() == v["plaintext"], name
        ct = bytearray.fromhex(v["ciphertext"])
        for a, c, t in ((bytes([aad[0] ^ 1]) + aad[1:], ct, tag), (aad, ct, bytes([tag[0] ^ 0x80]) + tag[1:])):
            body = bytearray(c)
            with pytest.raises(aead.DecryptionError):
                engine.chacha20poly1305_dec(key, nz, a, body, t)
            assert body == ct
        body = bytearray(ct)
        body[-1] ^= 1
        with pytest.raises(aead.DecryptionError):
            engine.chacha20poly1305_dec(key, nz, aad, body, tag)


def test_auto_routes_mixed_small_batches_to_flat():
    """Automatic kernel choice (rg_get_kernel / rg_last_kernel): the first IMIX batch runs the planned
    pipelined kernel, whose planner sees several size classes; the next ones run the flattened chunk
    stream until the 32nd call re-plans.  Every route gives the same bytes."""
    import torch

    from rustyguard_amd.device import DeviceBatch

    eng = aead.Engine(0)
    w = workloads.imix(5000)
    b = DeviceBatch(eng, w)
    outs, fams = [], []
    for _ in range(3):
        b.fill()
        b.seal()
        fams.append(eng.last_kernel())
        torch.cuda.synchronize()
        outs.append(b.buf.cpu().numpy().copy())
        b.open()
        fams.append(eng.last_kernel())
        torch.cuda.synchronize()
        assert (b.status.cpu().numpy()[: w.n] == 0).all()
    assert fams[0] == 0 and fams[1:] == [3] * 5  # the seal's planner already saw the mix
    assert all(np.array_equal(outs[0], o) for o in outs[1:])
    b.fill()
    ref = b.host_buf()
    oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, ref)
    assert np.array_equal(outs[0], ref)


def test_flat_first_launch_inside_graph_capture():
    """The flattened kernel's first launch on a context may happen inside a stream capture (the bench
    captures its step into a HIP graph): nothing may be allocated there."""
    import torch

    from rustyguard_amd.device import DeviceBatch

    eng = aead.Engine(0)
    eng.set_staged(3)
    w = workloads.imix(3000)
    b = DeviceBatch(eng, w)
    b.fill()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.seal()
    g.replay()
    torch.cuda.synchronize()
    got = b.host_buf()
    b.fill()
    ref = b.host_buf()
    oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, ref)
    assert np.array_equal(got, ref)


def test_per_message_key_wiped_from_device():
    """The per-message drop-in leaves no key in device memory (the reference zeroizes keys on drop,
    rustyguard-crypto/src/prim.rs:227-231): after enc, dec, a failed dec and the XChaCha pair, the
    device arena read back through the test hook holds none of the key bytes."""
    import ctypes

    from rustyguard_amd import _lib

    engine = aead.Engine(0, library=_lib.lib_test())  # the hook lives in the test library only
    key = bytes(range(0xA0, 0xC0))
    msg = bytearray(b"\x5a" * 200)
    tag = engine.chacha20poly1305_enc(key, aead.nonce(9), b"aad", msg)
    engine.chacha20poly1305_dec(key, aead.nonce(9), b"aad", msg, tag)
    with pytest.raises(aead.DecryptionError):
        engine.chacha20poly1305_dec(key, aead.nonce(9), b"aad", msg, bytes(16))
    xt = engine.xchacha20poly1305_enc(key, bytes(24), b"", msg)
    engine.xchacha20poly1305_dec(key, bytes(24), b"", msg, xt)
    out = (ctypes.c_uint8 * (1 << 16))()
    got = _lib.check(engine.library.rg_debug_read_arena(engine.handle, 0, out, len(out)), "rg_debug_read_arena",
                     engine.library)
    assert got > 0
    arena = bytes(out[:got])
    for w in range(0, 32, 8):  # no 8-byte run of the key anywhere
        assert key[w:w + 8] not in arena


def test_product_library_refuses_diagnostic_modes(engine):
    """a product context cannot be switched to a diagnostic seal mode (output that is
    not ciphertext with a success status) or given a stamp buffer; mode 0 stays accepted."""
    import torch

    for m in (1, 2, 3, 4, 7, 8):
        with pytest.raises(_lib.RgError):
            engine.set_debug_mode(m)
    engine.set_debug_mode(0)
    with pytest.raises(_lib.RgError):
        engine.set_debug_buffer(torch.zeros(64, dtype=torch.int64, device="cuda"))
    engine.set_debug_buffer(None)
