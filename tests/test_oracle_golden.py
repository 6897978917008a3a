"""Pin the CPU oracle before it is trusted as the checker.

Sources of truth:
  * the reference's own insta snapshots (rustyguard-crypto handshake-{4..7},
    rustyguard-core snapshot-3) -- bytes committed in tests/golden/;
  * RFC 8439 known answers (the algorithm graviola 0.2.0 implements);
  * OpenSSL EVP_chacha20_poly1305 multi-block vectors (generated here).
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import openssl_ref, oracle


def _seal(v):
    return oracle.aead_seal(bytes.fromhex(v["key"]), oracle.wg_nonce(v["counter"]), b"", bytes.fromhex(v["plaintext"]))


@pytest.mark.parametrize("v", load_golden("reference_snapshots.json")["transport_seals"], ids=lambda v: v["source"][:45])
def test_reference_transport_snapshots(v):
    # EncryptionKey::encrypt -> (ciphertext in place, tag) == insta snapshot
    ct, tag = _seal(v)
    assert ct.hex() == v["ciphertext"]
    assert tag.hex() == v["tag"]
    # DecryptionKey::decrypt round trip (rustyguard-crypto/src/lib.rs:548-549)
    pt = oracle.aead_open(bytes.fromhex(v["key"]), oracle.wg_nonce(v["counter"]), b"", ct, tag)
    assert pt == bytes.fromhex(v["plaintext"])


def test_reference_framed_packet_and_tamper():
    v = load_golden("reference_snapshots.json")["framed_packets"][0]
    keys = np.frombuffer(bytes.fromhex(v["key"]), np.uint8).reshape(1, 32)
    desc = np.zeros(1, oracle.DESC_DTYPE)
    pt = bytes.fromhex(v["plaintext"])
    desc["len"] = len(pt)
    buf = np.zeros(len(pt) + 32, np.uint8)
    buf[16:16 + len(pt)] = np.frombuffer(pt, np.uint8)
    oracle.seal_batch(keys, np.array([v["receiver"]], np.uint32), desc, np.array([v["counter"]], np.uint64), buf)
    assert buf.tobytes().hex() == v["frame"]
    # open the framed packet (Sessions::recv_message -> Message::Read)
    odesc = desc.copy()
    odesc["len"] = len(buf)
    b2 = buf.copy()
    st, ctr = oracle.open_batch(keys, odesc, b2)
    assert st[0] == oracle.OK and ctr[0] == v["counter"]
    assert b2[16:16 + len(pt)].tobytes() == pt
    # forged_packet_does_not_update_peer_endpoint: flip byte 47 -> DecryptionError, frame untouched
    b3 = buf.copy()
    b3[v["tamper_byte"]] ^= 1
    before = b3.copy()
    st, _ = oracle.open_batch(keys, odesc, b3)
    assert st[0] == oracle.DECRYPT_ERR
    assert np.array_equal(b3, before)


def test_rfc8439_known_answers():
    g = load_golden("rfc8439.json")
    for b in g["chacha20_block"]:
        out = oracle.chacha20_block(bytes.fromhex(b["key"]), b["counter"], bytes.fromhex(b["nonce"]))
        assert out.hex() == b["block"] and out.hex().startswith(b["block_prefix"])
    for p in g["poly1305"]:
        assert oracle.poly1305(bytes.fromhex(p["key"]), bytes.fromhex(p["message"])).hex() == p["tag"]
    for a in g["aead"]:
        ct, tag = oracle.aead_seal(bytes.fromhex(a["key"]), bytes.fromhex(a["nonce"]), bytes.fromhex(a["aad"]),
                                   bytes.fromhex(a["plaintext"]))
        assert tag.hex() == a["tag"] and ct.hex() == a["ciphertext"]


def test_openssl_vectors():
    g = load_golden("openssl_vectors.json")
    for v in g["wg_transport"]:
        ct, tag = _seal(v)
        assert (ct.hex(), tag.hex()) == (v["ciphertext"], v["tag"]), (len(v["plaintext"]) // 2, v["counter"])
    for v in g["general_aad"]:
        ct, tag = oracle.aead_seal(bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["aad"]),
                                   bytes.fromhex(v["plaintext"]))
        assert (ct.hex(), tag.hex()) == (v["ciphertext"], v["tag"])


@pytest.mark.skipif(not openssl_ref.available(), reason="libcrypto not present")
def test_oracle_vs_openssl_random():
    rng = np.random.default_rng(1234)
    for _ in range(200):
        ln = int(rng.integers(0, 2100))
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        ctr = int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2))
        pt = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        n = oracle.wg_nonce(ctr)
        assert oracle.aead_seal(key, n, b"", pt) == openssl_ref.seal(key, n, b"", pt)


def test_oracle_open_rejects_every_single_bit_flip_of_tag():
    key, pt = bytes(range(32)), b"x" * 64
    ct, tag = oracle.aead_seal(key, oracle.wg_nonce(7), b"", pt)
    for bit in range(128):
        t = bytearray(tag)
        t[bit // 8] ^= 1 << (bit % 8)
        assert oracle.aead_open(key, oracle.wg_nonce(7), b"", ct, bytes(t)) is None


def test_openssl_batch_baseline_matches_oracle():
    """The OpenSSL CPU baseline (oracle/rg_openssl_batch.c) computes the same frames as the oracle."""
    from rustyguard_amd import workloads as wl

    if not oracle.openssl_available():
        pytest.skip("libcrypto.so.3 not present")
    w = wl.imix(300)
    a = np.zeros(w.buf_bytes, np.uint8)
    oracle.synth_fill(a, w.desc, w.inner_len, w.data_seed)
    b = a.copy()
    oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, a)
    oracle.openssl_seal_batch(w.keys, w.receivers, w.desc, w.counters, b, nthreads=3)
    assert np.array_equal(a, b)
    od = w.open_desc()
    st = oracle.openssl_open_batch(w.keys, od, b, nthreads=2)
    assert (st == 0).all()
    a[int(od["offset"][7]) + 20] ^= 1
    st = oracle.openssl_open_batch(w.keys, od, a, nthreads=1)
    assert st[7] == oracle.DECRYPT_ERR and (np.delete(st, 7) == 0).all()


def test_xchacha_known_answer_and_vectors():
    """XChaCha20-Poly1305 (the cookie AEAD, rustyguard-crypto/src/prim.rs:202-224): the oracle's
    HChaCha20 reproduces draft-irtf-cfrg-xchacha-03 §2.2.1; the fixture seals open back and reject a
    flipped tag."""
    g = load_golden("xchacha.json")
    k = g["hchacha20_kat"]
    assert oracle.hchacha20(bytes.fromhex(k["key"]), bytes.fromhex(k["nonce"])).hex() == k["subkey"]
    for v in g["seals"]:
        key, nonce, aad = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["aad"])
        ct, tag = oracle.xaead_seal(key, nonce, aad, bytes.fromhex(v["plaintext"]))
        assert ct.hex() == v["ciphertext"] and tag.hex() == v["tag"]
        assert oracle.xaead_open(key, nonce, aad, ct, tag).hex() == v["plaintext"]
        bad = bytes([tag[0] ^ 1]) + tag[1:]
        assert oracle.xaead_open(key, nonce, aad, ct, bad) is None


def test_blake2s_reference_snapshots_and_vectors():
    """BLAKE2s behind HasMac (rustyguard-crypto/src/lib.rs:114-209): the oracle reproduces the
    reference's own blake2s_mac / blake2s_hash insta snapshots (prim.rs:477-489), RFC 7693
    Appendix B and hashlib-generated keyed MACs of handshake-message lengths."""
    g = load_golden("blake2s.json")
    m = g["reference_mac_snapshot"]
    assert oracle.blake2s(bytes.fromhex(m["msg"]), bytes.fromhex(m["key"]), 16).hex() == m["mac"]
    h = g["reference_hash_snapshot"]
    assert oracle.blake2s(bytes.fromhex(h["msg"])).hex() == h["hash"]
    assert oracle.blake2s(bytes.fromhex(g["rfc7693_abc"]["msg"])).hex() == g["rfc7693_abc"]["hash"]
    for v in g["keyed_macs"]:
        assert oracle.blake2s(bytes.fromhex(v["msg"]), bytes.fromhex(v["key"]), 16).hex() == v["mac"]


def test_message_type_dispatch():
    """Sessions::recv_message (rustyguard-core/src/lib.rs:619-628): the little-endian u32 type word
    selects handshake init / response / cookie (1, 2, 3: routed to the control plane, NOT_DATA) or
    data (4); every other value is Error::InvalidMessage."""
    import numpy as np

    keys = np.zeros((1, 32), np.uint8)
    types = [0, 1, 2, 3, 5, 0xFF, 0x104, 0xFFFFFFFF]
    buf = np.zeros(64 * len(types), np.uint8)
    desc = np.zeros(len(types), oracle.DESC_DTYPE)
    for k, t in enumerate(types):
        buf[64 * k:64 * k + 4] = np.frombuffer(np.uint32(t).tobytes(), np.uint8)
        desc[k] = (64 * k, 48, 0)
    st, _ = oracle.open_batch(keys, desc, buf)
    I, N = oracle.INVALID, oracle.NOT_DATA
    assert list(st) == [I, N, N, N, I, I, I, I]


def test_reference_handshake_vectors():
    """tests/golden/handshake_vectors.json (made by make_handshake.py from the reference's own
    snapshots): the oracle reproduces resp.empty (AEAD with a 32-byte AAD, handshake-3.snap) and
    BLAKE2s-128 reproduces the mac1 fields of the recorded initiation and response."""
    g = load_golden("handshake_vectors.json")
    v = g["aead_with_aad"]
    ct, tag = oracle.aead_seal(bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["aad"]), b"")
    assert ct == b"" and tag.hex() == v["tag"]
    m = g["handshake_macs"]
    init, resp = bytes.fromhex(m["initiation"]), bytes.fromhex(m["response"])
    assert oracle.blake2s(init[:116], bytes.fromhex(m["initiation_mac1_key"]), 16) == init[116:132]
    assert oracle.blake2s(resp[:60], bytes.fromhex(m["response_mac1_key"]), 16) == resp[60:76]


def test_reference_initiation_aead_fields():
    """The recorded initiation's encrypted_static (P = 32) and encrypted_timestamp (P = 12), both with
    AAD = the transcript hash (encrypt_handshake_init, rustyguard-crypto/src/lib.rs:287-344), re-derived
    by make_handshake.py: the oracle seals each to the snapshot's bytes and opens them back."""
    g = load_golden("handshake_vectors.json")
    init = bytes.fromhex(g["handshake_macs"]["initiation"])
    fields = g["initiation_aead"]
    for name, (lo, hi) in (("encrypted_static", (40, 88)), ("encrypted_timestamp", (88, 116))):
        v = fields[name]
        key, nz, aad, pt = (bytes.fromhex(v[k]) for k in ("key", "nonce", "aad", "plaintext"))
        ct, tag = oracle.aead_seal(key, nz, aad, pt)
        assert ct + tag == init[lo:hi] and ct.hex() == v["ciphertext"] and tag.hex() == v["tag"], name
        assert oracle.aead_open(key, nz, aad, ct, tag) == pt
        bad = bytearray(aad)
        bad[0] ^= 1
        assert oracle.aead_open(key, nz, bytes(bad), ct, tag) is None
