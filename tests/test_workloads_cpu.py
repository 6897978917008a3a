"""Synthetic workload generators (rustyguard_amd/workloads.py) -- CPU only.

They define the BASELINE configurations the GPU parity tests and bench.py
use, so their invariants are checked here, and their payload formula is
cross-checked between numpy, the C oracle and (in the GPU suite) the device
fill kernel.
"""
import numpy as np
import pytest

from oracle import oracle
from rustyguard_amd import workloads as wl


def test_mix64_numpy_matches_oracle():
    xs = np.random.default_rng(0).integers(0, 2**63, 200, dtype=np.uint64)
    xs[:3] = [0, 1, 2**64 - 1]
    got = wl.mix64(xs)
    for x, g in zip(xs, got):
        assert oracle.mix64(int(x)) == int(g)


def test_keys_formula():
    k = wl.make_keys(3)
    assert k.shape == (3, 32)
    for j in range(3):
        for t in range(4):
            v = oracle.mix64(wl.KEY_SEED + 4 * j + t)
            assert k[j, 8 * t: 8 * t + 8].tobytes() == v.to_bytes(8, "little")


def test_cfg2_shape():
    w = wl.build("cfg2")
    assert w.n == 65536
    assert (w.desc["len"] == 1504).all()  # L = 1500 padded to 16 (rustyguard-core/src/lib.rs:273-277)
    assert (w.desc["offset"] == np.arange(w.n, dtype=np.uint64) * 1536).all()
    assert (w.counters == np.arange(w.n)).all()
    assert (w.inner_len == 1500).all() and w.keys.shape == (1, 32)
    assert w.buf_bytes == 65536 * 1536


def test_cfg3_imix():
    w = wl.build("cfg3")
    assert w.n == 65536
    P = w.desc["len"].astype(np.int64)
    assert set(np.unique(P)) == {64, 576, 1504}
    frac = [(P == s).mean() for s in (64, 576, 1504)]
    assert abs(frac[0] - 7 / 12) < 0.01 and abs(frac[1] - 4 / 12) < 0.01 and abs(frac[2] - 1 / 12) < 0.01
    assert abs(P.mean() - 354.7) < 3
    off = w.desc["offset"].astype(np.int64)
    assert (off % 16 == 0).all()
    assert (off[1:] == off[:-1] + P[:-1] + 32).all()  # packed frames
    assert w.buf_bytes == int((P + 32).sum())


def test_cfg4_sessions():
    w = wl.build("cfg4")
    assert w.n == 256 * 4096 and w.keys.shape == (256, 32)
    sess = w.desc["key_idx"].astype(np.int64)
    assert (np.bincount(sess, minlength=256) == 4096).all()
    # per-session counters run 0..4095 in submission order (EncryptionKey::encrypt)
    order = np.argsort(sess, kind="stable")
    c = w.counters[order].reshape(256, 4096)
    assert (c == np.arange(4096)).all()
    # interleaved, not blocked by session
    assert (np.diff(sess[:1000]) != 0).mean() > 0.9


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_cfg5_shards_partition_the_batch(world):
    total = 1000
    seen = []
    for r in range(world):
        w = wl.shard(total, r, world)
        lo, hi = w.meta["shard"]
        assert w.n == hi - lo
        assert (w.counters == np.arange(lo, hi)).all()
        seen.extend(range(lo, hi))
    assert seen == list(range(total))


def test_oracle_synth_fill_formula():
    w = wl.imix(64)
    buf = np.zeros(w.buf_bytes, np.uint8)
    oracle.synth_fill(buf, w.desc, w.inner_len, w.data_seed)
    for i in range(w.n):
        o, P, L = int(w.desc["offset"][i]), int(w.desc["len"][i]), int(w.inner_len[i])
        words = wl.mix64(np.uint64(w.data_seed) + (np.uint64(i) << np.uint64(16)) + np.arange((P + 7) // 8,
                                                                                              dtype=np.uint64))
        want = words.astype("<u8").view(np.uint8)[:P].copy()
        want[L:] = 0  # zero padding up to P (rustyguard-tun/src/lib.rs:229-238)
        assert np.array_equal(buf[o + 16: o + 16 + P], want)
        assert not buf[o:o + 16].any() and not buf[o + 16 + P: o + 32 + P].any()


def test_open_desc_is_frame_length():
    w = wl.uniform(10, 100)
    od = w.open_desc()
    assert (od["len"] == w.desc["len"] + 32).all() and (od["offset"] == w.desc["offset"]).all()
