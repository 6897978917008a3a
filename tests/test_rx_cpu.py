"""Receiver-index table (rg_rx_table_build / rg_rx_table_find): the host half of the device-side
session lookup that mirrors Sessions::decrypt_packet's `peers_by_session` map
(rustyguard-core/src/lib.rs:646-650).  Pure host code: no GPU needed."""
import numpy as np
import pytest

from rustyguard_amd import aead
from rustyguard_amd._lib import RgError


def test_roundtrip_and_misses():
    rng = np.random.default_rng(11)
    rec = np.unique(rng.integers(0, 2**32, 3000, dtype=np.uint64).astype(np.uint32))[:2000]
    idx = rng.permutation(len(rec)).astype(np.uint32)
    t = aead.rx_table(rec, idx)
    assert t.shape[0] == 4096
    for r, k in zip(rec[:500], idx[:500]):
        assert aead.rx_find(t, int(r)) == int(k)
    present = set(rec.tolist())
    misses = [r for r in rng.integers(0, 2**32, 500, dtype=np.uint64).tolist() if r not in present]
    assert all(aead.rx_find(t, int(r)) == -1 for r in misses)


def test_colliding_receivers_probe_linearly():
    # receivers that all hash to one slot of an 8-slot table
    cap = 8
    slot = lambda r: ((r * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - 3)  # noqa: E731
    same = [r for r in range(1, 20000) if slot(r) == 5][:4]
    t = aead.rx_table(same, [10, 11, 12, 13], cap=cap)
    assert [aead.rx_find(t, r) for r in same] == [10, 11, 12, 13]
    assert sorted(t[:, 1].tolist()).count(0xFFFFFFFF) == cap - 4


@pytest.mark.parametrize("cap", [6, 4])
def test_bad_capacity_rejected(cap):
    with pytest.raises(RgError):
        aead.rx_table([1, 2, 3], [0, 1, 2], cap=cap)


def test_duplicates_and_reserved_index_rejected():
    with pytest.raises(RgError):
        aead.rx_table([7, 7], [0, 1])
    with pytest.raises(RgError):
        aead.rx_table([7], [0xFFFFFFFF])


def test_oracle_receiver_lookup_order():
    """The oracle's restatement of Sessions::recv_message -> decrypt_packet order
    (rustyguard-core/src/lib.rs:612-650): alignment, message type and 16-byte framing before the
    session lookup; an unknown session (Rejected) before the missing-tag DecryptionError."""
    from oracle import oracle
    from rustyguard_amd.workloads import DESC_DTYPE
    keys = np.zeros((1, 32), np.uint8)
    buf = np.zeros(1024, np.uint8)
    cases = [(8, 48, 4, 77, 4), (64, 40, 4, 99, 2), (128, 48, 1, 99, 5), (192, 16, 4, 99, 3),
             (256, 16, 4, 77, 1), (320, 48, 4, 99, 3), (384, 48, 4, 77, 1)]
    desc = np.zeros(len(cases), DESC_DTYPE)
    for i, (o, w, t, r, _) in enumerate(cases):
        desc[i] = (o, w, 0)
        buf[o:o + 4] = np.frombuffer(np.uint32(t).tobytes(), np.uint8)
        buf[o + 4:o + 8] = np.frombuffer(np.uint32(r).tobytes(), np.uint8)
    st, ctr, key = oracle.open_batch_rx(keys, [77], desc, buf)
    assert list(st) == [c[4] for c in cases]
    assert list(key) == [0xFFFFFFFF] * 4 + [0, 0xFFFFFFFF, 0]
