"""AntiReplay (rustyguard-utils/src/anti_replay.rs) -- host C implementation in librg_aead.

Runs without a GPU: the window is host-side state.
  * the reference's own unit tests (anti_replay.rs:66-108), transcribed;
  * its cargo-fuzz differential invariant (fuzz/fuzz_targets/anti_replay.rs:6-23)
    against a set-based model, on seeded random streams;
  * a restatement of anti_replay.rs in Python, compared operation by operation.
"""
import random

import pytest

from rustyguard_amd.aead import WINDOW_SIZE, AntiReplay


def check(r, n):
    if not r.would_accept(n):
        return False
    r.mark_seen(n)
    return True


def test_check_accept_and_mark():
    """anti_replay.rs:78-98"""
    replay = AntiReplay()
    for i in range(2048):
        assert check(replay, i * 2 + 1)
        assert not check(replay, i * 2 + 1)
        assert check(replay, i * 2)
        assert not check(replay, i * 2)
    for i in range(4096):
        assert not check(replay, i)
    assert check(replay, 4096 + 2048)
    assert not check(replay, 4097)
    assert check(replay, 65535)
    assert not check(replay, 10000)
    assert check(replay, 66000)


def test_unauthenticated_high_counter_does_not_lock_out():
    """anti_replay.rs:101-107 (RFC 6479 §3.4.3)"""
    replay = AntiReplay()
    assert check(replay, 5)
    assert replay.would_accept(1_000_000)
    assert check(replay, 6)


class PyAntiReplay:
    """Line-by-line restatement of rustyguard-utils/src/anti_replay.rs (usize = u64)."""

    BITMAP_LEN = 2048 // 64

    def __init__(self):
        self.bitmap = [0] * self.BITMAP_LEN
        self.last = 0

    def would_accept(self, n):
        if n > self.last:
            return True
        if self.last - n >= WINDOW_SIZE:
            return False
        return (self.bitmap[(n >> 6) & 31] >> (n & 63)) & 1 == 0

    def mark_seen(self, n):
        index, shift = n >> 6, n & 63
        if n > self.last:
            nxt = (self.last >> 6) + 1
            if index > nxt and index - nxt > self.BITMAP_LEN:
                self.bitmap = [0] * self.BITMAP_LEN
            else:
                for i in range(nxt, index + 1):
                    self.bitmap[i & 31] = 0
            self.last = n
        self.bitmap[index & 31] |= 1 << shift


def _streams(seed, count, length):
    rng = random.Random(seed)
    for _ in range(count):
        base = rng.choice([0, 1 << 20, (1 << 64) - 5000])
        spread = rng.choice([64, 3000, 10_000, 1 << 40])
        yield [min((1 << 64) - 1, base + rng.randrange(spread)) for _ in range(length)]


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_invariant_against_set_model(seed):
    """fuzz/fuzz_targets/anti_replay.rs: accepted == first sighting && not too old."""
    for data in _streams(seed, 40, 400):
        replay = AntiReplay()
        seen, last = set(), 0
        for d in data:
            allowed = d not in seen
            seen.add(d)
            too_old = d < last and last - d >= WINDOW_SIZE
            last = max(d, last)
            accepted = replay.would_accept(d)
            if accepted:
                replay.mark_seen(d)
            assert accepted == (allowed and not too_old), (d, last)


@pytest.mark.parametrize("seed", range(3))
def test_matches_python_restatement(seed):
    for data in _streams(100 + seed, 30, 500):
        a, b = AntiReplay(), PyAntiReplay()
        for d in data:
            assert a.would_accept(d) == b.would_accept(d)
            if b.would_accept(d) or random.Random(d).random() < 0.3:
                # also exercise mark_seen of accepted counters only, as callers must
                if b.would_accept(d):
                    a.mark_seen(d)
                    b.mark_seen(d)


def test_window_edges():
    r = AntiReplay()
    assert check(r, 10_000)
    assert check(r, 10_000 - (WINDOW_SIZE - 1))     # oldest still inside the window
    assert not check(r, 10_000 - WINDOW_SIZE)       # first one outside
    assert check(r, 10_001)
    assert not check(r, 10_001)
    # jump far ahead: the whole bitmap is cleared, old counters are too old
    assert check(r, 10_001 + 100_000)
    assert not check(r, 10_001)
    assert check(r, 10_001 + 100_000 - 1)
