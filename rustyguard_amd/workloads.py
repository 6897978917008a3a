"""Deterministic synthetic workloads for the BASELINE.json configurations.

SURVEY.md §8(d) conventions: L = inner plaintext length, P = roundup16(L) is
the AEAD payload (padding rule of rustyguard-core/src/lib.rs:273-277 and
rustyguard-tun/src/lib.rs:229-238), W = 16 + P + 16 the wire frame.
"1500-B packet" means L = 1500 -> P = 1504 -> W = 1536.

Generators (all from the stateless SplitMix64 finaliser ``mix64``):
  keys       key j = le64(mix64(KEY_SEED + 4 j + t)), t = 0..3
  receivers  session j's peer index = low 32 bits of mix64(RECV_SEED + j)
  payload    packet i inner bytes = le64(mix64(DATA_SEED + (i << 16) + word)),
             zero padding up to P (device fill: rg_synth_fill_dev); a cfg5 shard
             [lo, hi) uses seed DATA_SEED + (lo << 16), i.e. the global indices
  IMIX       class of packet i = mix64(IMIX_SEED + i) % 12:
             0-6 -> L=64, 7-10 -> L=576, 11 -> L=1500  (7:4:1 in expectation)
  sessions   cfg4: perm = stable argsort(mix64(SESS_SEED + i)); packet i
             belongs to session perm[i] % 256 (exactly 4096 each) and takes
             that session's next counter (EncryptionKey, prim.rs:386-394)
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

KEY_SEED = 0x7275737479  # "rusty"
RECV_SEED = 0x726563760000
DATA_SEED = 0x64617461
IMIX_SEED = 0x696D6978
SESS_SEED = 0x73657373

DESC_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("key_idx", "<u4")])
assert DESC_DTYPE.itemsize == 16

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def mix64(x) -> np.ndarray:
    """Vectorised SplitMix64 finaliser (wrapping uint64 arithmetic)."""
    z = np.asarray(x, dtype=np.uint64) + _G
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def make_keys(nkeys: int) -> np.ndarray:
    idx = np.arange(nkeys * 4, dtype=np.uint64) + np.uint64(KEY_SEED)
    return mix64(idx).astype("<u8").view(np.uint8).reshape(nkeys, 32).copy()


def make_receivers(nkeys: int) -> np.ndarray:
    return (mix64(np.arange(nkeys, dtype=np.uint64) + np.uint64(RECV_SEED)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def pad16(L):
    return (np.asarray(L, dtype=np.int64) + 15) // 16 * 16


@dataclass
class Workload:
    name: str
    desc: np.ndarray          # DESC_DTYPE, seal view: len = P
    counters: np.ndarray      # u64
    inner_len: np.ndarray     # u32, L per packet
    keys: np.ndarray          # u8 [nkeys, 32]
    receivers: np.ndarray     # u32 [nkeys]
    buf_bytes: int
    data_seed: int = DATA_SEED
    meta: dict = field(default_factory=dict)

    @property
    def n(self) -> int:
        return len(self.desc)

    @property
    def payload_bytes(self) -> int:
        return int(self.desc["len"].astype(np.int64).sum())

    @property
    def wire_bytes(self) -> int:
        return self.payload_bytes + 32 * self.n

    def open_desc(self) -> np.ndarray:
        """The same frames described for open (len = W = P + 32)."""
        d = self.desc.copy()
        d["len"] = d["len"] + 32
        return d


def _packed(P: np.ndarray, key_idx: np.ndarray, stride: int | None = None) -> tuple[np.ndarray, int]:
    n = len(P)
    desc = np.zeros(n, DESC_DTYPE)
    W = P.astype(np.uint64) + np.uint64(32)
    if stride is not None:
        desc["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(stride)
        total = n * stride
    else:
        off = np.zeros(n, np.uint64)
        if n > 1:
            off[1:] = np.cumsum(W[:-1], dtype=np.uint64)
        desc["offset"] = off
        total = int(W.sum())
    desc["len"] = P.astype(np.uint32)
    desc["key_idx"] = key_idx.astype(np.uint32)
    return desc, total


def uniform(n: int, L: int = 1500, name: str = "uniform", counter_base: int = 0, index_base: int = 0) -> Workload:
    """n packets of inner length L, one session key, sequential counters."""
    P = np.full(n, int(pad16(L)), np.int64)
    desc, total = _packed(P, np.zeros(n, np.uint32), stride=int(P[0]) + 32 if n else 0)
    ctr = np.arange(n, dtype=np.uint64) + np.uint64(counter_base)
    w = Workload(name, desc, ctr, np.full(n, L, np.uint32), make_keys(1), make_receivers(1), total,
                 meta={"L": L, "P": int(pad16(L)), "W": int(pad16(L)) + 32, "sessions": 1, "index_base": index_base})
    return w


def imix(n: int = 65536, name: str = "cfg3") -> Workload:
    cls = (mix64(np.arange(n, dtype=np.uint64) + np.uint64(IMIX_SEED)) % np.uint64(12)).astype(np.int64)
    L = np.where(cls < 7, 64, np.where(cls < 11, 576, 1500)).astype(np.int64)
    P = pad16(L)
    desc, total = _packed(P, np.zeros(n, np.uint32))
    ctr = np.arange(n, dtype=np.uint64)
    return Workload(name, desc, ctr, L.astype(np.uint32), make_keys(1), make_receivers(1), total,
                    meta={"mix": "64/576/1500 @ 7:4:1 (hash-assigned)", "mean_P": float(P.mean()), "sessions": 1})


def multi_session(sessions: int = 256, per_session: int = 4096, L: int = 1500, name: str = "cfg4") -> Workload:
    n = sessions * per_session
    order = np.argsort(mix64(np.arange(n, dtype=np.uint64) + np.uint64(SESS_SEED)), kind="stable")
    sess = (order % sessions).astype(np.int64)
    # running per-session counter in submission order
    ctr = np.zeros(n, np.uint64)
    srt = np.argsort(sess, kind="stable")
    ranks = np.empty(n, np.int64)
    ranks[srt] = np.arange(n) - np.repeat(np.arange(sessions) * per_session, per_session)
    ctr[:] = ranks.astype(np.uint64)
    P = np.full(n, int(pad16(L)), np.int64)
    desc, total = _packed(P, sess.astype(np.uint32), stride=int(P[0]) + 32)
    return Workload(name, desc, ctr, np.full(n, L, np.uint32), make_keys(sessions), make_receivers(sessions), total,
                    meta={"L": L, "P": int(pad16(L)), "W": int(pad16(L)) + 32, "sessions": sessions})


def shard(total: int, rank: int, world: int, L: int = 1500, name: str = "cfg5") -> Workload:
    """cfg5: `total` packets of one session split evenly across `world` GPUs by plain index range."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    w = uniform(hi - lo, L, name=name, counter_base=lo, index_base=lo)
    # payload of local packet k = that of global packet lo + k: the generator keys on
    # seed + (index << 16), so the shard's seed is advanced by lo << 16 (wrapping)
    w.data_seed = (DATA_SEED + (lo << 16)) % (1 << 64)
    w.meta.update({"total": total, "rank": rank, "world": world, "shard": [lo, hi]})
    return w


CONFIGS = {
    "cfg1": "Single 1500-B transport-data packet seal+open (CPU plumbing)",
    "cfg2": "64 Ki packets x 1500 B, one session key, seal then open, 1 MI355X",
    "cfg3": "64 Ki packets IMIX 64/576/1500, one session key, 1 MI355X",
    "cfg4": "256 sessions x 4 Ki packets, 1500 B, per-packet key gather, 1 MI355X",
    "cfg5": "8 Mi packets x 1500 B, one key, split evenly across GPUs (no collective)",
}


def build(name: str, rank: int = 0, world: int = 1) -> Workload:
    if name == "cfg1":
        return uniform(1, 1500, name="cfg1")
    if name == "cfg2":
        return uniform(65536, 1500, name="cfg2")
    if name == "cfg3":
        return imix(65536)
    if name == "cfg4":
        return multi_session(256, 4096, 1500)
    if name == "cfg5":
        return shard(8 * 1024 * 1024, rank, world)
    raise KeyError(name)
