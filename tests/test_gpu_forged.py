"""Forged frames in the benchmark geometries: every frame byte for byte against the oracle.

The reference's tamper contract (rustyguard-core/src/lib.rs:787-844: flip a byte, the packet is
rejected and nothing changes; rustyguard-crypto/src/prim.rs:190-201: DecryptionError leaves the
buffer as it came) is checked here in the layouts the benchmarks run, where the open kernels take
their fast store paths:

* config-2 shape (uniform 1504-byte payloads at a 1536-byte stride, >= 64 packets per wave): the
  pipelined kernel stores whole lines through its LDS ring, so other lanes write a lane's frame;
* tile batches of more than CUs x 512 uniform frames at a 1536-byte stride: the LDS-staged kernel's
  line-aligned (SH = 1) windows over two deal rounds, and config 4 (eight rounds: the grid-wide pool);
* IMIX (config 3) on the flattened chunk stream, where a lane's chunk range spans packets.

1 %, 10 % and 100 % of the frames are forged at a random byte of payload or tag; the GPU output
buffer and statuses must equal oracle.open_batch on the same tampered input, every byte.
"""
import numpy as np
import pytest

from oracle import oracle
from rustyguard_amd import workloads

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

FRACS = [0.01, 0.1, 1.0]


def _cus():
    return torch.cuda.get_device_properties(0).multi_processor_count


def _tamper(rng, od, buf, frac):
    """Flip one random bit at a random byte in [16, W) of a `frac` share of the frames (half of them
    in the tag); returns the forged indices."""
    n = len(od)
    k = max(1, int(round(frac * n)))
    pick = np.sort(rng.choice(n, size=k, replace=False))
    off = od["offset"][pick].astype(np.int64)
    W = od["len"][pick].astype(np.int64)
    in_tag = rng.random(k) < 0.5
    lo = np.where(in_tag, W - 16, 16)
    pos = off + lo + (rng.random(k) * (W - lo)).astype(np.int64)
    buf[pos] ^= (1 << rng.integers(0, 8, k)).astype(np.uint8)
    return pick


def _check(engine, w, frac, seed):
    from rustyguard_amd.device import DeviceBatch

    b = DeviceBatch(engine, w)
    b.fill()
    b.seal()
    torch.cuda.synchronize()
    assert (b.status[: w.n] == 0).all().item()
    od = w.open_desc()
    tampered = b.host_buf()
    pick = _tamper(np.random.default_rng(seed), od, tampered, frac)
    b.buf.copy_(torch.from_numpy(tampered))
    b.status.fill_(0xEE)
    b.open()
    torch.cuda.synchronize()
    want = tampered.copy()
    wst, wctr = oracle.open_batch(w.keys, od, want, nthreads=8)
    st = b.status[: w.n].cpu().numpy()
    assert (wst[pick] == oracle.DECRYPT_ERR).all()
    assert np.array_equal(st, wst)
    got = b.host_buf()
    if not np.array_equal(got, want):
        bad = np.nonzero(got != want)[0]
        frames = np.unique(np.searchsorted(od["offset"].astype(np.int64), bad, side="right") - 1)
        forged = np.isin(frames, pick)
        raise AssertionError(f"{len(bad)} bytes differ in {len(frames)} frames ({forged.sum()} forged), "
                             f"first byte {bad[0]}")
    ok = wst == 0
    assert np.array_equal(b.counters_out[: w.n].cpu().numpy().view(np.uint64)[ok], wctr[ok])
    del b
    torch.cuda.empty_cache()


@pytest.mark.parametrize("frac", FRACS)
@pytest.mark.parametrize("staged", [-1, 0])
def test_forged_cfg2_geometry(engine, staged, frac):
    """64 Ki x 1504-byte payloads at 1536-byte stride (config 2): the automatic choice and the pipelined
    kernel, both with LDS-ring line stores on open."""
    engine.set_staged(staged)
    try:
        _check(engine, workloads.build("cfg2"), frac, seed=11)
    finally:
        engine.set_staged(-1)


@pytest.mark.parametrize("frac", FRACS)
@pytest.mark.parametrize("plan", [2, 0])
def test_forged_tile_geometry(engine, plan, frac):
    """2 x CUs x 512 + 777 uniform frames at 1536-byte stride: the LDS-staged tile kernel with
    line-aligned windows over two deal rounds and a partial third (below the pool's eight), planner auto/off."""
    engine.set_staged(2)
    engine.set_plan(plan)
    try:
        _check(engine, workloads.uniform(2 * _cus() * 512 + 777, 1500, name="tiles"), frac, seed=12)
    finally:
        engine.set_staged(-1)
        engine.set_plan(2)


@pytest.mark.parametrize("frac", FRACS)
def test_forged_cfg4_geometry(engine, frac):
    """Config 4 (256 sessions x 4 Ki, per-packet key gather) under the automatic choice (tiles, eight deal
    rounds: the last one from the grid-wide pool)."""
    _check(engine, workloads.build("cfg4"), frac, seed=14)


@pytest.mark.parametrize("frac", FRACS)
@pytest.mark.parametrize("staged", [3, -1])
def test_forged_imix_flat(engine, staged, frac):
    """Config 3 (64 Ki IMIX, packed frames) on the flattened chunk stream and the automatic choice."""
    engine.set_staged(staged)
    try:
        _check(engine, workloads.build("cfg3"), frac, seed=13)
    finally:
        engine.set_staged(-1)
