"""Multi-process sharding on CPU (gloo, world_size 2).

The data path shards by plain index range with no collective (SURVEY.md
§8(e)); the only cross-rank traffic is the bench's timing barrier and
max-reduction.  Here two gloo ranks each seal their BASELINE-config-5 style
shard with the CPU oracle, gather the tags, and rank 0 checks that the union
is exactly the single-process result -- the same split bench.py --workload
cfg5 uses across GPUs.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

TOTAL = 2048


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rustyguard_amd import workloads

    w = workloads.shard(TOTAL, rank, world, L=176)
    # shard payload bytes are generated from the GLOBAL packet index
    w.data_seed = workloads.DATA_SEED
    tags = torch.from_numpy(_seal_tags_global(w))
    gathered = [torch.zeros_like(tags) for _ in range(world)]
    dist.all_gather(gathered, tags)
    # timing aggregation as in bench.py: MAX over ranks
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        out.put((torch.cat(gathered).numpy(), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def _seal_tags_global(w):
    """Seal a shard exactly as the whole batch would (global packet index in the payload generator)."""
    from oracle import oracle

    lo, _ = w.meta["shard"]
    buf = np.zeros(w.buf_bytes, np.uint8)
    for k in range(w.n):
        # payload of global packet lo + k
        from rustyguard_amd import workloads

        P = int(w.desc["len"][k])
        words = workloads.mix64(np.uint64(w.data_seed) + (np.uint64(lo + k) << np.uint64(16)) +
                                np.arange((P + 7) // 8, dtype=np.uint64))
        b = words.astype("<u8").view(np.uint8)[:P].copy()
        b[int(w.inner_len[k]):] = 0
        o = int(w.desc["offset"][k])
        buf[o + 16: o + 16 + P] = b
    oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, buf)
    off = w.desc["offset"].astype(np.int64)
    P = w.desc["len"].astype(np.int64)
    return np.stack([buf[o + 16 + p: o + 32 + p] for o, p in zip(off, P)])


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_seal_equals_single_process(world):
    from rustyguard_amd import workloads

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    tags, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = workloads.shard(TOTAL, 0, 1, L=176)
    want = _seal_tags_global(whole)
    assert tags.shape == want.shape
    assert np.array_equal(tags, want)
    assert tmax == float(world)
