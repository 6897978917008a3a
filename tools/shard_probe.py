#!/usr/bin/env python3
"""The per-GPU rate of config 5's strong split at each N of the driver's scaling run, on one GPU.

Rank 0's shard of `workloads.build("cfg5", 0, N)` (8 Mi / N packets of 1500 B) sealed then opened in place,
as bench.py's timed step does (a captured HIP graph, replayed; one event pair around `steps` replays).  On
a node every rank has a GPU of its own and nothing is exchanged, so N x this rate is what the N-GPU line
can reach; below it, the difference is the smaller batch per GPU (tile rounds, launch tail).
  usage: tools/shard_probe.py [N ...]   (default 1 2 4 8)
  RG_PROBE_SEGMENTS=K / RG_PROBE_STAGED=G / RG_PROBE_PLAN=P set the tile kernel's segments per packet, its
  window (family) and the planner before the probe (library defaults otherwise)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rustyguard_amd import workloads  # noqa: E402
from rustyguard_amd.aead import Engine  # noqa: E402
from rustyguard_amd.device import DeviceBatch  # noqa: E402


def probe(eng, world: int, steps: int = 10) -> dict:
    w = workloads.build("cfg5", 0, world)
    b = DeviceBatch(eng, w)
    b.fill()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            b.seal(stream=s)
            b.open(stream=s, counters_out=False)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.seal(stream=torch.cuda.current_stream())
        b.open(stream=torch.cuda.current_stream(), counters_out=False)
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(steps):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / steps
    out = {"world": world, "packets": w.n, "ms_per_step": round(ms, 4),
           "gib_s_per_gpu": round(2 * w.payload_bytes / (ms * 1e-3) / 2**30, 1)}
    del g, b
    torch.cuda.empty_cache()
    return out


def main():
    worlds = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
    eng = Engine(0)
    for env, fn in (("RG_PROBE_SEGMENTS", eng.set_segments), ("RG_PROBE_STAGED", eng.set_staged),
                    ("RG_PROBE_PLAN", eng.set_plan)):
        if os.environ.get(env):
            fn(int(os.environ[env]))
    for n in worlds:
        print(json.dumps(probe(eng, n)), flush=True)


if __name__ == "__main__":
    main()
