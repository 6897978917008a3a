#!/usr/bin/env python3
"""where the per-GPU rate goes between config 5's 8 Mi-packet batch (N = 1) and rank 0's
1 Mi shard (N = 8): 1642 -> 1488 GiB/s in round 5 (profiles/r5_shard_probe.jsonl).

Needs the diagnostic build (RG_AEAD_LIB=tools/build/librg_diag.so): the tile kernel's stamp rows (debug mode
3) carry each wave's section cycles and, since round 6, its wall-clock start and end (s_memrealtime, 100 MHz)
and the number of tiles it took.  Per shard size and op (seal, open), median over reps of:
  event_us     the launch, one HIP event pair on its stream (stamped run)
  plain_us     the same launch without stamps (debug mode 0), for the stamps' own cost
  span_us      last wave end - first wave start
  overhead_us  event - span: dispatch before the first wave and completion after the last (the L2 write-back)
  start_us     last wave start - first wave start (the dispatch ramp)
  tail_us      last wave end - mean wave end (the spread the launch waits for)
  wave_us      mean wave life; tiles per wave (min / mean / max); setup cycles per wave (mean)
  per_tile_us  mean wave life / mean tiles: the rate a wave works at once running
  clock_ghz    the waves' cycles (the stamps' section sums) over their wall time: the clock they ran at
  pool_items   mean grid-pool items per wave (an item is a tile or a segment of one, so items differ in size)
  usage: RG_AEAD_LIB=tools/build/librg_diag.so tools/shard_attrib.py [N ...]   (default 1 8)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustyguard_amd import workloads  # noqa: E402
from rustyguard_amd.aead import Engine  # noqa: E402
from rustyguard_amd.device import DeviceBatch  # noqa: E402


def timed(fn, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


def main():
    worlds = [int(x) for x in sys.argv[1:]] or [1, 8]
    eng = Engine(0)
    s = torch.cuda.current_stream()
    dbg = torch.zeros(8 * 256 * 32, dtype=torch.int64, device="cuda")
    eng.set_debug_buffer(dbg)
    for world in worlds:
        w = workloads.build("cfg5", 0, world)
        b = DeviceBatch(eng, w)
        b.fill()
        torch.cuda.synchronize()
        for _ in range(2):
            b.seal(stream=s)
            b.open(stream=s, counters_out=False)
        torch.cuda.synchronize()
        res = {"world": world, "packets": w.n}
        for op in ("seal", "open"):
            rows = []
            for rep in range(5):
                if op == "open":  # a freshly sealed batch for every measured open
                    eng.set_debug_mode(0)
                    b.seal(stream=s)
                fn = (lambda: b.seal(stream=s)) if op == "seal" else (lambda: b.open(stream=s, counters_out=False))
                eng.set_debug_mode(0)
                plain = timed(fn, s)
                if op == "open":
                    b.seal(stream=s)
                else:
                    b.open(stream=s, counters_out=False)  # back to plaintext: every seal starts alike
                dbg.zero_()
                eng.set_debug_mode(3)
                ev = timed(fn, s)
                eng.set_debug_mode(0)
                if op == "seal":
                    b.open(stream=s, counters_out=False)
                torch.cuda.synchronize()
                d = dbg.cpu().numpy().reshape(-1, 8)
                nw = int((d[:, 6] == 1).sum())
                a = d[:nw]
                t = d[nw:2 * nw]  # rows after the first block: start, end, tiles, hw id
                ok = t[:, 1] > 0
                a, t = a[ok], t[ok]
                st, en = t[:, 0].astype(np.float64), t[:, 1].astype(np.float64)
                span = (en.max() - st.min()) / 100.0
                cyc = a[:, 0:6].sum(axis=1).astype(np.float64)          # the wave's cycles, section by section
                wall = a[:, 7].astype(np.float64) * 10.0                  # ns (100 MHz ticks)
                rows.append({"clock_ghz": float(np.median(cyc / wall)), "pool_items": float(t[:, 6].mean())})
                rows[-1].update({"event_us": ev, "plain_us": plain, "span_us": span, "overhead_us": ev - span,
                                 "start_us": (st.max() - st.min()) / 100.0,
                             "tail_us": (en.max() - en.mean()) / 100.0,
                             "wave_us": float((en - st).mean()) / 100.0,
                             "tiles_min": int(t[:, 2].min()), "tiles_mean": float(t[:, 2].mean()),
                             "tiles_max": int(t[:, 2].max()), "setup_cycles": float(a[:, 0].mean()),
                             "waves": int(len(a))})
            med = {k: float(np.median([r[k] for r in rows])) for k in rows[0]}
            med["per_tile_us"] = med["wave_us"] / max(med["tiles_mean"], 1e-9)
            res[op] = {k: round(v, 3) for k, v in med.items()}
        print(json.dumps(res), flush=True)
        del b
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
