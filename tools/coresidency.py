#!/usr/bin/env python3
"""Round 4: are two waves of the pipelined kernel really resident on one SIMD at once?

Runs config 2's seal with per-wave stamps (debug mode 3) on a library built with
`tools/build_variant.sh lb2 -DRG_PIPE_LB2` (__launch_bounds__(256, 2) + an HW_ID / XCC_ID word in
each wave's stamp record), groups the waves by the SIMD they ran on (XCC, SE, SH, CU, SIMD from
HW_ID) and measures how long two waves of one SIMD were alive together.  Also prints the
occupancy the library computed (hipOccupancyMaxActiveBlocksPerMultiprocessor, via the
automatic workgroup count) and the compute-only (mode 1) numbers beside it."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustyguard_amd import workloads  # noqa: E402
from rustyguard_amd.aead import Engine  # noqa: E402
from rustyguard_amd.device import DeviceBatch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="cfg2")
ap.add_argument("--lanes", type=int, default=2)
ap.add_argument("--wg-per-cu", type=int, default=2)
ap.add_argument("--mode", type=int, default=3)
ap.add_argument("--tag", default="")
args = ap.parse_args()

eng = Engine(0)
eng.set_staged(0)
eng.set_plan(0)
eng.set_lanes_per_packet(args.lanes)
eng.set_wg_per_cu(args.wg_per_cu)
w = workloads.build(args.workload)
b = DeviceBatch(eng, w)
b.fill()
dbg = torch.zeros(8 * 256 * 64, dtype=torch.int64, device="cuda")
eng.set_debug_buffer(dbg)
res = []
for rep in range(3):
    eng.set_debug_mode(args.mode)
    dbg.zero_()
    b.seal()
    torch.cuda.synchronize()
    eng.set_debug_mode(0)
    b.open()
    torch.cuda.synchronize()
    d = dbg.cpu().numpy().reshape(-1, 8)
    d = d[d[:, 6] == 1]
    hw = (d[:, 3] & 0xFFFFFFFF).astype(np.int64)
    xcc = (d[:, 3] >> 32) & 0xF
    simd_key = (xcc << 16) | (hw & 0xFF30)  # SE/SH/CU bits 8-15, SIMD bits 4-5
    start = d[:, 4].astype(np.float64) / 100.0  # s_memrealtime: 100 MHz -> us
    end = start + d[:, 7].astype(np.float64) / 100.0
    t0 = start.min()
    keys, counts = np.unique(simd_key, return_counts=True)
    overlap, life = [], []
    for k in keys[counts == 2]:
        i, j = np.nonzero(simd_key == k)[0]
        ov = max(0.0, min(end[i], end[j]) - max(start[i], start[j]))
        overlap.append(ov / max(end[i] - start[i], end[j] - start[j]))
        life.append(max(end[i], end[j]) - min(start[i], start[j]))
    res.append({
        "waves": int(len(d)), "simds_seen": int(len(keys)),
        "waves_per_simd_hist": {int(c): int((counts == c).sum()) for c in np.unique(counts)},
        "distinct_wave_ids_per_simd_max": int(max(len(np.unique(hw[simd_key == k] & 0xF)) for k in keys)),
        "pair_overlap_frac_pct_0_10_50_90_100": [round(float(v), 3) for v in np.percentile(overlap, [0, 10, 50, 90, 100])]
        if overlap else None,
        "wave_us_median": round(float(np.median(end - start)), 2),
        "last_wave_end_us": round(float(end.max() - t0), 2),
        "start_spread_us": round(float(np.percentile(start - t0, 100)), 2),
        "cycles_per_wave_mean": float(d[:, 0].mean()),
        "prologue_cycles_mean_max": [float(d[:, 5].mean()), float(d[:, 5].max())],  # entry -> first unit's start
        "clock_ghz": round(float(d[:, 0].sum() / (d[:, 7].sum() / 100e6)) / 1e9, 3),
    })
out = {"workload": args.workload, "lanes": args.lanes, "wg_per_cu": args.wg_per_cu, "mode": args.mode,
       "lib": os.environ.get("RG_AEAD_LIB", "in-tree"), "reps": res}
os.makedirs("gpurun_out", exist_ok=True)
print(json.dumps(out))
