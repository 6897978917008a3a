#!/usr/bin/env python3
"""Per-wave s_memtime stamps of the batched kernels: section shares of the LDS-staged tile kernel
(debug mode 3), whole-wave cycles / wall time / start-end spread of the pipelined kernel."""
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
ap.add_argument("--staged", type=int, default=-1)
ap.add_argument("--wg-per-cu", type=int, default=0)
ap.add_argument("--plan", type=int, default=-1)
ap.add_argument("--segments", type=int, default=0)
ap.add_argument("--lanes", type=int, default=0)
ap.add_argument("--world", type=int, default=1, help="config 5: rank 0's shard of an N-GPU strong split")
ap.add_argument("--mode", type=int, default=3, help="seal debug mode while stamping (pipelined kernel: 1/2/4/5/6 too)")
args = ap.parse_args()
eng = Engine(0)
eng.set_staged(args.staged)
if args.wg_per_cu:
    eng.set_wg_per_cu(args.wg_per_cu)
if args.plan >= 0:
    eng.set_plan(args.plan)
eng.set_segments(args.segments)
if args.lanes:
    eng.set_lanes_per_packet(args.lanes)
w = workloads.build(args.workload, 0, args.world) if args.world > 1 else workloads.build(args.workload)
b = DeviceBatch(eng, w)
b.fill()
dbg = torch.zeros(8 * 256 * 32, dtype=torch.int64, device="cuda")
eng.set_debug_buffer(dbg)
eng.set_debug_mode(args.mode)
out = {}
for op in ("seal", "open"):
    for rep in range(3):
        # every measured open gets a freshly sealed batch (a repeated open would
        # fail the tag check and time the restore path instead)
        if op == "open":
            eng.set_debug_mode(0)
            b.seal()
            torch.cuda.synchronize()
            eng.set_debug_mode(args.mode)
        dbg.zero_()
        b.seal() if op == "seal" else b.open()
        torch.cuda.synchronize()
        if op == "seal":
            eng.set_debug_mode(0)
            b.open()  # restore plaintext so each seal starts from the same state
            torch.cuda.synchronize()
            eng.set_debug_mode(args.mode)
    d = dbg.cpu().numpy().reshape(-1, 8)
    os.makedirs("gpurun_out", exist_ok=True)
    np.save(f"gpurun_out/stamps_raw_{args.workload}_{op}.npy", d)
    d = d[d[:, 6] == 1]
    if not len(d):  # no stamps for this op in this mode
        continue
    if eng.kernel_for(w.n) == 0:
        # pipelined lane kernel: whole-wave cycles and wall time, start / end spread
        tot = d[:, 0].astype(np.float64)
        rt = d[:, 7].astype(np.float64) / 100e6
        t0 = d[:, 4].min()
        out[op] = {"waves": int(len(d)), "cycles_per_wave_mean": float(tot.mean()),
                   "wave_us_pct_0_10_50_90_100": [round(float(v), 2) for v in np.percentile(rt * 1e6, [0, 10, 50, 90, 100])],
                   "shader_clock_ghz": round(float(tot.sum() / rt.sum()) / 1e9, 3),
                   "start_us_pct_0_50_90_100": [round(float(v), 2) for v in np.percentile((d[:, 4] - t0) / 100.0, [0, 50, 90, 100])],
                   "end_us_pct_0_50_90_100": [round(float(v), 2) for v in np.percentile((d[:, 4] + d[:, 7] - t0) / 100.0, [0, 50, 90, 100])]}
        continue
    names = ["setup", "store", "dma_issue", "dma_wait", "chunk", "tail"]
    tot = d[:, :6].sum(axis=1)
    rt = d[:, 7].astype(np.float64) / 100e6  # s_memrealtime ticks at 100 MHz
    q = np.percentile(rt * 1e6, [0, 10, 50, 90, 99, 100])
    out[op] = {"waves": int(len(d)), "cycles_per_wave_mean": float(tot.mean()),
               "wave_us_mean": round(float(rt.mean()) * 1e6, 2),
               "wave_us_pct_0_10_50_90_99_100": [round(float(x), 1) for x in q],
               "shader_clock_ghz": round(float(tot.sum() / rt.sum()) / 1e9, 3),
               "share": {n: round(float(d[:, k].sum() / tot.sum()), 4) for k, n in enumerate(names)}}
print(json.dumps(out, indent=1))
