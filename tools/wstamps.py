#!/usr/bin/env python3
"""Step cycles of the pipelined kernel's line-store loop by unrolled position (t % 3), from a library
built with -DRG_PIPE_WSTAMP (tools/build_variant.sh wst -DRG_PIPE_WSTAMP; RG_AEAD_LIB points at it).
Per wave: slots 1-3 of its stamp record hold the summed cycles of the steps t = 3k, 3k+1, 3k+2, and
the same slots of a second block of records (seal) the cycles spent in an explicit vmcnt(16) wait before
the step's XOR."""
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
ap.add_argument("--mode", type=int, default=3)
args = ap.parse_args()
eng = Engine(0)
eng.set_plan(0)
w = workloads.build(args.workload)
b = DeviceBatch(eng, w)
b.fill()
dbg = torch.zeros(8 * 256 * 32, dtype=torch.int64, device="cuda")
eng.set_debug_buffer(dbg)
out = {}
P = int(w.desc["len"][0])
F = P // 64
steps = {k: sum(1 for t in range(2, F) if t % 3 == k) for k in range(3)}
for op in ("seal", "open"):
    for rep in range(3):
        eng.set_debug_mode(0)
        if op == "open":
            b.seal()
        torch.cuda.synchronize()
        eng.set_debug_mode(args.mode if op == "seal" else 3)
        dbg.zero_()
        b.seal() if op == "seal" else b.open()
        torch.cuda.synchronize()
        eng.set_debug_mode(0)
        if op == "seal":
            b.open()
        torch.cuda.synchronize()
    raw = dbg.cpu().numpy().reshape(-1, 8)
    nw = int((raw[:, 6] == 1).sum())
    d, ext = raw[:nw], raw[nw:2 * nw]
    if not nw:
        continue
    units = (w.n + len(d) * 64 - 1) // (len(d) * 64)  # packets per lane
    o = {"waves": int(len(d)), "cycles_per_wave": round(float(d[:, 0].mean()), 1),
         "flush_steps_per_position": steps}
    for k in range(3):
        o[f"t%3=={k}_cycles_per_step"] = round(float(d[:, 1 + k].mean()) / max(1, steps[k] * units), 1)
        o[f"t%3=={k}_vmcnt16_wait_per_step"] = round(float(ext[:, k].mean()) / max(1, steps[k] * units), 1)
    o["flush_share_of_wave"] = round(float(d[:, 1:4].sum(axis=1).mean() / d[:, 0].mean()), 4)
    out[op] = o
print(json.dumps(out, indent=1))
