#!/usr/bin/env python3
"""Phase times of the flattened kernel (rg_flat.hip, debug mode 3): per wave s_memtime at the end of
unit search, descriptor staging + chunk scan, phase A (one-time keys), phase C (chunk stream),
carries, phase F (tags) of its first sub-unit, and the wave's end.  Prints mean / max cycles per
phase over the waves, for seal and open."""
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
ap.add_argument("--workload", default="cfg3")
ap.add_argument("--plan", type=int, default=1)
ap.add_argument("--per-wave", action="store_true", help="also dump each wave's total with its unit's m and D")
args = ap.parse_args()
eng = Engine(0)
eng.set_staged(3)
eng.set_plan(args.plan)
w = workloads.build(args.workload)
b = DeviceBatch(eng, w)
b.fill()
dbg = torch.zeros(8 * 1024 * 2, dtype=torch.int64, device="cuda")
eng.set_debug_buffer(dbg)
names = ["search", "stage+scan", "phaseA", "phaseC", "carry", "phaseF", "end"]
res = {}
for op in ("seal", "open"):
    for rep in range(3):
        eng.set_debug_mode(0)
        if op == "open":
            b.seal()
        torch.cuda.synchronize()
        dbg.zero_()
        eng.set_debug_mode(3)
        b.seal() if op == "seal" else b.open()
        torch.cuda.synchronize()
        eng.set_debug_mode(0)
        if op == "seal":
            b.open()
        torch.cuda.synchronize()
    d = dbg.cpu().numpy().reshape(-1, 8).astype(np.int64)
    nwv = int((d[:1024, 0] != 0).sum())
    rt = d[nwv:2 * nwv, :2].astype(np.float64) / 100.0  # wall clock, us (s_memrealtime at 100 MHz)
    sub = d[nwv:2 * nwv, 2:8].copy()  # the cooperative search's steps (s_memtime), 0 = not reached
    sub_t0 = d[:nwv, 0:1]
    d = d[:nwv]
    d = d[d[:, 0] != 0]
    t0 = d[:, 0:1]
    rel = d - t0
    rel[d == 0] = -1
    out = {"waves": int(len(d))}
    prev = np.zeros(len(d), np.int64)
    for i, nm in enumerate(names, start=1):
        col = rel[:, i]
        ok = col >= 0
        seg = np.where(ok, col - prev, 0)
        out[nm] = {"mean_cyc": int(seg[ok].mean()) if ok.any() else None, "max_cyc": int(seg[ok].max()) if ok.any() else None}
        prev = np.where(ok, col, prev)
    out["wave_total"] = {"mean_cyc": int(rel[:, 7].mean()), "max_cyc": int(rel[:, 7].max())}
    out["slot_mean_from_start"] = [int(rel[:, i][rel[:, i] >= 0].mean()) if (rel[:, i] >= 0).any() else None
                                   for i in range(1, 8)]
    start = d[:, 0] - d[:, 0].min()
    out["start_spread_cyc"] = int(start.max())
    if len(rt) and rt[:, 0].min() > 0:
        r0 = rt[:, 0].min()
        out["wall_us_start_pct_0_50_100"] = [round(float(x), 2) for x in np.percentile(rt[:, 0] - r0, [0, 50, 100])]
        out["wall_us_end_pct_0_50_90_100"] = [round(float(x), 2) for x in np.percentile(rt[:, 1] - r0, [0, 50, 90, 100])]
        out["clock_ghz"] = round(float(rel[:, 7].sum() / ((rt[:, 1] - rt[:, 0]).sum() * 1e3)), 3)
    if (sub[:, 5] != 0).any():
        # search steps: coop entry (kernel arguments, setup), descriptor loads + LDS transpose, prefix and
        # wave total, first barrier, cut counts, second barrier
        okw = (sub != 0).all(axis=1) & (sub_t0[:, 0] != 0)
        st = np.concatenate([sub_t0[okw], sub[okw]], axis=1)
        dl = np.diff(st, axis=1)
        nm = ["entry", "desc_loads+transpose", "prefix", "barrier1", "cuts", "barrier2"]
        out["search_steps"] = {k: {"mean_cyc": int(dl[:, i].mean()), "max_cyc": int(dl[:, i].max())}
                               for i, k in enumerate(nm)}
    res[op] = out
    print(op, json.dumps(out), flush=True)
    if args.per_wave and op == "seal":
        # the unit each wave ran (wave id = unit id: one unit per wave), by the kernel's cut rule
        P = w.desc["len"].astype(np.int64)
        n = len(P)
        NU, G = len(d), 1024
        chunks = ((P + 15) // 16 + 3) // 4
        work = 1 + chunks
        rows = []
        raw = dbg.cpu().numpy().reshape(-1, 8).astype(np.int64)
        for u in range(NU):
            g = u * n // (G * NU)
            f0 = (g * G * NU + n - 1) // n
            f1 = min(NU, ((g + 1) * G * NU + n - 1) // n)
            kg, j, gb = f1 - f0, u - f0, g * G
            gn = min(G, n - gb)
            E = np.cumsum(work[gb:gb + gn])
            tot = int(E[-1])
            mid2 = E + np.concatenate([[0], E[:-1]])
            c0 = 0 if j == 0 else int((mid2 < 2 * (tot * j // kg)).sum())
            c1 = gn if j + 1 == kg else int((mid2 < 2 * (tot * (j + 1) // kg)).sum())
            m, D = c1 - c0, int(chunks[gb + c0:gb + c1].sum())
            r = raw[u]
            rows.append({"wave": u, "m": m, "D": D, "total": int(r[7] - r[0]) if r[0] else None})
        rows.sort(key=lambda x: -(x["total"] or 0))
        with open("gpurun_out/flat_per_wave.json", "w") as fo:
            json.dump(rows, fo)
        print("slowest", rows[:12], flush=True)
