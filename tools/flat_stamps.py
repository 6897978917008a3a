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
dbg = torch.zeros(8 * 1024 * 3, dtype=torch.int64, device="cuda")
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
        # search steps: entry (kernel arguments, setup), length loads + LDS transpose, prefix (+ the shared
        # prefix rows), the barrier, this wave's two cut points, and a sixth slot that round 5's single-barrier
        # search leaves empty (round 4 had a second barrier there; the round-5 deal record
        # profiles/r5_cfg3_deal_ab.txt labels the same six slots length loads + classes, class ranks,
        # barrier, sorted positions + unit lists, barrier).
        okw = (sub != 0).all(axis=1) & (sub_t0[:, 0] != 0)
        st = np.concatenate([sub_t0[okw], sub[okw]], axis=1)
        dl = np.diff(st, axis=1)
        nm = ["entry", "len_loads+transpose", "prefix", "barrier", "cut_points", "(none)"]
        out["search_steps"] = {k: {"mean_cyc": int(dl[:, i].mean()), "max_cyc": int(dl[:, i].max())}
                               for i, k in enumerate(nm)}
    res[op] = out
    print(op, json.dumps(out), flush=True)
    if args.per_wave and op == "seal":
        # each wave's first sub-unit as the kernel recorded it (third block of rows: packets m, chunks D,
        # steps S; XCC_ID / HW_ID), beside its phase cycles -- what the slowest waves have in common
        raw = dbg.cpu().numpy().reshape(-1, 8).astype(np.int64)
        info = raw[2 * nwv:3 * nwv]
        rows = []
        for u in range(nwv):
            r, ui = raw[u], int(info[u, 0])
            if not r[0]:
                continue
            hw = int(info[u, 1])
            rows.append({"wave": u, "m": ui & 0xFFFF, "D": (ui >> 16) & 0xFFFFFF, "S": ui >> 40,
                         "xcc": (hw >> 32) & 0xF, "total": int(r[7] - r[0]),
                         "phases": [int(r[i] - r[i - 1]) if r[i] and r[i - 1] else None for i in range(1, 8)]})
        rows.sort(key=lambda x: -x["total"])
        with open("gpurun_out/flat_per_wave.json", "w") as fo:
            json.dump(rows, fo)
        tot = np.array([x["total"] for x in rows], np.float64)
        for key in ("m", "S", "xcc"):
            v = np.array([x[key] for x in rows])
            out_k = {int(k): [int((v == k).sum()), int(tot[v == k].mean())] for k in np.unique(v)}
            print("by", key, "(count, mean cycles)", json.dumps(out_k), flush=True)
        print("slowest", rows[:8], flush=True)
