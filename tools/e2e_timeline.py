#!/usr/bin/env python3
"""Round 4: the host path's timeline from a rocprofv3 --kernel-trace --memory-copy-trace run of
tools/e2e_probe.py (tools/recipes.sh r4_e2etrace): for the last seal call, every H2D copy, kernel and D2H
blit in start order, relative to the call's first copy, with the gaps on each engine.
   usage: tools/e2e_timeline.py DIR [KERNEL_SUBSTRING]"""
import csv
import glob
import sys

d = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "seal"
ev = []
for r in csv.DictReader(open(glob.glob(f"{d}/*memory_copy_trace.csv")[0])):
    ev.append(("H2D" if "HOST_TO_DEVICE" in r["Direction"] else "D2H", int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for r in csv.DictReader(open(glob.glob(f"{d}/*kernel_trace.csv")[0])):
    n = r["Kernel_Name"]
    tag = "blit" if "rocclr_copyBuffer" in n else ("kern" if "rg::" in n else None)
    if tag:
        ev.append((tag if tag == "blit" else n.split("(")[0].split()[-1], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
ev.sort(key=lambda e: e[1])
# the last call of the named kernel family: its kernels and the copies between the first H2D before them
# and the last blit after them
ks = [i for i, e in enumerate(ev) if kname in e[0]]
last = ks[-1]
first = last
while first > 0 and (kname in ev[first - 1][0] or ev[first - 1][0] in ("H2D", "blit", "D2H")) and ev[last][1] - ev[first - 1][1] < 5e6:
    first -= 1
    if kname not in ev[first][0] and ev[first][0] not in ("H2D", "blit", "D2H"):
        break
# keep only events after the previous call's last kernel of another family
win = ev[first:]
end = max(e[2] for e in win if e[1] <= ev[last][2] + 2e6)
win = [e for e in win if e[1] <= end]
t0 = min(e[1] for e in win)
prev = {}
print(f"{'what':28s} {'start':>8s} {'end':>8s} {'us':>7s} {'gap':>7s}")
for n, s, e in win:
    lane = "H2D" if n == "H2D" else ("D2H" if n in ("blit", "D2H") else "kern")
    gap = (s - prev[lane]) / 1e3 if lane in prev else 0.0
    prev[lane] = e
    print(f"{n[:28]:28s} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {gap:7.1f}")
print(f"span {(end - t0) / 1e3:.1f} us")
