#!/usr/bin/env python3
"""Round 5: the host path's HIP API calls and GPU work on one clock (a rocprofv3 --hip-trace --kernel-trace
--memory-copy-trace run): for a window of slices, each API call of the pipeline and each copy / kernel.
   usage: tools/host_timeline.py DIR [N_KERNELS_BACK]"""
import csv
import glob
import sys

d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 12
keep = ("hipEventSynchronize", "hipEventQuery", "hipLaunchKernel", "hipMemcpyAsync", "hipEventRecord", "hipStreamWaitEvent")
ev = []
for r in csv.DictReader(open(glob.glob(d + "/*hip_api_trace.csv")[0])):
    if r["Function"] in keep:
        ev.append(("API " + r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for r in csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])):
    n = r["Kernel_Name"]
    tag = "GPU blit q" + r.get("Queue_Id", "?") if "copyBuffer" in n else ("GPU kern q" + r.get("Queue_Id", "?") if "rg::" in n else None)
    if tag:
        ev.append((tag, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for r in csv.DictReader(open(glob.glob(d + "/*memory_copy_trace.csv")[0])):
    ev.append(("GPU " + ("H2D" if "HOST_TO" in r["Direction"] else "D2H"), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
ev.sort(key=lambda e: e[1])
ks = [i for i, e in enumerate(ev) if e[0].startswith("GPU kern")]
i0 = ks[-back]
t0 = ev[i0][1]
last = None
for e in ev[i0 - 20:]:
    if e[0] == "API hipEventQuery" and last == "API hipEventQuery":
        continue  # a polling run: one line per run of queries
    last = e[0]
    print(f"{e[0]:28s} {(e[1] - t0) / 1e3:9.1f} {(e[2] - t0) / 1e3:9.1f} {(e[2] - e[1]) / 1e3:8.1f}")
