#!/usr/bin/env python3
"""Per-kernel duration, effective clock and issue counters from a rocprofv3 --pmc + --kernel-trace run."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not cc:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(cc[0])):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in agg.items():
        if not any(x in k for x in ("seal", "open", "tile", "plan", "pipe")):
            continue
        m = {c: sum(x) / len(x) for c, x in v.items()}
        us = sorted(dur[k])[len(dur[k]) // 2]
        clk = m.get("GRBM_GUI_ACTIVE", 0) / 8 / us / 1e3
        waves = m.get("SQ_WAVES", 1)
        print(f"{d.split('/')[-1]:14s} {k:36s} dur={us:8.1f}us clk={clk:.2f}GHz valu/wave={m.get('SQ_INSTS_VALU',0)/waves:9.0f} "
              f"wavecyc/wave={4*m.get('SQ_WAVE_CYCLES',0)/waves:9.0f} active={m.get('SQ_ACTIVE_INST_VALU',0)/max(m.get('SQ_WAVE_CYCLES',1),1):.2f} "
              f"wait={m.get('SQ_WAIT_ANY',0)/max(m.get('SQ_WAVE_CYCLES',1),1):.2f} waitinst={m.get('SQ_WAIT_INST_ANY',0)/max(m.get('SQ_WAVE_CYCLES',1),1):.2f}")
