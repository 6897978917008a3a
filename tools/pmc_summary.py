#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel over dispatches: tools/pmc_summary.py DIR [DIR...]"""
import csv
import collections
import glob
import sys

for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            if any(x in k for x in ("seal", "open", "chacha", "tile", "pipe", "flat", "rd_", "wr_", "k_phase")):
                print(d, k[:48], {c: round(sum(x) / len(x), 1) for c, x in sorted(v.items())})
