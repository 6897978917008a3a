#!/usr/bin/env python3
"""Summarise the `valu` step of tools/gpu_run.sh (rocprofv3 --pmc issue counters of the transport
kernels) into profiles/<tag>_valu_<workload>.json.

  tools/valu_profile.py --tag r2 gpurun_out/valu_cfg2 gpurun_out/valu_cfg3 ...

Units (MI355X_MICROARCH.md, PMC table): SQ_WAVE_CYCLES / SQ_ACTIVE_INST_VALU / SQ_WAIT_* count
quad-cycles summed over waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs.  Derived per kernel:
  clock_ghz       GRBM_GUI_ACTIVE / 8 / duration
  valu_insts_per_wave
  valu_active     SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (share of a wave's lifetime issuing VALU)
  wait_any        SQ_WAIT_ANY / SQ_WAVE_CYCLES           (parked on s_waitcnt / barrier)
  valu_busy       4 SQ_ACTIVE_INST_VALU / (SIMDs x GRBM_GUI_ACTIVE / 8)  (chip-wide VALU busy share)
"""
import argparse
import collections
import csv
import glob
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 256 * 4


def summarise(d):
    cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for f in cc:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k][r.get("Dispatch_Id", len(dur[k]))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = {}
    for k, v in agg.items():
        if not any(x in k for x in ("pipe_", "tile_kernel", "flat_", "plan")):
            continue
        m = {c: sum(x) / len(x) for c, x in v.items()}
        ds = sorted(dur[k].values())
        us = ds[len(ds) // 2]
        wc = max(m.get("SQ_WAVE_CYCLES", 1.0), 1.0)
        waves = max(m.get("SQ_WAVES", 1.0), 1.0)
        grbm = m.get("GRBM_GUI_ACTIVE", 0.0)
        out[k] = {"dispatches": len(ds), "duration_us_median": round(us, 2),
                  "clock_ghz": round(grbm / 8 / us / 1e3, 3) if us else None,
                  "waves": int(waves), "valu_insts_per_wave": round(m.get("SQ_INSTS_VALU", 0) / waves, 1),
                  "salu_insts_per_wave": round(m.get("SQ_INSTS_SALU", 0) / waves, 1),
                  "lds_insts_per_wave": round(m.get("SQ_INSTS_LDS", 0) / waves, 1),
                  "valu_active": round(m.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4),
                  "wait_any": round(m.get("SQ_WAIT_ANY", 0) / wc, 4),
                  "wait_inst_any": round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
                  "valu_busy": round(4 * m.get("SQ_ACTIVE_INST_VALU", 0) / (SIMDS * grbm / 8), 4) if grbm else None,
                  "raw_means": {c: round(x, 1) for c, x in sorted(m.items())}}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    for d in a.dirs:
        wl = os.path.basename(d.rstrip("/")).replace("valu_", "")
        res = {"source": f"rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES "
                         f"SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace, "
                         f"bench.py --workload {wl} --steps 5 --warmup 2 --no-cold (tools/gpu_run.sh valu), round {a.tag}",
               "workload": wl, "kernels": summarise(d)}
        p = os.path.join(REPO, "profiles", f"{a.tag}_valu_{wl}.json")
        with open(p, "w") as f:
            json.dump(res, f, indent=1)
        for k, v in res["kernels"].items():
            print(wl, k[:60], {x: v[x] for x in ("duration_us_median", "clock_ghz", "valu_insts_per_wave",
                                                  "valu_active", "wait_any", "valu_busy")})


if __name__ == "__main__":
    main()
