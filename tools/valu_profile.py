#!/usr/bin/env python3
"""Summarise the `valu` step of tools/gpu_run.sh (rocprofv3 --pmc issue counters of the transport
kernels) into profiles/<tag>_valu_<workload>.json.

  tools/valu_profile.py --tag r2 gpurun_out/valu_cfg2 gpurun_out/valu_cfg3 ...

Units (MI355X_MICROARCH.md, PMC table): SQ_WAVE_CYCLES / SQ_ACTIVE_INST_VALU / SQ_WAIT_* count
quad-cycles summed over waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs.  Derived per kernel:
  clock_ghz       the shader clock during the kernel: from in-kernel s_memtime / s_memrealtime stamps
                  (--clock WORKLOAD=GHZ, tools/stamps.py) when given; else GRBM_GUI_ACTIVE / 8 / duration,
                  but only for dispatches of >= 0.3 ms -- shorter ones read high (MI355X_MICROARCH.md:497:
                  round 2 committed 2.7-4.7 GHz for sub-0.1 ms kernels) and get null
  valu_insts_per_wave
  valu_active     SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (share of a wave's lifetime issuing VALU)
  wait_any        SQ_WAIT_ANY / SQ_WAVE_CYCLES           (parked on s_waitcnt / barrier)
  valu_busy       4 SQ_ACTIVE_INST_VALU / (SIMDs x clock x duration)  (chip-wide VALU busy share; null
                  without a trustworthy clock)

  tools/valu_profile.py --recompute profiles/r2c_valu_cfg2.json --clock cfg2=2.14   # fix a committed file
"""
import argparse
import collections
import csv
import glob
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 256 * 4


MIN_GRBM_US = 300.0


def derive(m: dict, us: float, clock: float | None) -> dict:
    """Clock and chip-wide VALU busy share of one kernel from its mean counters (see the module doc)."""
    grbm = m.get("GRBM_GUI_ACTIVE", 0.0)
    src = None
    if clock:
        src = "stamps"
    elif grbm and us >= MIN_GRBM_US:
        clock, src = grbm / 8 / us / 1e3, "grbm"
    busy = 4 * m.get("SQ_ACTIVE_INST_VALU", 0) / (SIMDS * clock * 1e3 * us) if clock and us else None
    return {"clock_ghz": round(clock, 3) if clock else None, "clock_source": src,
            "valu_busy": round(busy, 4) if busy is not None else None}


def summarise(d, clock=None):
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
        out[k] = {"dispatches": len(ds), "duration_us_median": round(us, 2), **derive(m, us, clock),
                  "waves": int(waves), "valu_insts_per_wave": round(m.get("SQ_INSTS_VALU", 0) / waves, 1),
                  "salu_insts_per_wave": round(m.get("SQ_INSTS_SALU", 0) / waves, 1),
                  "lds_insts_per_wave": round(m.get("SQ_INSTS_LDS", 0) / waves, 1),
                  "valu_active": round(m.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4),
                  "wait_any": round(m.get("SQ_WAIT_ANY", 0) / wc, 4),
                  "wait_inst_any": round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
                  "raw_means": {c: round(x, 1) for c, x in sorted(m.items())}}
    return out


def recompute(path: str, clocks: dict) -> None:
    """Re-derive clock_ghz / valu_busy of a committed profile from its raw counter means."""
    res = json.load(open(path))
    clock = clocks.get(res.get("workload"))
    for k, v in res["kernels"].items():
        v.update(derive(v["raw_means"], v["duration_us_median"], clock))
    res["clock_note"] = ("clock_ghz / valu_busy re-derived by tools/valu_profile.py --recompute: "
                         + (f"stamp clock {clock} GHz" if clock else "GRBM clock only for dispatches >= 0.3 ms"))
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res["kernels"].items():
        print(os.path.basename(path), k[:50], v["duration_us_median"], v["clock_ghz"], v["valu_busy"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag")
    ap.add_argument("--clock", action="append", default=[], help="WORKLOAD=GHZ from in-kernel stamps")
    ap.add_argument("--recompute", action="store_true", help="the arguments are committed profile JSON files")
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    clocks = {c.split("=")[0]: float(c.split("=")[1]) for c in a.clock}
    if a.recompute:
        for p in a.dirs:
            recompute(p, clocks)
        return
    for d in a.dirs:
        wl = os.path.basename(d.rstrip("/")).replace("valu_", "")
        res = {"source": f"rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES "
                         f"SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace, "
                         f"bench.py --workload {wl} --steps 5 --warmup 2 --no-cold (tools/gpu_run.sh valu), round {a.tag}",
               "workload": wl, "kernels": summarise(d, clocks.get(wl))}
        p = os.path.join(REPO, "profiles", f"{a.tag}_valu_{wl}.json")
        with open(p, "w") as f:
            json.dump(res, f, indent=1)
        for k, v in res["kernels"].items():
            print(wl, k[:60], {x: v[x] for x in ("duration_us_median", "clock_ghz", "valu_insts_per_wave",
                                                  "valu_active", "wait_any", "valu_busy")})


if __name__ == "__main__":
    main()
