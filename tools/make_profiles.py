#!/usr/bin/env python3
"""Turn rocprofv3 outputs under gpurun_out/ into the committed profiles/ files.

  tools/make_profiles.py --tag r1 --workload cfg2 --stats gpurun_out/prof \
      --fetch gpurun_out/pmc_fetch_cfg2 --write gpurun_out/pmc_write_cfg2 --bench gpurun_out/bench_default.log

Writes
  profiles/<tag>_<workload>_kernel_stats.csv   (rocprofv3 --kernel-trace --stats summary, verbatim)
  profiles/pmc_<workload>.json                 (per-launch HBM bytes the bench reads as roofline.traffic)

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3):
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (they do not fit one
pass), are reported in KiB, and on gfx950 FETCH_SIZE counts half the bytes of a
wide coalesced streaming read (16 B/lane, global_load and buffer_load ... lds
alike), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kind_of(name: str):
    """seal / open for the transport kernels, None otherwise."""
    if "staged_kernel<" in name or "tile_kernel<" in name:
        args = name.split("<", 1)[1].split(">", 1)[0].split(",")
        return "open" if args[1].strip() == "true" else "seal"
    if "flat_kernel<" in name:
        return "open" if name.split("<", 1)[1].startswith("true") else "seal"
    if "pipe_seal_kernel" in name:
        return "seal"
    if "pipe_open_kernel" in name:
        return "open"
    return None


def family_of(name: str) -> int:
    """rg_get_kernel value of a transport kernel: 0 pipelined lanes, 1/2 tile window."""
    if "pipe_" in name:
        return 0
    if "flat_kernel<" in name:
        return 3
    return int(name.split("<", 1)[1].split(",", 1)[0])


def counter_means(d: str):
    """Per-dispatch means of each counter for seal and open, over the dispatches of the kernel family
    that ran most often (automatic choice may route the first call of a run elsewhere)."""
    out = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
    names = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = kind_of(r["Kernel_Name"])
            if k:
                fam = family_of(r["Kernel_Name"])
                out[k][fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
                names[(k, fam)] = r["Kernel_Name"]
    means, picked = {}, {}
    for k, fams in out.items():
        fam = max(fams, key=lambda x: max(len(v) for v in fams[x].values()))
        means[k] = {c: sum(v) / len(v) for c, v in fams[fam].items()}
        picked[k] = names[(k, fam)]
    return means, picked


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench", help="bench log whose JSON line gives the algorithmic bytes")
    a = ap.parse_args()
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    if a.stats:
        src = glob.glob(f"{a.stats}/**/*kernel_stats.csv", recursive=True)[0]
        shutil.copy(src, os.path.join(prof, f"{a.tag}_{a.workload}_kernel_stats.csv"))
    if a.fetch and a.write:
        fetch, names = counter_means(a.fetch)
        write, _ = counter_means(a.write)
        alg, npk = {}, None
        if a.bench:
            for line in open(a.bench):
                if line.startswith("{"):
                    b = json.loads(line)
                    n = b["config"]["packets_per_gpu"]
                    p = b["config"]["mean_payload_bytes"] * n
                    alg = {"seal": int(2 * p + 32 * n), "open": int(2 * p + 33 * n)}
                    npk = n
        res = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), round {a.tag}",
               "workload": a.workload, "units": "bytes per launch; FETCH_SIZE KiB x 1024 x 2 (gfx950 correction), "
                                                "WRITE_SIZE KiB x 1024"}
        for k in ("seal", "open"):
            if k not in fetch or k not in write:
                continue
            rd = fetch[k]["FETCH_SIZE"] * 1024 * 2
            wr = write[k]["WRITE_SIZE"] * 1024
            res[k] = {"kernel": names[k], "family": family_of(names[k]), "fetch_size_kib_raw": round(fetch[k]["FETCH_SIZE"], 1),
                      "read_bytes": int(rd), "write_bytes": int(wr), "hbm_bytes_per_launch": int(rd + wr)}
            if npk:
                res[k]["packets_per_launch"] = npk
            if k in alg:
                res[k]["alg_bytes_per_launch"] = alg[k]
                res[k]["traffic_over_alg"] = round((rd + wr) / alg[k], 3)
        with open(os.path.join(prof, f"pmc_{a.workload}.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
