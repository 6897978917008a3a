#!/usr/bin/env python3
"""Benchmark: device-resident WireGuard transport-data ChaCha20-Poly1305 seal+open.

Metric (BASELINE.json): GiB/s + Mpkt/s device-resident ChaCha20-Poly1305
seal/open at 1/2/4/8 MI355X.

One step = one batch sealed (in place, header + tag framed) and then opened
(tag verified, plaintext restored).  N = 1 runs BASELINE config 2 ("64 Ki
packets x 1500 B, one session key, seal then open").  N > 1 runs BASELINE
config 5 ("8 Mi packets x 1500 B, one session key, batch split evenly across
the GPUs, no collective"): rank r seals and opens packets [r 8Mi/N,
(r+1) 8Mi/N) with their global counters (strong scaling).  The split is a
plain index range with no data-path collective; RCCL only carries the timing
barrier and the max-over-ranks reduction.

value = payload bytes through AEAD (seal + open, P bytes each) summed over
ranks / max-over-ranks wall time of the timed steps, in GiB/s.

Launch: `python bench.py --gpus N` starts N ranks itself (a torch.distributed.run
child process, before anything touches a GPU); the driver's own
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N` is
accepted too.  A WORLD_SIZE that disagrees with --gpus is an error (exit 2).

`--workload cfg1` times BASELINE config 1 instead: one 1500-B packet sealed and
opened on one CPU thread (ns/packet), plus the per-message GPU drop-in.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md "Chip-level parameters"
# VALU ceilings measured on the MI355X by tools/microbench.hip (profiles/r1c_microbench.json, best
# occupancy): ChaCha20 keystream bytes/s over the whole chip, and clamped Poly1305 bytes/s
CHACHA_PEAK_GBS = 2610.0
POLY_PEAK_GBS = 15765.0
# ... measured at these shader clocks (profiles/r1c_microbench.json "clock": 2.25-2.41 GHz, 2.39 at the best
# occupancy).  The AEAD kernels hold a lower clock under their own load; their clocks from per-wave
# s_memtime / s_memrealtime stamps of diagnostic builds (the product library has no stamps):
MICRO_CLOCK_GHZ = 2.39
KERNEL_CLOCK_GHZ = {
    "cfg2": (2.135, "profiles/r4_cfg2_twowave.txt (one wave per SIMD, 2.130-2.137 GHz)"),
    "cfg3": (2.15, "profiles/r4_cfg3_flat_ab.txt, r4_cfg3_search_ab.txt, r4_cfg3_xcd_ab.txt (flattened kernel stamps, 2.09-2.19 GHz by box)"),
    "cfg4": (2.09, "profiles/r3_valu_cfg4.json (GRBM quotient over a ~1 ms dispatch)"),
    "cfg5": (2.09, "as cfg4: the same tile kernel on 8 Mi packets"),
}


def valu_ceiling_gbs(desc_len, is_open: bool) -> float:
    """Payload bytes/s the chip's VALU could seal (open) at the measured ChaCha20 / Poly1305 rates:
    per packet ceil(P/64) + 1 keystream blocks (one-time key) and P/16 + 1 Poly1305 blocks."""
    P = np.asarray(desc_len, dtype=np.float64) - (32 if is_open else 0)
    t = ((np.ceil(P / 64) + 1) * 64 / CHACHA_PEAK_GBS + (P / 16 + 1) * 16 / POLY_PEAK_GBS).sum()
    return float(P.sum() / t) if t > 0 else 0.0


def rooflines(dominant: str, achieved: float, dom_alg: int, traffic, pay_gbs: float, ceil_gbs: float, clk):
    """The line's `roofline` and `valu_roofline` objects.

    roofline.bound is what limits the kernels by the counters: integer VALU issue (ChaCha20 ARX + Poly1305
    multiplies; 0.71-0.95 of the chip's VALU cycles issuing at HBM traffic ~1.0x of the algorithmic bytes,
    DESIGN.md §5), not HBM.  achieved / peak / frac / traffic stay the HBM figures of the
    dominant kernel (the contract's fields); roofline.valu beside them is the seal's fraction of the VALU
    ceiling, at the microbenchmarks' clock and at the kernel's own (clock recorded by a diagnostic build,
    not measured in this run: clock_assumed)."""
    roof = {"bound": "valu", "kernel": dominant, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "alg_bytes_per_launch": dom_alg,
            "note": "achieved = algorithmic bytes (seal 2P+32, open 2P+33 per packet) / mean launch time "
                    "(one HIP event pair per launch on the launch stream, seal->open pairs) against the HBM "
                    "peak; the kernels are VALU-bound: roofline.valu is the seal's fraction of the VALU ceiling"}
    valu = {"kernel": "seal", "achieved": round(pay_gbs, 2), "peak": round(ceil_gbs, 2), "unit": "GB/s of payload",
            "frac": round(pay_gbs / ceil_gbs, 4) if ceil_gbs else None,
            "basis": f"ChaCha20 {CHACHA_PEAK_GBS:.0f} GB/s + Poly1305 {POLY_PEAK_GBS:.0f} GB/s chip rates measured by "
                     f"tools/microbench.hip at {MICRO_CLOCK_GHZ} GHz; one-time-key block per packet"}
    if clk and ceil_gbs:
        # the same fraction against the ceiling scaled to the clock the kernel holds under its own load (VERDICT
        # r3); that clock varies by box (2.09-2.19 GHz) and is not measured here: clock_assumed
        valu.update({"kernel_clock_ghz": clk[0], "basis_clock_ghz": MICRO_CLOCK_GHZ,
                     "frac_at_kernel_clock": round(pay_gbs / (ceil_gbs * clk[0] / MICRO_CLOCK_GHZ), 4),
                     "clock_assumed": True, "clock_source": clk[1]})
    roof["valu"] = {k: valu.get(k) for k in ("kernel", "achieved", "peak", "unit", "frac", "frac_at_kernel_clock",
                                             "clock_assumed")}
    return roof, valu


METRIC = "GiB/s + Mpkt/s device-resident ChaCha20-Poly1305 seal/open, 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default=None, choices=["cfg1", "cfg2", "cfg3", "cfg4", "cfg5"],
                    help="BASELINE config (default: cfg2 on one GPU, the cfg5 split on several)")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per packet (0 = auto)")
    ap.add_argument("--wg-per-cu", type=int, default=0, help="resident workgroups per CU (0 = auto, -1 = plain grid)")
    ap.add_argument("--staged", type=int, default=-1,
                    help="kernel: -1 automatic (default), 0 pipelined lanes, 1/2 LDS-staged tiles with that window")
    ap.add_argument("--plan", type=int, default=-1, help="size-class planner: 0 off, 1 on, 2 auto, -1 library default (auto)")
    ap.add_argument("--segments", type=int, default=0, help="segments per packet for the tile kernels (0 = auto)")
    ap.add_argument("--debug-mode", type=int, default=0, help="seal diagnostics (invalid output): 1 compute-only, 2 memory-only")
    ap.add_argument("--frame-shift", type=int, default=0,
                    help="diagnostics: add this many bytes (multiple of 16) to every frame offset")
    ap.add_argument("--split", type=int, default=1,
                    help="sub-batches per step: seal of part k+1 overlaps open of part k on a second stream")
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a captured HIP graph")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU baseline budget: port and OpenSSL, 1 thread and all cores, 5 runs each (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="all-core thread count (0 = this host's share)")
    ap.add_argument("--cpu-study", action="store_true",
                    help="only the CPU baselines' scaling study (free / pinned / pinned + private slices), no GPU")
    ap.add_argument("--e2e", action="store_true", help="also time the pinned host->GPU->host path")
    ap.add_argument("--single-process", action="store_true",
                    help="one process and one thread drive all --gpus N GPUs (rg_group: config 5's split, "
                         "rg_{seal,open}_batch_dev_multi) instead of one rank per GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch/validate the ranks, print each rank's plan as JSON and exit before any GPU work")
    ap.add_argument("--forged", default="0.01,0.1",
                    help="also time the open with these fractions of forged tags, comma-separated (0 = skip)")
    ap.add_argument("--no-cold", dest="cold", action="store_false",
                    help="skip the cold-cache pass (profiling runs: keeps per-kernel averages to the step's regime)")
    ap.add_argument("--no-verify", dest="verify", action="store_false",
                    help="skip the status check after the timed region (on by default, outside the timing)")
    return ap.parse_args()


def kernel_label(args, eng, w) -> str:
    k = eng.last_kernel()  # the family the timed launches actually ran
    if k < 0:
        k = eng.kernel_for(w.n)
    plan = ({0: "off", 1: "on"}).get(args.plan, "auto")
    if k == 3:
        return (f"flattened chunk stream (units of equal work cut inside the kernel, chunks dealt evenly "
                f"over 64 lanes), planner {plan}")
    if k == 0:
        return (f"pipelined lanes ({eng.lanes_per_packet(w.n)} lane(s)/packet without plan, 3 chunks in flight, "
                f"Poly1305 in keystream rounds), planner {plan}")
    return f"lds-staged tiles, {k} chunks/window, planner {plan}, segments {args.segments or 'auto'}"


def host_cpu_info() -> dict:
    """What the CPU baselines ran on: model, the machine's logical CPUs and this process's share."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity": aff}


def cgroup_cpu_quota():
    """The job's CPU quota from its cgroup (v2 cpu.max, else v1 cfs quota / period) in CPUs, or None when
    unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def all_core_threads(requested: int):
    """(threads, how): the host's CPU share for the all-core baseline -- the smallest of the affinity mask,
    the cgroup CPU quota (cpu.max, rounded down) and OMP_NUM_THREADS (16 per GPU on the GPU box, where
    nproc and the affinity mask show the whole 256-CPU machine)."""
    aff = host_cpu_info()["affinity"]
    quota = cgroup_cpu_quota()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    limits = {"affinity": aff}
    if quota is not None:
        limits["cgroup_cpu_max"] = quota
    if omp > 0:
        limits["OMP_NUM_THREADS"] = omp
    if requested:
        return requested, {"requested": requested, **limits}
    t = max(1, min([aff] + ([int(quota)] if quota is not None else []) + ([omp] if omp > 0 else [])))
    return t, limits


CPU_SAMPLE = 65536  # packets: >= 64 Ki; config 2's whole batch


def cgroup_throttle():
    """(periods throttled, µs throttled) of the job's cgroup (v2 cpu.stat), or None: the CPU quota at work."""
    try:
        d = {}
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                d[k] = int(v)
        return d.get("nr_throttled", 0), d.get("throttled_usec", 0)
    except (OSError, ValueError):
        return None


def _cpulist(text: str):
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def pick_cpus(n: int, node=None, spread_l3: bool = True):
    """n CPUs of this process's affinity mask for pinned baseline workers: one hardware thread per core
    (the first sibling), on one NUMA node -- `node` if it has n, else the node with the most -- dealt
    round-robin over the node's L3 domains (CCDs), so that the workers neither migrate nor share a core
    and their slices spread over every L3 and CCD link; None if the mask cannot give n."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    allowed = set(aff)

    def read_list(path, default):
        try:
            with open(path) as f:
                return tuple(_cpulist(f.read()))
        except (OSError, ValueError):
            return default

    def spread(cpus):
        seen, doms = set(), {}
        for c in cpus:
            sib = read_list(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list", (c,))
            if sib in seen:
                continue
            seen.add(sib)
            l3 = read_list(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list", ())
            doms.setdefault(l3, []).append(c)
        lists = [doms[k] for k in sorted(doms, key=lambda k: min(k) if k else -1)]
        if not spread_l3:
            return [c for lst in lists for c in lst]
        out, i = [], 0
        while any(lists):
            lst = lists[i % len(lists)]
            if lst:
                out.append(lst.pop(0))
            i += 1
        return out

    nodes = {}
    try:
        for d in os.listdir("/sys/devices/system/node"):
            if d.startswith("node") and d[4:].isdigit():
                with open(f"/sys/devices/system/node/{d}/cpulist") as f:
                    nodes[int(d[4:])] = spread([c for c in _cpulist(f.read()) if c in allowed])
    except OSError:
        nodes = {}
    if not nodes:
        nodes = {0: spread(aff)}
    order = sorted(nodes, key=lambda k: (k != node, -len(nodes[k])))
    for k in order:
        if len(nodes[k]) >= n:
            return nodes[k][:n]
    return None


def cpu_mhz(cpus):
    """Mean current clock (MHz, /proc/cpuinfo) of the given CPUs, or None where the kernel does not say."""
    want, cur, out = set(cpus), None, []
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("processor"):
                    cur = int(line.split(":")[1])
                elif line.startswith("cpu MHz") and cur in want:
                    out.append(float(line.split(":")[1]))
    except (OSError, ValueError):
        return None
    return sum(out) / len(out) if out else None


def _proc_stat():
    """Per-CPU (busy, total) jiffies from /proc/stat, or None."""
    out = {}
    try:
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3:4].isdigit():
                    v = line.split()
                    nums = [int(x) for x in v[1:]]
                    idle = nums[3] + (nums[4] if len(nums) > 4 else 0)
                    out[int(v[0][3:])] = (sum(nums) - idle, sum(nums))
    except (OSError, ValueError):
        return None
    return out


def _siblings(cpus):
    out = []
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                out.extend(x for x in _cpulist(f.read()) if x != c)
        except OSError:
            pass
    return out


def cpu_busy(before, after, cpus):
    """Busy share of the given CPUs between two _proc_stat() readings."""
    if not before or not after:
        return None
    b = t = 0
    for c in cpus:
        if c in before and c in after:
            b += after[c][0] - before[c][0]
            t += after[c][1] - before[c][1]
    return round(b / t, 3) if t else None


class _MhzSampler:
    """Samples cpu_mhz(cpus) every 0.1 s on a thread while the C pool runs (ctypes drops the GIL)."""

    def __init__(self, cpus):
        import threading

        self.cpus, self.samples, self.stop = cpus, [], threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True) if cpus else None

    def _run(self):
        while not self.stop.wait(0.1):
            m = cpu_mhz(self.cpus)
            if m is not None:
                self.samples.append(m)

    def __enter__(self):
        if self.t:
            self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        if self.t:
            self.t.join()

    def mean(self):
        return round(sum(self.samples) / len(self.samples)) if self.samples else None


def cpu_rate(w, impl: str, threads: int, rep_seconds: float, reps: int = 3, cpus=None, local: bool = False,
             sample: int = CPU_SAMPLE):
    """Median of `reps` timed runs of seal+open over a sample of the workload (its first CPU_SAMPLE
    packets) by a persistent pool of `threads` workers (oracle/rg_openssl_batch.c rg_cpu_bench: threads
    and OpenSSL cipher contexts live for the whole run, one untimed round first): GiB/s of payload and
    Mpkt/s.  cpus pins worker t to cpus[t]; local gives each worker a first-touched private copy of its
    slice.  throttled_ms: the cgroup's CPU-quota throttling during the runs."""
    from oracle import oracle  # checker / baseline only

    n = min(w.n, sample)
    desc = w.desc[:n].copy()
    base = int(desc["offset"][0])
    desc["offset"] -= np.uint64(base)
    span = int(desc["offset"][-1]) + int(desc["len"][-1]) + 32
    buf = np.zeros(span, np.uint8)
    oracle.synth_fill(buf, desc, w.inner_len[:n], w.data_seed)
    plain = buf.copy()
    ctr = w.counters[:n]
    payload = int(desc["len"].astype(np.int64).sum())
    runs = []
    th0 = cgroup_throttle()
    ps0 = _proc_stat()
    with _MhzSampler(list(cpus) if cpus else None) as mhz:
        for _ in range(reps):
            el, rounds = oracle.cpu_bench(impl, threads, w.keys, w.receivers, desc, ctr, buf, rep_seconds,
                                          cpus=cpus, local=local)
            runs.append((2 * payload * rounds / el / 2**30, 2 * n * rounds / el / 1e6))
    th1 = cgroup_throttle()
    ps1 = _proc_stat()
    pay = np.zeros(span, bool)  # payload bytes (headers and tags are rewritten by every seal)
    for o, ln in zip(desc["offset"].astype(np.int64), desc["len"].astype(np.int64)):
        pay[o + 16:o + 16 + ln] = True
    assert np.array_equal(buf[pay], plain[pay]), "a seal+open round did not give the plaintext back"
    gib = sorted(r[0] for r in runs)[reps // 2]
    mpkt = sorted(r[1] for r in runs)[reps // 2]
    out = {"value": round(gib, 4), "unit": "GiB/s", "cores": threads, "mpkt_s": round(mpkt, 4),
           "runs_gib_s": [round(r[0], 4) for r in runs], "median_of": reps, "n_sample": n,
           "mean_payload": round(payload / n, 1)}
    if th0 is not None and th1 is not None:
        out["throttled_ms"] = round((th1[1] - th0[1]) / 1000.0, 1)
    if mhz.mean() is not None:
        out["cpu_mhz"] = mhz.mean()  # the workers' CPUs while they ran
    if cpus and ps0 and ps1:
        # how busy the workers' CPUs, their SMT siblings (not ours: another job's threads share the core) and
        # the whole machine were while the pool ran
        out["busy"] = {"workers": cpu_busy(ps0, ps1, cpus), "siblings": cpu_busy(ps0, ps1, _siblings(cpus)),
                       "machine": cpu_busy(ps0, ps1, list(ps0))}
    return out


def cpu_baselines(w, seconds: float, threads_how):
    """CPU baselines of BASELINE.md §2, in the same run as the GPU numbers: the C restatement
    (kind "port": the reference's Rust + graviola 0.2.0 path cannot be built here -- no cargo, crate
    not vendored) and OpenSSL EVP ChaCha20-Poly1305 (an assembly-optimised stand-in for graviola),
    each on 1 thread and on the host's share of cores, median of 3 runs over a 64 Ki-packet sample.
    The all-core figure is the better of two placements, both pinned one worker per core on one NUMA node
    with private first-touched slices: spread over the node's L3 domains (CCDs), and compact (the first
    cores).  The port scales best spread, OpenSSL compact (bench.py --cpu-study).
    scaling = all-core rate / (threads x 1-thread rate), with the workers' clock, the cgroup's quota
    throttling and how busy the workers' SMT siblings were, which together say what stops it."""
    from oracle import oracle

    threads, limits = threads_how
    info = host_cpu_info()
    placements = [(name, cp) for name, cp in (("spread", pick_cpus(threads)),
                                               ("compact", pick_cpus(threads, spread_l3=False))) if cp]
    if not placements:
        placements = [("unpinned", None)]
    impls = ["port"] + (["openssl"] if oracle.openssl_available() else [])
    rep = max(0.2, seconds / (len(impls) * (1 + len(placements)) * 3))
    out = {}
    for impl in impls:
        first = placements[0][1]
        one = cpu_rate(w, impl, 1, rep, cpus=first[:1] if first else None, local=first is not None)
        tried = {}
        for name, cp in placements:
            tried[name] = cpu_rate(w, impl, threads, rep, cpus=cp, local=cp is not None)
        best = max(tried, key=lambda k: tried[k]["value"])
        many = tried[best]
        what = ("C RFC 8439 restatement (oracle/rg_oracle.c)" if impl == "port" else
                f"{oracle.openssl_version()} EVP_chacha20_poly1305, re-keyed per packet (oracle/rg_openssl_batch.c)")
        cp = dict(placements)[best]
        placement = (f"pinned one per core on one NUMA node, {best} (CPUs {sorted(cp)[0]}..{sorted(cp)[-1]}), private "
                     f"first-touched slices" if cp else "unpinned (the affinity mask cannot give one core per worker)")
        d = dict(many)
        d["kind"] = "port" if impl == "port" else "openssl (stand-in for graviola)"
        d["one_thread"] = {k: one[k] for k in ("value", "unit", "mpkt_s", "runs_gib_s", "cpu_mhz") if k in one}
        eff = many["value"] / (threads * one["value"]) if one["value"] > 0 else None
        sc = {"speedup": round(many["value"] / one["value"], 2) if one["value"] else None,
              "efficiency": round(eff, 3) if eff is not None else None, "threads": threads,
              "thread_limits": limits, "placement": placement,
              "by_placement_gib_s": {k: v["value"] for k, v in tried.items()}}
        m1, mn = one.get("cpu_mhz"), many.get("cpu_mhz")
        if m1 and mn:
            sc["cpu_mhz"] = {"one_thread": m1, "all_threads": mn}
        if "throttled_ms" in many:
            sc["throttled_ms"] = many["throttled_ms"]
        if many.get("busy"):
            sc["busy"] = many["busy"]
        if eff is not None and eff < 0.9:
            why = []
            if m1 and mn and mn < 0.95 * m1:
                why.append(f"the workers' clock: {m1} MHz on 1 thread, {mn} MHz on {threads}")
            if many.get("throttled_ms", 0) > 0.05 * 3 * rep * 1000:
                why.append(f"cgroup quota throttling {many['throttled_ms']} ms over the runs")
            sib = (many.get("busy") or {}).get("siblings")
            if sib is not None and sib > 0.2:
                why.append(f"the workers' SMT siblings {sib:.0%} busy with other work")
            vals = sorted(v["value"] for v in tried.values())
            if not why and len(vals) > 1 and vals[-1] > 1.1 * vals[0]:
                why.append("state shared between the workers: the rate follows where they sit ("
                           + ", ".join(f"{k} {v['value']:.2f}" for k, v in tried.items())
                           + " GiB/s) while the clock, the quota and the SMT siblings are not the cause")
            sc["limit"] = "; ".join(why) or (
                "neither the workers' clock, the cgroup quota nor their SMT siblings (read beside the runs); "
                "bench.py --cpu-study separates placement, private slices, an L3-sized sample and the re-key")
        d["scaling"] = sc
        d["sample"] = (f"first {many['n_sample']} packets of {w.name} (mean P={many['mean_payload']}) sealed then "
                       f"opened by a persistent pool (threads and cipher contexts kept across rounds; {placement}), "
                       f"{rep:.2f} s per run, median of 3 runs on {threads} threads and on 1 thread; {what}")
        d.update(info)
        out[impl] = d
    return out.get("port"), out.get("openssl")


def cpu_study(args):
    """The all-core CPU baseline's scaling, without the GPU (bench.py --cpu-study): each
    implementation on 1 thread and on the host's share, with the workers free to migrate, pinned one per
    core on the first cores of one NUMA node (compact), pinned spread over its L3 domains, spread with
    private first-touched slices (the default line's placement), and that on a 16 Ki-packet sample (slices
    that fit the L3s).  The workers' clock and the cgroup's quota throttling are read beside each run."""
    from oracle import oracle
    from rustyguard_amd import workloads

    w = workloads.build("cfg2")
    threads, limits = all_core_threads(args.cpu_threads)
    cpus = pick_cpus(threads)
    rep = max(0.3, args.cpu_seconds / 24)
    res = {"threads": threads, "thread_limits": limits, "cpus": cpus, **host_cpu_info(), "rep_seconds": rep,
           "runs": []}
    impls = ["port"] + (["openssl", "openssl-keyed-once"] if oracle.openssl_available() else [])
    compact = pick_cpus(threads, spread_l3=False)
    res["cpus_compact"] = compact
    # (name, cpus, private slices, sample packets)
    modes = [("free", None, False, CPU_SAMPLE), ("compact", compact, False, CPU_SAMPLE),
             ("spread", cpus, False, CPU_SAMPLE), ("spread+local", cpus, True, CPU_SAMPLE),
             ("spread+local, 16 Ki sample", cpus, True, 16384)]
    for impl in impls:
        for name, cp, loc, smp in modes:
            if name != "free" and cp is None:
                continue
            one = cpu_rate(w, impl, 1, rep, cpus=cp[:1] if cp else None, local=loc, sample=smp)
            many = cpu_rate(w, impl, threads, rep, cpus=cp, local=loc, sample=smp)
            res["runs"].append({"impl": impl, "mode": name, "threads": threads, "sample": smp,
                                "gib_s": many["value"], "runs_gib_s": many["runs_gib_s"],
                                "one_thread_gib_s": one["value"],
                                "speedup": round(many["value"] / one["value"], 2),
                                "efficiency": round(many["value"] / (threads * one["value"]), 3),
                                "cpu_mhz": [one.get("cpu_mhz"), many.get("cpu_mhz")],
                                "busy": [one.get("busy"), many.get("busy")],
                                "throttled_ms": many.get("throttled_ms")})
            print(json.dumps(res["runs"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


def bench_cfg1(args):
    """BASELINE config 1: a single 1500-B transport packet (L = 1500, P = 1504) sealed then opened on
    one CPU thread -- ns/packet for the C restatement and for OpenSSL -- plus the per-message GPU
    drop-in (rg_chacha20poly1305_enc/_dec: H2D, kernel, D2H per call) for comparison."""
    from oracle import oracle
    from rustyguard_amd import workloads

    w = workloads.build("cfg1")
    key = w.keys[0].tobytes()
    P = int(w.desc["len"][0])
    iters = 20000
    res = {}
    for impl in ["port"] + (["openssl"] if oracle.openssl_available() else []):
        oracle.time_one(impl, key, P, iters // 10)
        runs = [oracle.time_one(impl, key, P, iters) for _ in range(5)]
        seal_ns = sorted(r[0] for r in runs)[2]
        open_ns = sorted(r[1] for r in runs)[2]
        res[impl] = {"seal_ns": round(seal_ns, 1), "open_ns": round(open_ns, 1),
                     "seal_open_ns": round(seal_ns + open_ns, 1), "median_of": 5, "iters": iters}
    gpu = None
    try:
        import torch

        if torch.cuda.is_available():
            from rustyguard_amd.aead import Engine, nonce

            eng = Engine(0)
            pt = bytearray(np.random.default_rng(1).integers(0, 256, P, dtype=np.uint8).tobytes())
            for _ in range(20):
                t = eng.chacha20poly1305_enc(key, nonce(0), b"", pt)
                eng.chacha20poly1305_dec(key, nonce(0), b"", pt, t)
            ts, to = [], []
            for i in range(200):
                t0 = time.perf_counter()
                t = eng.chacha20poly1305_enc(key, nonce(i), b"", pt)
                t1 = time.perf_counter()
                eng.chacha20poly1305_dec(key, nonce(i), b"", pt, t)
                t2 = time.perf_counter()
                ts.append(t1 - t0)
                to.append(t2 - t1)
            gpu = {"seal_us": round(float(np.median(ts)) * 1e6, 2), "open_us": round(float(np.median(to)) * 1e6, 2),
                   "note": "per-message drop-in rg_chacha20poly1305_enc/_dec (host buffers: H2D + kernel + D2H + "
                           "sync per call), median of 200"}
            eng.close()
    except Exception as e:  # the CPU measurement stands on its own
        gpu = {"error": str(e)}
    best = res.get("openssl", res["port"])
    out = {"metric": "ns/packet, single 1500-B transport packet seal+open on one CPU thread (BASELINE config 1)",
           "value": best["seal_open_ns"], "unit": "ns/packet", "n_gpus": 0, "higher_is_better": False,
           "vs_baseline": None, "dtype": "u32", "data": "synthetic",
           "config": {"workload": f"cfg1: {workloads.CONFIGS['cfg1']}", "payload_bytes": P, "wire_bytes": P + 32},
           "cpu": res, "gpu_per_message": gpu, **host_cpu_info(),
           "note": "value = OpenSSL EVP (stand-in for graviola 0.2.0, which cannot be built here) when libcrypto is "
                   "present, else the C restatement"}
    print(json.dumps(out), flush=True)


def launch_ranks(n: int) -> int:
    """Start n ranks of this script under torch.distributed.run as a child process (nothing here has
    touched a GPU yet) and return its exit code."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


MALL_BYTES = 256 * 2**20  # MI355X Infinity Cache (memory-side, in front of HBM)


def forged_open_timing(w, b, stream, frac: float, verify: bool):
    """Open time when a fraction of the batch carries forged tags (last tag byte flipped after the
    seal), beside the clean open timed the same way: every rep (seal, flip, open) is enqueued while a
    spin kernel holds the stream, so the events bracket the open kernel and not the host's time to
    submit it (round 2's numbers included that gap, ~20 us per open).  A forged frame is left as it
    came (checked byte for byte on the last rep).  DESIGN.md §4.1."""
    import torch

    rng = np.random.default_rng(7)
    k = max(1, int(round(frac * w.n)))
    pick = np.sort(rng.choice(w.n, size=k, replace=False))
    pos = (w.desc["offset"][pick] + np.uint64(16) + w.desc["len"][pick].astype(np.uint64) + np.uint64(15))
    idx = torch.from_numpy(pos.astype(np.int64)).to(b.buf.device)
    reps = 5

    def run(forge: bool, keep_last: bool):
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(reps)]
        before = None
        with torch.cuda.stream(stream):
            torch.cuda._sleep(int(2e7))  # ~10 ms: longer than enqueueing the reps
        for r, e in enumerate(evs):
            b.seal(stream=stream)
            with torch.cuda.stream(stream):
                if forge:
                    b.buf[idx] ^= 1
                if keep_last and r == reps - 1:
                    before = b.buf.clone()  # the submitted (tampered) frames of the last rep
            e[0].record(stream)
            b.open(stream=stream, counters_out=False)
            e[1].record(stream)
        torch.cuda.synchronize()
        return sorted(e[0].elapsed_time(e[1]) for e in evs)[reps // 2], before

    clean_ms, _ = run(False, False)
    open_ms, before = run(True, verify)
    st = b.status[: w.n].cpu().numpy()
    if verify:
        bad = np.zeros(w.n, bool)
        bad[pick] = True
        assert (st[bad] == 1).all() and (st[~bad] == 0).all(), "forged-batch statuses"
        # a rejected frame is left exactly as it came (prim.rs:190-201): every byte of every forged frame
        off = torch.from_numpy(w.desc["offset"][pick].astype(np.int64)).to(b.buf.device)
        wl = torch.from_numpy(w.desc["len"][pick].astype(np.int64) + 32).to(b.buf.device)
        span = int(wl.max().item())
        ar = torch.arange(span, device=b.buf.device)
        for g in range(0, k, 32768):
            pos_ = off[g:g + 32768, None] + ar[None, :]
            m = ar[None, :] < wl[g:g + 32768, None]
            pos_ = pos_[m]
            assert torch.equal(b.buf[pos_], before[pos_]), "a forged frame was not restored byte for byte"
        del before
    b.fill(stream=stream)  # back to the synthetic plaintext the later checks start from
    torch.cuda.synchronize()
    return {"forged_frac": round(k / w.n, 4), "open_ms": round(open_ms, 5), "clean_open_ms": round(clean_ms, 5),
            "ratio": round(open_ms / clean_ms, 3), "open_gib_s": round(w.payload_bytes / (open_ms / 1e3) / 2**30, 3),
            "how": "median of 5 event-timed opens enqueued behind a spin kernel, clean and forged batches alike"}


def forged_fracs(spec: str) -> list:
    """--forged: comma-separated fractions in (0, 1]; 0 or empty = no forged-open legs."""
    out = [float(x) for x in str(spec).split(",") if x.strip()]
    if any(f < 0 or f > 1 for f in out):
        raise SystemExit(f"bench.py: --forged fractions must lie in [0, 1], got {spec!r}")
    return [f for f in out if f > 0]


def hbm_copy_rate(stream, nbytes: int = 1 << 30, reps: int = 5):
    """Achievable HBM bandwidth on this GPU for comparison with the 8 TB/s spec peak: a device-to-device
    copy of a 1 GiB buffer (4x the Infinity Cache, so it streams from HBM), (read + written bytes) /
    time, median of `reps` event-timed copies.  Outside the timed region."""
    import torch

    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    src.fill_(1)
    with torch.cuda.stream(stream):
        dst.copy_(src)  # warm-up
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in evs:
            e0.record(stream)
            dst.copy_(src)
            e1.record(stream)
    torch.cuda.synchronize()
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs)[reps // 2]
    del src, dst
    return {"gb_s": round(2 * nbytes / (ms / 1e3) / 1e9, 1), "bytes": 2 * nbytes,
            "how": "torch copy_ of a 1 GiB device buffer, read + write bytes / time, median of 5"}


def cold_cache_timing(eng, w, b, stream, verify: bool):
    """Per-launch seal / open time when the batch is not cache resident: a batch smaller than the
    256 MB Infinity Cache stays there between a step's seal and open and across steps.  Copies
    spanning twice that cache are sealed back to back between two events, then opened back to back,
    so every launch reads data last touched ~512 MB of traffic earlier.  Reported beside the step
    numbers only."""
    import torch

    from rustyguard_amd.device import DeviceBatch

    copies = int(min(64, max(2, -(-2 * MALL_BYTES // max(w.buf_bytes, 1)))))
    batches = [b] + [DeviceBatch(eng, w) for _ in range(copies - 1)]
    for x in batches[1:]:
        x.fill()
    torch.cuda.synchronize()
    reps = 3
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
    for e in evs:
        e[0].record(stream)
        for x in batches:
            x.seal(stream=stream)
        e[1].record(stream)
        for x in batches:
            x.open(stream=stream, counters_out=False)
        e[2].record(stream)
    torch.cuda.synchronize()
    if verify:
        for x in batches:
            assert (x.status[: w.n] == 0).all().item(), "open failed in the cold-cache pass"
    seal_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / (reps * copies)
    open_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / (reps * copies)
    pay = w.payload_bytes
    return {"copies": copies, "working_set_mb": round(copies * w.buf_bytes / 1e6, 1),
            "seal_ms": round(seal_ms, 5), "open_ms": round(open_ms, 5),
            "gib_s": round(2 * pay / ((seal_ms + open_ms) / 1e3) / 2**30, 3)}


def expected_payload(w, k: int) -> np.ndarray:
    """Synthetic plaintext of packet k (the generator of rustyguard_amd/workloads.py)."""
    from rustyguard_amd import workloads

    P = int(w.desc["len"][k])
    words = workloads.mix64(np.uint64(w.data_seed) + (np.uint64(k) << np.uint64(16)) +
                            np.arange((P + 7) // 8, dtype=np.uint64))
    out = words.astype("<u8").view(np.uint8)[:P].copy()
    out[int(w.inner_len[k]):] = 0
    return out


def strict_check(w, b, stream):
    """Outside the timed region: one more seal and open with the statuses preset to a sentinel (a
    kernel that skipped a packet would leave it), and a sample of frames checked byte for byte --
    sealed: header {4, receiver, counter} and payload != plaintext; opened: payload == plaintext."""
    import torch

    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([[0, w.n - 1], rng.choice(w.n, min(w.n, 254), replace=False)]))
    exp = {int(k): expected_payload(w, int(k)) for k in idx}

    def frames():
        out = {}
        for k in idx:
            o, p = int(w.desc["offset"][k]), int(w.desc["len"][k])
            out[int(k)] = b.buf[o:o + p + 32].cpu().numpy()
        return out

    b.status.fill_(0xEE)
    b.seal(stream=stream)
    torch.cuda.synchronize()
    assert (b.status[: w.n] == 0).all().item(), "seal skipped or failed packets"
    for k, fr in frames().items():
        hdr = np.frombuffer(fr[:16].tobytes(), "<u4")
        key = int(w.desc["key_idx"][k])
        assert hdr[0] == 4 and hdr[1] == int(w.receivers[key]), f"seal header of packet {k}"
        assert int(hdr[2]) | (int(hdr[3]) << 32) == int(w.counters[k]), f"seal counter of packet {k}"
        if len(exp[k]) >= 16:
            assert not np.array_equal(fr[16:16 + len(exp[k])], exp[k]), f"packet {k} left in plaintext"
    b.status.fill_(0xEE)
    b.open(stream=stream, counters_out=False)
    torch.cuda.synchronize()
    assert (b.status[: w.n] == 0).all().item(), "open skipped or failed packets"
    for k, fr in frames().items():
        assert np.array_equal(fr[16:16 + len(exp[k])], exp[k]), f"open did not restore packet {k}"


def bench_single_process(args):
    """--single-process: the bench line of one process driving --gpus N GPUs through an rg_group."""
    import torch

    if "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
        print("bench.py: --single-process is one process; do not launch it under torch.distributed.run",
              file=sys.stderr)
        sys.exit(2)
    share = os.environ.get("RG_BENCH_SHARE_GPU") == "1"
    ndev = torch.cuda.device_count()
    if not share and ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {ndev} GPU(s) visible", file=sys.stderr)
        sys.exit(2)
    devices = [0] * args.gpus if share else list(range(args.gpus))
    sp = single_process_run(devices, args.steps, args.warmup, args.verify)
    out = {"metric": METRIC, "value": sp["gib_s"], "unit": "GiB/s", "n_gpus": args.gpus, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": sp["ms_per_step"], "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (SplitMix64 payload, fixed-seed keys; rustyguard_amd/workloads.py)",
           "config": {"workload": "cfg5: " + __import__("rustyguard_amd.workloads", fromlist=["CONFIGS"]).CONFIGS["cfg5"]
                                  + f" (strong split over {args.gpus} GPU(s), one process, one thread)",
                      "parallelism": f"group{args.gpus} (one rg_ctx per GPU, no collective)"},
           "mpkt_s": sp["mpkt_s"], "single_process": sp}
    try:
        out["e2e_multi"] = e2e_multi_run(devices, verify=args.verify)
    except Exception as e:  # the device-resident line stands without it
        out["e2e_multi"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if share:
        out["rehearsal"] = f"RG_BENCH_SHARE_GPU=1: {args.gpus} contexts on one GPU -- not a scaling measurement"
    print(json.dumps(out), flush=True)


def run_legs(rank: int, world: int, workload: str, args) -> list:
    """What a rank runs after the timed steps.  With N > 1 rank 0 also makes the line self-contained:
    the same workload's whole batch on its one GPU (the strong-scaling base, `base_1gpu`) and the CPU
    baselines; the other ranks wait at the final barrier."""
    legs = ["timed"]
    if rank == 0:
        if world > 1 and workload == "cfg5":
            legs.append("base_1gpu")
            legs.append("single_process")
            legs.append("e2e_multi")
        if args.cpu_seconds > 0:
            legs.append("cpu_baseline")
    return legs


def base_one_gpu(eng, steps: int = 3):
    """Config 5's whole 8 Mi-packet batch sealed and opened on this rank's GPU alone (graph-replayed
    steps, as the timed region): the 1-GPU base of the strong-scaling split, measured in the same run."""
    import torch

    from rustyguard_amd import workloads
    from rustyguard_amd.device import DeviceBatch

    w = workloads.build("cfg5", 0, 1)
    b = DeviceBatch(eng, w)
    b.fill()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    b.seal(stream=s)
    b.open(stream=s, counters_out=False)  # warm-up (planner state, caches)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        b.seal(stream=s)
        b.open(stream=s, counters_out=False)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ok = bool((b.status[: w.n] == 0).all().item())
    out = {"workload": f"cfg5 whole batch ({w.n} packets) on one GPU", "steps": steps,
           "gib_s": round(2 * w.payload_bytes * steps / el / 2**30, 3), "ms_per_step": round(el / steps * 1e3, 4),
           "statuses_ok": ok}
    del b
    torch.cuda.empty_cache()
    return out


def single_process_run(devices, steps: int, warmup: int, verify: bool = True):
    """One process and one thread driving every GPU of `devices` (include/rg_aead.h "several GPUs, one
    thread": an rg_group with a context per device): config 5's strong split, shard k on device k, device
    resident; a step is the seal of every shard then the open of every shard, each enqueued on the
    shard's own stream by rg_seal_batch_dev_multi / rg_open_batch_dev_multi.  Timed by the host clock
    between full synchronisations of every device (as the step loop above)."""
    import torch

    from rustyguard_amd import workloads
    from rustyguard_amd.aead import Group
    from rustyguard_amd.device import DeviceBatch

    g = Group(devices)
    n = len(devices)
    batches, streams = [], []
    for k, d in enumerate(devices):
        w = workloads.build("cfg5", k, n)
        with torch.cuda.device(d):
            s = torch.cuda.Stream(device=d)
            b = DeviceBatch(g.engine(k), w, device=f"cuda:{d}")
            b.fill(stream=s)
        batches.append(b)
        streams.append(s)
    seal = Group.shards([{"keys": b.keys, "receivers": b.receivers, "desc": b.desc_seal, "counters": b.counters,
                          "buf": b.buf, "status": b.status, "stream": s} for b, s in zip(batches, streams)], True)
    opn = Group.shards([{"keys": b.keys, "desc": b.desc_open, "buf": b.buf, "status": b.status, "stream": s}
                        for b, s in zip(batches, streams)], False)

    def sync():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    def step():
        g.seal_dev(seal)
        g.open_dev(opn)

    for _ in range(max(warmup, 1)):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    el = time.perf_counter() - t0
    ok = all(bool((b.status[: b.w.n] == 0).all().item()) for b in batches) if verify else None
    payload = sum(b.w.payload_bytes for b in batches)
    out = {"devices": list(devices), "contexts": n, "steps": steps, "packets": sum(b.w.n for b in batches),
           "gib_s": round(2 * payload * steps / el / 2**30, 3), "ms_per_step": round(el / steps * 1e3, 4),
           "mpkt_s": round(2 * sum(b.w.n for b in batches) * steps / el / 1e6, 3), "statuses_ok": ok,
           "how": "one thread: rg_seal_batch_dev_multi + rg_open_batch_dev_multi per step over an rg_group, "
                  "host clock between full device synchronisations"}
    del batches, seal, opn
    g.close()
    torch.cuda.empty_cache()
    return out


def e2e_multi_run(devices, reps: int = 3, verify: bool = True):
    """Packets that start and end in pinned host memory (the reference's UDP buffers,
    rustyguard-tun/src/main.rs:41-57), driven over several GPUs from ONE calling thread (the reference's
    single event loop, rustyguard-core/src/lib.rs:349-352): rg_seal_batch_host_multi then
    rg_open_batch_host_multi on config 5's whole batch (8 Mi x 1500 B, 12.9 GB of frames) in one host
    buffer whose parts sit on their contexts' NUMA nodes, pinned (aead.placed_host_buffer; the line's
    `placement`), split by equal work over the group's contexts (one per entry of `devices`), each
    running its own three-stream H2D -> kernel -> D2H slice pipeline from a worker thread of the library
    (round 5; no context waits on another's GPU).  Beside it the same batch through one context (device
    devices[0]) -- the e2e speed-up of the group.  Median of `reps` timed passes after one warm pass;
    every open must verify, and sampled payloads must come back to what they were before the first seal."""
    from rustyguard_amd import workloads
    from rustyguard_amd.aead import Group, placed_host_buffer

    w = workloads.build("cfg5", 0, 1)
    # the frames placed per part on each context's NUMA node and pinned (round 6)
    g0 = Group(list(devices))
    try:
        buf, placement = placed_host_buffer(g0, w.desc, w.buf_bytes)
    finally:
        g0.close()
    od = w.open_desc()
    rng = np.random.default_rng(11)
    pick = np.unique(np.concatenate([[0, w.n - 1], rng.choice(w.n, 256, replace=False)]))
    before = {int(k): buf[int(w.desc["offset"][k]) + 16:int(w.desc["offset"][k]) + 16 + int(w.desc["len"][k])].copy()
              for k in pick}
    out = {"workload": f"cfg5 whole batch ({w.n} packets, {w.buf_bytes / 1e9:.1f} GB of frames) in pinned host memory",
           "reps": reps, "placement": placement}
    runs = [("group", list(devices))] + ([("one_context", [devices[0]])] if len(devices) > 1 else [])
    for name, devs in runs:
        g = Group(devs)
        try:
            g.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)  # warm: slot buffers, key tables
            st, _ = g.open_host(w.keys, od, buf)
            assert (st == 0).all(), "e2e warm open"
            ts, to = [], []
            for _ in range(reps):
                t0 = time.perf_counter()
                st = g.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)
                t1 = time.perf_counter()
                so, _ = g.open_host(w.keys, od, buf)
                t2 = time.perf_counter()
                if verify:
                    assert (st == 0).all() and (so == 0).all(), "e2e seal/open statuses"
                ts.append(t1 - t0)
                to.append(t2 - t1)
        finally:
            g.close()
        tsm, tom = sorted(ts)[reps // 2], sorted(to)[reps // 2]
        out[name] = {"devices": devs, "seal_gib_s": round(w.payload_bytes / tsm / 2**30, 3),
                     "open_gib_s": round(w.payload_bytes / tom / 2**30, 3),
                     "seal_open_gib_s": round(2 * w.payload_bytes / (tsm + tom) / 2**30, 3),
                     "seal_mpkt_s": round(w.n / tsm / 1e6, 3), "open_mpkt_s": round(w.n / tom / 1e6, 3),
                     "wire_gb_s_per_dir": round(w.wire_bytes / min(tsm, tom) / 1e9, 2),
                     "seal_s": round(tsm, 4), "open_s": round(tom, 4)}
    if verify:
        for k, v in before.items():
            o = int(w.desc["offset"][k]) + 16
            assert np.array_equal(buf[o:o + len(v)], v), f"e2e packet {k} not restored by seal + open"
    if "one_context" in out:
        out["speedup"] = round(out["group"]["seal_open_gib_s"] / out["one_context"]["seal_open_gib_s"], 3)
    out["how"] = ("one calling thread: rg_{seal,open}_batch_host_multi over an rg_group (the library drives each context's "
                  "pipeline from a worker thread of its own), 8 MiB slices, 3 slots per context, "
                  "descriptors/counters/statuses in mapped host memory; host clock per call, median of reps")
    del buf
    return out


def load_traffic(workload: str):
    p = os.path.join(REPO, "profiles", f"pmc_{workload}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if args.single_process:
        bench_single_process(args)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and args.workload != "cfg1":
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.workload != "cfg1" and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
              f"{world}-rank run as {args.gpus} GPUs", file=sys.stderr)
        sys.exit(2)
    if args.workload == "cfg1":
        bench_cfg1(args)
        return
    if args.cpu_study:
        cpu_study(args)
        return
    workload = args.workload or ("cfg2" if world == 1 else "cfg5")
    if args.dry_run:
        plan = {"rank": int(os.environ.get("RANK", "0")), "world": world, "gpus": args.gpus,
                "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "workload": workload}
        if world > 1:
            plan["legs"] = run_legs(plan["rank"], world, workload, args)
        plan["forged"] = forged_fracs(args.forged)  # forged-open legs after the timed region
        line = json.dumps(plan) + "\n"
        os.write(1, line.encode())  # one write: ranks sharing the pipe never interleave a line
        return
    import torch

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the N > 1 path on a one-GPU box (RG_BENCH_SHARE_GPU=1): every rank on device 0, the
    # bookkeeping collectives over gloo on CPU tensors (RCCL refuses two ranks on one GPU).  Never a
    # scaling measurement: the ranks share one GPU, and the line says so.
    share = os.environ.get("RG_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    torch.cuda.set_device(local)
    dist = None
    coll_dev = "cuda"
    if world > 1:
        import torch.distributed as dist

        if share:
            dist.init_process_group("gloo")
            coll_dev = "cpu"
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    # CPU-side barrier for the end of the run: ranks waiting for rank 0's extra legs must not hold a
    # spinning RCCL kernel on their GPUs while rank 0's single-process leg runs there
    cpu_group = dist.new_group(backend="gloo") if dist is not None else None

    from rustyguard_amd import workloads
    from rustyguard_amd.aead import Engine
    from rustyguard_amd.device import DeviceBatch

    def configured_engine():
        e = Engine(local)
        if args.lanes:
            e.set_lanes_per_packet(args.lanes)
        if args.wg_per_cu:
            e.set_wg_per_cu(args.wg_per_cu)
        if args.debug_mode:
            e.set_debug_mode(args.debug_mode)
        if args.staged != -1:
            e.set_staged(args.staged)
        if args.plan >= 0:
            e.set_plan(args.plan)
        if args.segments:
            e.set_segments(args.segments)
        return e

    eng = configured_engine()
    eng_open = configured_engine() if args.split > 1 else eng  # opens run beside seals: own planner scratch
    if workload == "cfg5":
        w = workloads.build("cfg5", rank, world)  # strong split of the 8 Mi batch
    else:
        w = workloads.build(workload)
    if args.frame_shift:  # layout experiment: every frame moved by the same 16-B multiple
        assert args.frame_shift % 16 == 0
        w.desc["offset"] += np.uint64(args.frame_shift)
        w.buf_bytes += args.frame_shift
    b = DeviceBatch(eng, w)
    b.fill()
    torch.cuda.synchronize()

    # One step = seal the batch then open it (both in place).  With --split K the batch is K
    # contiguous packet ranges: seal of range k runs on the step's stream, open of range k on a
    # second stream once that seal is done, so open k overlaps seal k+1 and each launch's ramp-down
    # and write drain hide behind the next one (the same packets, the same work).
    # Captured once into a HIP graph (torch.cuda.CUDAGraph drives HIP stream
    # capture) and replayed, so launch latency does not sit between steps.
    ostream = torch.cuda.Stream()
    parts = b.parts(args.split) if args.split > 1 else None

    def enqueue(s_):
        if parts is None:
            b.seal(stream=s_)
            b.open(stream=s_, counters_out=False)
            return
        ostream.wait_stream(s_)
        for p in parts:
            b.seal(stream=s_, part=p)
            ev = torch.cuda.Event()
            ev.record(s_)
            ostream.wait_event(ev)
            b.open(stream=ostream, counters_out=False, part=p, engine=eng_open)
        s_.wait_stream(ostream)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(max(args.warmup, 1)):
            enqueue(side)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            enqueue(torch.cuda.current_stream())
        graph.replay()
        torch.cuda.synchronize()
    stream = torch.cuda.current_stream()

    def step():
        if graph is not None:
            graph.replay()
        else:
            enqueue(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    step_ms = e0.elapsed_time(e1) / args.steps
    if args.verify:
        assert (b.status[: w.n] == 0).all().item(), "open failed after timed steps"

    # per-kernel timing for the roofline: seal -> open pairs on the step's batch
    # (the same work and cache state as a step), one HIP event pair around each
    # launch on the launch stream, averaged over the pairs.  The stream is first held
    # by a spin kernel while every pair is enqueued, so that the GPU runs them back to
    # back: an event then brackets the kernel, not the host's time to submit it.
    reps = max(args.steps, 10)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(reps)]
    with torch.cuda.stream(stream):
        torch.cuda._sleep(int(2e7))  # ~10 ms of GPU clock cycles: longer than enqueueing the pairs
    for e in evs:
        e[0].record(stream)
        b.seal(stream=stream)
        e[1].record(stream)
        e[2].record(stream)
        b.open(stream=stream, counters_out=False)
        e[3].record(stream)
    torch.cuda.synchronize()
    seal_each = sorted(e[0].elapsed_time(e[1]) for e in evs)
    open_each = sorted(e[2].elapsed_time(e[3]) for e in evs)
    seal_ms = sum(seal_each) / reps
    open_ms = sum(open_each) / reps
    if args.verify:
        assert (b.status[: w.n] == 0).all().item(), "open failed in the kernel-timing pass"
    cold = cold_cache_timing(eng, w, b, stream, args.verify) if args.cold and w.buf_bytes < MALL_BYTES else None
    forged = [forged_open_timing(w, b, stream, f, args.verify) for f in forged_fracs(args.forged)] or None
    copy_ceiling = hbm_copy_rate(stream) if rank == 0 else None
    if args.verify:
        strict_check(w, b, stream)

    t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    tmax = float(t.item())

    payload = w.payload_bytes
    total_payload = 2 * payload * args.steps * world  # seal + open
    total_pkts = 2 * w.n * args.steps * world
    value = total_payload / tmax / 2**30
    seal_alg = 2 * payload + 32 * w.n        # read P, write P + header + tag
    open_alg = 2 * payload + 33 * w.n        # read P + header + tag, write P + status
    dominant = "seal" if seal_ms >= open_ms else "open"
    dom_ms, dom_alg = (seal_ms, seal_alg) if dominant == "seal" else (open_ms, open_alg)
    achieved = dom_alg / (dom_ms / 1e3) / 1e9
    pmc = load_traffic(workload)
    traffic = None
    # only counters of the kernel family this run used (a kernel change makes them stale)
    if pmc and pmc.get(dominant) and pmc[dominant].get("family") == eng.last_kernel():
        traffic = pmc[dominant].get("hbm_bytes_per_launch")
        n_pmc = pmc[dominant].get("packets_per_launch")
        if traffic and n_pmc and n_pmc != w.n:
            # counters taken on another shard size of the same geometry (config 5 on one GPU vs a rank's
            # shard): HBM bytes per packet carried over
            traffic = int(round(traffic * w.n / n_pmc))

    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(tmax / args.steps * 1e3, 4),
        "gpu_ms_per_step": round(step_ms, 5),
        "graph": graph is not None,
        "higher_is_better": True,
        "scaling": "strong" if workload == "cfg5" else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (SplitMix64 payload, fixed-seed keys; rustyguard_amd/workloads.py)",
        "config": {"workload": f"{w.name}: {workloads.CONFIGS[w.name]}" +
                               (f" (strong split: {w.meta['total']} packets over {world} GPU(s), "
                                f"{w.n} per GPU)" if workload == "cfg5" else ""),
                   "packets_per_gpu": w.n,
                   "payload_bytes_per_packet": int(w.desc["len"][0]) if w.n else 0,
                   "mean_payload_bytes": round(payload / max(w.n, 1), 2), "wire_bytes_per_gpu": w.wire_bytes,
                   "sessions": int(w.meta.get("sessions", 1)), "parallelism": f"split{world} (no collective)",
                   "kernel": kernel_label(args, eng, w), "split": args.split,
                   "wg_per_cu": args.wg_per_cu or "auto"},
        "mpkt_s": round(total_pkts / tmax / 1e6, 3),
        "seal_ms": round(seal_ms, 5),
        "open_ms": round(open_ms, 5),
        "seal_ms_median": round(seal_each[reps // 2], 5),  # the median beside the mean
        "open_ms_median": round(open_each[reps // 2], 5),
        "seal_gib_s": round(payload / (seal_ms / 1e3) / 2**30 * world, 3),
        "open_gib_s": round(payload / (open_ms / 1e3) / 2**30 * world, 3),
        "seal_mpkt_s": round(w.n / (seal_ms / 1e3) / 1e6 * world, 3),
        # the same rate counted in wire bytes W = P + 32 per packet (header + tag), SURVEY §8(d)
        "wire_gib_s": round(2 * w.wire_bytes * args.steps * world / tmax / 2**30, 3),
    }
    ceil_gbs = valu_ceiling_gbs(w.desc["len"], False)
    out["roofline"], out["valu_roofline"] = rooflines(dominant, achieved, dom_alg, traffic, payload / (seal_ms / 1e3) / 1e9,
                                                      ceil_gbs, KERNEL_CLOCK_GHZ.get(workload))
    if pmc:
        out["roofline"]["pmc_source"] = pmc.get("source")
    if copy_ceiling:
        # the spec peak stays the denominator; the copy rate is what a plain streaming kernel reaches here
        out["roofline"]["copy_achievable"] = copy_ceiling
        out["roofline"]["frac_of_copy"] = round(achieved / copy_ceiling["gb_s"], 4)
    if cold:
        # the cold-cache leg's own HBM roofline fraction (the step above runs on a cache-resident batch)
        cold_dom_ms = cold["seal_ms"] if dominant == "seal" else cold["open_ms"]
        cold["roofline"] = {"kernel": dominant, "achieved": round(dom_alg / (cold_dom_ms / 1e3) / 1e9, 2),
                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(dom_alg / (cold_dom_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        cold["vs_warm"] = {"seal": round(cold["seal_ms"] / seal_ms, 3), "open": round(cold["open_ms"] / open_ms, 3),
                           "gib_s": round(cold["gib_s"] / (2 * payload / ((seal_ms + open_ms) / 1e3) / 2**30), 3)}
        out["cold_cache"] = cold
    if forged:
        out["forged_open"] = forged
    # the host path (never `value`), on request: its 8 MiB slice launches would otherwise sit in a rocprofv3
    # summary of the default command beside the batch launches the roofline is quoted on (round 4:
    # profiles/r4_default_kernel_stats.csv, average 62 us against 78 us); a failure there is reported, not fatal
    if rank == 0 and args.e2e:
        try:
            out["e2e"] = e2e_host(eng, w, b)
        except Exception as e:  # noqa: BLE001 -- an auxiliary leg: the line stands without it
            out["e2e"] = {"error": repr(e)[:300]}
    legs = run_legs(rank, world, workload, args)
    if world == 1 and workload == "cfg2":
        out["note"] = ("N = 1 runs BASELINE config 2 (the configuration the metric is quoted on); N > 1 runs config 5's "
                       "strong split, whose line carries its own 1-GPU base (base_1gpu) and speed-up")
    if "base_1gpu" in legs:
        del b
        torch.cuda.empty_cache()
        base = base_one_gpu(eng)
        out["base_1gpu"] = base
        out["base_1gpu_gib_s"] = base["gib_s"]
        out["speedup"] = round(value / base["gib_s"], 3) if base["gib_s"] else None
    if "single_process" in legs:
        # the same split driven by ONE process and ONE thread over every GPU (rg_group), beside the
        # one-process-per-GPU value above; the other ranks wait on a CPU barrier meanwhile
        devs = [0] * world if share else list(range(world))
        if not share and torch.cuda.device_count() < world:
            out["single_process"] = {"skipped": f"rank 0 sees {torch.cuda.device_count()} GPU(s), not {world}"}
        else:
            try:
                out["single_process"] = single_process_run(devs, max(3, min(args.steps, 10)), 2, args.verify)
            except Exception as e:  # an extra leg: never lose the timed line for it
                out["single_process"] = {"error": f"{type(e).__name__}: {e}"}
    if "e2e_multi" in legs:
        # packets from and to pinned host memory over every GPU, one thread; the other
        # ranks wait on the CPU barrier meanwhile
        devs = [0] * world if share else list(range(world))
        if not share and torch.cuda.device_count() < world:
            out["e2e_multi"] = {"skipped": f"rank 0 sees {torch.cuda.device_count()} GPU(s), not {world}"}
        else:
            try:
                out["e2e_multi"] = e2e_multi_run(devs, verify=args.verify)
            except Exception as e:  # an extra leg: never lose the timed line for it
                out["e2e_multi"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if "cpu_baseline" in legs:
        port, ossl = cpu_baselines(w, args.cpu_seconds, all_core_threads(args.cpu_threads))
        out["cpu_baseline"] = port
        if ossl:
            out["cpu_openssl"] = ossl
    if share and world > 1:
        out["rehearsal"] = (f"RG_BENCH_SHARE_GPU=1: {world} ranks shared one GPU over gloo -- a functional rehearsal of "
                            "the N > 1 path, not a scaling measurement")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier(group=cpu_group)  # the other ranks wait (on the CPU) for rank 0's extra legs
        dist.destroy_process_group()


def pcie_ceiling(nbytes: int):
    """Pinned-host <-> device copy rates: H2D alone, D2H alone and both directions at once -- the ceiling
    the end-to-end path is measured against.  Measured by tools/build/pcie (tools/pcie.hip, built by
    __graft_entry__.build()) in a child process: hipMemcpyAsync on two hipStreamNonBlocking streams it
    creates first, timed with HIP events.  In this process the same copies on two of torch's streams ran
    the two directions one after the other (28.5 GB/s per direction against pcie.hip's 48), with torch's
    pinned buffers and with hipHostMalloc ones alike -- most likely the two pool streams we were handed
    share one of the process's GPU_MAX_HW_QUEUES=4 hardware queues (not verified).  The in-process figure is kept as the fallback when the tool is absent
    and is labelled as the lower bound it is."""
    import subprocess

    tool = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "build", "pcie")
    if os.path.exists(tool):
        try:
            p = subprocess.run([tool, str(max(1, nbytes >> 20))], capture_output=True, text=True, timeout=120)
            if p.returncode == 0:
                d = json.loads(p.stdout.strip().splitlines()[-1])
                g = d["gb_s_per_direction"]
                return {"h2d_gb_s": g["h2d_copy"], "d2h_gb_s": g["d2h_copy"], "bidir_gb_s_per_dir": g["both_copies"],
                        "bidir_16MiB_pieces_gb_s_per_dir": g["both_copies_16MiB_pieces"], "bytes": d["bytes"],
                        "how": "tools/build/pcie in a child process: hipMemcpyAsync on two non-blocking streams, "
                               "hipHostMalloc buffers, HIP events"}
            print(f"pcie tool failed ({p.returncode}): {p.stderr[-500:]}", file=sys.stderr)
        except (OSError, subprocess.SubprocessError, ValueError, KeyError, IndexError) as e:
            print(f"pcie tool failed: {e!r}", file=sys.stderr)
    try:
        return dict(_pcie_in_process(nbytes), lower_bound=True)
    except (OSError, RuntimeError) as e:  # the ceiling only: the e2e rates stand without it
        return {"error": f"in-process PCIe ceiling failed: {e!r}"[:300]}


def _pcie_in_process(nbytes: int):
    """Fallback: the copies on two of torch's streams (may share a hardware queue, so `bidir` is a lower
    bound)."""
    import ctypes

    import torch

    hip = None
    for name in ("libamdhip64.so.7", "libamdhip64.so.6", "libamdhip64.so"):  # torch's HIP runtime (the loaded copy)
        try:
            hip = ctypes.CDLL(name)
            break
        except OSError:
            continue
    if hip is None:
        return {"error": "libamdhip64 not loadable: no in-process PCIe ceiling"}
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipMemcpyAsync.restype = ctypes.c_int
    h_src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def copy(dst, src, kind, s):  # kind 1: host -> device, 2: device -> host
        rc = hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()), nbytes, kind,
                                ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipMemcpyAsync failed: {rc}")

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        return sorted(t)[reps // 2]

    def h2d():
        copy(d_a, h_src, 1, s1)

    def d2h():
        copy(h_dst, d_b, 2, s2)

    def both():
        h2d()
        d2h()

    t_h2d, t_d2h, t_both = timed(h2d), timed(d2h), timed(both)
    return {"h2d_gb_s": round(nbytes / t_h2d / 1e9, 2), "d2h_gb_s": round(nbytes / t_d2h / 1e9, 2),
            "bidir_gb_s_per_dir": round(nbytes / t_both / 1e9, 2), "bytes": nbytes,
            "how": "hipMemcpyAsync on two torch streams, pinned buffers, median of 5"}


def e2e_host(eng, w, b):
    """Packets that start and end in pinned host memory (a UDP socket buffer): rg_{seal,open}_batch_host,
    H2D -> kernel -> D2H pipelined over three streams in 8 MiB slices, so one slice's upload runs beside
    another's download.  Rates per PCIe direction are the wire bytes W = P + 32 moved each way."""
    import torch

    from rustyguard_amd.aead import host_alloc

    buf = host_alloc(w.buf_bytes)
    b.fill()  # the synthetic plaintext frames, generated on the device and copied to the pinned buffer
    torch.cuda.synchronize()
    torch.from_numpy(buf).copy_(b.buf[: w.buf_bytes])
    od = w.open_desc()
    eng.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)  # warm
    eng.open_host(w.keys, od, buf)
    reps = 5
    ts, to = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        eng.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)
        t1 = time.perf_counter()
        st, _ = eng.open_host(w.keys, od, buf)
        t2 = time.perf_counter()
        assert (st == 0).all()
        ts.append(t1 - t0)
        to.append(t2 - t1)
    tsm, tom = sorted(ts)[reps // 2], sorted(to)[reps // 2]
    p, wire = w.payload_bytes, w.wire_bytes
    ceil = pcie_ceiling(min(w.buf_bytes, 256 << 20))
    return {"seal_gib_s": round(p / tsm / 2**30, 3), "open_gib_s": round(p / tom / 2**30, 3),
            "seal_mpkt_s": round(w.n / tsm / 1e6, 3), "open_mpkt_s": round(w.n / tom / 1e6, 3),
            "seal_gb_s_per_dir": round(wire / tsm / 1e9, 2), "open_gb_s_per_dir": round(wire / tom / 1e9, 2),
            "pcie_ceiling": ceil,
            "note": "pinned hipHostMalloc frames, H2D+kernel+D2H over 3 streams, 8 MiB slices, descriptors/counters/statuses in mapped host memory; median of 5"}


if __name__ == "__main__":
    main()
