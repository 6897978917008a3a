#!/usr/bin/env python3
"""Config 3: a cycle model that bounds the flattened kernel's seal from below, CPU only.

The kernel (rg_flat.hip) runs one wave per SIMD, one unit of whole packets per wave, and the launch lasts as
long as its slowest wave.  The model replays the kernel's unit cut on the config-3 batch (tools/cut_sim.py's
`cuts`, the cooperative search's rule: groups of 4096 packets, work 1 + 8 x chunks, midpoint rule) and gives
every unit each phase at a floor, in two tiers:

  issue floor   the VALU issue cycles of the phase's work at one wave per SIMD, every latency hidden;
  chain floor   the issue floor plus the phase's dependent memory round trips at idle-chip latencies
                (MI355X_MICROARCH.md: HBM miss ~900, L2 hit ~200, LDS ~50 cycles; a workgroup barrier ~100):
                at one wave per SIMD a wave has no other work to issue while its own chain waits.

Per-phase constants and where they come from:
  STEP      4694  one 64-byte chunk step (ChaCha20 block + four Poly1305 blocks + XOR + cursor), the same
                  step code with no memory at all: config 2's pipelined seal in diagnostic mode 1 (compute
                  only), 116 958 cycles per wave (profiles/r5_stamps_ilp.txt) less one key block and the tag,
                  over its 24 steps.
  OTK       3800  one ChaCha20 block per lane (the one-time keys, phase A; profiles/HISTORY.md §8.2).
  QUAD      0.36  x OTK per 16 packets past 64 in a sub-unit (the lane-quad key blocks; rg_flat.hip).
  POW        714  one square-and-multiply step of a carry power (issue-bound: the right-to-left A/B made it
                  longer, profiles/r5_cfg3_pow_r2l_ab.txt): 5.0 k measured for six steps and the final multiply.
  TAGPASS    500  one pass of phase F over 64 packets: fold, length block, one clamped multiply (17
                  v_mad_u64_u32 at 8 cycles), finish (~400 issue cycles) and its LDS reads.
  SEARCH_I   600  the search's own VALU (length transpose, 16-wide serial prefix, one wave scan, the cut
                  ballots: ~150 instructions at 4 cycles).
  SEARCH_L  1500  its chain: kernel-argument loads (276 measured on the open, the shorter of the two),
                  the length loads from HBM (900), the transpose's LDS round trip, the barrier, three
                  dependent LDS round trips of the cut.
  STAGE_I    400  staging's VALU (descriptor checks, two chunk-count scans, the lane markers' scans).
  STAGE_L    550  its chain: descriptors from L2 (200), then the key row that the descriptor names (200),
                  three LDS round trips.
  MISC_A     400  phase A besides the key blocks (headers, status, the LDS rows).
Launch and drain (the launch's event less its waves' span) are taken as measured, not modelled.

Usage: tools/cfg3_floor.py [stamps]   (stamps: a tools/flat_stamps.py output; default the round-6 profile)
Prints the per-phase table (measured mean / slowest wave beside the two floors) and the bound on the seal."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from cut_sim import cuts  # noqa: E402

from rustyguard_amd import workloads  # noqa: E402

STEP, OTK, QUAD, POW, TAGPASS = 4694, 3800, 0.36, 714, 500
SEARCH_I, SEARCH_L, STAGE_I, STAGE_L, MISC_A = 600, 1500, 400, 550, 400
DEFAULT_STAMPS = "profiles/r6_cfg3_flat_stamps.txt"


def unit_shapes(P):
    """Every unit of the kernel's cut: packets m, chunks D, steps S, carry power steps (wave-uniform)."""
    nb = P // 16                                   # data blocks per packet
    ch = np.maximum((nb + 3) // 4, 1)              # chunks (a P = 0 packet holds one empty chunk)
    m_all, d_all = cuts(ch, 1, 8)
    out = []
    s = 0
    for m, _ in zip(m_all, d_all):
        c = ch[s:s + m]
        b = nb[s:s + m]
        cs = np.concatenate([[0], np.cumsum(c)])     # chunk start of each packet, D at the end
        D = int(cs[-1])
        pb = -1
        for lane in range(64):
            hi = ((lane + 1) * D) >> 6
            lo = (lane * D) >> 6
            if hi <= lo:
                continue
            k = int(np.searchsorted(cs, hi - 1, side="right") - 1)   # the packet of the lane's last chunk
            t_end = hi - int(cs[k])                                  # its chunks through this lane
            e = int(b[k]) - 4 * t_end
            if e > 0:
                pb = max(pb, e.bit_length() - 1)
        out.append((int(m), D, (D + 63) // 64, pb))
        s += m
    return out


def floors(m, S, pb):
    if m <= 64:
        extra = 0.0
    elif m <= 96:  # lane quads: 16 key blocks per pass
        extra = np.ceil((m - 64) / 16) * QUAD * OTK
    else:          # a second one-lane pass (sub-units hold at most 128 packets)
        extra = OTK + MISC_A
    a_issue = OTK + MISC_A + extra
    carry = POW * (max(pb, 0) + 1) if pb >= 0 else 0
    tags = TAGPASS * int(np.ceil(m / 64))
    issue = {"search": SEARCH_I, "staging": STAGE_I, "phaseA": a_issue, "phaseC": S * STEP, "carry": carry,
             "phaseF": tags}
    chain = dict(issue)
    chain["search"] += SEARCH_L
    chain["staging"] += STAGE_L
    return issue, chain


def measured(path):
    if not os.path.exists(path):
        return None
    for line in open(path):
        if line.startswith("seal {"):
            return json.loads(line[5:])
    return None


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_STAMPS
    P = workloads.build("cfg3").desc["len"].astype(np.int64)
    units = unit_shapes(P)
    rows = [floors(m, S, pb) for m, _, S, pb in units]
    tot_i = np.array([sum(i.values()) for i, _ in rows])
    tot_c = np.array([sum(c.values()) for _, c in rows])
    worst = int(np.argmax(tot_c))
    ms = np.array([u[0] for u in units])
    print(f"config 3: {len(P)} packets in {len(units)} units; packets per unit {ms.min()}-{ms.max()}, "
          f"steps {sorted(set(u[2] for u in units))}, carry power steps {sorted(set(u[3] for u in units))}")
    meas = measured(path)
    phases = ["search", "staging", "phaseA", "phaseC", "carry", "phaseF"]
    key = {"staging": "stage+scan"}
    print(f"{'phase':8s} | {'measured mean / max':>20s} | {'issue floor':>11s} | {'chain floor':>11s}  (slowest unit: m={units[worst][0]})")
    for ph in phases:
        mm = ""
        if meas:
            d = meas[key.get(ph, ph)]
            mm = f"{d['mean_cyc']:>9d} / {d['max_cyc']:<8d}"
        i, c = rows[worst]
        print(f"{ph:8s} | {mm:>20s} | {int(i[ph]):>11d} | {int(c[ph]):>11d}")
    wt = f"{meas['wave_total']['mean_cyc']} / {meas['wave_total']['max_cyc']}" if meas else ""
    print(f"{'wave':8s} | {wt:>20s} | {int(tot_i.max()):>11d} | {int(tot_c.max()):>11d}")
    if not meas:
        return
    clock = meas["clock_ghz"] * 1e9
    span_end = meas["wall_us_end_pct_0_50_90_100"][3]
    kernel_us = float(os.environ.get("CFG3_SEAL_US", "0")) or None
    drain = (kernel_us - span_end) if kernel_us else None
    fl_i = tot_i.max() / clock * 1e6
    fl_c = tot_c.max() / clock * 1e6
    print(f"kernel clock {meas['clock_ghz']} GHz: slowest wave at its floor {fl_i:.1f} us (issue) / {fl_c:.1f} us "
          f"(chain); measured waves end by {span_end:.1f} us")
    if drain is not None:
        print(f"seal {kernel_us:.2f} us measured (rocprofv3); launch + drain {drain:.2f} us measured -> seal floor "
              f"{fl_i + drain:.1f} us (issue) / {fl_c + drain:.1f} us (chain)")


if __name__ == "__main__":
    main()
