#!/usr/bin/env python3
"""Config 3: what the flattened kernel's unit cuts could buy (CPU only, no GPU).

Replays the cooperative search's cut rule (rg_flat.hip: groups of 4096 packets, unit work wpkt + wchk x chunks,
midpoint rule against targets 2 floor(tot (j0 + b) / kgc)) on the config-3 batch for several packet weights,
and prices each unit with the per-wave cycles measured by packet count (profiles/r4_cfg3_perwave_final.txt:
m <= 64 59.7 k, 65-80 62.7 k, 81-92 64.1 k) plus 6.2 k cycles per chunk step beyond six.  The kernel's time
follows the slowest unit."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rustyguard_amd import workloads  # noqa: E402

GROUP, UNITS = 4096, 1024


def cuts(chunks, wpkt, wchk):
    n = len(chunks)
    kgc = UNITS * GROUP // n
    m_out, d_out = [], []
    for g in range(n // GROUP):
        c = chunks[g * GROUP:(g + 1) * GROUP]
        E = np.cumsum(wpkt + wchk * c)
        mid2 = E + np.concatenate([[0], E[:-1]])
        t2 = 2 * np.floor(E[-1] / kgc * np.arange(kgc + 1)).astype(np.int64)
        cnt = np.searchsorted(mid2, t2, side="left")
        cnt[0], cnt[-1] = 0, GROUP
        for j in range(kgc):
            m_out.append(cnt[j + 1] - cnt[j])
            d_out.append(max(int(np.maximum(c[cnt[j]:cnt[j + 1]], 1).sum()), 0))
    return np.array(m_out), np.array(d_out)


def price(m, d):
    steps = (d + 63) // 64
    return 59700 + np.where(m > 64, 3000, 0) + np.where(m > 80, 1400, 0) + np.where(m > 96, 3000, 0) + 6200 * (steps - 6)


def main():
    P = workloads.build("cfg3").desc["len"].astype(np.int64)
    chunks = (P + 63) // 64
    print(f"config 3: {len(P)} packets, chunks per packet {dict((int(a), int(b)) for a, b in zip(*np.unique(chunks, return_counts=True)))}")
    print("wpkt wchk | packets per unit | >64 | >80 | chunks per unit | units > 6 steps | model max / mean cycles")
    for wpkt in (1, 2, 4, 8, 16, 32, 64):
        m, d = cuts(chunks, wpkt, 8)
        c = price(m, d)
        print(f"{wpkt:4d} {8:4d} | {m.min():3d}-{m.max():3d} | {np.mean(m > 64):.2f} | {np.mean(m > 80):.3f} | "
              f"{d.min()}-{d.max()} | {int(np.sum(d > 384)):4d} | {c.max()} / {c.mean():.0f}")
    print("equal packet counts (64 per unit):", end=" ")
    d = np.array([int(chunks[i:i + 64].sum()) for i in range(0, len(chunks), 64)])
    print(f"chunks {d.min()}-{d.max()}, units > 6 steps {int(np.sum(d > 384))}, model max {price(np.full(len(d), 64), d).max()}")


if __name__ == "__main__":
    main()
