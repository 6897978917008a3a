#!/usr/bin/env python3
"""Large-batch diagnostic: seal/open a BASELINE config on one GPU and check samples against the oracle.

  python tools/diag_large.py --workload cfg5 [--n N]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg5")
    ap.add_argument("--n", type=int, default=0)
    a = ap.parse_args()
    import torch

    from oracle import oracle
    from rustyguard_amd import workloads
    from rustyguard_amd.aead import Engine
    from rustyguard_amd.device import DeviceBatch

    w = workloads.build(a.workload) if not a.n else workloads.shard(a.n, 0, 1)
    print("n", w.n, "buf bytes", w.buf_bytes, flush=True)
    eng = Engine(0)
    b = DeviceBatch(eng, w)
    b.fill()
    torch.cuda.synchronize()
    b.seal()
    torch.cuda.synchronize()
    st = b.status[: w.n].cpu().numpy()
    print("seal status histogram", np.bincount(st, minlength=6).tolist(), flush=True)
    # sample packets: first, around 4 GiB boundaries, last
    idx = set(range(0, 64)) | set(range(w.n - 64, w.n))
    off = w.desc["offset"].astype(np.int64)
    for g in range(1, 8):
        k = int(np.searchsorted(off, g << 32))
        idx |= set(range(max(0, k - 70), min(w.n, k + 70)))
    idx = np.array(sorted(i for i in idx if 0 <= i < w.n))
    bad = []
    for i in idx:
        o, P = int(off[i]), int(w.desc["len"][i])
        got = b.buf[o: o + P + 32].cpu().numpy()
        one = np.zeros(1, workloads.DESC_DTYPE)
        one[0] = (0, P, int(w.desc["key_idx"][i]))
        ref = np.zeros(P + 32, np.uint8)
        # plaintext from the generator formula (global index i)
        words = workloads.mix64(np.uint64(w.data_seed) + (np.uint64(i) << np.uint64(16)) +
                                np.arange((P + 7) // 8, dtype=np.uint64))
        pt = words.astype("<u8").view(np.uint8)[:P].copy()
        pt[int(w.inner_len[i]):] = 0
        ref[16:16 + P] = pt
        oracle.seal_batch(w.keys, w.receivers, one, w.counters[i:i + 1], ref)
        if not np.array_equal(got, ref):
            bad.append(i)
    print("sampled", len(idx), "mismatched", len(bad), "first", bad[:10],
          "offsets", [int(off[i]) for i in bad[:5]], flush=True)
    b.open()
    torch.cuda.synchronize()
    st = b.status[: w.n].cpu().numpy()
    print("open status histogram", np.bincount(st, minlength=6).tolist(), flush=True)
    nz = np.nonzero(st)[0]
    if len(nz):
        print("first failing", nz[:10].tolist(), "offsets", off[nz[:10]].tolist(), "last", nz[-3:].tolist(),
              "count", len(nz), flush=True)


if __name__ == "__main__":
    main()
