#!/usr/bin/env python3
"""Throughput of the SURVEY 8(f) rows beside the transport AEAD (one MI355X):

  mac1   rg_mac_verify_batch_dev: 1 Mi handshake-initiation messages (148 B), mac1 checked under the
         message's own key, and under an 8-peer scan (RG_KEY_SCAN, wg-proxy)
  rx     rg_open_batch_dev_rx vs rg_open_batch_dev on config 4 frames (256 sessions): the cost of
         resolving every frame's session from its header on the device

Prints one JSON object.  Synthetic data (random messages: every MAC check does the full work and
rejects, which costs the same as accepting)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustyguard_amd import aead, workloads  # noqa: E402
from rustyguard_amd.device import DeviceBatch  # noqa: E402
from rustyguard_amd.workloads import DESC_DTYPE  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    eng = aead.Engine(0)
    out = {}
    # ---------------------------------------------------------------- mac1
    n, L = 1 << 20, 148
    rng = np.random.default_rng(5)
    keys = torch.from_numpy(rng.integers(0, 256, (8, 32), dtype=np.uint8)).cuda()
    desc = np.zeros(n, DESC_DTYPE)
    desc["offset"] = np.arange(n, dtype=np.uint64) * 160
    desc["len"] = L
    desc["key_idx"] = rng.integers(0, 8, n)
    buf = torch.randint(0, 256, (n * 160,), dtype=torch.uint8, device="cuda")
    d = torch.from_numpy(desc.view(np.uint8).reshape(-1, 16)).cuda()
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ms_own = timed(lambda: eng.mac_verify_dev(keys, 1, d, buf, st))
    desc["key_idx"] = aead.KEY_SCAN
    ds = torch.from_numpy(desc.view(np.uint8).reshape(-1, 16)).cuda()
    ms_scan = timed(lambda: eng.mac_verify_dev(keys, 1, ds, buf, st))
    out["mac1"] = {"messages": n, "bytes_each": L, "own_key_ms": round(ms_own, 4),
                   "own_key_mmsg_s": round(n / ms_own / 1e3, 1), "scan8_ms": round(ms_scan, 4),
                   "scan8_mmsg_s": round(n / ms_scan / 1e3, 1)}
    # ------------------------------------------------------------------ rx
    w = workloads.build("cfg4")  # 256 sessions: a real table
    b = DeviceBatch(eng, w)
    b.fill()
    torch.cuda.synchronize()
    table = torch.from_numpy(aead.rx_table(w.receivers, np.arange(len(w.receivers), dtype=np.uint32))).cuda()

    def seal_open(rx):
        b.seal()
        if rx:
            eng.open_dev_rx(b.keys, table, b.desc_open, b.buf, b.status)
        else:
            eng.open_dev(b.keys, b.desc_open, b.buf, b.status)

    # alternating repetitions, medians: box-to-box and run-to-run noise on a 2 ms
    # step is larger than the ~50 us being measured
    t_open, t_rx = [], []
    for _ in range(7):
        t_open.append(timed(lambda: seal_open(False), 10))
        t_rx.append(timed(lambda: seal_open(True), 10))
    assert (b.status[: w.n] == 0).all().item()
    ms_open, ms_rx = float(np.median(t_open)), float(np.median(t_rx))
    out["rx"] = {"workload": "cfg4 (1 Mi packets, 256 sessions)", "seal_open_ms": round(ms_open, 4),
                 "seal_open_rx_ms": round(ms_rx, 4), "resolve_overhead_us": round((ms_rx - ms_open) * 1e3, 2),
                 "note": "medians of 7 alternating repetitions of 10 steps; the rx_resolve kernel itself is in the "
                         "rocprofv3 kernel stats"}
    # ------------------------------------------------------------ sessions
    # the device-resident session layer on config-2 geometry (64 Ki x 1504 B, one session): B seals
    # with rg_send_batch_dev (fresh counters every round), A receives with rg_recv_batch_dev; the host
    # half (rg_recv_batch_dev_finish: in-order anti-replay pass, flags, status write-back) is timed
    # on its own
    import time

    w = workloads.build("cfg2")
    b = DeviceBatch(eng, w)
    b.fill()
    rng = np.random.default_rng(9)
    k1, k2 = rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    sa, sb = aead.Sessions(eng, 4), aead.Sessions(eng, 4)
    slot_a = sa.insert(0x1111, 0x2222, k1, k2)
    slot_b = sb.insert(0x2222, 0x1111, k2, k1)
    slots = np.full(w.n, slot_b, np.uint32)
    t_send, t_gpu, t_fin = [], [], []
    for it in range(12):
        b.fill()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sb.send_batch_dev(slots, b.desc_seal, b.buf, b.status)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        sa.recv_batch_dev(b.desc_open, b.buf, b.status)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        st, sl, fl = sa.recv_batch_dev_finish(w.n)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        assert (st == 0).all() and (sl == slot_a).all()
        if it >= 2:
            t_send.append(t1 - t0)
            t_gpu.append(t2 - t1)
            t_fin.append(t3 - t2)
    med = lambda x: float(np.median(x)) * 1e3  # noqa: E731
    out["sessions"] = {"workload": "cfg2 geometry, one session", "packets": w.n,
                       "send_batch_dev_ms": round(med(t_send), 4), "recv_batch_dev_ms": round(med(t_gpu), 4),
                       "recv_finish_ms": round(med(t_fin), 4),
                       "recv_mpkt_s": round(w.n / (med(t_gpu) + med(t_fin)) / 1e3, 2),
                       "note": "wall-clock medians of 10 rounds, each call followed by a device sync; finish is "
                               "the host's in-order anti-replay pass plus the status write-back"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
