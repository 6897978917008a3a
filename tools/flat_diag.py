#!/usr/bin/env python3
"""Quick correctness probe of the flattened kernel on a few batch sizes (GPU): seal vs oracle,
which waves ran (debug stamps), statuses pre-set to a sentinel so a kernel that does not run shows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from rustyguard_amd import workloads  # noqa: E402
from rustyguard_amd.aead import Engine  # noqa: E402

eng = Engine(0)
eng.set_staged(3)
eng.set_plan(1)
dbg = torch.zeros(8 * 4096, dtype=torch.int64, device="cuda")
eng.set_debug_buffer(dbg)
for n in (1, 7, 3000, 65536):
    w = workloads.imix(n)
    buf = np.zeros(w.buf_bytes, np.uint8)
    oracle.synth_fill(buf, w.desc, w.inner_len, w.data_seed)
    want = buf.copy()
    oracle.seal_batch(w.keys, w.receivers, w.desc, w.counters, want)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    b = t(buf)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    dbg.zero_()
    eng.set_debug_mode(3)
    eng.seal_dev(t(w.keys), t(w.receivers.view(np.int32)), t(w.desc.view(np.uint8).reshape(-1, 16)),
                 t(w.counters.view(np.int64)), b, st)
    torch.cuda.synchronize()
    eng.set_debug_mode(0)
    got = b.cpu().numpy()
    d = dbg.cpu().numpy().reshape(-1, 8)
    ran = np.nonzero(d[:, 7])[0]
    started = np.nonzero((d[:, 6] & 0xFFFF0000) == 0xABCD0000)[0]
    print("started", len(started), "wv values", np.unique(d[started, 6] & 0xFF) if len(started) else None)
    print(n, "status", np.unique(st.cpu().numpy(), return_counts=True), "match", np.array_equal(got, want),
          "waves_ran", len(ran), "min", ran.min() if len(ran) else None, "max", ran.max() if len(ran) else None,
          flush=True)
