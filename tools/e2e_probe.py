#!/usr/bin/env python3
"""Round 4: the host-memory path (rg_{seal,open}_batch_host) on config 2 by pipeline slice size, against
the link's duplex ceiling (tools/pcie.hip).  Prints one JSON line per slice size: median of 5 seal and open
calls, GiB/s of payload and GB/s of wire bytes per PCIe direction."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustyguard_amd import workloads  # noqa: E402
from rustyguard_amd.aead import Engine, host_alloc  # noqa: E402
from rustyguard_amd.device import DeviceBatch  # noqa: E402

w = workloads.build(sys.argv[1] if len(sys.argv) > 1 else "cfg2")
eng = Engine(0)
b = DeviceBatch(eng, w)
b.fill()
torch.cuda.synchronize()
buf = host_alloc(w.buf_bytes)
torch.from_numpy(buf).copy_(b.buf[: w.buf_bytes])
del b
od = w.open_desc()
for mib in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,4,8,16,32").split(",")]:
    eng.set_host_slice(mib << 20)
    eng.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)
    st, _ = eng.open_host(w.keys, od, buf)
    assert (st == 0).all()
    ts, to = [], []
    for _ in range(5):
        t0 = time.perf_counter()
        eng.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)
        t1 = time.perf_counter()
        st, _ = eng.open_host(w.keys, od, buf)
        t2 = time.perf_counter()
        assert (st == 0).all()
        ts.append(t1 - t0)
        to.append(t2 - t1)
    tsm, tom = sorted(ts)[2], sorted(to)[2]
    print(json.dumps({"workload": w.name, "slice_mib": mib, "seal_ms": round(tsm * 1e3, 3), "open_ms": round(tom * 1e3, 3),
                      "seal_gib_s": round(w.payload_bytes / tsm / 2**30, 2), "open_gib_s": round(w.payload_bytes / tom / 2**30, 2),
                      "seal_gb_s_per_dir": round(w.wire_bytes / tsm / 1e9, 2), "open_gb_s_per_dir": round(w.wire_bytes / tom / 1e9, 2)}),
          flush=True)
