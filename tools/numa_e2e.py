#!/usr/bin/env python3
"""the host path's end-to-end rate with the frames on the GPU's own NUMA node and on the
other node(s) (1-GPU box).  The frame buffer is an anonymous mapping bound to a node with rg_numa_bind
(mbind MPOL_BIND + MPOL_MF_MOVE), first-touched, pinned with rg_host_register, then sealed and opened through
rg_seal_batch_host / rg_open_batch_host (config 2's batch: 64 Ki x 1504-B payloads, 96 MiB of frames) --
median of 5 of each.  Prints one JSON line per node the process may bind to, plus the GPU's node and the
nodes visible (a node the job's cpuset excludes is reported as refused)."""
import ctypes
import json
import mmap
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rustyguard_amd import _lib, workloads  # noqa: E402
from rustyguard_amd.aead import Engine, _vp  # noqa: E402


def nodes():
    base = "/sys/devices/system/node"
    try:
        return sorted(int(d[4:]) for d in os.listdir(base) if d.startswith("node") and d[4:].isdigit())
    except OSError:
        return [0]


def main():
    eng = Engine(0)
    L = eng.library
    gpu_node = L.rg_numa_node(eng.handle)
    w = workloads.build("cfg2")
    plain = np.random.default_rng(1).integers(0, 256, w.buf_bytes, dtype=np.uint8)
    od = w.open_desc()
    out = {"gpu": 0, "gpu_numa_node": gpu_node, "nodes": nodes(), "cpus_allowed": len(os.sched_getaffinity(0)),
           "bytes": int(w.buf_bytes), "runs": []}
    for node in nodes():
        mm = mmap.mmap(-1, w.buf_bytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        buf = np.frombuffer(mm, np.uint8)
        p = buf.ctypes.data_as(ctypes.c_void_p)
        rc = L.rg_numa_bind(p, buf.nbytes, node)
        if rc != 0:
            out["runs"].append({"node": node, "refused": L.rg_last_error().decode()})
            del p, buf  # the exported pointers into the mapping go before it closes
            mm.close()
            continue
        buf[:] = plain  # first touch: the pages land on the bound node
        _lib.check(L.rg_host_register(p, buf.nbytes), "rg_host_register", L)
        seal_t, open_t = [], []
        for _ in range(6):
            t0 = time.perf_counter()
            st = eng.seal_host(w.keys, w.receivers, w.desc, w.counters, buf)
            t1 = time.perf_counter()
            st2, _ = eng.open_host(w.keys, od, buf)
            t2 = time.perf_counter()
            assert (st == 0).all() and (st2 == 0).all()
            seal_t.append(t1 - t0)
            open_t.append(t2 - t1)
        pay = np.ones(w.buf_bytes, bool)  # the payload bytes: sealed then opened in place -> back to plain
        for o in range(0, w.buf_bytes, 1536):
            pay[o:o + 16] = False
            pay[o + 1520:o + 1536] = False
        ok = bool(np.array_equal(buf[pay], plain[pay]))
        _lib.check(L.rg_host_unregister(p), "rg_host_unregister", L)
        sm, om = sorted(seal_t[1:])[2], sorted(open_t[1:])[2]
        pay = w.payload_bytes
        out["runs"].append({"node": node, "local": node == gpu_node, "seal_ms": round(sm * 1e3, 3),
                            "open_ms": round(om * 1e3, 3), "seal_gib_s": round(pay / sm / 2**30, 2),
                            "open_gib_s": round(pay / om / 2**30, 2), "round_trip_ok": ok})
        del p, buf
        mm.close()
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
