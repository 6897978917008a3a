"""Device-resident batches: a Workload's arrays copied into HBM as torch tensors.

torch is only plumbing here (allocation, streams, events); every byte of
AEAD work is done by librg_aead's HIP kernels.
"""
from __future__ import annotations

import numpy as np

from .aead import Engine
from .workloads import Workload


class DeviceBatch:
    def __init__(self, engine: Engine, w: Workload, device: str = "cuda"):
        import torch

        self.engine, self.w = engine, w
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        self.keys = t(w.keys.reshape(-1, 32))
        self.receivers = t(w.receivers.view(np.int32))
        self.desc_seal = t(w.desc.view(np.uint8).reshape(-1, 16))
        self.desc_open = t(w.open_desc().view(np.uint8).reshape(-1, 16))
        self.counters = t(w.counters.view(np.int64))
        self.inner_len = t(w.inner_len.view(np.int32))
        self.buf = torch.zeros(w.buf_bytes, dtype=torch.uint8, device=device)
        self.status = torch.zeros(max(w.n, 1), dtype=torch.uint8, device=device)
        self.counters_out = torch.zeros(max(w.n, 1), dtype=torch.int64, device=device)

    def fill(self, stream=None):
        """Synthetic plaintext (see workloads.py) written on the device."""
        self.engine.synth_fill_dev(self.desc_seal, self.inner_len, self.buf, self.w.data_seed, stream=stream)

    def seal(self, stream=None, with_header: bool = True, part=None, engine=None):
        """Seal packets [a, b) when `part` = (a, b) (all of them by default), on `engine` (default: the
        batch's).  Concurrent calls on different streams need different engines: an engine's planner
        scratch is stream-ordered (a second stream while the first one's batch is in flight is refused)."""
        a, b = part if part is not None else (0, self.w.n)
        (engine or self.engine).seal_dev(self.keys, self.receivers if with_header else None, self.desc_seal[a:b],
                                         self.counters[a:b], self.buf, self.status[a:b], stream=stream)

    def open(self, stream=None, counters_out: bool = True, part=None, engine=None):
        a, b = part if part is not None else (0, self.w.n)
        (engine or self.engine).open_dev(self.keys, self.desc_open[a:b], self.buf, self.status[a:b],
                                         self.counters_out[a:b] if counters_out else None, stream=stream)

    def parts(self, k: int):
        """k contiguous packet ranges of near-equal size."""
        n = self.w.n
        return [(i * n // k, (i + 1) * n // k) for i in range(k)]

    def host_buf(self) -> np.ndarray:
        return self.buf.cpu().numpy()
