"""CPU checks of the single-process multi-GPU split (rg_split_batch, include/rg_aead.h "several GPUs,
one thread"): contiguous index ranges of about equal AEAD work, computed on the host before anything is
enqueued (packets are independent, so any split gives the one-context result)."""
import numpy as np
import pytest

from rustyguard_amd import aead, workloads


def _work(desc, open_=False):
    P = desc["len"].astype(np.int64) - (32 if open_ else 0)
    return np.clip(P, 0, 1 << 20) + 64


@pytest.mark.parametrize("parts", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_split_is_contiguous_and_balanced(parts, cfg):
    w = workloads.build(cfg)
    b = aead.split_batch(w.desc, parts)
    assert b[0] == 0 and b[-1] == w.n and (np.diff(b) >= 0).all()
    wk = _work(w.desc)
    per = np.array([wk[b[k]:b[k + 1]].sum() for k in range(parts)])
    # each part within one packet's work of the ideal share
    assert np.abs(per - wk.sum() / parts).max() <= wk.max()


def test_split_open_counts_the_frame_overhead_out():
    w = workloads.build("cfg3")
    od = w.open_desc()
    assert np.array_equal(aead.split_batch(od, 4, open_=True), aead.split_batch(w.desc, 4))


def test_split_small_and_empty_batches():
    d = np.zeros(3, dtype=workloads.DESC_DTYPE)
    d["len"] = [1504, 16, 0]
    b = aead.split_batch(d, 8)
    assert b[0] == 0 and b[-1] == 3 and (np.diff(b) >= 0).all()
    e = np.zeros(0, dtype=workloads.DESC_DTYPE)
    assert list(aead.split_batch(e, 4)) == [0, 0, 0, 0, 0]
