"""The CPU baseline loops bench.py times beside the GPU legs (oracle/batch.c *_mt: the reference's
per-record loops on several host threads, contiguous record shards, one output region per
thread): on every thread count they produce exactly the single-threaded oracle's results."""
from __future__ import annotations

import numpy as np
import pytest

import spec_amd
from oracle import oracle as O
from spec_amd import workload


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_encode_flat_mt_matches_serial(threads):
    n = 2000
    s = spec_amd.FLAT16
    cols, heaps = workload.flat16(n, seed=5)
    hl = [heaps.get(f) for f in range(len(s))]
    want, want_ends = O.encode_flat_batch(s.tags, s.kinds, cols, hl, n)
    cap = 4 * want.size + (1 << 16)
    run, out, ends = O.encode_flat_batch_mt(s.tags, s.kinds, cols, hl, n, cap, threads)
    run()
    share = cap // threads
    for t in range(threads):
        r0, r1 = n * t // threads, n * (t + 1) // threads
        base = int(want_ends[r0 - 1]) if r0 else 0
        assert np.array_equal(ends[r0:r1], want_ends[r0:r1] - base)
        assert np.array_equal(out[t * share: t * share + int(ends[r1 - 1])], want[base: int(want_ends[r1 - 1])])


@pytest.mark.parametrize("threads", [1, 4])
def test_nested_mt_matches_serial(threads):
    n = 1500
    w = workload.nested(n, 11)
    stream, ends = O.encode_nested_batch(w)
    want = O.decode_nested_batch(stream, ends)
    enc, dec, out, e2, got = O.nested_batch_mt(w, stream, ends, 4 * stream.size + (1 << 16), threads)
    enc()
    dec()
    share = (4 * stream.size + (1 << 16)) // threads
    for t in range(threads):
        r0, r1 = n * t // threads, n * (t + 1) // threads
        base = int(ends[r0 - 1]) if r0 else 0
        assert np.array_equal(e2[r0:r1], ends[r0:r1] - base)
        assert np.array_equal(out[t * share: t * share + int(e2[r1 - 1])], stream[base: int(ends[r1 - 1])])
    m = int(w["item_begin"][-1])
    for k in ("id", "seq", "name", "status"):
        assert np.array_equal(got[k], want[k]), k
    for k in ("key", "value", "label", "item_status"):
        assert np.array_equal(got[k][:m], want[k]), k
