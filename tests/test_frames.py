"""mpx framing ([u32 BE size][message], mpx/conn_reader.go:179-194): the host frame indexer
against a Python walk of the heads, incomplete tails and capacity limits (CPU, no GPU)."""
from __future__ import annotations

import numpy as np

import spec_amd
from oracle import oracle as O
from spec_amd import FLAT16, workload


def walk(buf):
    p, ends = 0, []
    while p + 4 <= len(buf):
        z = int.from_bytes(bytes(buf[p:p + 4]), "big")
        if p + 4 + z > len(buf):
            break
        p += 4 + z
        ends.append(p)
    return ends, p


def test_frames_index_matches_walk():
    n = 500
    cols, heaps = workload.flat16(n, seed=2)
    stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
    fr = spec_amd.make_frames(stream, ends)
    assert fr.size == stream.size + 4 * n
    got, used = spec_amd.frames_index(fr)
    want, wused = walk(fr)
    assert list(got) == want and used == wused == fr.size
    o_ends, o_used = O.frames_read(fr, n)  # the oracle's mpx read loop
    assert np.array_equal(o_ends, got) and o_used == used
    assert np.array_equal(got, np.cumsum(np.diff(np.concatenate([[0], ends])) + 4))
    # records are recovered exactly
    starts = np.concatenate([[0], got[:-1]]).astype(np.int64) + 4
    for i in range(0, n, 37):
        s0 = int(ends[i - 1]) if i else 0
        assert bytes(fr[starts[i]:got[i]]) == bytes(stream[s0:int(ends[i])])


def test_frames_index_incomplete_and_capacity():
    recs = [b"abc", b"", b"x" * 300]
    buf = b"".join(len(r).to_bytes(4, "big") + r for r in recs)
    arr = np.frombuffer(buf + b"\x00\x00\x01\x00zz", dtype=np.uint8)  # incomplete 4th frame
    got, used = spec_amd.frames_index(arr)
    assert list(got) == [7, 11, 315] and used == 315
    got, used = spec_amd.frames_index(arr, cap=2)
    assert list(got) == [7, 11] and used == 11
    got, used = spec_amd.frames_index(np.zeros(0, np.uint8), cap=1)
    assert len(got) == 0 and used == 0
